"""The C ABI (include/render.h): the library loads without a GPU, exports every declared symbol,
and the structs match render-cpp/render.hpp:7-21.  Failure semantics of render.cpp:160-176."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

from swift3drenderer_amd import abi
from swift3drenderer_amd.renderer import LIB_PATH, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, 'include', 'render.h')).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;', text)))


def test_header_declares_the_reference_symbol():
    fns = declared_functions()
    assert 'updateAndRender' in fns
    assert len(fns) >= 10


def test_library_exports_every_declared_symbol():
    lib = load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(['nm', '-D', '--defined-only', LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r' T (\w+)', out))
    assert set(declared_functions()) <= exported


def test_dylib_name_exists():
    # the Swift main loop dlopens "render.dylib" (main.swift:96, Makefile:19)
    assert os.path.exists(os.path.join(os.path.dirname(LIB_PATH), 'render.dylib'))


def test_struct_layouts():
    assert ctypes.sizeof(abi.PixelData) == 24
    assert abi.PixelData.bufferSize.offset == 20
    assert ctypes.sizeof(abi.Input) == 24
    assert abi.Input.mouse_x.offset == 16 and abi.Input.mouse_y.offset == 20


def test_header_compiles_as_c_and_layout_matches(tmp_path):
    src = tmp_path / 't.c'
    src.write_text('#include "render.h"\n#include <stddef.h>\n'
                   '_Static_assert(sizeof(PixelData) == 24, "PixelData");\n'
                   '_Static_assert(sizeof(Input) == 24, "Input");\n'
                   '_Static_assert(offsetof(Input, mouse) == 16, "mouse");\n'
                   'int main(void) { return 0; }\n')
    subprocess.run(['gcc', '-std=c11', '-Wall', '-Werror', '-I', os.path.join(ROOT, 'include'), str(src),
                    '-o', str(tmp_path / 't')], check=True)


def test_missing_data_bin_exits_666(tmp_path):
    """render.cpp:173: no data.bin next to the library -> exit(666) (exit status 666 & 255)."""
    code = ('import ctypes, sys; sys.path.insert(0, %r)\n'
            'from swift3drenderer_amd.renderer import load_library\n'
            'from swift3drenderer_amd.abi import PixelData, Input\n'
            'import numpy as np\n'
            'lib = load_library()\n'
            'lib.s3r_configure(b%r, -1)\n'
            'buf = np.zeros((4, 4), dtype=np.uint32)\n'
            'pd = PixelData(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 4, 4, 4, 64)\n'
            'lib.updateAndRender(ctypes.byref(pd), ctypes.byref(Input()))\n') % (ROOT, str(tmp_path / 'none.bin'))
    env = dict(os.environ)
    env.pop('S3R_DATA_PATH', None)
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True)
    assert r.returncode == 666 & 255


def test_malformed_data_bin_exits(tmp_path):
    bad = tmp_path / 'bad.bin'
    bad.write_bytes(b'\x05' + bytes(20))     # truncated
    code = ('import ctypes, sys; sys.path.insert(0, %r)\n'
            'from swift3drenderer_amd.renderer import load_library\n'
            'from swift3drenderer_amd.abi import PixelData, Input\n'
            'import numpy as np\n'
            'lib = load_library()\n'
            'lib.s3r_configure(b%r, -1)\n'
            'buf = np.zeros((4, 4), dtype=np.uint32)\n'
            'pd = PixelData(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 4, 4, 4, 64)\n'
            'lib.updateAndRender(ctypes.byref(pd), ctypes.byref(Input()))\n') % (ROOT, str(bad))
    r = subprocess.run([sys.executable, '-c', code], capture_output=True)
    assert r.returncode == 666 & 255
    assert b'malformed' in r.stderr


def test_render_bands_rejects_bad_arguments():
    lib = load_library()
    i = abi.Input()
    assert lib.s3r_render_bands(ctypes.byref(i), 16, 16, 0, 1, 0, None, None) == -1
    assert lib.s3r_render_bands(ctypes.byref(i), 16, 16, 4, 2, 2, None, None) == -1
    # an Input instance passes straight through (POINTER(Input) argtype, Input.of identity)
    assert abi.Input.of(i) is i
    assert lib.s3r_render_bands(i, 16, 16, 0, 1, 0, None, None) == -1


def test_unregister_host_is_a_no_op_for_unknown_pointers():
    """s3r_unregister_host on NULL or on memory the library never page-locked touches no device."""
    import numpy as np
    lib = load_library()
    lib.s3r_unregister_host(None)
    a = np.zeros(16, dtype=np.uint32)
    lib.s3r_unregister_host(ctypes.c_void_p(a.ctypes.data))
