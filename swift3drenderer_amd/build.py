"""Build the gfx950 shared library in-tree (hipcc, no cmake) -- the reference's Makefile:18-19 step.

Produces ``swift3drenderer_amd/librender.so`` (+ ``render.dylib``, the name the Swift main loop
dlopens) and ``swift3drenderer_amd/data.bin`` (the default scene, found next to the library the way
``render.cpp:160-176`` searches, like ``Makefile:12-13`` generating data.bin at build time).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
BUILD = os.path.join(ROOT, 'build')
LIB = os.path.join(PKG, 'librender.so')
DYLIB = os.path.join(PKG, 'render.dylib')
DATA = os.path.join(PKG, 'data.bin')

HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('S3R_ARCH', 'gfx950')
# -ffp-contract=off: no FMA contraction (bit parity with the x86 reference build); no fast-math:
# IEEE-correct division and sqrt.
# -fno-slp-vectorize: no SLP packing of adjacent f32 ops into v_pk_*_f32 (the packing adds operand
# moves; measured 66.9 -> 64.1 us per 4K fragment launch, tile raster 784 -> 748 us on the stress scene).
FLAGS = ['-O3', '-std=c++17', f'--offload-arch={ARCH}', '-fPIC', '-ffp-contract=off', '-fno-slp-vectorize',
         '-fno-fast-math', '-Wall', '-Wno-unused-function', '-Wno-bitwise-instead-of-logical', f'-I{os.path.join(ROOT, "include")}']
SOURCES = ['kernels.hip', 'render_api.cpp']
# host-only C++ (no HIP): compiled by g++ so x86 intrinsics stay out of the HIP compilation
HOST_SOURCES = ['host_fill.cpp', 'clusters.cpp']
HOST_FLAGS = ['-O3', '-std=c++17', '-fPIC', '-Wall']


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


STATS_LIB = os.path.join(PKG, 'librender_stats.so')


def build_variant(tag: str, defines: dict, verbose: bool = False) -> str:
    """A tuning variant (build/librender_<tag>.so) with extra -D knobs; tools/variants.sh."""
    bdir = os.path.join(BUILD, tag)
    os.makedirs(bdir, exist_ok=True)
    lib_path = os.path.join(BUILD, f'librender_{tag}.so')
    extra = [f'-D{k}={v}' for k, v in defines.items() if not k.startswith('-')]
    extra += [k for k in defines if k.startswith('-')]          # raw compiler flags: {"-mllvm -x=y": 1}
    extra = [a for e in extra for a in (e.split(' ') if e.startswith('-mllvm') else [e])]
    objs = []
    for src in SOURCES:
        o = os.path.join(bdir, src + '.o')
        subprocess.run([HIPCC, *FLAGS, *extra, '-x', 'hip', '-c', os.path.join(CSRC, src), '-o', o], check=True)
        objs.append(o)
    objs += _host_objects(bdir, False)
    subprocess.run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', *objs, '-o', lib_path, '-ldl'], check=True)
    return lib_path


def _host_objects(bdir: str, force: bool, verbose: bool = False):
    objs = []
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src + '.o')
        objs.append(o)
        if force or not _newer(o, [s]):
            cmd = ['g++', *HOST_FLAGS, '-c', s, '-o', o]
            if verbose:
                print(' '.join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
    return objs


def build_library(force: bool = False, verbose: bool = False, stats: bool = False, ablate: int = 0) -> str:
    """stats=True builds the diagnostic variant (-DS3R_STATS, walker iteration counters) as
    librender_stats.so; ablate=k builds a timing-only variant with parts of the fragment stage
    removed (wrong pixels; tools/ablate.sh).  The product library has neither."""
    tag = 'stats' if stats else (f'ablate{ablate}' if ablate else '')
    bdir = os.path.join(BUILD, tag) if tag else BUILD
    lib_path = os.path.join(BUILD, f'librender_{tag}.so') if ablate else (STATS_LIB if stats else LIB)
    extra = (['-DS3R_STATS'] if stats else []) + ([f'-DS3R_ABLATE={ablate}'] if ablate else [])
    os.makedirs(bdir, exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith('.h')]
    headers.append(os.path.join(ROOT, 'include', 'render.h'))
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src + '.o')
        objs.append(o)
        if force or not _newer(o, [s, *headers]):
            cmd = [HIPCC, *FLAGS, *extra, '-x', 'hip', '-c', s, '-o', o]
            if verbose:
                print(' '.join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
    objs += _host_objects(bdir, force, verbose)
    if force or not _newer(lib_path, objs):
        cmd = [HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', *objs, '-o', lib_path, '-ldl']
        if verbose:
            print(' '.join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    if not tag and not _newer(DYLIB, [LIB]):
        shutil.copyfile(LIB, DYLIB)
    return lib_path


def build_data(force: bool = False) -> str:
    from . import scene
    if force or not os.path.exists(DATA):
        scene.write_named('full', DATA)
    return DATA


HOST_SRC = os.path.join(ROOT, 'host', 'main_loop.cpp')
HOST_BIN = os.path.join(ROOT, 'host', 'main_loop')


def build_host(force: bool = False) -> str:
    """The C++ counterpart of main.swift's loop (dlopen + per-frame updateAndRender); plain g++."""
    if force or not _newer(HOST_BIN, [HOST_SRC, os.path.join(ROOT, 'include', 'render.h')]):
        subprocess.run(['g++', '-O2', '-std=c++17', '-Wall', HOST_SRC, '-ldl', '-o', HOST_BIN], check=True)
    return HOST_BIN


def main():
    build_library(force='--force' in sys.argv, verbose=True)
    if '--stats' in sys.argv:
        build_library(force='--force' in sys.argv, verbose=True, stats=True)
    build_data()
    build_host()
    print(LIB)


if __name__ == '__main__':
    main()
