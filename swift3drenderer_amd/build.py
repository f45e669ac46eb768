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
FLAGS = ['-O3', '-std=c++17', f'--offload-arch={ARCH}', '-fPIC', '-ffp-contract=off',
         '-fno-fast-math', '-Wall', '-Wno-unused-function', f'-I{os.path.join(ROOT, "include")}']
SOURCES = ['kernels.hip', 'render_api.cpp']


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build_library(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith('.h')]
    headers.append(os.path.join(ROOT, 'include', 'render.h'))
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src + '.o')
        objs.append(o)
        if force or not _newer(o, [s, *headers]):
            cmd = [HIPCC, *FLAGS, '-x', 'hip', '-c', s, '-o', o]
            if verbose:
                print(' '.join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
    if force or not _newer(LIB, objs):
        cmd = [HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', *objs, '-o', LIB, '-ldl']
        if verbose:
            print(' '.join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    if not _newer(DYLIB, [LIB]):
        shutil.copyfile(LIB, DYLIB)
    return LIB


def build_data(force: bool = False) -> str:
    from . import scene
    if force or not os.path.exists(DATA):
        scene.write_named('full', DATA)
    return DATA


def main():
    build_library(force='--force' in sys.argv, verbose=True)
    build_data()
    print(LIB)


if __name__ == '__main__':
    main()
