"""ctypes loader for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module; the product path (``swift3drenderer_amd``) never does.  See ``render_oracle.c`` for what the
oracle restates and why its parity is *unpinned* (the reference has no golden vectors and cannot be
built without Apple's simd header).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from swift3drenderer_amd.abi import Input, pixel_data_for

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'liboracle.so')


def build() -> str:
    subprocess.run(['make', '-s', '-C', HERE], check=True)
    return LIB


_lib = None
VARIANTS = ('fma', 'fma_fast', 'rsqrt12', 'rsqrt_nr', 'tan_double')   # oracle/Makefile `variants` (sensitivity only)


def _declare(l):
    l.oracle_set_data_path.argtypes = [ctypes.c_char_p]
    l.oracle_updateAndRender.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    l.oracle_camera_matrix.argtypes = [ctypes.POINTER(ctypes.c_float)]
    l.oracle_factor.restype = ctypes.c_float
    l.oracle_scale.restype = ctypes.c_float
    l.oracle_repeat_add.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_uint32]
    l.oracle_repeat_add.restype = ctypes.c_float
    l.oracle_set_row_windows.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]
    l.oracle_set_row_windows.restype = ctypes.c_int
    return l


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = _declare(ctypes.CDLL(LIB))
    return _lib


def variant_lib(name: str):
    """A sensitivity variant of the oracle (oracle/Makefile `variants`), NOT the parity oracle."""
    if name not in VARIANTS:
        raise ValueError(name)
    subprocess.run(['make', '-s', '-C', HERE, 'variants'], check=True)
    return _declare(ctypes.CDLL(os.path.join(HERE, '_build', f'liboracle_{name}.so')))


class OracleRenderer:
    """Stateful like the reference (one scene, one camera); ``reset`` reloads a data.bin.  ``lib``: a
    variant_lib() for sensitivity studies (default: the parity oracle)."""

    def __init__(self, data_path: str, lib_=None):
        self._l = lib_
        self.reset(data_path)

    def _lib(self):
        return self._l if self._l is not None else lib()

    def reset(self, data_path: str):
        self._lib().oracle_set_data_path(data_path.encode())

    def update_and_render(self, width: int, height: int, inp, out: np.ndarray | None = None):
        if out is None:
            out = np.zeros((height, width), dtype=np.uint32)
        pd = pixel_data_for(out)
        i = Input.of(inp)
        self._lib().oracle_updateAndRender(ctypes.byref(pd), ctypes.byref(i))
        return out

    def set_row_windows(self, windows):
        """Rasterise only rows in the [y0, y1) windows (others are walked, not drawn; [] = all rows):
        a test extension for checking full-size frames on a few rows (render_oracle.c)."""
        flat = (ctypes.c_uint32 * max(1, 2 * len(windows)))(*[v for w in windows for v in w])
        if self._lib().oracle_set_row_windows(flat, len(windows)) != 0:
            raise ValueError('at most 32 row windows')

    def camera_matrix(self) -> np.ndarray:
        m = (ctypes.c_float * 12)()
        self._lib().oracle_camera_matrix(m)
        return np.array(m, dtype=np.float32).reshape(3, 4)

    def factor(self) -> float:
        return self._lib().oracle_factor()

    def scale(self) -> float:
        return self._lib().oracle_scale()


def repeat_add(s: float, d: float, n: int) -> float:
    return lib().oracle_repeat_add(s, d, n)


def render_pose(data_path: str, pose_script, width: int, height: int, extra_frames: int = 0, lib_=None):
    """Run a pose script from a fresh state and return the last frame."""
    r = OracleRenderer(data_path, lib_)
    out = None
    for t in pose_script:
        out = r.update_and_render(width, height, t)
    hold = (0, 0, 0, 0) + tuple(pose_script[-1][4:6])
    for _ in range(extra_frames):
        out = r.update_and_render(width, height, hold)
    return out
