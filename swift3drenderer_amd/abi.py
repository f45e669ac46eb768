"""ctypes mirror of the reference's C-ABI structs (``render-cpp/render.hpp:7-21``).

``PixelData`` is 24 bytes and ``Input`` is 24 bytes with ``mouse`` (a ``simd_float2``) at offset 16;
these are the exact layouts the Swift main loop passes (``main.swift:13-27``, ``:121``).
"""
from __future__ import annotations

import ctypes


class PixelData(ctypes.Structure):
    _fields_ = [('buffer', ctypes.POINTER(ctypes.c_uint32)),
                ('width', ctypes.c_uint32),
                ('height', ctypes.c_uint32),
                ('bytesPerPixel', ctypes.c_uint32),
                ('bufferSize', ctypes.c_uint32)]


class Input(ctypes.Structure):
    _fields_ = [('up', ctypes.c_float),
                ('down', ctypes.c_float),
                ('left', ctypes.c_float),
                ('right', ctypes.c_float),
                ('mouse_x', ctypes.c_float),
                ('mouse_y', ctypes.c_float)]

    @classmethod
    def of(cls, t):
        """Build from an (up, down, left, right, mouse.x, mouse.y) tuple (an Input passes through)."""
        if isinstance(t, cls):
            return t
        return cls(*(float(v) for v in t))


assert ctypes.sizeof(PixelData) == 24
assert ctypes.sizeof(Input) == 24 and Input.mouse_x.offset == 16


def pixel_data_for(arr) -> PixelData:
    """A PixelData over a C-contiguous uint32 numpy array of shape (H, W)."""
    h, w = arr.shape
    assert arr.dtype.itemsize == 4 and arr.flags['C_CONTIGUOUS']
    ptr = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    return PixelData(ptr, w, h, 4, 4 * w * h)
