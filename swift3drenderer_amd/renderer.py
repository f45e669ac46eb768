"""Host-side mirror of the reference's plugin interface: ``updateAndRender(PixelData*, Input*)``.

This loads the in-tree gfx950 library (``librender.so``) and calls it through its C ABI exactly
the way the Swift main loop does (``main.swift:96-98`` dlopen/dlsym, ``:121`` the call).  There is
no CPU fallback: if the library is missing or cannot be loaded this raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .abi import Input, pixel_data_for

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('S3R_LIB') or os.path.join(PKG, 'librender.so')

EXPORTS = ['updateAndRender', 's3r_configure', 's3r_configure_devices', 's3r_devices', 's3r_shutdown',
           's3r_set_raster_path', 's3r_raster_path', 's3r_unregister_host', 's3r_host_pinned', 's3r_host_stats',
           's3r_render_bands', 's3r_bands_to_host', 's3r_band_rows_local', 's3r_timing', 's3r_timing_collect',
           's3r_scene_counts', 's3r_camera', 's3r_debug_set_frame_count', 's3r_set_delivery', 's3r_delivery',
           's3r_fill_profile', 's3r_tile_stats']

_lib = None
# host frames of update_and_render(out=None), one per shape, kept for the process: the library may
# hold a hipHostRegister registration on them (render_api.cpp host_pinned)
_HOST_FRAMES: dict = {}


def load_library(path: str = LIB_PATH):
    """dlopen the rasterizer (RTLD_NOW, like main.swift:96) and declare its C signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f'{path} is missing: run __graft_entry__.build() (no CPU fallback exists)')
    lib = ctypes.CDLL(path, mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    lib.updateAndRender.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.updateAndRender.restype = None
    lib.s3r_configure.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.s3r_configure.restype = ctypes.c_int
    lib.s3r_shutdown.argtypes = []
    lib.s3r_set_raster_path.argtypes = [ctypes.c_int]
    lib.s3r_set_raster_path.restype = ctypes.c_int
    lib.s3r_raster_path.argtypes = []
    lib.s3r_raster_path.restype = ctypes.c_int
    lib.s3r_render_bands.argtypes = [ctypes.POINTER(Input), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.s3r_render_bands.restype = ctypes.c_int64
    lib.s3r_band_rows_local.argtypes = [ctypes.c_uint32] * 4
    lib.s3r_band_rows_local.restype = ctypes.c_uint32
    lib.s3r_timing.argtypes = [ctypes.c_int]
    lib.s3r_timing_collect.argtypes = [ctypes.POINTER(ctypes.c_double)]
    lib.s3r_scene_counts.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    lib.s3r_camera.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.s3r_bands_to_host.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.s3r_bands_to_host.restype = ctypes.c_int64
    lib.s3r_unregister_host.argtypes = [ctypes.c_void_p]
    lib.s3r_unregister_host.restype = None
    lib.s3r_debug_set_frame_count.argtypes = [ctypes.c_uint32]
    lib.s3r_debug_set_frame_count.restype = None
    lib.s3r_configure_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_uint32]
    lib.s3r_configure_devices.restype = ctypes.c_int
    lib.s3r_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    lib.s3r_devices.restype = ctypes.c_int
    lib.s3r_host_pinned.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.s3r_host_pinned.restype = ctypes.c_int
    lib.s3r_host_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    lib.s3r_host_stats.restype = None
    lib.s3r_set_delivery.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.s3r_set_delivery.restype = ctypes.c_int
    lib.s3r_delivery.argtypes = []
    lib.s3r_delivery.restype = ctypes.c_int
    lib.s3r_fill_profile.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    lib.s3r_fill_profile.restype = ctypes.c_uint32
    lib.s3r_tile_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    lib.s3r_tile_stats.restype = None
    if hasattr(lib, 's3r_deinterleave_bands'):     # (optional: A/B runs load earlier builds via S3R_LIB)
        lib.s3r_deinterleave_bands.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        lib.s3r_deinterleave_bands.restype = ctypes.c_int
    if hasattr(lib, 's3r_device_profile'):
        lib.s3r_device_profile.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
        lib.s3r_device_profile.restype = ctypes.c_uint32
    if hasattr(lib, 's3r_cluster_stats'):         # (optional: A/B runs load earlier builds via S3R_LIB)
        lib.s3r_cluster_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
        lib.s3r_cluster_stats.restype = None
    missing = [name for name in EXPORTS if not hasattr(lib, name)]
    if missing:
        raise RuntimeError(f'{path} does not export {missing}: rebuild it (__graft_entry__.build())')
    _lib = lib
    return lib


def band_rows_local(height: int, band: int, nparts: int, part: int) -> int:
    return int(load_library().s3r_band_rows_local(height, band, nparts, part))


def band_row_ids(height: int, band: int, nparts: int, part: int) -> np.ndarray:
    """Frame rows owned by `part`, in the order they are stored locally."""
    y = np.arange(height)
    return y[(y // band) % nparts == part]


class Renderer:
    """Stateful like the reference: one scene, one camera, lazy init on the first call."""

    def __init__(self, data_path: str | None = None, device: int = -1):
        self.lib = load_library()
        self.configure(data_path, device)

    def configure(self, data_path: str | None, device: int = -1):
        self.lib.s3r_configure(data_path.encode() if data_path else None, device)

    def configure_devices(self, device_ids, band: int = 0):
        """updateAndRender over several devices (interleaved row bands, each device copying its rows
        into the caller's buffer); [] = one device.  Drops all state like configure()."""
        ids = (ctypes.c_int * max(len(device_ids), 1))(*device_ids)
        if self.lib.s3r_configure_devices(ids, len(device_ids), band) != 0:
            raise ValueError(f'bad device list {device_ids!r}')

    def frame_band(self, height: int, nparts: int) -> int:
        """Rows per band of an updateAndRender frame over nparts devices (include/render.h s3r_frame_band)."""
        f = self.lib.s3r_frame_band
        f.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        f.restype = ctypes.c_uint32
        return int(f(height, nparts))

    def devices(self):
        out = (ctypes.c_int * 64)()
        n = self.lib.s3r_devices(out, 64)
        return list(out[:n])

    def host_pinned(self, arr: np.ndarray) -> bool:
        """Whether the library holds a successful page-lock covering the array's bytes."""
        return bool(self.lib.s3r_host_pinned(ctypes.c_void_p(arr.ctypes.data), arr.nbytes))

    def host_stats(self) -> dict:
        out = (ctypes.c_uint64 * 12)()
        self.lib.s3r_host_stats(out)
        keys = ('pinned_frames', 'pageable_frames', 'registrations', 'merges', 'held', 'stale', 'copy_frames',
                'direct_frames', 'fill_frames', 'fill_threads', 'link_bytes', 'fill_gpu_eighths')
        return dict(zip(keys, (int(v) for v in out)))

    def fill_profile(self) -> dict:
        """Host fill profile since the last call (include/render.h s3r_fill_profile), means per frame in
        us: entry to frame start (pre), then after the start: launches issued, devices drained, fill
        threads done, joined; per thread its CPU, mean finish and pixels per frame."""
        out = (ctypes.c_uint64 * (8 + 4 * 64))()
        n = self.lib.s3r_fill_profile(out, 64)
        f = max(int(out[0]), 1)
        us = lambda v: round(v / f / 1e3, 1)
        return {'frames': int(out[0]), 'pre_us': us(out[1]), 'issued_us': us(out[2]), 'dev_end_us': us(out[3]),
                'fill_end_us': us(out[4]), 'joined_us': us(out[5]), 'placed': bool(out[6]),
                'node': ctypes.c_int64(out[7]).value,
                'threads': [{'cpu': int(out[8 + 4 * t]), 'end_us': us(out[9 + 4 * t]), 'px': int(out[10 + 4 * t] // f),
                             'covered_us': us(out[11 + 4 * t])} for t in range(n)]}

    def tile_stats(self) -> dict:
        """Tile path list sizing (include/render.h s3r_tile_stats)."""
        out = (ctypes.c_uint64 * 4)()
        self.lib.s3r_tile_stats(out)
        return {'readbacks': int(out[0]), 'overflows': int(out[1]), 'last_pairs': int(out[2]),
                'last_live': int(out[3])}

    def device_profile(self) -> list:
        """Per device behind updateAndRender since the last call (include/render.h
        s3r_device_profile): mean finish time of its part (us after the call's entry) and its link
        bytes in the last frame."""
        out = (ctypes.c_uint64 * (4 * 64))()
        n = self.lib.s3r_device_profile(out, 64)
        return [{'device': int(out[4 * i]), 'frames': int(out[4 * i + 1]),
                 'finish_us': round(out[4 * i + 2] / max(out[4 * i + 1], 1) / 1e3, 2),
                 'link_bytes': int(out[4 * i + 3])} for i in range(n)]

    def cluster_stats(self) -> dict:
        """Tile path clusters (include/render.h s3r_cluster_stats)."""
        out = (ctypes.c_uint64 * 4)()
        self.lib.s3r_cluster_stats(out)
        return {'clusters': int(out[0]), 'culling': bool(out[1]), 'last_kept': int(out[2]),
                'permuted': bool(out[3])}

    DELIVERIES = {'env': -1, 'auto': 0, 'copy': 1, 'direct': 2, 'fill': 3}

    def set_delivery(self, mode='auto', fill_threads: int = -1):
        """updateAndRender's delivery into the caller's buffer: 'auto', 'copy', 'direct', 'fill' (host
        fill with `fill_threads` threads), or 'env' (S3R_DELIVERY); include/render.h."""
        if self.lib.s3r_set_delivery(self.DELIVERIES.get(mode, mode), int(fill_threads)) != 0:
            raise ValueError(f'bad delivery {mode!r} / {fill_threads}')

    def delivery(self) -> str:
        return {v: k for k, v in self.DELIVERIES.items()}[self.lib.s3r_delivery()]

    def update_and_render(self, width: int, height: int, inp, out: np.ndarray | None = None) -> np.ndarray:
        """updateAndRender into a host uint32 (H, W) buffer (the reference's contract).

        The library may page-lock (hipHostRegister) the caller's buffer and keeps that registration
        for the buffer's pointer, like the reference app's long-lived double buffer (main.swift:117):
        a caller passing `out` keeps it alive while it uses the library.  Without `out` the frame goes
        through a buffer this object owns, and a copy is returned."""
        own = out is None
        if own:
            out = _HOST_FRAMES.get((height, width))
            if out is None:
                out = _HOST_FRAMES[(height, width)] = np.empty((height, width), dtype=np.uint32)
        pd = pixel_data_for(out)
        i = Input.of(inp)
        self.lib.updateAndRender(ctypes.byref(pd), ctypes.byref(i))
        return out.copy() if own else out

    def render_bands(self, inp, width: int, height: int, band: int, nparts: int, part: int, dev_ptr: int,
                     stream: int = 0) -> int:
        """Render one part of an interleaved row-band split into device memory at dev_ptr, on the
        HIP stream `stream` (0 = the default stream, i.e. torch's default stream)."""
        r = self.lib.s3r_render_bands(Input.of(inp), width, height, band, nparts, part, dev_ptr, stream or None)
        if r < 0:
            raise ValueError('s3r_render_bands: bad arguments')
        return int(r)

    def bands_to_host(self, dev_ptr: int, width: int, height: int, band: int, nparts: int, part: int,
                      host: np.ndarray, stream: int = 0) -> int:
        """Copy one part's rows (device, compact) into their rows of the host frame `host` (H x W
        uint32, C-contiguous) on `stream`, asynchronously (s3r_bands_to_host)."""
        if host.dtype != np.uint32 or host.shape != (height, width) or not host.flags['C_CONTIGUOUS']:
            raise ValueError('host frame must be a C-contiguous (height, width) uint32 array')
        r = self.lib.s3r_bands_to_host(ctypes.c_void_p(dev_ptr), width, height, band, nparts, part,
                                       ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(stream or None))
        if r < 0:
            raise ValueError('s3r_bands_to_host: bad arguments')
        return int(r)

    def unregister_host(self, host: np.ndarray):
        """Drop the page-lock bands_to_host took on `host` (before the array is freed / unmapped)."""
        self.lib.s3r_unregister_host(ctypes.c_void_p(host.ctypes.data))

    def set_raster_path(self, mode: str | int):
        """'auto' | 'rows' | 'tiles' (or 0/1/2): the fragment-stage strategy, include/render.h."""
        m = {'auto': 0, 'rows': 1, 'tiles': 2}.get(mode, mode)
        if self.lib.s3r_set_raster_path(int(m)) != 0:
            raise ValueError(f'unknown raster path {mode!r}')

    def raster_path(self) -> str:
        return {1: 'rows', 2: 'tiles'}[self.lib.s3r_raster_path()]

    def timing(self, enable: bool):
        self.lib.s3r_timing(1 if enable else 0)

    def timing_collect(self):
        out = (ctypes.c_double * 3)()
        self.lib.s3r_timing_collect(out)
        return out[0], out[1], int(out[2])

    def timing_stages(self) -> dict:
        """Summed HIP-event ms since timing(True) (include/render.h s3r_timing_stages): fragment
        stage, whole frame, geometry / setup stage, and the frame count; resets like timing_collect."""
        out = (ctypes.c_double * 4)()
        self.lib.s3r_timing_stages(out)
        return {'frag_ms': out[0], 'frame_ms': out[1], 'frames': int(out[2]), 'geo_ms': out[3]}

    def scene_counts(self):
        out = (ctypes.c_uint64 * 8)()
        self.lib.s3r_scene_counts(out)
        return list(out)

    def camera(self):
        m = (ctypes.c_float * 12)()
        f = ctypes.c_float()
        self.lib.s3r_camera(m, ctypes.byref(f))
        return np.array(m, dtype=np.float32).reshape(3, 4), f.value

    def debug_set_frame_count(self, frame_no: int):
        """Test hook: continue the frame count (the frames' uint32 tags) at frame_no."""
        self.lib.s3r_debug_set_frame_count(frame_no)

    def shutdown(self):
        self.lib.s3r_shutdown()


def render_pose(r: Renderer, data_path: str, pose_script, width: int, height: int, extra_frames: int = 0):
    """Fresh state, run a pose script, return the last frame (mirrors oracle.render_pose)."""
    r.configure(data_path)
    out = None
    for t in pose_script:
        out = r.update_and_render(width, height, t)
    hold = (0, 0, 0, 0) + tuple(pose_script[-1][4:6])
    for _ in range(extra_frames):
        out = r.update_and_render(width, height, hold)
    return out
