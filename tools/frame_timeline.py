#!/usr/bin/env python3
"""Where one synchronous updateAndRender frame's time goes, without a tracer (timing build
build/librender_wgt.so; run on the GPU box).

The geometry and fragment workgroups of the timing build stamp the GPU's 100 MHz wall clock
(kernels.hip S3R_GWT / S3R_WGT), so one frame delivered into a main.swift-style double buffer
(host-fill delivery by default) splits into: the geometry launch's span, the gap until the first
fragment workgroup starts (k_sky_flags and the dispatch between them), the fragment launch's span;
the rest of the call's host-measured time is launch latency before the geometry and the host's
wait / fill end / return after the last fragment workgroup.

    python tools/frame_timeline.py [--frames 20] [--delivery fill]
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--scene', default='full')
    ap.add_argument('--pose', default='P_over')
    ap.add_argument('--width', type=int, default=3840)
    ap.add_argument('--height', type=int, default=2160)
    ap.add_argument('--delivery', default='fill')
    ap.add_argument('--frames', type=int, default=20)
    ap.add_argument('--dump', default=None, help='save the last frame\'s workgroup records (.npz)')
    a = ap.parse_args()
    os.environ.setdefault('S3R_LIB', os.path.join(ROOT, 'build', 'librender_wgt.so'))
    from bench import DoubleBuffer
    from swift3drenderer_amd import poses, scene
    from swift3drenderer_amd.abi import Input
    from swift3drenderer_amd.renderer import Renderer
    path = os.path.join(tempfile.mkdtemp(), 's.bin')
    scene.write_named(a.scene, path)
    r = Renderer(path, device=0)
    lib = r.lib
    for f in (lib.s3r_stats_geo_times, lib.s3r_stats_wg_times):
        f.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
        f.restype = ctypes.c_uint32
    r.set_delivery(a.delivery, -1)
    W, H = a.width, a.height
    buf = DoubleBuffer(W, H)
    for t in poses.script(a.pose):
        lib.updateAndRender(ctypes.byref(buf.next()), ctypes.byref(Input.of(t)))
    hold = Input.of(poses.hold(a.pose))
    for _ in range(30):
        lib.updateAndRender(ctypes.byref(buf.next()), ctypes.byref(hold))
    geo = (ctypes.c_uint64 * (4 * 16384))()
    frag = (ctypes.c_uint64 * (12 * 65536))()
    rows = []
    for k in range(a.frames):
        lib.s3r_stats_geo_times(geo, 16384)                     # clear
        t0 = time.perf_counter()
        lib.updateAndRender(ctypes.byref(buf.next()), ctypes.byref(hold))
        call = (time.perf_counter() - t0) * 1e6
        n = lib.s3r_stats_geo_times(geo, 16384)
        g = np.frombuffer(geo, dtype=np.uint64)[: 4 * n].reshape(n, 4).astype(np.int64)
        g = g[g[:, 0] > 0]
        m = lib.s3r_stats_wg_times(frag, 65536)
        fr = np.frombuffer(frag, dtype=np.uint64)[: 12 * m].reshape(m, 12).astype(np.int64)
        fr = fr[fr[:, 3] > 0]
        g0, g1 = g[:, 0].min(), g[:, 3].max()
        f0, f1 = fr[:, 0].min(), fr[:, 3].max()
        rows.append([call, (g1 - g0) * 0.01, (f0 - g1) * 0.01, (f1 - f0) * 0.01, call - (f1 - g0) * 0.01])
    if a.dump:
        np.savez(a.dump, geo=g, frag=fr)
    v = np.array(rows)
    med = np.median(v, axis=0)
    out = {'delivery': a.delivery, 'frames': a.frames, 'call_us': round(med[0], 1), 'geometry_span_us': round(med[1], 1),
           'geometry_to_fragment_us': round(med[2], 1), 'fragment_span_us': round(med[3], 1),
           'host_outside_gpu_us': round(med[4], 1), 'host_stats': r.host_stats()}
    print(json.dumps(out))
    r.shutdown()
    buf.free()


if __name__ == '__main__':
    main()
