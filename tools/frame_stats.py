#!/usr/bin/env python3
"""Diagnostic: walker iteration counters of the fragment kernel (librender_stats.so, -DS3R_STATS).

    python tools/frame_stats.py [--scene full] [--pose P_over] [--width 3840] [--height 2160] [--device]

--device: frames left in HBM (s3r_render_bands: k_geometry walks every segment start) instead of
updateAndRender into a host buffer (row starts only, the fragment walks along its rows).
"""
import argparse
import ctypes
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ['row_walk', 'chunk_walk', 'pixel_walk', 'irregular_comp', 'pixel_tests', 'batches']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--scene', default='full')
    ap.add_argument('--pose', default='P_over')
    ap.add_argument('--width', type=int, default=3840)
    ap.add_argument('--height', type=int, default=2160)
    ap.add_argument('--device', action='store_true')
    a = ap.parse_args()
    from swift3drenderer_amd import build, poses, scene, renderer
    path = build.build_library(stats=True)
    lib = renderer.load_library(path)
    lib.s3r_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    d = tempfile.mkdtemp()
    data = os.path.join(d, a.scene + '.bin')
    scene.write_named(a.scene, data)
    r = renderer.Renderer(data)
    if a.device:
        import torch
        buf = torch.empty((a.height, a.width), dtype=torch.int32, device='cuda')
        st = torch.cuda.current_stream().cuda_stream
        frame = lambda t: (r.render_bands(t, a.width, a.height, a.height, 1, 0, buf.data_ptr(), st),
                           torch.cuda.synchronize())
    else:
        frame = lambda t: r.update_and_render(a.width, a.height, t)
    for t in poses.script(a.pose):
        frame(t)
    out = (ctypes.c_uint64 * 16)()
    lib.s3r_stats(out, 1)
    frame(poses.hold(a.pose))
    lib.s3r_stats(out, 0)
    segs = (a.width + 1023) // 1024
    waves = a.height * segs
    print(f'{a.scene}/{a.pose} {a.width}x{a.height}: {waves} waves')
    for k, n in enumerate(NAMES):
        print(f'  {n:15s} lane-sum {out[2 * k]:>14d}  per-wave(sum of wave-max) {out[2 * k + 1]:>12d}'
              f'  per wave {out[2 * k + 1] / waves:10.1f}')
    print(f'  k_geometry: row-walk iterations sum {out[12]} max/lane {out[13]}; segment walks sum {out[14]} max/lane {out[15]}')
    lib.s3r_stats_geometry.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    g = (ctypes.c_uint64 * 8)()
    lib.s3r_stats_geometry(g)
    print(f'  k_geometry wall clock: max WG setup {g[0] * 10 / 1e3:.2f} us, max WG {g[1] * 10 / 1e3:.2f} us, '
          f'first start -> last end {(g[3] - g[2]) * 10 / 1e3:.2f} us')


if __name__ == '__main__':
    main()
