#!/usr/bin/env python3
"""Per-workgroup timeline of one k_geometry launch (timing build build/librender_wgt.so, see
tools/wg_timeline.py; run on the GPU box, ideally with S3R_SERIAL=1).

Each geometry workgroup (slot, block of 128 local rows; record slot * 64 + row block) stamps the 100 MHz wall clock at its start,
after thread 0 set the slot up, after the bins were set, and when its last wave finished the row /
segment-start walks.  Prints the launch span and the phase durations of live and dead slots.

    python tools/geo_timeline.py [--scene full --pose P_over --width 3840 --height 2160 --nparts 1]
"""
import argparse
import ctypes
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--scene', default='full')
    ap.add_argument('--pose', default='P_over')
    ap.add_argument('--width', type=int, default=3840)
    ap.add_argument('--height', type=int, default=2160)
    ap.add_argument('--nparts', type=int, default=1)
    ap.add_argument('--band', type=int, default=16)
    ap.add_argument('--delivered', action='store_true',
                    help='updateAndRender frames into a host buffer (row starts only) instead of HBM frames')
    a = ap.parse_args()
    import torch
    from swift3drenderer_amd import poses, renderer, scene
    lib = renderer.load_library(os.environ.get('S3R_LIB') or os.path.join(ROOT, 'build', 'librender_wgt.so'))
    lib.s3r_stats_geo_times.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    lib.s3r_stats_geo_times.restype = ctypes.c_uint32
    d = tempfile.mkdtemp()
    data = os.path.join(d, a.scene + '.bin')
    scene.write_named(a.scene, data)
    W, H, N = a.width, a.height, a.nparts
    B = a.band if N > 1 else H
    r = renderer.Renderer(data, device=0)
    buf = torch.empty((H, W), dtype=torch.int32, device='cuda')
    st = torch.cuda.current_stream().cuda_stream
    host = np.empty((H, W), dtype=np.uint32)

    def frame(t):
        if a.delivered:
            r.update_and_render(W, H, t, host)
        else:
            r.render_bands(t, W, H, B, N, 0, buf.data_ptr(), st)
    for t in poses.script(a.pose):
        frame(t)
    for _ in range(20):
        frame(poses.hold(a.pose))
    torch.cuda.synchronize()
    out = (ctypes.c_uint64 * (4 * 16384))()
    lib.s3r_stats_geo_times(out, 16384)           # clear
    frame(poses.hold(a.pose))
    torch.cuda.synchronize()
    n = lib.s3r_stats_geo_times(out, 16384)
    t = np.frombuffer(out, dtype=np.uint64)[: 4 * n].reshape(n, 4).astype(np.int64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    rel = (t - t0) * 0.01
    idx = np.nonzero(np.frombuffer(out, dtype=np.uint64)[: 4 * n].reshape(n, 4)[:, 0] > 0)[0]
    live = t[:, 2] > 0
    print(f'{a.scene}/{a.pose} {W}x{H} part 0 of {N}: {len(t)} geometry workgroups ({live.sum()} live), '
          f'span {rel[:, 3].max():.1f} us')
    for lab, m in [('live', live), ('dead', ~live)]:
        if not m.any():
            continue
        for name, v in [('start', rel[m, 0]), ('setup', rel[m, 1] - rel[m, 0]),
                        ('walks', (rel[m, 3] - rel[m, 2]) if lab == 'live' else rel[m, 3] - rel[m, 1]),
                        ('total', rel[m, 3] - rel[m, 0])]:
            p = np.percentile(v, [10, 50, 90, 100])
            print(f'  {lab} {name:6s} p10 {p[0]:7.2f}  p50 {p[1]:7.2f}  p90 {p[2]:7.2f}  max {p[3]:7.2f} us')
    wt = rel[:, 3] - rel[:, 2]
    for i in np.argsort(-np.where(live, wt, -1))[:6]:
        g = int(idx[i])
        print(f'  slow walk: slot {g // 64} row block {g % 64}: start {rel[i, 0]:.2f} setup {rel[i, 1] - rel[i, 0]:.2f} '
              f'walks {wt[i]:.2f} us')
    r.shutdown()


if __name__ == '__main__':
    main()
