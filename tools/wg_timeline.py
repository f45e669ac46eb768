#!/usr/bin/env python3
"""Per-workgroup timeline of one k_fragment launch (timing build build/librender_wgt.so, made here by
`python -c "from swift3drenderer_amd.build import build_variant; build_variant('wgt', {'S3R_WGTIME': 1})"`;
run on the GPU box).

Each fragment workgroup stamps the 100 MHz wall clock at its start, after its triangle list is in
LDS, after its walk state is loaded, and at its end.  Prints the launch span, the phase durations
(percentiles over workgroups) and how many workgroups were in flight over time.

    python tools/wg_timeline.py [--scene full --pose P_over --width 3840 --height 2160 --nparts 1]
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
    a = ap.parse_args()
    import torch
    from swift3drenderer_amd import build, poses, renderer, scene
    lib = renderer.load_library(os.path.join(ROOT, 'build', 'librender_wgt.so'))
    lib.s3r_stats_wg_times.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    lib.s3r_stats_wg_times.restype = ctypes.c_uint32
    d = tempfile.mkdtemp()
    data = os.path.join(d, a.scene + '.bin')
    scene.write_named(a.scene, data)
    W, H, N = a.width, a.height, a.nparts
    B = a.band if N > 1 else H
    r = renderer.Renderer(data, device=0)
    buf = torch.empty((H, W), dtype=torch.int32, device='cuda')
    st = torch.cuda.current_stream().cuda_stream
    for t in poses.script(a.pose):
        r.render_bands(t, W, H, B, N, 0, buf.data_ptr(), st)
    for _ in range(20):
        r.render_bands(poses.hold(a.pose), W, H, B, N, 0, buf.data_ptr(), st)
    torch.cuda.synchronize()
    out = (ctypes.c_uint64 * (12 * 65536))()
    n = lib.s3r_stats_wg_times(out, 65536)
    t = np.frombuffer(out, dtype=np.uint64)[: 12 * n].reshape(n, 12).astype(np.int64)
    t = t[t[:, 3] > 0]
    t0 = t[:, 0].min()
    rel = (t - t0) * 0.01          # us
    span = rel[:, 3].max()
    print(f'{a.scene}/{a.pose} {W}x{H} part 0 of {N}: {len(t)} workgroups, launch span {span:.1f} us')
    for name, v in [('list', rel[:, 1] - rel[:, 0]), ('state', rel[:, 2] - rel[:, 1]),
                    ('chunks', rel[:, 3] - rel[:, 2]), ('total', rel[:, 3] - rel[:, 0]), ('start', rel[:, 0])]:
        p = np.percentile(v, [10, 50, 90, 99])
        print(f'  {name:7s} p10 {p[0]:7.2f}  p50 {p[1]:7.2f}  p90 {p[2]:7.2f}  p99 {p[3]:7.2f}  mean {v.mean():7.2f} us')
    # wave 0's chunk-loop phases (shader clock, summed over the workgroup's chunks) by list length
    cyc = t[:, 4:7].astype(np.float64)
    tot = rel[:, 3] - rel[:, 0]
    heavy = tot >= np.percentile(tot, 90)
    for lab, m in [('all', np.ones(len(t), bool)), ('slowest 10%', heavy)]:
        c = cyc[m].mean(axis=0)
        print(f'  wave-0 cycles ({lab}): batch0 {c[0]:.0f}  later batches {c[1]:.0f}  shade+store {c[2]:.0f}; '
              f'list length mean {t[m, 7].mean():.1f} max {t[m, 7].max()}')
        print(f'      per workgroup (wave 0): slow-path chunks {t[m, 8].mean():.2f}, non-linear chunks {t[m, 9].mean():.2f}, '
              f'live triangles tested {t[m, 10].mean():.2f}')
    if os.environ.get('S3R_WGT_DUMP'):
        np.save(os.environ['S3R_WGT_DUMP'], t)
    edges = np.linspace(0, span, 11)
    live = [int(((rel[:, 0] <= e) & (rel[:, 3] > e)).sum()) for e in edges[:-1]]
    print('  in flight at 0%,10%..90% of the span:', live)
    r.shutdown()


if __name__ == '__main__':
    main()
