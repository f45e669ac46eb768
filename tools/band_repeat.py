#!/usr/bin/env python3
"""Repeat tests/test_multi.py::test_gpu_band_parts_reassemble's sequence many times in one process
(GPU box) and report every mismatch with its rows and parts: a search for an intermittent band-part
difference (open issue).

    python tools/band_repeat.py [--iters 40] [--lpt-first]
"""
import argparse
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=40)
    ap.add_argument('--lpt-first', action='store_true',
                    help='before each split, 10 pipelined 640x480 frames on another stream with the '
                         'longest-first order forced on (the GPU suite\'s preceding test)')
    a = ap.parse_args()
    import torch
    from swift3drenderer_amd import poses, scene
    from swift3drenderer_amd.renderer import Renderer
    from swift3drenderer_amd.multi import assemble, band_rows
    d = tempfile.mkdtemp()
    path = os.path.join(d, 'full.bin')
    scene.write_named('full', path)
    r = Renderer()
    dev = torch.device('cuda', 0)
    W, H = 800, 600
    bad = 0
    runs = 0
    for it in range(a.iters):
        for nparts, band in [(2, 16), (3, 16), (8, 16), (8, 1), (5, 7)]:
            r.configure(path)
            if a.lpt_first:
                os.environ['S3R_LPT_MIN'] = '0'
                s2 = torch.cuda.Stream()
                bufs = [torch.empty((480, 640), dtype=torch.int32, device=dev) for _ in range(10)]
                for k, b in enumerate(bufs):
                    with torch.cuda.stream(s2):
                        r.render_bands((0, 0, 0, 0, 3.0 * k, -150 + k), 640, 480, 480, 1, 0, b.data_ptr(),
                                       s2.cuda_stream)
                torch.cuda.synchronize()
                del os.environ['S3R_LPT_MIN']
            st = torch.cuda.current_stream(dev).cuda_stream
            full = torch.empty((H, W), dtype=torch.int32, device=dev)
            for t in poses.script('P_over'):
                r.render_bands(t, W, H, H, 1, 0, full.data_ptr(), st)
            torch.cuda.synchronize()
            parts = []
            hold = poses.hold('P_over')
            for p in range(nparts):
                rows = band_rows(H, band, nparts, p)
                buf = torch.full((max(rows, 1), W), -1, dtype=torch.int32, device=dev)
                r.render_bands(hold, W, H, band, nparts, p, buf.data_ptr(), st)
                parts.append(buf.cpu().numpy()[:rows])
            torch.cuda.synchronize()
            got = assemble(parts, H, band)
            want = full.cpu().numpy()
            runs += 1
            if not np.array_equal(got, want):
                bad += 1
                ys, xs = np.nonzero(got != want)
                print(f'iter {it} nparts {nparts} band {band}: {len(ys)} px differ, rows {ys.min()}-{ys.max()}, '
                      f'parts {sorted({(int(y) // band) % nparts for y in ys})}, first (x={xs[0]}, y={ys[0]}) '
                      f'parts {got[ys[0], xs[0]] & 0xFFFFFFFF:#x} whole {want[ys[0], xs[0]] & 0xFFFFFFFF:#x}', flush=True)
        print(f'iter {it}: {bad} mismatches in {runs} splits', flush=True)
    r.shutdown()
    print(f'done: {bad} mismatches in {runs} splits')


if __name__ == '__main__':
    main()
