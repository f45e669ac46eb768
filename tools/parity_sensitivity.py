#!/usr/bin/env python3
"""How far do the reference semantics this build could not pin move the pixels?  

The parity oracle (oracle/render_oracle.c) fixes one reading of render.cpp: x86-64 semantics, no FMA
contraction, simd_fast_normalize as 1/sqrtf, config.scale from tanf.  An Apple build of the reference
may differ at exactly those points.  This renders the golden cases with each
sensitivity variant of the oracle (oracle/Makefile `variants`) and counts, against the parity oracle:
pixels that differ at all, pixels with any RGB channel off by more than 1 LSB (north_star's
tolerance), and the largest channel difference.

    python tools/parity_sensitivity.py [--out profiles/r03_parity_sensitivity.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.oracle import VARIANTS, render_pose, variant_lib  # noqa: E402
from swift3drenderer_amd import poses, scene  # noqa: E402

CASES = [('full', 'P_id', 640, 480), ('full', 'P_over', 640, 480), ('full', 'P_clip', 640, 480),
         ('full', 'P_floor', 640, 480), ('flat', 'P_over', 640, 480), ('tetra', 'P_tetra', 640, 480),
         ('full', 'P_over', 1920, 1080), ('full', 'P_id', 1920, 1080)]


def compare(a: np.ndarray, b: np.ndarray) -> dict:
    ch = [np.abs(((a >> s) & 255).astype(np.int32) - ((b >> s) & 255).astype(np.int32)) for s in (16, 8, 0)]
    worst = np.maximum(np.maximum(ch[0], ch[1]), ch[2])
    covered = int((b != 0x1E1E1E).sum())
    return {'pixels': int(a.size), 'covered': covered, 'differ': int((a != b).sum()),
            'beyond_1lsb': int((worst > 1).sum()), 'max_channel_diff': int(worst.max())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default=None)
    ap.add_argument('--cases', type=int, default=len(CASES))
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix='s3r_sens_')
    paths = {}
    for name in ('full', 'flat', 'tetra'):
        paths[name] = os.path.join(tmp, f'{name}.bin')
        scene.write_named(name, paths[name])
    libs = {v: variant_lib(v) for v in VARIANTS}
    rows = []
    for sc, pose, w, h in CASES[:a.cases]:
        ref = render_pose(paths[sc], poses.script(pose), w, h, extra_frames=1)
        for v, lib in libs.items():
            got = render_pose(paths[sc], poses.script(pose), w, h, extra_frames=1, lib_=lib)
            r = {'case': f'{sc}/{pose}/{w}x{h}', 'variant': v, **compare(got, ref)}
            rows.append(r)
            print(json.dumps(r), flush=True)
    summary = {}
    for v in VARIANTS:
        rs = [r for r in rows if r['variant'] == v]
        cov = sum(r['covered'] for r in rs)
        summary[v] = {'differ': sum(r['differ'] for r in rs), 'beyond_1lsb': sum(r['beyond_1lsb'] for r in rs),
                      'covered': cov, 'beyond_1lsb_frac_of_covered': round(sum(r['beyond_1lsb'] for r in rs) / max(cov, 1), 6),
                      'max_channel_diff': max(r['max_channel_diff'] for r in rs)}
    print(json.dumps({'summary': summary}))
    if a.out:
        with open(a.out, 'w') as f:
            json.dump({'cases': rows, 'summary': summary}, f, indent=1)


if __name__ == '__main__':
    main()
