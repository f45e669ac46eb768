#!/usr/bin/env python3
"""Regenerate tests/golden/frames.{npz,json} from the CPU oracle.

The reference has no golden vectors and cannot be built here (Apple simd), so these
fixtures pin the oracle (itself cross-checked against tests/pyref.py) -- any change to the oracle's
output must be deliberate.  Small frames are stored; larger ones by SHA-256 only.
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.oracle import render_pose  # noqa: E402
from swift3drenderer_amd import poses, scene  # noqa: E402

CASES = [  # (scene, pose, w, h, store)
    ('full', 'P_id', 160, 120, True), ('full', 'P_over', 160, 120, True), ('full', 'P_clip', 160, 120, True),
    ('flat', 'P_over', 160, 120, True), ('tetra', 'P_tetra', 160, 120, True), ('full', 'P_floor', 160, 120, True),
    ('full', 'P_id', 640, 480, False), ('full', 'P_over', 640, 480, False), ('full', 'P_clip', 640, 480, False),
    ('tetra', 'P_tetra', 640, 480, False), ('full', 'P_over', 1920, 1080, False),
]


def main():
    d = tempfile.mkdtemp()
    meta, arrays = {}, {}
    for sc, pose, w, h, store in CASES:
        path = os.path.join(d, sc + '.bin')
        if not os.path.exists(path):
            scene.write_named(sc, path)
        img = render_pose(path, poses.script(pose), w, h)
        key = f'{sc}_{pose}_{w}x{h}'
        meta[key] = {'scene': sc, 'pose': pose, 'w': w, 'h': h, 'sha256': hashlib.sha256(img.tobytes()).hexdigest()}
        if store:
            arrays[key] = img
    np.savez_compressed(os.path.join(HERE, 'frames.npz'), **arrays)
    with open(os.path.join(HERE, 'frames.json'), 'w') as f:
        json.dump(meta, f, indent=1)


if __name__ == '__main__':
    main()
