"""The CPU oracle (oracle/render_oracle.c) against an independent pure-Python restatement
(tests/pyref.py) on small frames, against its committed golden fixtures (tests/golden/), and
known-answer checks of single rules of render.cpp."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle.oracle import OracleRenderer, render_pose, repeat_add
from swift3drenderer_amd import poses

GOLD = os.path.join(os.path.dirname(__file__), 'golden')

SMALL = [('full', 'P_id'), ('full', 'P_over'), ('full', 'P_clip'), ('full', 'P_strafe'), ('flat', 'P_over'),
         ('tetra', 'P_tetra'), ('full', 'P_floor')]


@pytest.mark.parametrize('scene_name,pose', SMALL)
def test_oracle_matches_python_restatement(scene_dir, scene_name, pose):
    from pyref import render_pose as py_render
    script = poses.script(pose)
    want = py_render(scene_dir[scene_name], script, 64, 48)
    got = render_pose(scene_dir[scene_name], script, 64, 48)
    assert np.array_equal(got, want), f'{int((got != want).sum())} pixels differ'


@pytest.mark.parametrize('scene_name,pose', [('full', 'P_over'), ('full', 'P_clip'), ('full', 'P_floor'),
                                             ('regular', 'P_over')])
def test_oracle_matches_python_restatement_200x150(scene_dir, scene_name, pose):
    from pyref import render_pose as py_render
    script = poses.script(pose)
    want = py_render(scene_dir[scene_name], script, 200, 150)
    got = render_pose(scene_dir[scene_name], script, 200, 150)
    assert np.array_equal(got, want), f'{int((got != want).sum())} pixels differ'


def test_oracle_golden_frames(scene_dir):
    """Frames pinned by tests/golden/make_golden.py (small ones stored, larger ones by SHA-256)."""
    z = np.load(os.path.join(GOLD, 'frames.npz'))
    meta = json.load(open(os.path.join(GOLD, 'frames.json')))
    for key, m in meta.items():
        img = render_pose(scene_dir[m['scene']], poses.script(m['pose']), m['w'], m['h'])
        if key in z.files:
            assert np.array_equal(img, z[key]), key
        assert hashlib.sha256(img.tobytes()).hexdigest() == m['sha256'], key


def test_empty_view_is_background(scene_dir):
    # looking straight up: nothing in view; every pixel RGB(30,30,30) (render.cpp:96, :282)
    img = render_pose(scene_dir['full'], [(0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 0, -2000)], 40, 30)
    assert np.all(img == 0x1E1E1E)


def test_buffer_size_fill(scene_dir):
    """memset_pattern4 fills bufferSize bytes (render.cpp:282)."""
    r = OracleRenderer(scene_dir['tetra'])
    out = np.zeros((10, 8), dtype=np.uint32)
    r.update_and_render(8, 10, (0, 0, 0, 0, 0, 0), out)
    assert np.all(out == 0x1E1E1E)


def test_resize_keeps_factor_when_area_unchanged(scene_dir):
    """render.cpp:276-279: the raster factor is recomputed only when W*H changes."""
    r = OracleRenderer(scene_dir['full'])
    a = r.update_and_render(64, 48, (0, 0, 0, 0, 0, 0))
    b = r.update_and_render(48, 64, (0, 0, 0, 0, 0, 0))     # same area: factor from height 48 kept
    r2 = OracleRenderer(scene_dir['full'])
    c = r2.update_and_render(48, 64, (0, 0, 0, 0, 0, 0))    # fresh: factor from height 64
    assert not np.array_equal(b, c)
    assert a.shape == (48, 64)


def test_translation_uses_pre_rotation_axes(scene_dir):
    """render.cpp:136-139 runs before :140-150: moving and turning in one call moves along the old
    axes, so (move+turn) != (turn, then move)."""
    r1 = OracleRenderer(scene_dir['full'])
    r1.update_and_render(16, 16, (0, 0, 0, 0, 0, 0))
    r1.update_and_render(16, 16, (10, 0, 0, 0, 50, 0))
    m1 = r1.camera_matrix()
    r2 = OracleRenderer(scene_dir['full'])
    r2.update_and_render(16, 16, (0, 0, 0, 0, 0, 0))
    r2.update_and_render(16, 16, (0, 0, 0, 0, 50, 0))
    r2.update_and_render(16, 16, (10, 0, 0, 0, 50, 0))
    assert not np.allclose(m1[:, 3], r2.camera_matrix()[:, 3])


def test_repeat_add_is_sequential():
    s = np.float32(0.3)
    d = np.float32(1e-3)
    want = s
    for _ in range(777):
        want = np.float32(want + d)
    assert np.float32(repeat_add(float(s), float(d), 777)) == want


@pytest.mark.parametrize('scene_name,pose', [('full', 'P_over'), ('full', 'P_clip')])
def test_row_windows_equal_full_frame_rows(scene_dir, scene_name, pose):
    """The oracle's row-window mode (rows outside the windows walked, not drawn) gives the full
    frame's pixels on the window rows and the background elsewhere."""
    from oracle.oracle import OracleRenderer
    W, H = 320, 240
    full = render_pose(scene_dir[scene_name], poses.script(pose), W, H)
    r = OracleRenderer(scene_dir[scene_name])
    wins = [(0, 9), (100, 117), (239, 240)]
    r.set_row_windows(wins)
    out = None
    for t in poses.script(pose):
        out = r.update_and_render(W, H, t)
    mask = np.zeros(H, dtype=bool)
    for a, b in wins:
        mask[a:b] = True
    assert np.array_equal(out[mask], full[mask])
    assert (out[~mask] == 0x1E1E1E).all()
    assert (full[mask] != 0x1E1E1E).any()


# config.scale = near * tan(fov / 2) with fov = (float)M_PI / 5 (render.cpp:89-92) and
# factor = near * height / (2 * scale) (render.cpp:279), pinned to the correctly rounded float32
# values: tan(fov / 2) lies 0.18 ulp from its float, far from a rounding tie, so every faithful tanf
# (glibc's, Apple's) and a double-precision tan rounded to float give these same bits.
SCALE_BITS = 0x3D05164D
FACTOR_BITS = {240: 0x43B8A938, 480: 0x4438A938, 1080: 0x44CFBE5F, 2160: 0x454FBE5F, 4320: 0x45CFBE5F}


def f32_bits(x) -> int:
    return int(np.float32(x).view(np.uint32))


def test_config_scale_known_answer():
    import math
    f32 = np.float32
    half = f32(f32(math.pi) / f32(5)) / f32(2)
    tan_f = f32(math.tan(float(half)))
    assert f32_bits(f32(0.1) * tan_f) == SCALE_BITS
    r = OracleRenderer.__new__(OracleRenderer)
    r._l = None
    assert f32_bits(r.scale()) == SCALE_BITS


@pytest.mark.parametrize('height', sorted(FACTOR_BITS))
def test_factor_known_answer(scene_dir, height):
    r = OracleRenderer(scene_dir['tetra'])
    r.update_and_render(8, height, (0, 0, 0, 0, 0, 0))
    assert f32_bits(r.factor()) == FACTOR_BITS[height]


def test_parity_sensitivity_tool_runs():
    """tools/parity_sensitivity.py: the variants build and load, and the one that
    cannot move pixels (double-precision tan, same float bits) moves none."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, 'tools', 'parity_sensitivity.py'), '--cases', '1'],
                       capture_output=True, text=True, timeout=300, check=True)
    summary = json.loads(r.stdout.strip().splitlines()[-1])['summary']
    assert summary['tan_double']['differ'] == 0
    assert summary['rsqrt12']['differ'] > 0          # the approximate rsqrt does move pixels
