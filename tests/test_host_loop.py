"""The C++ main-loop driver (host/main_loop.cpp, the counterpart of main.swift:96-153): it dlopens
the library and calls updateAndRender per frame with a double-buffered caller-owned buffer and a
scripted Input sequence.  On the GPU its dumped frames must equal the CPU oracle fed the same
input sequence, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, 'host', 'flythrough.txt')


@pytest.fixture(scope='module')
def host_bin():
    from swift3drenderer_amd import build
    return build.build_host()


def read_script(path):
    """Input tuples per frame, expanded exactly as main_loop.cpp:load_script + its frame loop."""
    steps = []
    with open(path) as f:
        for line in f:
            if line.startswith('#') or line == '\n':
                continue
            v = line.split()
            if len(v) >= 6:
                steps.append((tuple(np.float32(x) for x in v[:6]), int(v[6]) if len(v) > 6 else 1))
    return steps


def inputs_for(steps, frames):
    out, last = [], (0, 0, 0, 0, 0, 0)
    for inp, n in steps:
        for _ in range(n):
            out.append(inp)
            last = inp
    while len(out) < frames:
        out.append((0, 0, 0, 0, last[4], last[5]))
    return out[:frames]


def read_ppm(path):
    with open(path, 'rb') as f:
        data = f.read()
    head = data.split(b'\n', 3)
    w, h = map(int, head[1].split())
    rgb = np.frombuffer(head[3], dtype=np.uint8).reshape(h, w, 3).astype(np.uint32)
    return (rgb[..., 0] << 16) | (rgb[..., 1] << 8) | rgb[..., 2]


def test_host_loop_missing_data_exits_666(host_bin, tmp_path):
    """render.cpp:173 behaviour seen through the driver: exit(666) before any device work."""
    from swift3drenderer_amd.build import LIB
    env = dict(os.environ, S3R_DATA_PATH=str(tmp_path / 'none.bin'))
    r = subprocess.run([host_bin, '--lib', LIB, '--frames', '1', '--size', '8', '8'], env=env,
                       capture_output=True)
    assert r.returncode == 666 & 255


def test_host_loop_bad_library(host_bin, tmp_path):
    r = subprocess.run([host_bin, '--lib', str(tmp_path / 'nope.so')], capture_output=True)
    assert r.returncode == 1 and b'dlopen' in r.stderr


def test_script_expansion():
    steps = read_script(SCRIPT)
    seq = inputs_for(steps, sum(n for _, n in steps) + 3)
    assert seq[0] == steps[0][0]
    assert seq[-1][:4] == (0, 0, 0, 0) and seq[-1][4:] == steps[-1][0][4:]


@pytest.mark.gpu
def test_host_loop_matches_oracle(host_bin, scene_dir, tmp_path):
    from oracle.oracle import OracleRenderer
    from swift3drenderer_amd.build import LIB
    W, H, frames, every = 320, 240, 481, 60
    env = dict(os.environ, S3R_DATA_PATH=scene_dir['full'])
    prefix = str(tmp_path / 'f')
    r = subprocess.run([host_bin, '--lib', LIB, '--size', str(W), str(H), '--frames', str(frames),
                        '--script', SCRIPT, '--dump', prefix, str(every)], env=env, capture_output=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    seq = inputs_for(read_script(SCRIPT), frames)
    o = OracleRenderer(scene_dir['full'])
    checked = 0
    for f, inp in enumerate(seq):
        ref = o.update_and_render(W, H, inp)
        if f % every == 0:
            got = read_ppm(f'{prefix}_{f:05d}.ppm')
            bad = int(np.count_nonzero(got != (ref & 0xFFFFFF)))
            assert bad == 0, f'frame {f}: {bad} pixels differ'
            checked += 1
    assert checked == (frames - 1) // every + 1
