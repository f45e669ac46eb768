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
SESSION = os.path.join(ROOT, 'host', 'session.txt')
f32 = np.float32


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


def expand_session(path, frames, width, height):
    """Per-frame (W, H, Input) of a main_loop script, restated from the reference's own sources:
    input.swift:75-93 (macOS keys / captured mouse, iOS sticks), main.swift:156-165 (resize), in
    float32 like the Swift Input struct.  The Input persists across frames like main.swift's `input`;
    after the script the movement keys are released and the mouse held."""
    steps = []
    with open(path) as f:
        for line in f:
            v = line.split()
            if not v or v[0].startswith('#'):
                continue
            if v[0] == 'mac':
                steps.append(('mac', v[1], f32(v[2]), f32(v[3]), int(v[4]) if len(v) > 4 else 1))
            elif v[0] == 'ios':
                steps.append(('ios', *(f32(x) for x in v[1:5]), int(v[5]) if len(v) > 5 else 1))
            elif v[0] == 'resize':
                steps.append(('resize', int(v[1]), int(v[2])))
            else:
                steps.append(('raw', tuple(f32(x) for x in v[:6]), int(v[6]) if len(v) > 6 else 1))
    inp, mouse, out, w, h = [f32(0)] * 6, [f32(0), f32(0)], [], width, height
    for st in steps:
        if st[0] == 'resize':
            w, h = st[1], st[2]
            continue
        for _ in range(st[-1]):
            if st[0] == 'raw':
                inp = list(st[1])
            elif st[0] == 'mac':
                speed = f32(2) if '+' in st[1] else f32(1)                  # input.swift:78
                inp[0], inp[1] = (speed if k in st[1] else f32(0) for k in 'ws')   # up, down
                inp[2], inp[3] = (speed if k in st[1] else f32(0) for k in 'ad')   # left, right
                mouse = [f32(mouse[0] + st[2]), f32(mouse[1] + st[3])]           # :43-44
                inp[4], inp[5] = mouse                                           # :84
            else:
                lx, ly, rx, ry = st[1:5]
                inp[0], inp[1], inp[2], inp[3] = ly, f32(-ly), f32(-lx), lx      # :87-90
                inp[4] = f32(inp[4] + f32(f32(6) * rx))                          # :91
                inp[5] = f32(inp[5] + f32(f32(6) * ry))
            out.append((w, h, tuple(inp)))
    while len(out) < frames:
        lw, lh, li = out[-1] if out else (w, h, (f32(0),) * 6)
        out.append((lw, lh, (f32(0),) * 4 + tuple(li[4:])))
    return out[:frames]


def read_log(path):
    rows = []
    with open(path) as f:
        for line in f:
            v = line.split()
            rows.append((int(v[1]), int(v[2]), tuple(f32(x) for x in v[3:9])))
    return rows


@pytest.fixture(scope='module')
def stub_lib(tmp_path_factory):
    """A stand-in render library for CPU tests of the driver's own logic (script, input mapping,
    resize): its updateAndRender fills the caller's buffer with a marker and nothing else."""
    d = tmp_path_factory.mktemp('stub')
    src = d / 'stub.c'
    src.write_text('#include "render.h"\n'
                   'void updateAndRender(const PixelData *p, const Input *in) {\n'
                   '  (void)in; for (uint32_t i = 0; i < p->bufferSize / 4; i++) p->buffer[i] = 0x123456u; }\n')
    so = d / 'libstub.so'
    subprocess.run(['gcc', '-O1', '-shared', '-fPIC', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(so)],
                   check=True)
    return str(so)


def test_session_script_inputs_and_resizes(host_bin, stub_lib, tmp_path):
    """main_loop feeds updateAndRender the Input and frame size input.swift / main.swift would: shift
    doubles the key value, iOS sticks give negative left/right/up/down and accumulate the mouse, and
    resizes change W x H (and the realloc'ed double buffer) mid-run."""
    frames = 240
    log = str(tmp_path / 'log.txt')
    r = subprocess.run([host_bin, '--lib', stub_lib, '--size', '320', '240', '--frames', str(frames),
                        '--script', SESSION, '--log', log], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    got = read_log(log)
    want = expand_session(SESSION, frames, 320, 240)
    assert len(got) == frames
    for f, (g, w) in enumerate(zip(got, want)):
        assert g == w, f'frame {f}: driver {g} vs input.swift restatement {w}'
    sizes = {(w, h) for w, h, _ in got}
    assert sizes == {(320, 240), (400, 300), (256, 200)}
    assert any(i[2] < 0 or i[3] < 0 for _, _, i in got)          # iOS: negative left / right
    assert any(i[0] == 2 for _, _, i in got)                      # shift: speed 2


@pytest.mark.gpu
def test_host_loop_session_matches_oracle(host_bin, scene_dir, tmp_path):
    """The scripted session (keys, mouse, sticks, three resizes) through the real library: dumped
    frames equal the oracle's for the same per-frame (W, H, Input) sequence."""
    from oracle.oracle import OracleRenderer
    from swift3drenderer_amd.build import LIB
    frames, every = 240, 10
    env = dict(os.environ, S3R_DATA_PATH=scene_dir['full'])
    prefix = str(tmp_path / 's')
    log = str(tmp_path / 'log.txt')
    r = subprocess.run([host_bin, '--lib', LIB, '--size', '320', '240', '--frames', str(frames), '--script', SESSION,
                        '--dump', prefix, str(every), '--log', log], env=env, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    seq = expand_session(SESSION, frames, 320, 240)
    assert read_log(log) == seq
    o = OracleRenderer(scene_dir['full'])
    for f, (w, h, inp) in enumerate(seq):
        ref = o.update_and_render(w, h, inp)
        if f % every == 0:
            got = read_ppm(f'{prefix}_{f:05d}.ppm')
            assert got.shape == (h, w)
            bad = int(np.count_nonzero(got != (ref & 0xFFFFFF)))
            assert bad == 0, f'frame {f} ({w}x{h}): {bad} pixels differ'


def parse_loop_report(text):
    rep = {}
    for line in text.splitlines():
        v = line.split()
        if line.startswith('frames '):
            rep['mean_ms'] = float(v[v.index('updateAndRender') + 1])
            rep['median_ms'] = float(v[v.index('median') + 1])
        elif v and v[0] == 'host_stats':
            rep.update({v[k]: int(v[k + 1]) for k in range(1, len(v) - 1, 2)})
        elif v and v[0] == 'halves_pinned':
            rep['halves_pinned'] = (int(v[1]), int(v[2]))
    return rep


@pytest.mark.gpu
def test_host_loop_4k_double_buffer_pinned(host_bin, scene_dir):
    """The reference's double buffer (one malloc of 2 * bufferSize, halves alternating,
    main.swift:117-118, :164) at 3840x2160: both halves are page-locked (the registration of the
    second half is merged with the first's across the shared seam page) and no frame takes a
    pageable copy."""
    from swift3drenderer_amd.build import LIB
    env = dict(os.environ, S3R_DATA_PATH=scene_dir['full'])
    r = subprocess.run([host_bin, '--lib', LIB, '--size', '3840', '2160', '--frames', '300'], env=env,
                       capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    rep = parse_loop_report(r.stdout.decode())
    print(rep)
    assert rep['halves_pinned'] == (1, 1), rep
    assert rep['pageable_frames'] == 0 and rep['pinned_frames'] == 300, rep
