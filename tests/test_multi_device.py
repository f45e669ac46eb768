"""Several GPUs behind updateAndRender itself (render_api.cpp, s3r_configure_devices / S3R_DEVICES).

The reference's caller is one process and one thread: main.swift:121 calls updateAndRender
(render.cpp:264-265) once per frame.  With N devices configured the library splits every frame into
interleaved 16-row bands, each device renders its bands and copies them straight into
their rows of the caller's buffer over its own link.  On the one-GPU test box the N "devices" are N
independent renderers on GPU 0 (their own scene replicas, buffer sets, streams and worker threads):
the split, the threads and the per-part delivery are exercised; only the N physical links are not.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from swift3drenderer_amd import poses
from swift3drenderer_amd.renderer import band_row_ids, band_rows_local, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- CPU: bookkeeping and configuration
@pytest.mark.parametrize('n', [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize('h', [1, 5, 15, 16, 17, 240, 333, 1080, 2160, 4320])
def test_band_rows_partition_the_frame(n, h):
    """Every frame row belongs to exactly one part; each part's row count is what the library sizes
    its device buffer and its copies by."""
    seen = np.zeros(h, dtype=int)
    for p in range(n):
        ids = band_row_ids(h, 16, n, p)
        assert band_rows_local(h, 16, n, p) == len(ids)
        assert np.all(np.diff(ids) > 0)
        assert np.all((ids // 16) % n == p)
        seen[ids] += 1
    assert np.all(seen == 1)


def test_configure_devices_arguments():
    lib = load_library()
    ids = (ctypes.c_int * 3)(0, 1, 2)
    out = (ctypes.c_int * 8)()
    try:
        assert lib.s3r_configure_devices(ids, 3, 16) == 0
        assert lib.s3r_devices(out, 8) == 3 and list(out[:3]) == [0, 1, 2]
        assert lib.s3r_devices(out, 1) == 3                          # count beyond max_ids
        bad = (ctypes.c_int * 2)(0, -1)
        assert lib.s3r_configure_devices(bad, 2, 16) == -1
        assert lib.s3r_configure_devices(None, 2, 16) == -1
        assert lib.s3r_configure_devices(ids, 65, 16) == -1
        assert lib.s3r_configure_devices(ids, -1, 16) == -1
    finally:
        assert lib.s3r_configure_devices(None, 0, 0) == 0
    lib.s3r_configure(None, 3)
    assert lib.s3r_devices(out, 8) == 1 and out[0] == 3              # one device: s3r_configure's
    lib.s3r_configure(None, -1)


def test_devices_from_environment():
    """S3R_DEVICES is how a caller that binds only updateAndRender (the Swift app) asks for N GPUs."""
    code = ('import ctypes, sys; sys.path.insert(0, %r)\n'
            'from swift3drenderer_amd.renderer import load_library\n'
            'lib = load_library(); out = (ctypes.c_int * 8)()\n'
            'n = lib.s3r_devices(out, 8); print(n, list(out[:n]))\n') % ROOT
    for env_val, want in (('0,1,2,3', '4 [0, 1, 2, 3]'), ('2, 5', '2 [2, 5]'), ('x', '1 [-1]')):
        env = dict(os.environ, S3R_DEVICES=env_val)
        r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, check=True)
        assert r.stdout.strip() == want, (env_val, r.stdout, r.stderr)


# ---------------------------------------------------------------- GPU: frames against the oracle
def diff_report(a, b):
    d = a != b
    n = int(d.sum())
    if n == 0:
        return 'identical'
    ys, xs = np.nonzero(d)
    return f'{n} pixels differ, first at (x={xs[0]}, y={ys[0]}): gpu {a[ys[0], xs[0]]:06x} oracle {b[ys[0], xs[0]]:06x}'


@pytest.fixture
def multi(gpu_renderer):
    """The session renderer, returned to one device afterwards."""
    yield gpu_renderer
    gpu_renderer.configure_devices([])


def frames_vs_oracle(r, path, seq, devices, band=0):
    """Run (W, H, Input) frames through updateAndRender on `devices` parts, into the halves of one
    2 * bufferSize allocation used alternately (main.swift:117-118, :164), against the oracle."""
    from oracle.oracle import OracleRenderer
    r.configure_devices(devices, band)
    r.configure(path)
    o = OracleRenderer(path)
    mem, cur = None, 0
    for k, (w, h, inp) in enumerate(seq):
        if mem is None or mem.size != 2 * w * h:
            mem, cur = np.empty(2 * w * h, dtype=np.uint32), 0     # realloc on resize (main.swift:164)
        half = mem[cur * w * h:(cur + 1) * w * h].reshape(h, w)
        cur ^= 1
        got = r.update_and_render(w, h, inp, half)
        want = o.update_and_render(w, h, inp)
        assert np.array_equal(got, want), f'frame {k} {w}x{h} on {len(devices)} parts: ' + diff_report(got, want)
    assert r.devices() == list(devices)


def pose_frames(pose, w, h, extra=2):
    script = poses.script(pose)
    return [(w, h, t) for t in script] + [(w, h, poses.hold(pose))] * extra


@pytest.mark.gpu
@pytest.mark.parametrize('w,h', [(3840, 2160), (7680, 4320)])
def test_eight_parts_full_frames(multi, scene_dir, w, h):
    """BASELINE config 3's frame and config 4's (7680x4320, its 8-way split) through updateAndRender
    on 8 parts: bit-identical to the oracle."""
    frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_over', w, h), [0] * 8)


@pytest.mark.gpu
@pytest.mark.parametrize('n', [2, 3, 4])
@pytest.mark.parametrize('scene_name,pose,w,h', [('full', 'P_over', 1000, 333), ('full', 'P_clip', 640, 480),
                                                 ('flat', 'P_over', 1920, 1080), ('full', 'P_id', 17, 5),
                                                 ('regular', 'P_floor', 1280, 720)])
def test_parts_match_oracle(multi, scene_dir, n, scene_name, pose, w, h):
    frames_vs_oracle(multi, scene_dir[scene_name], pose_frames(pose, w, h), [0] * n)


@pytest.mark.gpu
def test_parts_resize_and_flythrough(multi, scene_dir):
    """Camera moving every frame, resizes (new W x H, a reallocated double buffer) and band heights
    that do not divide the frame."""
    rng = np.random.default_rng(5)
    mouse = np.array([0.0, -120.0])
    seq = []
    for k in range(20):
        w, h = [(640, 480), (333, 250), (800, 600)][k // 7]
        keys = rng.integers(0, 2, 4) * rng.uniform(0, 10, 4)
        mouse += rng.normal(0, 10, 2)
        seq.append((w, h, (*keys, *mouse)))
    frames_vs_oracle(multi, scene_dir['full'], seq, [0, 0, 0], band=7)


@pytest.mark.gpu
def test_parts_tile_path(multi, scene_dir):
    """The tile fragment path split across parts (forced on the packaged scene)."""
    try:
        multi.set_raster_path('tiles')
        frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_over', 1280, 720), [0] * 4)
    finally:
        multi.set_raster_path('auto')


@pytest.mark.gpu
def test_parts_pin_the_callers_double_buffer(multi, scene_dir):
    """With parts on several devices every frame still lands in a page-locked buffer: both halves of
    the double buffer are registered (merged at the seam page), no frame is copied pageable."""
    w, h = 1920, 1080
    frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_over', w, h, extra=6), [0] * 4)
    st = multi.host_stats()
    assert st['pageable_frames'] == 0 and st['pinned_frames'] >= 9, st


@pytest.mark.gpu
@pytest.mark.parametrize('mode,fill', [('copy', -1), ('direct', -1), ('fill', 1), ('fill', 3), ('fill', 16),
                                       ('auto', -1)])
@pytest.mark.parametrize('devices', [[0], [0, 0, 0]])
def test_delivery_modes_match_oracle(multi, scene_dir, mode, fill, devices):
    """Every delivery of updateAndRender -- rendered into HBM and copied over the link, written by the
    fragment kernel straight into the caller's buffer, or host fill (covered bins by the GPU, sky bins
    by `fill` host threads; render_api.cpp) -- gives the oracle's frames, on one device and on three
    parts, at 4K (384-px bins) and 1080p (128-px bins)."""
    try:
        multi.set_delivery(mode, fill)
        frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_over', 1920, 1080), devices)
        frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_id', 3840, 2160, extra=1), devices)
        st = multi.host_stats()                      # (counters restart at each configure)
        used = mode if mode != 'auto' else 'fill'
        assert st[f'{used}_frames'] == 2 and st['pinned_frames'] == 2, st
        assert multi.delivery() == mode
    finally:
        multi.set_delivery('env')


@pytest.mark.gpu
def test_host_fill_sparse_and_empty_frames(multi, scene_dir, tmp_path):
    """Host fill when nothing is visible (every bin sky) and when the scene is empty."""
    from swift3drenderer_amd import scene
    empty = str(tmp_path / 'empty.bin')
    scene.write_scene(scene.Scene(), empty)
    frames_vs_oracle(multi, empty, pose_frames('P_over', 640, 480), [0])
    away = [(640, 480, (0, 0, 0, 0, 0, 0)), (640, 480, (0, 0, 0, 0, 4000.0, 0.0)), (640, 480, (0, 0, 0, 0, 8000.0, 0.0))]
    frames_vs_oracle(multi, scene_dir['full'], away, [0, 0])
    assert multi.host_stats()['fill_frames'] > 0


@pytest.mark.gpu
@pytest.mark.parametrize('split', [0, 3, 8])
@pytest.mark.parametrize('devices', [[0], [0, 0]])
def test_host_fill_split_matches_oracle(multi, scene_dir, monkeypatch, split, devices):
    """Host fill with a fixed share of the sky bins (S3R_FILL_GPU eighths) written by the GPU instead
    of the fill threads -- the adaptive split's every position gives the oracle's frames."""
    monkeypatch.setenv('S3R_FILL_GPU', str(split))
    multi.set_delivery('fill')
    try:
        frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_over', 1920, 1080), devices)
        frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_clip', 3840, 2160, extra=1), devices)
        st = multi.host_stats()
        assert st['fill_gpu_eighths'] == split and st['fill_frames'] == 3, st
    finally:
        multi.set_delivery('env')


def l3_domains():
    """CPU -> last-level-cache domain id, from sysfs (empty where the topology is not exposed)."""
    import glob
    dom = {}
    for path in glob.glob('/sys/devices/system/cpu/cpu[0-9]*/cache/index3/shared_cpu_list'):
        cpu = int(path.split('/cpu/cpu')[1].split('/')[0])
        dom[cpu] = open(path).read().strip()
    return dom


@pytest.mark.gpu
@pytest.mark.parametrize('pin', ['1', '0'])
def test_host_fill_thread_placement(multi, scene_dir, monkeypatch, pin):
    """Host fill threads placed one per CPU domain (render_api.cpp fill_placement): frames still match
    the oracle, the profile reports the placement and the buffer's node, and the threads' last CPUs lie
    in distinct last-level-cache domains; S3R_FILL_PIN=0 leaves them to the scheduler."""
    monkeypatch.setenv('S3R_FILL_PIN', pin)
    multi.set_delivery('fill', 4)            # (restarts the fill threads: placement is redone)
    try:
        multi.fill_profile()
        frames_vs_oracle(multi, scene_dir['full'], pose_frames('P_over', 1920, 1080, extra=4), [0])
        prof = multi.fill_profile()
        assert prof['frames'] >= 5 and len(prof['threads']) == 4, prof
        assert sum(t['px'] for t in prof['threads']) > 0
        dom = l3_domains()
        if pin == '0':
            assert not prof['placed'], prof
        elif len(set(dom.values())) >= 4:
            assert prof['placed'], prof
            assert len({dom[t['cpu']] for t in prof['threads']}) == 4, (prof, dom)
    finally:
        multi.set_delivery('env')
