"""GPU parity: frames from the gfx950 library (through its C ABI) == the CPU oracle, bit for bit.

Bar: bit-exact u32 frames (stricter than north_star's +-1 LSB per RGB channel).  The oracle is the
plain-C restatement of render.cpp (oracle/render_oracle.c; parity unpinned, see its header).
"""
import numpy as np
import pytest

from oracle.oracle import render_pose as oracle_render_pose
from swift3drenderer_amd import poses
from swift3drenderer_amd.renderer import render_pose

pytestmark = pytest.mark.gpu


def diff_report(a, b):
    d = a != b
    n = int(d.sum())
    if n == 0:
        return 'identical'
    ys, xs = np.nonzero(d)
    ch = [np.abs(((a >> s) & 255).astype(int) - ((b >> s) & 255).astype(int)).max() for s in (16, 8, 0)]
    return f'{n} pixels differ, first at (x={xs[0]}, y={ys[0]}): gpu {a[ys[0], xs[0]]:06x} oracle {b[ys[0], xs[0]]:06x}; max |d| per channel {ch}'


CASES = [
    ('full', 'P_id', 640, 480),
    ('full', 'P_over', 640, 480),
    ('full', 'P_clip', 640, 480),
    ('full', 'P_floor', 640, 480),
    ('full', 'P_strafe', 640, 480),
    ('flat', 'P_over', 640, 480),
    ('tetra', 'P_tetra', 640, 480),
    ('full', 'P_over', 320, 240),
    ('full', 'P_id', 1920, 1080),
    ('full', 'P_over', 1920, 1080),
    ('full', 'P_clip', 1920, 1080),
    ('flat', 'P_over', 1920, 1080),
    ('regular', 'P_over', 1280, 720),
    ('regular', 'P_floor', 1280, 720),
    ('full', 'P_over', 1000, 333),     # width not a multiple of the 512-pixel segment
    ('full', 'P_id', 17, 5),           # tiny frame
    ('full', 'P_over', 3840, 2160),    # BASELINE config 3 (the bench workload)
    ('full', 'P_id', 3840, 2160),
    ('full', 'P_over', 7680, 4320),    # BASELINE config 4's frame, whole on one GPU
]


@pytest.mark.parametrize('scene_name,pose,w,h', CASES)
def test_frame_matches_oracle(gpu_renderer, scene_dir, scene_name, pose, w, h):
    path = scene_dir[scene_name]
    script = poses.script(pose)
    want = oracle_render_pose(path, script, w, h, extra_frames=1)
    got = render_pose(gpu_renderer, path, script, w, h, extra_frames=1)
    assert np.array_equal(got, want), diff_report(got, want)


def test_clip_slots_follow_the_near_plane(gpu_renderer, scene_dir):
    """k_geometry leaves out the clip-appended slots (and marks their records dead) when the host finds
    no triangle crossing the near plane (render_api.cpp near_plane_crossing, render.cpp:308): poses that
    cross it and poses that do not, alternating in one session, each frame against the oracle."""
    path = scene_dir['full']
    for pose in ['P_clip', 'P_over', 'P_clip', 'P_id', 'P_clip', 'P_floor']:
        script = poses.script(pose)
        want = oracle_render_pose(path, script, 640, 480, extra_frames=1)
        got = render_pose(gpu_renderer, path, script, 640, 480, extra_frames=1)
        assert np.array_equal(got, want), (pose, diff_report(got, want))


def test_slot_cull_turning_camera(gpu_renderer, scene_dir):
    """k_geometry launches only the slots the host does not surely reject (render_api.cpp cull_slots:
    behind the near plane, off the frame, back faces and slivers of area < 10, render.cpp:306-317): the
    camera turns through a full circle and pitches, so triangles leave the frame on every side and turn
    their backs, each frame against the oracle (tiny and wide frames too)."""
    from oracle.oracle import OracleRenderer
    for name, w, h in [('full', 320, 240), ('regular', 256, 96), ('full', 33, 7)]:
        path = scene_dir[name]
        o = OracleRenderer(path)
        gpu_renderer.configure(path)
        for k in range(30):
            inp = (0, 0, 0, 0, 24.0 * k, 40.0 * np.sin(k / 3.0))
            want = o.update_and_render(w, h, inp)
            got = gpu_renderer.update_and_render(w, h, inp)
            assert np.array_equal(got, want), f'{name} {w}x{h} frame {k} {inp}: ' + diff_report(got, want)


def test_resize_between_calls(gpu_renderer, scene_dir):
    """render.cpp:275-280: factor changes only when W*H changes; camera state carries over."""
    from oracle.oracle import OracleRenderer
    path = scene_dir['full']
    o = OracleRenderer(path)
    gpu_renderer.configure(path)
    seq = [(640, 480, (0, 0, 0, 0, 0, 0)), (640, 480, (0, 0, 0, 0, 0, -150)), (320, 240, (0, 150, 0, 0, 0, -150)),
           (480, 640, (0, 0, 0, 0, 0, -90)), (640, 480, (0, 0, 3, 0, 10, -90)), (800, 600, (0, 0, 0, 0, 10, -90))]
    for w, h, inp in seq:
        want = o.update_and_render(w, h, inp)
        got = gpu_renderer.update_and_render(w, h, inp)
        assert np.array_equal(got, want), f'{w}x{h} {inp}: ' + diff_report(got, want)


def test_long_walk_sequence(gpu_renderer, scene_dir):
    """A flythrough: per-frame camera updates, clipping on and off."""
    from oracle.oracle import OracleRenderer
    path = scene_dir['full']
    o = OracleRenderer(path)
    gpu_renderer.configure(path)
    rng = np.random.default_rng(7)
    mouse = np.zeros(2)
    for k in range(24):
        keys = rng.integers(0, 2, 4) * rng.uniform(0, 20, 4)
        mouse += rng.normal(0, 15, 2)
        inp = (*keys, *mouse)
        want = o.update_and_render(480, 320, inp)
        got = gpu_renderer.update_and_render(480, 320, inp)
        assert np.array_equal(got, want), f'frame {k} {inp}: ' + diff_report(got, want)


def test_pipelined_frames_on_mixed_streams(gpu_renderer, scene_dir):
    """Frames issued without waiting (more in flight than the 4 buffer sets), alternating between two
    caller streams, with tile-path frames and a host-buffer updateAndRender in between: every frame
    equals the oracle's frame for the same input sequence.  Exercises the event-free buffer-set reuse
    (render_api.cpp wait_set_free), the stream hand-off and the row/tile path switch."""
    import torch
    from oracle.oracle import OracleRenderer
    path = scene_dir['full']
    o = OracleRenderer(path)
    gpu_renderer.configure(path)
    W, H = 320, 240
    rng = np.random.default_rng(11)
    inputs, wants = [], []
    mouse = np.array([0.0, -120.0])
    for k in range(18):                      # the oracle first, so the GPU frames go out back to back
        keys = rng.integers(0, 2, 4) * rng.uniform(0, 10, 4)
        mouse += rng.normal(0, 12, 2)
        inputs.append((*keys, *mouse))
        wants.append(o.update_and_render(W, H, inputs[-1]))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = []
    for k, inp in enumerate(inputs):
        if k == 7:
            gpu_renderer.set_raster_path('tiles')
        if k == 10:
            gpu_renderer.set_raster_path('auto')
        if k == 13:
            got = gpu_renderer.update_and_render(W, H, inp)          # host buffer, the library's own stream
            assert np.array_equal(got, wants[k]), f'frame {k} (updateAndRender): ' + diff_report(got, wants[k])
            continue
        buf = torch.empty((H, W), dtype=torch.int32, device='cuda')
        st = streams[(k // 3) % 2]
        with torch.cuda.stream(st):
            gpu_renderer.render_bands(inp, W, H, H, 1, 0, buf.data_ptr(), st.cuda_stream)
        bufs.append((k, buf))
    torch.cuda.synchronize()
    for k, buf in bufs:
        got = buf.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, wants[k]), f'frame {k}: ' + diff_report(got, wants[k])


def test_empty_scene(gpu_renderer, tmp_path):
    """A data.bin without triangles (or textures): every pixel is the background (render.cpp:282)."""
    from swift3drenderer_amd import scene
    path = str(tmp_path / 'empty.bin')
    scene.write_scene(scene.Scene(), path)
    script = poses.script('P_over')
    want = oracle_render_pose(path, script, 160, 120)
    got = render_pose(gpu_renderer, path, script, 160, 120)
    assert np.array_equal(got, want), diff_report(got, want)
    assert (got == 0x1E1E1E).all()


@pytest.mark.parametrize('w,h', [(1, 1), (1, 300), (300, 1), (65, 2), (2, 65), (385, 7)])
def test_thin_frames(gpu_renderer, scene_dir, w, h):
    """Single-pixel, single-row and single-column frames; widths just past a chunk / a segment."""
    script = poses.script('P_over')
    want = oracle_render_pose(scene_dir['full'], script, w, h)
    got = render_pose(gpu_renderer, scene_dir['full'], script, w, h)
    assert np.array_equal(got, want), diff_report(got, want)


def test_nothing_visible(gpu_renderer, scene_dir):
    """Camera turned away from every triangle (all culled off screen, render.cpp:312-315)."""
    script = [(0, 0, 0, 0, 4000.0, 0.0), (0, 0, 0, 0, 8000.0, 0.0)]
    want = oracle_render_pose(scene_dir['full'], script, 320, 240)
    got = render_pose(gpu_renderer, scene_dir['full'], script, 320, 240)
    assert np.array_equal(got, want), diff_report(got, want)


def stacked_quads_scene(path, n=160, size=1.0):
    """n coloured quads (2n triangles) stacked in front of the identity camera, slightly shifted and
    tilted so that their depths interleave; every 10th repeats the previous depth (tie order).
    size = 1 fills the view; smaller quads cover the centre."""
    from swift3drenderer_amd import scene
    sc = scene.Scene()
    rng = np.random.default_rng(3)
    z = -5.0
    for i in range(n):
        if i % 10:
            z -= 0.05
        dx, dy, tilt = (rng.uniform(-0.6, 0.6) * size, rng.uniform(-0.4, 0.4) * size,
                        rng.uniform(-0.3, 0.3) * size)
        a, b = 4 * size, 3 * size
        k = len(sc.vertices)
        sc.vertices += [scene.v3(-a + dx, -b + dy, z - tilt), scene.v3(a + dx, -b + dy, z + tilt),
                        scene.v3(-a + dx, b + dy, z - tilt), scene.v3(a + dx, b + dy, z + tilt)]
        sc.vertex_indexes += [k, k + 2, k + 1, k + 1, k + 2, k + 3]
        j = len(sc.attributes)
        cols = [tuple(float(c) for c in rng.uniform(0, 255, 3)) for _ in range(4)]
        nrm = scene.v3(0, 0, 1)
        sc.attributes += [(nrm, ("c", scene.v3(*cols[q]))) for q in (0, 2, 1, 1, 2, 3)]
        sc.attribute_indexes += list(range(j, j + 6))
    scene.write_scene(sc, path)


def test_row_path_list_overflow(gpu_renderer, tmp_path):
    """320 stacked triangles cover every fragment workgroup: more than the 128 a workgroup lists from
    its bin's pair records (kPairMax), so the row path takes its in-kernel slot-scan rounds (build_list)."""
    path = str(tmp_path / 'stack.bin')
    stacked_quads_scene(path)
    for w, h in ((320, 240), (1280, 720)):
        ident = [(0, 0, 0, 0, 0, 0)]
        want = oracle_render_pose(path, ident, w, h)
        got = render_pose(gpu_renderer, path, ident, w, h)
        assert gpu_renderer.raster_path() == 'rows'
        assert (want != 0x1E1E1E).mean() > 0.5
        assert np.array_equal(got, want), f'{w}x{h}: ' + diff_report(got, want)


def _parts_vs_oracle(r, path, script, W, H, nparts, band, parts):
    import torch
    from swift3drenderer_amd.multi import band_row_ids
    want = oracle_render_pose(path, script, W, H)
    r.configure(path)
    dev = torch.device('cuda', 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    hold = (0, 0, 0, 0) + tuple(script[-1][4:6])
    scratch = torch.empty((H, W), dtype=torch.int32, device=dev)
    for t in script:                                         # the script's camera, one frame each
        r.render_bands(t, W, H, band, nparts, 0, scratch.data_ptr(), st)
    torch.cuda.synchronize()
    for p in parts:
        ids = band_row_ids(H, band, nparts, p)
        buf = torch.full((max(len(ids), 1), W), -1, dtype=torch.int32, device=dev)
        n = r.render_bands(hold, W, H, band, nparts, p, buf.data_ptr(), st)
        assert n == len(ids)
        got = buf.cpu().numpy().view(np.uint32)[:n]
        assert np.array_equal(got, want[ids]), f'part {p} of {nparts}: ' + diff_report(got, want[ids])


def test_small_parts_match_oracle(gpu_renderer, scene_dir):
    """Every GPU's rows of an 8-way 4K split (128-px fragment segments at this size): each part is
    bit-identical to the oracle's rows of the whole frame."""
    _parts_vs_oracle(gpu_renderer, scene_dir['full'], poses.script('P_over'), 3840, 2160, 8, 16, range(8))


def test_small_parts_overflow(gpu_renderer, tmp_path):
    """The list-overflow rounds (more than 128 triangles per workgroup) in one GPU's rows of an
    8-way 4K split."""
    path = str(tmp_path / 'stack-small.bin')
    stacked_quads_scene(path, size=0.08)
    _parts_vs_oracle(gpu_renderer, path, [(0, 0, 0, 0, 0, 0)], 3840, 2160, 8, 16, (0, 5))


def test_longest_first_order(gpu_renderer, scene_dir, monkeypatch):
    """Longest-first fragment order (k_geometry's order column from earlier frames' per-bin costs,
    render_api.cpp kLptMinBins) forced on for every frame size: held, moving, resized and pipelined
    frames all equal the oracle's -- the order is a permutation of the bins, never a change of pixels."""
    import torch
    from oracle.oracle import OracleRenderer
    monkeypatch.setenv('S3R_LPT_MIN', '0')
    path = scene_dir['full']
    o = OracleRenderer(path)
    gpu_renderer.configure(path)
    seq = [(640, 480, (0, 0, 0, 0, 0, -150))] * 3 + [(640, 480, (2, 0, 1, 0, 5, -150)), (320, 240, (0, 0, 0, 0, 0, -150)),
                                                  (800, 600, (0, 3, 0, 0, -4, -140)), (800, 600, (0, 0, 0, 0, 0, -140))]
    for k, (w, h, inp) in enumerate(seq):
        want = o.update_and_render(w, h, inp)
        got = gpu_renderer.update_and_render(w, h, inp)
        assert np.array_equal(got, want), f'frame {k} {w}x{h}: ' + diff_report(got, want)
    W, H = 640, 480
    inputs = [(0, 0, 0, 0, 3.0 * k, -150 + k) for k in range(10)]
    wants = [o.update_and_render(W, H, inp) for inp in inputs]
    st = torch.cuda.Stream()
    bufs = []
    for inp in inputs:                      # back to back: several frames in flight
        buf = torch.empty((H, W), dtype=torch.int32, device='cuda')
        with torch.cuda.stream(st):
            gpu_renderer.render_bands(inp, W, H, H, 1, 0, buf.data_ptr(), st.cuda_stream)
        bufs.append(buf)
    torch.cuda.synchronize()
    for k, buf in enumerate(bufs):
        got = buf.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, wants[k]), f'pipelined frame {k}: ' + diff_report(got, wants[k])


@pytest.mark.parametrize('scene_name,pose,w,h', [('full', 'P_over', 640, 480), ('full', 'P_clip', 640, 480),
                                                 ('flat', 'P_over', 640, 480), ('tetra', 'P_tetra', 640, 480),
                                                 ('regular', 'P_floor', 1280, 720), ('full', 'P_id', 1000, 333)])
@pytest.mark.parametrize('waterfall', [False, True])
def test_widest_segments_match_oracle(gpu_renderer, scene_dir, monkeypatch, scene_name, pose, w, h, waterfall):
    """Small frames forced onto the widest fragment segments (S3R_MIN_BLOCKS=1: 384-pixel segments,
    the launch shape of 4K and 8K frames), with the shading by per-lane gathers or by the waterfall
    over the wave's distinct winners (S3R_WATERFALL_BINS=0: the 4K / 8K instance): every frame equals
    the oracle's."""
    monkeypatch.setenv('S3R_MIN_BLOCKS', '1')
    monkeypatch.setenv('S3R_WATERFALL_BINS', '0' if waterfall else '1000000000')
    path = scene_dir[scene_name]
    script = poses.script(pose)
    want = oracle_render_pose(path, script, w, h, extra_frames=1)
    got = render_pose(gpu_renderer, path, script, w, h, extra_frames=1)
    assert np.array_equal(got, want), diff_report(got, want)


@pytest.mark.parametrize('height', [240, 480, 1080, 2160, 4320])
def test_factor_known_answer_gpu(gpu_renderer, scene_dir, height):
    """The library's raster factor (render.cpp:279, host float32) has the correctly rounded bits
    pinned in tests/test_oracle.py."""
    from test_oracle import FACTOR_BITS, f32_bits
    gpu_renderer.configure(scene_dir['tetra'])
    gpu_renderer.update_and_render(8, height, (0, 0, 0, 0, 0, 0))
    _, factor = gpu_renderer.camera()
    assert f32_bits(factor) == FACTOR_BITS[height]
