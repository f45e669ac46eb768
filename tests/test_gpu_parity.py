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
]


@pytest.mark.parametrize('scene_name,pose,w,h', CASES)
def test_frame_matches_oracle(gpu_renderer, scene_dir, scene_name, pose, w, h):
    path = scene_dir[scene_name]
    script = poses.script(pose)
    want = oracle_render_pose(path, script, w, h, extra_frames=1)
    got = render_pose(gpu_renderer, path, script, w, h, extra_frames=1)
    assert np.array_equal(got, want), diff_report(got, want)


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
