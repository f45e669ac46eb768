"""Bounded waits (render_api.cpp "bounded waits"): a stage that is late past the
library's deadline ends the process with exit status 86 and a message naming the stage, the kernel
waited for, the device and the frame -- a dlopen'ed library never hangs its caller (the reference's
failure contract is exit(666), render.cpp:173).

Each case runs one child process with a test hook:
  * S3R_TEST_HOLD_MS: a kernel that spins that long (and then exits by itself) in front of every
    frame's geometry / tile setup -- the frame is late, never lost;
  * S3R_TEST_ARRIVALS_EXTRA: k_geometry's sky-flag publishers wait for one geometry workgroup more
    than the launch has, so their device spin runs into its clock deadline (S3R_SPIN_MS).
The hooks act from the second frame on: the child renders one frame, prints the time, then renders
the frame that is held.  The test asserts the exit status, the message, and that the process ended
within the deadline plus slack -- well before the hold would have let the frame finish.
"""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STALL_EXIT = 86

CHILD = r'''
import sys, time
sys.path.insert(0, {root!r})
from swift3drenderer_amd import poses, scene
from swift3drenderer_amd.renderer import Renderer
scene.write_named('full', {data!r})
r = Renderer({data!r}, device=0)
mode = {mode!r}
if mode == 'tiles':
    import torch
    r.set_raster_path('tiles')
    buf = torch.empty((240, 320), dtype=torch.int32, device='cuda')
    r.render_bands(poses.hold('P_over'), 320, 240, 240, 1, 0, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print('T0', time.time(), flush=True)
    r.render_bands(poses.hold('P_over'), 320, 240, 240, 1, 0, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
else:
    r.set_delivery(mode)
    r.update_and_render(320, 240, poses.hold('P_over'))
    print('T0', time.time(), flush=True)
    r.update_and_render(320, 240, poses.hold('P_over'))
print('FRAME DONE', flush=True)
'''


def run_child(tmp_path, mode, env_extra, limit=60):
    env = dict(os.environ)
    env.update(env_extra)
    code = CHILD.format(root=ROOT, data=str(tmp_path / 'full.bin'), mode=mode)
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=limit)
    end = time.time()
    t0 = [float(l.split()[1]) for l in r.stdout.splitlines() if l.startswith('T0 ')]
    return r, (end - t0[0]) if t0 else None


def check_stall(r, elapsed, deadline_s, hold_s, *needles):
    msg = f'rc {r.returncode}\nstdout:\n{r.stdout}\nstderr:\n{r.stderr}'
    assert r.returncode == STALL_EXIT, msg
    assert 'FRAME DONE' not in r.stdout, msg
    assert 's3r: stall:' in r.stderr, msg
    for n in needles:
        assert n in r.stderr, msg
    assert elapsed is not None and deadline_s <= elapsed + 0.05, msg
    # the deadline, plus the watchdog's period and process teardown; the hold would take hold_s
    assert elapsed < min(deadline_s + 2.0, hold_s - 0.5), msg


@pytest.mark.gpu
def test_late_geometry_ends_the_frame_call_at_the_deadline(tmp_path):
    """Row path, copy delivery: the frame's stream is held past S3R_WAIT_MS; the watchdog armed
    around the part's stream synchronisation ends the process and names the stage."""
    r, el = run_child(tmp_path, 'copy', {'S3R_TEST_HOLD_MS': '5000', 'S3R_WAIT_MS': '600'})
    check_stall(r, el, 0.6, 5.0, 'updateAndRender: the frame part rendered and copied', 'device 0')


@pytest.mark.gpu
def test_late_geometry_under_host_fill_ends_at_the_deadline(tmp_path):
    """Row path, host fill: the fill threads' flag wait and the part's synchronisation are both
    bounded -- whichever reaches the deadline first ends the process."""
    r, el = run_child(tmp_path, 'fill', {'S3R_TEST_HOLD_MS': '5000', 'S3R_WAIT_MS': '600'})
    check_stall(r, el, 0.6, 5.0, 'device 0')


@pytest.mark.gpu
def test_withheld_tile_summary_ends_at_the_deadline(tmp_path):
    """Tile path, asynchronous frame (s3r_render_bands): the setup's summary is withheld past the
    deadline; the host's summary wait polls the geometry stream and ends the process."""
    r, el = run_child(tmp_path, 'tiles', {'S3R_TEST_HOLD_MS': '5000', 'S3R_WAIT_MS': '600'})
    check_stall(r, el, 0.6, 5.0, "tile path: the frame's setup summary", 'k_tile_setup')


@pytest.mark.gpu
def test_inflated_arrivals_end_the_publisher_spin(tmp_path):
    """Host fill: the publishers wait for one arrival more than the launch has.  Their device spin
    stops at S3R_SPIN_MS and stores the error words; a fill thread reports the row block and the
    arrival counts and ends the process -- long before the host deadline."""
    r, el = run_child(tmp_path, 'fill', {'S3R_TEST_ARRIVALS_EXTRA': '1', 'S3R_SPIN_MS': '300', 'S3R_WAIT_MS': '20000'})
    check_stall(r, el, 0.3, 20.0, "sky-flag publisher of row block", 'geometry workgroups arrived')


def test_stall_exit_status_is_declared():
    """The exit status the tests expect is the library's (s3r_kernels.h kStallExit)."""
    text = open(os.path.join(ROOT, 'swift3drenderer_amd', 'csrc', 's3r_kernels.h')).read()
    assert f'constexpr int kStallExit = {STALL_EXIT};' in text
