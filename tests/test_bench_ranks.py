"""bench.py's one-process-per-GPU leg (the driver's N-GPU run): every rank renders its
interleaved bands, the parts are gathered to rank 0 and de-interleaved, per-rank times are taken with
a barrier + sync on both sides and the max over ranks reported.  On CPU with gloo (world size 2 and
3): a stub renders each rank's rows of a known frame, the real BandGather gathers them, and the leg's
summary must say the gathered frame equals the whole frame.  The GPU form (RCCL, one rank) is
test_bench_ranks_leg_one_rank_gpu."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, frame, band, steps, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench
    from swift3drenderer_amd.multi import BandGather, band_row_ids, band_rows
    h, w = frame.shape
    bg = BandGather(w, h, band, world, rank, torch.device('cpu'))
    mine = torch.from_numpy(frame[band_row_ids(h, band, world, rank)].view(np.int32).copy())
    calls = {'part': 0}

    def render_part():                       # what s3r_render_bands writes for this rank
        calls['part'] += 1
        bg.send[: len(mine)] = mine

    def allgather_f(x):
        out = [None] * world
        dist.all_gather_object(out, float(x))
        return out

    whole = (lambda: torch.from_numpy(frame.view(np.int32))) if rank == 0 else None
    res = bench.ranks_leg(render_part, whole, lambda: None, lambda: bg.gather(), dist.barrier, allgather_f,
                          w, h, band, world, rank, steps, 4)
    summary = bench.ranks_summary(res, w, h, band, world, steps, 1000.0,
                                  [band_rows(h, band, world, p) for p in range(world)], 'gloo') if rank == 0 else None
    q.put((rank, calls['part'], summary))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,band', [(2, 16), (3, 7)])
def test_ranks_leg_gloo(world, band):
    rng = np.random.default_rng(world)
    frame = rng.integers(0, 1 << 24, size=(100, 37), dtype=np.uint32)
    steps = 5
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frame, band, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    by_rank = {r: (calls, s) for r, calls, s in got}
    # every rank rendered: warm-up + the device pass + the gathered pass (+ its warm-up) + the check frame
    for r in range(world):
        assert by_rank[r][0] == 4 + steps + 2 + steps + 1
    s = by_rank[0][1]
    assert s['gathered_equals_whole_frame'] is True
    assert s['processes'] == world and len(s['per_rank_device_ms']) == world
    assert s['max_rank_device_ms'] == max(s['per_rank_device_ms'])
    assert s['device_fps_N'] > 0 and s['gathered_fps'] > 0
    assert s['device_efficiency_per_gpu'] == round(s['device_fps_N'] / (world * 1000.0), 4)
    assert sum(s['rows_per_rank']) == frame.shape[0]
    json.dumps(s)


def test_bench_parse_ranks_options():
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse(['--ranks-leg', '--rank-devices', '0,0', '--gather-backend', 'gloo'])
    assert a.ranks_leg and a.rank_devices == '0,0' and a.gather_backend == 'gloo'
    assert bench.rank_device(a, 1, torch) == 0


@pytest.mark.gpu
def test_bench_ranks_leg_one_rank_gpu(tmp_path):
    """bench.py with one rank and the ranks leg on: the part rendered into HBM, the RCCL gather (world
    size 1) and the de-interleave kernel; the gathered frame equals rank 0's whole frame."""
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(free_port()))
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--ranks-leg', '--steps', '20', '--warmup', '5',
           '--no-cpu-baseline', '--width', '1280', '--height', '720']
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    line = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith('{')][-1])
    rl = line['ranks']
    assert rl['gathered_equals_whole_frame'] is True
    assert rl['processes'] == 1 and rl['device_fps_N'] > 0 and rl['gathered_fps'] > 0
    assert rl['gather'].startswith('rccl')
