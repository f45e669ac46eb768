#!/usr/bin/env python3
"""Benchmark: frames/s and Mpixels/s of updateAndRender's frame at 3840x2160 on the packaged scene.

Step = one frame of the hot path (render.cpp:264-384): camera update, vertex transform, triangle
setup/clip/cull, fragment stage, with the frame left in device memory (HBM-resident value; the
PCIe-inclusive updateAndRender rate is reported separately as `e2e_fps_with_d2h`).  With N GPUs
the frame's rows are split into interleaved bands (band g -> rank g % N) and every rank renders its
bands into its own HBM: `value` counts frames whose rows are all rendered, left where they were
rendered, as the one-GPU frame is left in its GPU's HBM.  Reassembling every frame on rank 0 with
one RCCL gather over xGMI (torch.distributed, nccl backend) is timed in a second loop and reported
as `gathered_fps`; the frame is then 33 MB per 4K frame moving over xGMI, and that loop is bound by
rank 0's xGMI ingest, not by rendering (multi-GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'frames/sec + Mpixels/s at 3840x2160, data.bin scene; 1/2/4/8-GPU scaling'
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md, HBM3E peak (spec)
TRI_SETUP_BYTES = 240    # sizeof(TriSetup)
RASTER_REC_BYTES = 64    # sizeof(RasterRec), tile path


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=200)
    p.add_argument('--warmup', type=int, default=20)
    p.add_argument('--width', type=int, default=3840)
    p.add_argument('--height', type=int, default=2160)
    p.add_argument('--scene', default='full')
    p.add_argument('--pose', default='P_over')
    p.add_argument('--band', type=int, default=16, help='rows per interleaved band (multi-GPU)')
    p.add_argument('--cpu-seconds', type=float, default=10.0, help='CPU-baseline sample budget')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-e2e', action='store_true')
    p.add_argument('--backend', default='nccl', help="torch.distributed backend: nccl (RCCL) or gloo "
                   "(rehearsal only: gathers through host memory)")
    return p.parse_args()


def cpu_model() -> str:
    try:
        out = subprocess.run(['lscpu'], capture_output=True, text=True).stdout
        for line in out.splitlines():
            if line.startswith('Model name'):
                return line.split(':', 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or 'unknown'


def cpu_baseline(data_path, script, hold, w, h, budget_s):
    """The CPU oracle (a single-threaded C restatement of render.cpp) on this host, bounded sample."""
    from oracle.oracle import OracleRenderer
    r = OracleRenderer(data_path)
    for t in script:
        r.update_and_render(w, h, t)
    import numpy as np
    out = np.empty((h, w), dtype=np.uint32)
    frames, t0 = 0, time.perf_counter()
    while True:
        r.update_and_render(w, h, hold, out)
        frames += 1
        el = time.perf_counter() - t0
        if (el >= budget_s and frames >= 3) or el >= 3 * budget_s or frames >= 2000:
            break
    return frames / el, frames, el


def load_traffic(workload_key):
    """HBM bytes per fragment launch from the committed rocprofv3 --pmc summary (profiles/)."""
    p = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(workload_key, {}).get('hbm_bytes_per_launch')
    except Exception:
        return None


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit('--gpus N>1 needs torch.distributed.run with N processes')
    # one process per GPU; on a box with fewer GPUs than ranks (a gloo rehearsal) ranks share them
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if a.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(a.backend)

    from swift3drenderer_amd import poses, scene
    from swift3drenderer_amd.multi import BandGather
    from swift3drenderer_amd.renderer import Renderer

    tmp = tempfile.mkdtemp(prefix=f's3r_bench_{rank}_')
    data_path = os.path.join(tmp, f'{a.scene}.bin')
    scene.write_named(a.scene, data_path)

    W, H, B = a.width, a.height, a.band
    N = world
    script = poses.script(a.pose)
    hold = poses.hold(a.pose)
    from swift3drenderer_amd.abi import Input
    hold_in = Input.of(hold)                 # built once: the timed loops pass it straight through

    r = Renderer(data_path, device=local)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    rows = r.lib.s3r_band_rows_local(H, B, N, rank) if N > 1 else H
    local_buf = torch.empty((max(rows, 1), W), dtype=torch.int32, device=dev)
    if N > 1:
        # gloo rehearsal (one box, ranks sharing a GPU): the same gather through host memory
        gdev = dev if a.backend == 'nccl' else torch.device('cpu')
        bg = BandGather(W, H, B, N, rank, gdev)

    def render(inp):
        """One frame: this rank's rows of the frame into its device buffer (HBM-resident)."""
        if N == 1:
            r.render_bands(inp, W, H, H, 1, 0, local_buf.data_ptr(), sptr)
        elif a.backend == 'nccl':
            r.render_bands(inp, W, H, B, N, rank, bg.send.data_ptr(), sptr)   # straight into the send buffer
        else:
            r.render_bands(inp, W, H, B, N, rank, local_buf.data_ptr(), sptr)

    def gathered(inp):
        """One frame reassembled on rank 0: render, then one gather (RCCL over xGMI)."""
        render(inp)
        if a.backend != 'nccl':
            bg.send[:rows].copy_(local_buf[:rows].cpu())
        bg.gather()

    def timed(fn, k):
        """k frames between barrier + sync pairs; the max over ranks of the elapsed time."""
        if N > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn(hold_in)
        torch.cuda.synchronize(dev)
        if N > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if N > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev if a.backend == 'nccl' else 'cpu')
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    for t in script:                     # pose script (first call initialises), untimed
        render(t)
    for _ in range(a.warmup):
        render(hold)
    torch.cuda.synchronize(dev)

    # value: frames rendered, each frame's rows left in the HBM of the ranks that own them (N = 1:
    # the whole frame in one GPU's HBM).  No HIP-event timing inside this loop.
    el = timed(render, a.steps)

    # device-side kernel times from HIP events, in a separate pass of the same frames
    r.timing(True)
    for _ in range(a.steps):
        render(hold)
    frag_ms, frame_ms, nfr = r.timing_collect()
    r.timing(False)

    # the same frames reassembled on rank 0 by one gather per frame (reported beside value)
    gathered_fps = None
    e2e_multi = None
    if N > 1:
        for _ in range(3):
            gathered(hold)
        kg = max(10, min(100, a.steps))
        gathered_fps = kg / timed(gathered, kg)
        # the same frames delivered into ONE host frame shared by the node's ranks (/dev/shm), each
        # rank copying its own bands over its own GPU's PCIe link (s3r_bands_to_host): the
        # multi-GPU counterpart of updateAndRender's host buffer
        from swift3drenderer_amd.multi import HostFrame
        hf = HostFrame(W, H, rank)
        src = bg.send if a.backend == 'nccl' else local_buf

        def delivered(inp):
            render(inp)
            r.bands_to_host(src.data_ptr(), W, H, B, N, rank, hf.frame, sptr)

        for _ in range(3):
            delivered(hold)
        e2e_multi = kg / timed(delivered, kg)
        r.unregister_host(hf.frame)            # before the mapping goes away
        hf.close()

    fps = a.steps / el
    counts = r.scene_counts()      # V, I, A, texels, slots, tile pairs, path
    nv, ni, na, ntex, nslots, pairs, path = counts[:7]
    if path == 2:
        # tile path, fragment stage = k_tile_raster + k_tile_resolve: framebuffer rows, the per-pixel
        # (1/z, slot) keys written and read back, and per (slot, tile) pair its list entry + 64-B record
        kernel = 'k_tile_raster+k_tile_resolve'
        frag_bytes = 4 * W * rows + 16 * W * rows + (4 + RASTER_REC_BYTES) * pairs
    else:
        # row path, k_fragment: this rank's framebuffer rows + the ripmap texels it may sample + the
        # triangle setup records it reads
        kernel = 'k_fragment'
        frag_bytes = 4 * W * rows + 4 * ntex + TRI_SETUP_BYTES * nslots
    frag_avg_s = frag_ms / 1e3 / max(nfr, 1)
    achieved = frag_bytes / frag_avg_s / 1e9
    workload = f'{a.scene}/{a.pose}/{W}x{H}/N{N}'

    result = None
    if rank == 0:
        e2e = None
        if not a.no_e2e and N == 1:
            # updateAndRender into a caller-owned host buffer: includes the D2H over PCIe
            host = np.empty((H, W), dtype=np.uint32)
            r.configure(data_path, local)
            for t in script:
                r.update_and_render(W, H, t, host)
            for _ in range(5):
                r.update_and_render(W, H, hold, host)
            n_e2e = max(20, min(200, a.steps))
            t1 = time.perf_counter()
            for _ in range(n_e2e):
                r.update_and_render(W, H, hold, host)
            e2e = n_e2e / (time.perf_counter() - t1)
        cpu = None
        if not a.no_cpu_baseline and N == 1:
            cfps, cframes, cel = cpu_baseline(data_path, script, hold, W, H, a.cpu_seconds)
            cpu = {'value': round(cfps, 4), 'unit': 'frames/s', 'cores': 1, 'kind': 'port',
                   'sample': f'{cframes} frames of {a.scene}/{a.pose} at {W}x{H} in {cel:.1f} s, single thread, '
                             f'oracle/render_oracle.c (gcc -O2) on {cpu_model()}'}
        result = {
            'metric': METRIC,
            'value': round(fps, 3),
            'unit': 'frames/s',
            'n_gpus': N,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': round(el / a.steps * 1e3, 5),
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic: deterministic data.bin-format scene (SplitMix64 geometry, procedural ripmaps)',
            'config': {'workload': f'updateAndRender frame, scene {a.scene} ({nslots // 2} triangles, '
                                   f'{ntex >> 18} ripmap textures), pose {a.pose}, {W}x{H}',
                       'fragment_path': {1: 'rows', 2: 'tiles'}.get(path, '?'),
                       'scene': a.scene, 'pose': a.pose, 'width': W, 'height': H,
                       'band_rows': B if N > 1 else H, 'parallelism': f'rows{N}' + (' (interleaved bands; gather timed separately)' if N > 1 else '')},
            'mpixels_per_s': round(fps * W * H / 1e6, 2),
            'device_frame_ms': round(frame_ms / max(nfr, 1), 5),
            'fragment_kernel_ms': round(frag_avg_s * 1e3, 5),
            # N = 1: updateAndRender into a host buffer; N > 1: every rank's bands into one shared host frame
            'e2e_fps_with_d2h': round(e2e, 3) if e2e else (round(e2e_multi, 3) if e2e_multi else None),
            'gathered_fps': round(gathered_fps, 3) if gathered_fps else None,
            'roofline': {'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBS, 5), 'traffic': load_traffic(workload),
                         'kernel': kernel, 'algorithmic_bytes_per_launch': frag_bytes},
            'cpu_baseline': cpu,
        }
        print(json.dumps(result), flush=True)
    r.shutdown()
    if N > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == '__main__':
    main()
