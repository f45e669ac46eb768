#!/usr/bin/env python3
"""Benchmark: frames/s and Mpixels/s of updateAndRender at 3840x2160 on the packaged scene
(BASELINE.json metric).

A step is one call of the reference's boundary, ``updateAndRender(PixelData*, Input*)``
(render.cpp:264-384): camera update, geometry, fragment stage, and the finished frame in the
caller's HOST buffer when the call returns -- timed the way the reference's main loop times it
(main.swift:120-122), one call at a time, into a caller-owned buffer allocated the way main.swift
allocates it: ONE malloc of 2 * bufferSize whose halves are used alternately (main.swift:117-118,
:164).  ``value`` = 1 / the median wall time of those calls, over at least 200 timed frames
(whatever --steps says; the count used is reported in ``steps``) after at least 20 warm-up frames.

N GPUs: the reference's caller is one process on one thread, so the N GPUs sit behind that one call
(s3r_configure_devices): rank 0 calls updateAndRender with devices 0..N-1, each rendering its
interleaved 16-row bands and copying them into their rows of the caller's buffer over its own PCIe
link -- that is ``value``.  Then every rank renders its own part on its own GPU (one process per GPU,
``ranks``): the part left in HBM (``device_fps_N`` = frames / the slowest rank's time) and the
parts gathered to rank 0 over xGMI by one RCCL gather plus the de-interleave kernel
(``gathered_fps``), each with its per-GPU efficiency against rank 0's whole frame on one GPU.
Scaling is strong (a fixed frame).

Beside ``value``: ``device_fps`` (one GPU, frames pipelined and left in HBM: s3r_render_bands),
the ``roofline`` of the fragment kernel (HIP events on its stream during updateAndRender frames),
and ``cpu_baseline`` (the single-threaded CPU oracle on this host, a bounded sample).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'frames/sec + Mpixels/s at 3840x2160, data.bin scene; 1/2/4/8-GPU scaling'
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md, HBM3E peak (spec)
LINK_PEAK_GBS = 63.0     # MI355X_MICROARCH.md, host link PCIe Gen5 x16 per direction (spec)
TRI_SETUP_BYTES = 240    # sizeof(TriSetup)
ENTRY_SOURCE_BYTES = 12 + 3 * 16   # tile path, per binned entry: the 3 vertex indices and 3 corners the
                                    # raster rebuilds its record from (Tile frames without records)
MIN_TIMED = 200          # >= 200 frames after 20 warm-up frames
MIN_WARMUP = 20


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=MIN_TIMED)
    p.add_argument('--warmup', type=int, default=MIN_WARMUP)
    p.add_argument('--width', type=int, default=3840)
    p.add_argument('--height', type=int, default=2160)
    p.add_argument('--scene', default='full')
    p.add_argument('--pose', default='P_over')
    p.add_argument('--band', type=int, default=0,
                   help='rows per interleaved band (multi-GPU); 0: the library\'s choice by fragment path '
                        '(s3r_frame_band: 16 on the row path, two bands per GPU on the tile path)')
    p.add_argument('--devices', default=None,
                   help='comma-separated device ids behind updateAndRender (default 0..N-1; ids may repeat '
                        'to rehearse N parts on one GPU)')
    p.add_argument('--cpu-seconds', type=float, default=10.0, help='CPU-baseline sample budget')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-device', action='store_true', help='skip the device-resident (HBM) rate')
    p.add_argument('--data', default=None,
                   help='data.bin path to reuse across runs (the deterministic scene is written there when missing)')
    p.add_argument('--ranks-leg', action='store_true',
                   help='run the one-process-per-GPU leg (on by default when WORLD_SIZE > 1; with one rank: '
                        'the single-rank RCCL gather)')
    p.add_argument('--rank-devices', default=None,
                   help='comma-separated GPU of each rank in the ranks leg (default: LOCAL_RANK); repeated '
                        'ids rehearse ranks on one GPU and then need --gather-backend gloo')
    p.add_argument('--ranks-extra', default=None,
                   help='further WxH frames for the ranks leg, comma-separated (default with N > 1: 7680x4320, '
                        'BASELINE config 4 -- the 8-GPU row-strip + RCCL gather config; "none": only the main frame)')
    p.add_argument('--gather-backend', default='nccl', choices=('nccl', 'gloo'),
                   help='the ranks leg\'s gather: nccl (RCCL over xGMI) or gloo (a rehearsal through host copies)')
    return p.parse_args(argv)


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


def textured_scene(path, nv, ni, na, ntex) -> bool:
    """Whether any attribute of the data.bin is textured (its disc tag, App. A, at +32 of the 48-B
    record): only then can a frame sample texels.  Memory-mapped; a scene without textures is not
    scanned."""
    if not ntex or not na:
        return False
    import numpy as np
    off = 16 + 16 * nv + 16 + 8 * (ni + ni % 2) + 16
    rec = np.memmap(path, dtype=np.uint8, mode='r', offset=off, shape=(na, 48))
    return bool(rec[:, 32:36].any())


def frame_roofline(W, H, nv, ni, na, ntex, textured, device_s, delivered_s):
    """SURVEY.md §8(d)'s whole-frame bytes B = 4 W H (framebuffer) + 16 V + 16 I + 48 A (the scene;
    both index arrays at 8 B) + the texels when a textured triangle exists, against the device
    frame time and the delivered (updateAndRender) median."""
    b = 4 * W * H + 16 * nv + 16 * ni + 48 * na + (4 * ntex if textured else 0)
    out = {'bytes_per_frame': b, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
           'formula': '4WH + 16V + 16I + 48A (+ 4 x texels if textured), SURVEY.md 8(d)'}
    for k, t in (('device', device_s), ('delivered', delivered_s)):
        if t:
            out[f'achieved_{k}'] = round(b / t / 1e9, 2)
            out[f'frac_{k}'] = round(b / t / 1e9 / HBM_PEAK_GBS, 5)
    return out


def library_sha256():
    """SHA-256 of the library this process renders with (the one renderer.load_library opened)."""
    import hashlib
    from swift3drenderer_amd.renderer import LIB_PATH
    try:
        with open(LIB_PATH, 'rb') as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def load_traffic(workload_key, field='hbm_bytes_per_launch'):
    """HBM bytes per launch (the fragment kernel's, or with field='setup_hbm_bytes_per_launch' the
    tile path's setup) from the committed rocprofv3 --pmc summary (profiles/pmc_traffic.json,
    tools/pmc_traffic.py) -- only when that PMC pass measured this very library (its SHA-256 recorded
    beside the bytes): a figure from another build is not reported.  Returns (bytes, provenance)."""
    p = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        with open(p) as f:
            e = json.load(f).get(workload_key, {})
    except Exception:
        return None, None
    v = e.get(field)
    if v is None:
        return None, None
    if not e.get('library_sha256') or e['library_sha256'] != library_sha256():
        return None, 'profiles/pmc_traffic.json measured another build of the library: not reported'
    kern = e.get('setup_kernel' if field.startswith('setup') else 'kernel', '?')
    return v, f"{e.get('source', '?')}; kernel {kern}; library sha256 {e['library_sha256'][:12]}"


class DoubleBuffer:
    """main.swift:117-118, :164: one malloc of 2 * bufferSize, halves used alternately."""

    def __init__(self, w, h, line_offset=None):
        """line_offset (probes only): the buffer placed that many bytes past a 64-B line boundary
        instead of where malloc puts it (glibc: 16 B past one)."""
        import numpy as np
        from swift3drenderer_amd.abi import PixelData
        self.libc = ctypes.CDLL(None)
        self.libc.malloc.restype = ctypes.c_void_p
        self.libc.malloc.argtypes = [ctypes.c_size_t]
        self.libc.free.argtypes = [ctypes.c_void_p]
        self.size = 4 * w * h
        self.raw = self.libc.malloc(2 * self.size + (128 if line_offset is not None else 0))
        if not self.raw:
            raise MemoryError('malloc of the double buffer failed')
        self.ptr = self.raw if line_offset is None else ((self.raw + 63) & ~63) + line_offset
        self.halves = [PixelData(ctypes.cast(self.ptr + k * self.size, ctypes.POINTER(ctypes.c_uint32)), w, h, 4,
                                 self.size) for k in (0, 1)]
        self.cur = 0
        self.np = np

    def next(self):
        pd = self.halves[self.cur]
        self.cur ^= 1
        return pd

    def half(self, k):
        return (ctypes.c_uint8 * self.size).from_address(self.ptr + k * self.size)

    def free(self):
        self.libc.free(self.raw)


def main(argv=None):
    a = parse(argv)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    if world == 1 and a.gpus > 1:
        raise SystemExit('--gpus N>1 needs torch.distributed.run with N processes')
    N = max(world, 1)
    ranks_on = world > 1 or a.ranks_leg
    if world > 1 or ranks_on:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29511')
        os.environ.setdefault('RANK', '0')
        os.environ.setdefault('WORLD_SIZE', '1')
        # control (barriers, the max over ranks); the ranks leg's gather has its own group
        dist.init_process_group('gloo')

    def barrier():
        if dist.is_initialized():
            dist.barrier()

    result = None
    if rank == 0:
        result = run_rank0(a, N, np, torch)
    barrier()
    if ranks_on:
        frames = [(a.width, a.height)]
        extra = a.ranks_extra if a.ranks_extra is not None else ('7680x4320' if world > 1 else 'none')
        if extra != 'none':
            frames += [tuple(int(v) for v in f.split('x')) for f in extra.split(',') if f]
        for k, (w, h) in enumerate(frames):
            fps1 = result['device_fps'] if rank == 0 and result and k == 0 else None
            rl = run_ranks_leg(a, rank, N, np, torch, dist, w, h, fps1)
            if rank == 0:
                result['ranks' if k == 0 else f'ranks_{w}x{h}'] = rl
    if rank == 0:
        print(json.dumps(result), flush=True)
    barrier()
    if dist.is_initialized():
        dist.destroy_process_group()
    return result


def rank_device(a, rank, torch):
    """The GPU of this rank in the ranks leg: --rank-devices, else LOCAL_RANK."""
    if a.rank_devices:
        ids = [int(x) for x in a.rank_devices.split(',')]
        return ids[rank % len(ids)]
    return int(os.environ.get('LOCAL_RANK', str(rank)))


def ranks_leg(render_part, render_whole, sync, gather, barrier, allgather_f, W, H, B, N, rank, steps, warmup,
              clock=time.perf_counter):
    """One process per GPU: this rank's part of every frame.

    render_part(): issue one frame of this rank's interleaved bands into its send buffer (asynchronous);
    gather(): the collective that brings every rank's part to rank 0 and de-interleaves it there
    (returns rank 0's frame, else None); render_whole(): rank 0's reference, the whole frame on its one
    GPU (None elsewhere); sync(): the device drained; barrier(); allgather_f(x): every rank's float.
    Returns, on every rank, per-rank part times and the max over ranks of the device-resident pass and
    of the gathered pass (each K frames, barrier + sync on both sides), and whether rank 0's gathered
    frame equals its whole frame."""
    for _ in range(warmup):
        render_part()
    sync()

    def timed(body):
        barrier()
        sync()
        t0 = clock()
        for _ in range(steps):
            body()
        sync()
        t = clock() - t0
        barrier()
        return allgather_f(t)

    dev_times = timed(render_part)

    def frame():
        render_part()
        gather()

    for _ in range(max(2, warmup // 4)):
        frame()
    sync()
    gat_times = timed(frame)
    render_part()
    got = gather()
    sync()
    same = None
    if rank == 0 and render_whole is not None:
        want = render_whole()
        sync()
        same = bool(got is not None and want is not None and got.shape == want.shape and bool((got == want).all()))
    return {'device_s': dev_times, 'gathered_s': gat_times, 'gathered_equals_whole': same}


_GROUPS = {}


def run_ranks_leg(a, rank, N, np, torch, dist, W, H, device_fps_1):
    """The ranks leg on this rank for a W x H frame: its own GPU, its own library state, the part it
    owns.  device_fps_1 (rank 0): the whole frame's device-resident rate on one GPU; None: rank 0
    measures it here first, the same way (frames pipelined into HBM), while the others wait."""
    from swift3drenderer_amd import poses, scene
    from swift3drenderer_amd.abi import Input
    from swift3drenderer_amd.multi import BandGather, band_rows
    from swift3drenderer_amd.renderer import Renderer

    dev_id = rank_device(a, rank, torch)
    torch.cuda.set_device(dev_id)
    dev = torch.device('cuda', dev_id)
    tmp = tempfile.mkdtemp(prefix=f's3r_rank{rank}_')
    data_path = os.path.join(tmp, f'{a.scene}.bin')
    scene.write_named(a.scene, data_path)
    script, hold_in = poses.script(a.pose), Input.of(poses.hold(a.pose))
    st = torch.cuda.current_stream(dev)
    steps = max(a.steps, MIN_TIMED)
    if rank == 0 and not device_fps_1:
        r1 = Renderer(data_path, device=dev_id)
        frame = torch.empty((H, W), dtype=torch.int32, device=dev)
        for t in script:
            r1.render_bands(t, W, H, H, 1, 0, frame.data_ptr(), st.cuda_stream)
        for _ in range(max(a.warmup, MIN_WARMUP)):
            r1.render_bands(hold_in, W, H, H, 1, 0, frame.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            r1.render_bands(hold_in, W, H, H, 1, 0, frame.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        device_fps_1 = steps / (time.perf_counter() - t0)
        del frame
    dist.barrier()
    r = Renderer(data_path, device=dev_id)
    B = a.band or r.frame_band(H, N)
    if N == 1:
        B = H
    nccl = a.gather_backend == 'nccl'
    if nccl and 'nccl' not in _GROUPS:
        _GROUPS['nccl'] = dist.new_group(backend='nccl')      # (one communicator for every frame size)
    group = _GROUPS.get('nccl') if nccl else None
    bg = BandGather(W, H, B, N, rank, dev)
    if not nccl:
        cpu = BandGather(W, H, B, N, rank, torch.device('cpu'))
    for t in script:
        r.render_bands(t, W, H, B, N, rank, bg.send.data_ptr(), st.cuda_stream)

    def render_part():
        r.render_bands(hold_in, W, H, B, N, rank, bg.send.data_ptr(), st.cuda_stream)

    def gather():
        if nccl:
            return bg.gather(group=group)
        cpu.send.copy_(bg.send)                       # rehearsal: through host copies over gloo
        out = cpu.gather()
        return out.to(dev) if rank == 0 else None

    whole = None
    if rank == 0:
        ref = torch.empty((H, W), dtype=torch.int32, device=dev)

        def whole():
            r2 = Renderer(data_path, device=dev_id)   # (the library is per process: a fresh state, whole frame)
            for t in script:
                r2.render_bands(t, W, H, H, 1, 0, ref.data_ptr(), st.cuda_stream)
            r2.render_bands(hold_in, W, H, H, 1, 0, ref.data_ptr(), st.cuda_stream)
            return ref

    def allgather_f(x):
        out = [None] * N
        dist.all_gather_object(out, float(x))
        return out

    res = ranks_leg(render_part, whole, lambda: torch.cuda.synchronize(dev), gather, dist.barrier, allgather_f,
                    W, H, B, N, rank, steps, max(a.warmup, MIN_WARMUP))
    r.shutdown()
    shutil.rmtree(tmp, ignore_errors=True)
    if rank != 0:
        return None
    out = ranks_summary(res, W, H, B, N, steps, device_fps_1, [band_rows(H, B, N, p) for p in range(N)],
                         'rccl (torch.distributed nccl) gather + s3r_deinterleave_bands' if nccl else
                         'gloo gather through host copies (rehearsal) + index_select')
    out['frame'] = f'{a.scene}/{a.pose}/{W}x{H}'
    return out


def ranks_summary(res, W, H, B, N, steps, device_fps_1, rows, gather_desc):
    """The ranks leg's JSON: per-rank frame times, the slowest rank, device-resident and gathered
    frames/s and their per-GPU efficiency fps(N) / (N fps(1)), fps(1) = rank 0's whole frame on one
    GPU in this run (device_fps)."""
    dev_ms = [t / steps * 1e3 for t in res['device_s']]
    gat_ms = [t / steps * 1e3 for t in res['gathered_s']]
    dfps = steps / max(res['device_s'])
    gfps = steps / max(res['gathered_s'])
    eff = (lambda f: round(f / (N * device_fps_1), 4)) if device_fps_1 else (lambda f: None)
    return {
        'processes': N, 'band_rows': B, 'rows_per_rank': rows,
        'per_rank_device_ms': [round(x, 5) for x in dev_ms],
        'max_rank_device_ms': round(max(dev_ms), 5),
        'device_fps_N': round(dfps, 3),
        'device_mpixels_per_s': round(dfps * W * H / 1e6, 2),
        'device_efficiency_per_gpu': eff(dfps),
        'per_rank_gathered_ms': [round(x, 5) for x in gat_ms],
        'gathered_fps': round(gfps, 3),
        'gathered_efficiency_per_gpu': eff(gfps),
        'fps_1': round(device_fps_1, 3) if device_fps_1 else None,
        'gather': gather_desc,
        'gathered_equals_whole_frame': res['gathered_equals_whole'],
        'note': 'every rank renders its interleaved bands of the frame on its own GPU (s3r_render_bands, '
                'frames pipelined, left in HBM); device_fps_N = frames / the slowest rank\'s time; gathered_fps '
                'adds one gather of the parts to rank 0 and the de-interleave per frame; efficiency = fps(N) / '
                '(N x fps(1)), fps(1) = rank 0\'s whole frame on one GPU (device_fps)',
    }


def run_rank0(a, N, np, torch):
    from swift3drenderer_amd import poses, scene
    from swift3drenderer_amd.abi import Input
    from swift3drenderer_amd.renderer import Renderer

    ndev = torch.cuda.device_count()
    devices = [int(x) for x in a.devices.split(',')] if a.devices else list(range(N))
    if not a.devices and ndev < N:
        raise SystemExit(f'--gpus {N}: only {ndev} GPUs visible (use --devices to rehearse parts on one GPU)')
    tmp = None
    if a.data and os.path.exists(a.data):
        data_path = a.data
    elif a.data:
        data_path = a.data
        scene.write_named(a.scene, data_path)
    else:
        tmp = tempfile.mkdtemp(prefix='s3r_bench_')
        data_path = os.path.join(tmp, f'{a.scene}.bin')
        scene.write_named(a.scene, data_path)
    W, H, B = a.width, a.height, a.band
    script = poses.script(a.pose)
    hold = poses.hold(a.pose)
    hold_in = Input.of(hold)
    steps = max(a.steps, MIN_TIMED)
    warmup = max(a.warmup, MIN_WARMUP)

    torch.cuda.set_device(devices[0])
    dev = torch.device('cuda', devices[0])
    r = Renderer(data_path, device=devices[0])
    r.configure_devices(devices if len(devices) > 1 else [], B)
    r.configure(data_path, devices[0])
    lib = r.lib
    buf = DoubleBuffer(W, H)

    def call(inp):
        lib.updateAndRender(ctypes.byref(buf.next()), ctypes.byref(inp))

    for t in script:                       # the pose script (the first call initialises), untimed
        call(Input.of(t))
    for _ in range(warmup):
        call(hold_in)

    # value: synchronous updateAndRender calls, each timed like main.swift:120-122
    r.device_profile()                     # (reset the per-device and fill profiles: timed calls only)
    r.fill_profile()
    per = np.empty(steps)
    refs = [ctypes.byref(h) for h in buf.halves]
    in_ref = ctypes.byref(hold_in)
    uar = lib.updateAndRender
    clock = time.perf_counter
    torch.cuda.synchronize(dev)
    t_start = clock()
    for k in range(steps):
        t0 = clock()
        uar(refs[buf.cur], in_ref)
        per[k] = clock() - t0
        buf.cur ^= 1
    torch.cuda.synchronize(dev)
    total = clock() - t_start
    median_s = float(np.median(per))
    fps = 1.0 / median_s

    # both halves carry the held pose's frame; the pin state the frames were delivered with
    host = r.host_stats()
    per_device = r.device_profile()        # each device's part: finish time after the call's entry, link bytes
    fill_prof = r.fill_profile()           # host fill: devices' / fill threads' finish per frame (fill frames)
    halves_pinned = [bool(lib.s3r_host_pinned(ctypes.c_void_p(buf.ptr + k * buf.size), buf.size)) for k in (0, 1)]
    used = [m for m in ('copy', 'direct', 'fill') if host[f'{m}_frames'] > 0]
    link_bytes = host['link_bytes']

    def timed_calls(n):
        t = np.empty(n)
        for k in range(n):
            t0 = clock()
            uar(refs[buf.cur], in_ref)
            t[k] = clock() - t0
            buf.cur ^= 1
        return t

    # the same calls through each delivery into the caller's buffer (render_api.cpp "deliveries")
    modes = {}
    nm = min(steps, 100)
    for mode in ('copy', 'direct', 'fill'):
        r.set_delivery(mode)
        timed_calls(10)
        tm = timed_calls(nm)
        hs = r.host_stats()
        modes[mode] = {'fps': round(1.0 / float(np.median(tm)), 3), 'median_ms': round(float(np.median(tm)) * 1e3, 5),
                       'link_bytes_per_frame': hs['link_bytes']}
    r.set_delivery('env')
    timed_calls(10)

    # fragment-kernel time on device 0's stream (HIP events) within the delivered frames, in a
    # separate pass of the same calls (with direct / host-fill delivery its stores cross the link)
    r.timing(True)
    nt = min(steps, MIN_TIMED)
    for _ in range(nt):
        call(hold_in)
    st_dl = r.timing_stages()
    dl_frag_ms, dl_frame_ms, dl_nfr, dl_geo_ms = st_dl['frag_ms'], st_dl['frame_ms'], st_dl['frames'], st_dl['geo_ms']
    r.timing(False)

    counts = r.scene_counts()      # V, I, A, texels, slots, tile pairs, path
    nv, ni, na, ntex, nslots, pairs, path = counts[:7]
    B = B or r.frame_band(H, len(devices))          # (the library's choice, now that the path is known)
    rows0 = r.lib.s3r_band_rows_local(H, B, len(devices), 0) if len(devices) > 1 and H > B else H

    def kernel_bytes(rows):
        if path == 2:
            # tile path, fragment stage = k_tile_raster<true> (raster and shading fused) + the short
            # k_tile_resolve_deferred: the framebuffer rows, and per binned (slot, tile) entry its 4-B bin
            # entry and the indices and corners its record is rebuilt from (pairs: the frame's binned
            # entries, s3r_scene_counts)
            return 'k_tile_raster (fused) + k_tile_resolve_deferred', 4 * W * rows + (4 + ENTRY_SOURCE_BYTES) * pairs
        # row path, k_fragment: the framebuffer rows + the ripmap texels it may sample + the triangle
        # setup records it reads
        return 'k_fragment', 4 * W * rows + 4 * ntex + TRI_SETUP_BYTES * nslots

    # device-resident rate of one GPU: whole frames pipelined into HBM (no host copy), and the HBM
    # roofline of the fragment kernel from HIP events on its stream in a second pass of those frames
    device_fps = None
    frag_ms, frame_ms, nfr, geo_ms, roof_rows, roof_launch = dl_frag_ms, dl_frame_ms, dl_nfr, dl_geo_ms, rows0, 'delivered frames'
    if not a.no_device:
        r.configure_devices([], B)
        r.configure(data_path, devices[0])
        out = torch.empty((H, W), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)
        for t in script:
            r.render_bands(t, W, H, H, 1, 0, out.data_ptr(), stream.cuda_stream)
        for _ in range(warmup):
            r.render_bands(hold_in, W, H, H, 1, 0, out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            r.render_bands(hold_in, W, H, H, 1, 0, out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        device_fps = steps / (time.perf_counter() - t0)
        r.timing(True)
        for _ in range(nt):
            r.render_bands(hold_in, W, H, H, 1, 0, out.data_ptr(), stream.cuda_stream)
        st_dv = r.timing_stages()
        frag_ms, frame_ms, nfr, geo_ms = st_dv['frag_ms'], st_dv['frame_ms'], st_dv['frames'], st_dv['geo_ms']
        r.timing(False)
        roof_rows, roof_launch = H, 'whole frame into HBM, frames pipelined (device_fps pass)'
        del out
    kernel, frag_bytes = kernel_bytes(roof_rows)
    frame_roof = frame_roofline(W, H, nv, ni, na, ntex, textured_scene(data_path, nv, ni, na, ntex),
                                1.0 / device_fps if device_fps else None, median_s)
    frag_avg_s = frag_ms / 1e3 / max(nfr, 1)
    achieved = frag_bytes / frag_avg_s / 1e9
    workload = f'{a.scene}/{a.pose}/{W}x{H}/N1'
    if path == 2 and device_fps:
        # the tile path reads no per-vertex attributes beyond the winners' (§8(d)'s 48 A bytes are not its
        # traffic): the PMC-measured bytes of its setup and fused raster per frame over the device frame
        cb = [load_traffic(workload, 'setup_hbm_bytes_per_launch')[0], load_traffic(workload)[0]]
        if all(cb):
            frame_roof['counter_bytes_per_frame'] = int(sum(cb))
            frame_roof['counter_frac_device'] = round(sum(cb) * device_fps / 1e9 / HBM_PEAK_GBS, 5)

    cpu = None
    if not a.no_cpu_baseline and len(devices) == 1:
        cfps, cframes, cel = cpu_baseline(data_path, script, hold, W, H, a.cpu_seconds)
        cpu = {'value': round(cfps, 4), 'unit': 'frames/s', 'cores': 1, 'kind': 'port',
               'sample': f'{cframes} frames of {a.scene}/{a.pose} at {W}x{H} in {cel:.1f} s, single thread, '
                         f'oracle/render_oracle.c (gcc -O2) on {cpu_model()}'}
    r.shutdown()
    buf.free()
    if tmp:
        shutil.rmtree(tmp, ignore_errors=True)

    frame_bytes = 4 * W * H
    traffic, traffic_src = load_traffic(workload)
    setup_traffic, setup_src = load_traffic(workload, 'setup_hbm_bytes_per_launch')
    return {
        'metric': METRIC,
        'value': round(fps, 3),
        'unit': 'frames/s',
        'n_gpus': N,
        'steps': steps,
        'warmup': warmup,
        'steps_requested': a.steps,
        'warmup_requested': a.warmup,
        'steps_note': f'at least {MIN_TIMED} timed / {MIN_WARMUP} warm-up calls whatever --steps / --warmup say '
                      '(SURVEY.md 8(d): fps = 1 / median of >= 200 calls)',
        'ms_per_step': round(total / steps * 1e3, 5),
        'higher_is_better': True,
        'scaling': 'strong',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic: deterministic data.bin-format scene (SplitMix64 geometry, procedural ripmaps)',
        'config': {'workload': f'updateAndRender into the caller\'s host double buffer, scene {a.scene} '
                               f'({nslots // 2} triangles, {ntex >> 18} ripmap textures), pose {a.pose}, {W}x{H}',
                   'fragment_path': {1: 'rows', 2: 'tiles'}.get(path, '?'),
                   'scene': a.scene, 'pose': a.pose, 'width': W, 'height': H, 'devices': devices,
                   'band_rows': B if len(devices) > 1 else H,
                   'parallelism': f'rows{len(devices)}' + (' (interleaved bands, per-device D2H into the caller buffer, '
                                                           'one process)' if len(devices) > 1 else '')},
        'mpixels_per_s': round(fps * W * H / 1e6, 2),
        'median_ms': round(median_s * 1e3, 5),
        'p10_ms': round(float(np.percentile(per, 10)) * 1e3, 5),
        'p90_ms': round(float(np.percentile(per, 90)) * 1e3, 5),
        'fps_mean': round(steps / total, 3),
        'frame_GB_per_s': round(frame_bytes / median_s / 1e9, 3),
        'delivery': {'mode': used[0] if len(used) == 1 else used, 'fill_threads': host['fill_threads'],
                     'fill_gpu_eighths': host['fill_gpu_eighths'], 'link_bytes_per_frame': link_bytes, 'modes': modes,
                     'per_device': per_device, 'fill_profile': fill_prof},
        'link_roofline': {'bound': 'pcie', 'achieved': round(link_bytes / median_s / 1e9, 2),
                          'peak': LINK_PEAK_GBS * len(devices), 'unit': 'GB/s',
                          'frac': round(link_bytes / median_s / 1e9 / (LINK_PEAK_GBS * len(devices)), 5),
                          'note': 'bytes the devices sent over their host links per frame / median frame time; '
                                  f'{len(devices)} x PCIe Gen5 x16'},
        'host_buffer': {'halves_pinned': halves_pinned, 'pinned_frames': host['pinned_frames'],
                        'pageable_frames': host['pageable_frames']},
        'device_fps': round(device_fps, 3) if device_fps else None,
        'device_frame_ms': round(1e3 / device_fps, 5) if device_fps else None,
        # HIP events from a frame's first launch to its fragment stage's end (frames pipelined: includes
        # the wait behind earlier frames' stages)
        'device_frame_latency_ms': round(frame_ms / max(nfr, 1), 5),
        'fragment_kernel_ms': round(frag_avg_s * 1e3, 5),
        'fragment_kernel_ms_delivered': round(dl_frag_ms / max(dl_nfr, 1), 5),
        # the geometry stage (row path: k_geometry; tile path: cluster cull, setup, clip and binning), HIP
        # events on its stream from the frame's first launch to the stage's end, same frames as roofline
        'setup_ms': round(geo_ms / max(nfr, 1), 5),
        'setup_bytes_per_frame': (16 * nv + 4 * ni + 4 * pairs) if path == 2 else None,
        'setup_traffic': setup_traffic if path == 2 else None,
        'setup_traffic_source': setup_src if path == 2 else None,
        'setup_bytes_note': ('tile path, a lower bound: vertices 16 B and indices 4 B read, a 4-B bin entry '
                             'written per binned entry; the setup writes no raster record except for the clip\'s '
                             'slots (rare; not counted); setup_traffic: the PMC bytes per frame of the same '
                             'library (tools/pmc_traffic.py)') if path == 2 else None,
        'roofline': {'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(achieved / HBM_PEAK_GBS, 5), 'traffic': traffic, 'traffic_source': traffic_src,
                     'kernel': kernel, 'algorithmic_bytes_per_launch': frag_bytes,
                     'launch': roof_launch, 'frame': frame_roof},
        'cpu_baseline': cpu,
    }


if __name__ == '__main__':
    main()
