#!/usr/bin/env python3
"""Where does a bench frame's time go beyond the fragment kernel?  (run on the GPU box)

Prints, for the bench workload: host enqueue time per frame (no sync), wall time per frame with
sync at the end, and the HIP-event fragment / frame times.  Usage:
    python tools/overhead_probe.py [--scene full --pose P_over --width 3840 --height 2160 --steps 400]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--scene', default='full')
    p.add_argument('--pose', default='P_over')
    p.add_argument('--width', type=int, default=3840)
    p.add_argument('--height', type=int, default=2160)
    p.add_argument('--steps', type=int, default=400)
    p.add_argument('--nparts', type=int, default=1, help='emulate one rank of an N-GPU band split')
    p.add_argument('--band', type=int, default=16)
    p.add_argument('--data', default=None, help='use (and create if missing) this data.bin instead of a temp file')
    a = p.parse_args()
    import torch
    from swift3drenderer_amd import poses, scene
    from swift3drenderer_amd.renderer import Renderer
    torch.cuda.set_device(0)
    path = a.data or os.path.join(tempfile.mkdtemp(), 's.bin')
    if not os.path.exists(path):
        scene.write_named(a.scene, path)
    W, H = a.width, a.height
    r = Renderer(path, device=0)
    N, B = a.nparts, (a.band if a.nparts > 1 else H)
    buf = torch.empty((H, W), dtype=torch.int32, device='cuda')
    sptr = torch.cuda.current_stream().cuda_stream
    from swift3drenderer_amd.abi import Input
    script, hold = poses.script(a.pose), Input.of(poses.hold(a.pose))   # built once, as bench.py does
    for t in script:
        r.render_bands(t, W, H, B, N, 0, buf.data_ptr(), sptr)
    for _ in range(50):
        r.render_bands(hold, W, H, B, N, 0, buf.data_ptr(), sptr)
    torch.cuda.synchronize()
    res = {}
    # host enqueue rate
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r.render_bands(hold, W, H, B, N, 0, buf.data_ptr(), sptr)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res['host_enqueue_us'] = (t1 - t0) / a.steps * 1e6
    res['wall_us'] = (t2 - t0) / a.steps * 1e6
    # event timing
    r.timing(True)
    for _ in range(a.steps):
        r.render_bands(hold, W, H, B, N, 0, buf.data_ptr(), sptr)
    frag, frame, n = r.timing_collect()
    r.timing(False)
    res['frag_us'] = frag / n * 1e3
    res['frame_us'] = frame / n * 1e3
    # Python + ctypes cost of one library call that does nothing on the GPU
    from swift3drenderer_amd.abi import Input
    t0 = time.perf_counter()
    for _ in range(a.steps):
        Input.of(hold)
        r.lib.s3r_band_rows_local(H, B, N, 0)
    res['python_ctypes_us'] = (time.perf_counter() - t0) / a.steps * 1e6
    res['serial'] = bool(os.environ.get('S3R_SERIAL'))
    res['nparts'] = N
    print(json.dumps(res), flush=True)
    r.shutdown()


if __name__ == '__main__':
    main()
