#!/usr/bin/env python3
"""Every part of an N-way band split timed, not just part 0 (run on the GPU box).

One rank of an N-GPU frame renders only its interleaved bands; an N-GPU frame ends when its SLOWEST
part ends.  For each config and N = 1, 2, 4, 8 this renders every part p < N on the one GPU, frames
pipelined and left in HBM (s3r_render_bands, as a rank does), and reports per part its frame period
and, per N, max / mean over the parts and the per-GPU efficiency fps(1) / (N x slowest part's
period).  Bands: the library's choice (s3r_frame_band) unless --band.  One JSON line per (config, N).

    python tools/parts_all.py --out profiles/r05_parts_all.jsonl [--configs 3,4,5] [--steps 200]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    '3': ('full', 'P_over', 3840, 2160),
    '3id': ('full', 'P_id', 3840, 2160),
    '4': ('full', 'P_over', 7680, 4320),
    '5': ('icosa-stress', 'P_id', 3840, 2160),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--configs', default='3,4,5')
    p.add_argument('--nparts', default='1,2,4,8')
    p.add_argument('--steps', type=int, default=200)
    p.add_argument('--band', type=int, default=0)
    p.add_argument('--out', default=None)
    p.add_argument('--stress-data', default='/tmp/s3r_stress.bin')
    a = p.parse_args()
    import torch
    from swift3drenderer_amd import poses, scene, stress
    from swift3drenderer_amd.abi import Input
    from swift3drenderer_amd.renderer import Renderer
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream().cuda_stream
    tmp = tempfile.mkdtemp()
    lines = []
    for c in a.configs.split(','):
        name, pose, W, H = CONFIGS[c]
        if name == 'icosa-stress':
            path = a.stress_data
            if not os.path.exists(path):
                stress.write_named(name, path)
        else:
            path = os.path.join(tmp, f'{name}.bin')
            scene.write_named(name, path)
        r = Renderer(path, device=0)
        script, hold = poses.script(pose), Input.of(poses.hold(pose))
        buf = torch.empty((H, W), dtype=torch.int32, device='cuda')
        for t in script:                   # the pose, once (its movement keys would move the camera again)
            r.render_bands(t, W, H, H, 1, 0, buf.data_ptr(), st)
        fps1 = None
        for N in [int(x) for x in a.nparts.split(',')]:
            B = (a.band or r.frame_band(H, N)) if N > 1 else H
            parts = []
            for part in range(N):
                for _ in range(20):
                    r.render_bands(hold, W, H, B, N, part, buf.data_ptr(), st)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    r.render_bands(hold, W, H, B, N, part, buf.data_ptr(), st)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / a.steps
                parts.append(round(dt * 1e6, 2))
            slow, mean = max(parts), sum(parts) / len(parts)
            if N == 1:
                fps1 = 1e6 / slow
            line = {'config': c, 'scene': name, 'pose': pose, 'W': W, 'H': H, 'N': N, 'band': B,
                    'part_us': parts, 'slowest_us': slow, 'mean_us': round(mean, 2),
                    'max_over_mean': round(slow / mean, 4), 'fps_N': round(1e6 / slow, 1),
                    'part0_fps': round(1e6 / parts[0], 1),
                    'efficiency_per_gpu': round((1e6 / slow) / (N * fps1), 4)
                    if fps1 else None,
                    'path': r.raster_path()}
            print(json.dumps(line), flush=True)
            lines.append(line)
        r.shutdown()
        del buf
    if a.out:
        with open(a.out, 'w') as f:
            for ln in lines:
                f.write(json.dumps(ln) + '\n')


if __name__ == '__main__':
    main()
