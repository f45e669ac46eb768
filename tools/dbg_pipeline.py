#!/usr/bin/env python3
"""Debug helper (GPU box): the mixed-stream pipelined sequence of
tests/test_gpu_parity.py::test_pipelined_frames_on_mixed_streams, synchronising after every frame
to find the first call that leaves a HIP error behind."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from swift3drenderer_amd import scene
    from swift3drenderer_amd.renderer import Renderer
    d = tempfile.mkdtemp()
    path = os.path.join(d, 'full.bin')
    scene.write_named('full', path)
    r = Renderer(path)
    W, H = 320, 240
    rng = np.random.default_rng(11)
    mouse = np.array([0.0, -120.0])
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    sync_each = '--sync' in sys.argv
    for k in range(18):
        keys = rng.integers(0, 2, 4) * rng.uniform(0, 10, 4)
        mouse += rng.normal(0, 12, 2)
        inp = (*keys, *mouse)
        if k == 7:
            r.set_raster_path('tiles')
        if k == 10:
            r.set_raster_path('auto')
        try:
            if k == 13:
                r.update_and_render(W, H, inp)
            else:
                buf = torch.empty((H, W), dtype=torch.int32, device='cuda')
                st = streams[(k // 3) % 2]
                with torch.cuda.stream(st):
                    r.render_bands(inp, W, H, H, 1, 0, buf.data_ptr(), st.cuda_stream)
            if sync_each:
                torch.cuda.synchronize()
                _ = buf.cpu()
            print('frame', k, 'ok', flush=True)
        except Exception as e:
            print('frame', k, 'FAILED:', e, flush=True)
            return
    torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()
