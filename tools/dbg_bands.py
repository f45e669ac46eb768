import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
from swift3drenderer_amd import poses, scene
from swift3drenderer_amd.renderer import Renderer
from swift3drenderer_amd.multi import assemble, band_rows, band_row_ids
from oracle.oracle import render_pose as orc
scene.write_named('full', '/tmp/full.bin')
W, H = 800, 600
r = Renderer('/tmp/full.bin', device=0)
dev = torch.device('cuda', 0)
st = torch.cuda.current_stream(dev).cuda_stream
full = torch.empty((H, W), dtype=torch.int32, device=dev)
for t in poses.script('P_over'):
    r.render_bands(t, W, H, H, 1, 0, full.data_ptr(), st)
torch.cuda.synchronize()
f = full.cpu().numpy().view(np.uint32)
o = orc('/tmp/full.bin', poses.script('P_over'), W, H)
print('full vs oracle diff', (f != o).sum())
for nparts, band in [(2, 16), (1, 600)]:
    parts = []
    for p in range(nparts):
        rows = band_rows(H, band, nparts, p)
        buf = torch.full((max(rows, 1), W), -1, dtype=torch.int32, device=dev)
        n = r.render_bands(poses.hold('P_over'), W, H, band, nparts, p, buf.data_ptr(), st)
        torch.cuda.synchronize()
        b = buf.cpu().numpy().view(np.uint32)[:rows]
        ids = band_row_ids(H, band, nparts, p)
        d = (b != o[ids])
        bad_rows = np.nonzero(d.any(1))[0]
        print(nparts, band, p, 'rows', rows, 'n', n, 'bad rows', len(bad_rows), bad_rows[:10], 'first vals', b[bad_rows[:1], :8] if len(bad_rows) else '')
