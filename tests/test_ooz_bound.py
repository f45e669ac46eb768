"""The tile path's 1/z bound (kernels.hip ooz_bound, include/render.h s3r_ooz_bound), on the CPU:
for random triangles set up the way render.cpp:311-336 sets them up (float32, its operation order),
every 1/z the reference's own walk produces at a covered pixel -- `wy += dy` per row, `w += dx` per
pixel (render.cpp:374, :378), coverage w >= 0 (:362), 1/z = (r0 w0 + r1 w1) + r2 w2 (:363) -- must
not exceed the bound: k_tile_raster skips a triangle whose bound is below the tile's current winners
(strict '>' at :364), so a bound that is too small would drop a winning fragment."""
import ctypes

import numpy as np

from swift3drenderer_amd.renderer import load_library

F = np.float32


def ooz_bound(ws, dx, dy, rvz, xmin, xmax, ymin, ymax):
    lib = load_library()
    f = lib.s3r_ooz_bound
    f.restype = ctypes.c_float
    P = ctypes.POINTER(ctypes.c_float)
    f.argtypes = [P, P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    arr = [np.ascontiguousarray(v, dtype=F) for v in (ws, dx, dy, rvz)]
    return F(f(*[a.ctypes.data_as(P) for a in arr], xmin, xmax, ymin, ymax))


def edge(ax, ay, bx, by, cx, cy):
    """EDGE_FUNCTION (render.cpp:9) in float32, its operation order."""
    return F(F(F(cx - ax) * F(ay - by)) + F(F(cy - ay) * F(bx - ax)))


def setup(v, sw, sh):
    """render.cpp:311-336 for screen-space corners v[i] = (x, y, z): None when culled."""
    xs, ys, zs = [F(p[0]) for p in v], [F(p[1]) for p in v], [F(p[2]) for p in v]
    area = edge(xs[0], ys[0], xs[1], ys[1], xs[2], ys[2])
    if max(xs) < 0 or max(ys) < 0 or min(xs) >= sw or min(ys) >= sh or area < 10:
        return None
    ooa = F(F(1) / area)
    xmin, xmax = int(max(F(0), min(xs))), int(min(F(sw - 1), max(xs)))
    ymin, ymax = int(max(F(0), min(ys))), int(min(F(sh - 1), max(ys)))
    px, py = F(xmin + F(0.5)), F(ymin + F(0.5))
    ws = [F(edge(xs[1], ys[1], xs[2], ys[2], px, py) * ooa), F(edge(xs[2], ys[2], xs[0], ys[0], px, py) * ooa),
          F(edge(xs[0], ys[0], xs[1], ys[1], px, py) * ooa)]
    dx = [F(F(ys[1] - ys[2]) * ooa), F(F(ys[2] - ys[0]) * ooa), F(F(ys[0] - ys[1]) * ooa)]
    dy = [F(F(xs[2] - xs[1]) * ooa), F(F(xs[0] - xs[2]) * ooa), F(F(xs[1] - xs[0]) * ooa)]
    rvz = [F(F(1) / z) for z in zs]
    return ws, dx, dy, rvz, xmin, xmax, ymin, ymax


def max_walked_ooz(ws, dx, dy, rvz, xmin, xmax, ymin, ymax):
    """The largest 1/z of a covered pixel, walked exactly as render.cpp walks (sequential float32 adds)."""
    nr, nc = ymax - ymin + 1, xmax - xmin + 1
    a = []
    for i in range(3):
        col = np.full(nr, dy[i], dtype=F)
        col[0] = ws[i]
        wy = np.add.accumulate(col, dtype=F)                       # wy += dy, row by row (:378)
        grid = np.full((nr, nc), dx[i], dtype=F)
        grid[:, 0] = wy
        a.append(np.add.accumulate(grid, axis=1, dtype=F))         # w += dx, pixel by pixel (:374)
    cov = (a[0] >= 0) & (a[1] >= 0) & (a[2] >= 0)                  # :362
    ooz = (F(rvz[0]) * a[0] + F(rvz[1]) * a[1]) + F(rvz[2]) * a[2]  # :363
    return float(ooz[cov].max()) if cov.any() else None


def test_bound_holds_for_random_triangles():
    rng = np.random.default_rng(20261017)
    sw, sh = F(3840), F(2160)
    checked = 0
    for case in range(2500):
        size = [4, 12, 40, 150][case % 4]
        c = rng.uniform([0, 0], [3840, 2160])
        v = []
        for _ in range(3):
            z = F(rng.choice([rng.uniform(0.1, 1.0), rng.uniform(1, 60), rng.uniform(60, 5000)]))
            v.append((F(c[0] + rng.normal(0, size)), F(c[1] + rng.normal(0, size)), z))
        st = setup(v, sw, sh)
        if st is None:
            continue
        ws, dx, dy, rvz, xmin, xmax, ymin, ymax = st
        if (xmax - xmin + 1) * (ymax - ymin + 1) > 400_000:
            continue
        m = max_walked_ooz(*st)
        if m is None:
            continue
        b = ooz_bound(*st)
        assert np.isfinite(b) and b >= m, (case, b, m, st)
        checked += 1
    assert checked > 800


def test_bound_edge_cases():
    # a sliver whose walked values hover around zero at an edge, and corners at the near plane
    for v in [[(100.25, 50.5, 0.1), (164.75, 51.0, 0.1), (130.0, 52.0, 0.1)],
              [(0.5, 0.5, 0.100001), (3839.5, 0.5, 4000.0), (0.5, 2159.5, 0.5)],
              [(10.0, 10.0, 1.0), (30.0, 10.0, 1.0), (10.0, 30.0, 1.0)]]:
        st = setup(v, F(3840), F(2160))
        assert st is not None
        m = max_walked_ooz(*st)
        assert m is not None and ooz_bound(*st) >= m
