"""The icosahedron stress scene (BASELINE config 5) -- generated vectorized, streamed to data.bin.

``addIcosahedron`` (data-generator/main.swift:260-373) repeated ``n`` times with a random frame,
centre and radius per icosahedron: 12 n vertices, 20 n triangles, 60 n attributes (flat colour,
per-face normals), no textures.  n = 1 000 000 is a 4.03 GB data.bin.

Placement (tuned as that row asks): centres fill the default camera's
view frustum -- depth uniform in [5, 60] in front of the camera, x and y uniform across 1.05x the
half-extents the projection covers at that depth for a 16:9 frame (render.cpp:279, :288:
factor = H / (2 tan(fov/2)), fov = pi/5) -- and the radius is proportional to depth,
r = depth * u, u uniform in [0.0025, 0.004], so every icosahedron projects to a 8-13 px radius at
3840x2160 and its front faces to ~10-60 px^2 (the survey's fixed radius range [0.1, 0.4] over that
depth range gives near objects of 100+ px radius, ~7 G fragments per frame: fragment-bound, not
the triangle-bound case this config is for).

Randomness: a counter-based SplitMix64 stream (seed in the scene name); the orientation frame uses
rejection-sampled cube points and only +, -, *, /, sqrt in float32 -- IEEE-exact operations, so the
file is bit-identical on every machine (no libm transcendental).  The arithmetic of the icosahedron
itself follows ``scene.add_icosahedron`` / main.swift in Swift's expression order.
"""
from __future__ import annotations

import os
import re

import numpy as np

from .scene import ICOSA_COLOURS, ICOSA_FACES, ORANGE

F = np.float32
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
CHUNK = 1 << 16                     # icosahedra per generation chunk
DEPTH = (5.0, 60.0)
RADIUS_PER_DEPTH = (0.0025, 0.004)
HALF_X = F(0.5773503)               # 1920 / (2160 / (2 tan(pi/10)))  ~ (W/2) / factor at 16:9
HALF_Y = F(0.3249197)               # tan(pi/10)
ATTEMPTS = 40                       # rejection sampling: P(all fail) = (1 - pi/6)^40 ~ 2e-13


def _splitmix(counter: np.ndarray) -> np.ndarray:
    """SplitMix64 output for state = seed + (i+1)*golden (counter already includes the seed)."""
    with np.errstate(over='ignore'):
        z = counter + GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _uniform(seed: int, stream: int, idx: np.ndarray, lo: float, hi: float) -> np.ndarray:
    """float32 uniform in [lo, hi) for (stream, idx): 24 random bits, exact float32 arithmetic."""
    with np.errstate(over='ignore'):
        ctr = np.uint64(seed) + (np.uint64(stream) << np.uint64(40)) * GOLDEN + idx.astype(np.uint64) * GOLDEN
    bits = (_splitmix(ctr) >> np.uint64(40)).astype(np.float32)        # [0, 2^24)
    return F(lo) + F(hi - lo) * (bits * F(1.0 / (1 << 24)))


def _dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def _cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1)


def _normalize(a):
    r = F(1.0) / np.sqrt(_dot(a, a))
    return a * r[..., None]


def _unit_points(seed: int, stream: int, ids: np.ndarray) -> np.ndarray:
    """Per id, the first accepted of ATTEMPTS cube points p with 1/64 < |p|^2 <= 1, normalized."""
    n = ids.size
    out = np.zeros((n, 3), dtype=F)
    todo = np.ones(n, dtype=bool)
    for k in range(ATTEMPTS):
        base = ids.astype(np.uint64) * np.uint64(3 * ATTEMPTS) + np.uint64(3 * k)
        p = np.stack([_uniform(seed, stream, base + np.uint64(c), -1.0, 1.0) for c in range(3)], axis=-1)
        d = _dot(p, p)
        ok = todo & (d > F(1 / 64)) & (d <= F(1))
        out[ok] = p[ok]
        todo &= ~ok
        if not todo.any():
            break
    if todo.any():
        raise RuntimeError('stress scene: rejection sampling exhausted')
    return _normalize(out)


def _frames(seed: int, ids: np.ndarray):
    """randomUnitAxis (main.swift:23-32) restated: x, then y = normalize(x cross q), z = x cross y."""
    x = _unit_points(seed, 1, ids)
    q = _unit_points(seed, 2, ids)
    par = np.abs(_dot(x, q)) > F(0.999)          # nearly parallel: take another candidate
    if par.any():
        q[par] = _unit_points(seed, 3, ids[par])
    y = _normalize(_cross(x, q))
    z = _cross(x, y)
    return x, y, z


def _icosa_vertices(x, y, z):
    """scene.icosa_unit_vertices, vectorized (main.swift:262-277)."""
    phi = F(F(np.sqrt(F(5)) + F(1)) / F(2))
    l_ = F(F(1) / F(np.sqrt(F(phi + F(2)))))
    k = F(phi * l_)
    mk = F(-k)
    ml = F(-l_)
    return np.stack([k * x + l_ * y, k * x - l_ * y, mk * x + l_ * y, mk * x - l_ * y,
                     l_ * x + k * z, ml * x + k * z, l_ * x - k * z, ml * x - k * z,
                     k * y + l_ * z, k * y - l_ * z, mk * y + l_ * z, mk * y - l_ * z], axis=1)


def _chunk(seed: int, lo: int, hi: int):
    """Vertices (m, 12, 3) and per-face normals (m, 20, 3) of icosahedra [lo, hi)."""
    ids = np.arange(lo, hi, dtype=np.uint64)
    x, y, z = _frames(seed, ids)
    depth = _uniform(seed, 4, ids, *DEPTH)
    cx = _uniform(seed, 5, ids, -1.05, 1.05) * HALF_X * depth
    cy = _uniform(seed, 6, ids, -1.05, 1.05) * HALF_Y * depth
    r = depth * _uniform(seed, 7, ids, *RADIUS_PER_DEPTH)
    p = np.stack([cx, cy, -depth], axis=-1)
    v = r[:, None, None] * _icosa_vertices(x, y, z) + p[:, None, :]          # r * q + p
    f = np.array(ICOSA_FACES)
    a, b, c = v[:, f[:, 0]], v[:, f[:, 1]], v[:, f[:, 2]]
    nrm = _normalize(_cross(c - a, b - a))                                   # main.swift:69-72
    return v.astype(F), nrm.astype(F)


def _colour_table() -> np.ndarray:
    """(20, 3, 4) float32 colour payloads (rgb + pad), main.swift:310-371."""
    t = np.zeros((20, 3, 4), dtype=F)
    for fi in range(20):
        cols = ICOSA_COLOURS.get(fi, (ORANGE, ORANGE, ORANGE))
        for k in range(3):
            t[fi, k, :3] = cols[k]
    return t


def write_stress(path: str, n: int, seed: int = 1) -> int:
    """Stream the n-icosahedron scene to `path` in the data.bin layout (scene.py docstring)."""
    nv, ni = 12 * n, 60 * n
    faces = np.array(ICOSA_FACES, dtype=np.int64).reshape(-1)
    cols = _colour_table()
    hdr = lambda k: np.array([k, 0], dtype=np.uint64).tobytes()     # noqa: E731
    total = 0
    with open(path, 'wb') as fo:
        def w(b):
            nonlocal total
            fo.write(b)
            total += len(b)
        # vertices: float4 (x, y, z, 1)
        w(hdr(nv))
        for lo in range(0, n, CHUNK):
            hi = min(n, lo + CHUNK)
            v, _ = _chunk(seed, lo, hi)
            v4 = np.ones((hi - lo, 12, 4), dtype=F)
            v4[..., :3] = v
            w(v4.tobytes())
        # vertex indices: icosahedron i uses vertices 12 i + ICOSA_FACES
        w(hdr(ni))
        for lo in range(0, n, CHUNK):
            hi = min(n, lo + CHUNK)
            idx = (np.arange(lo, hi, dtype=np.int64)[:, None] * 12 + faces[None, :]).reshape(-1)
            w(idx.tobytes())
        if ni % 2:
            w(bytes(8))
        # attributes: 48 B each, three per face (normal, colour payload, tag 0)
        w(hdr(ni))
        for lo in range(0, n, CHUNK):
            hi = min(n, lo + CHUNK)
            _, nrm = _chunk(seed, lo, hi)
            rec = np.zeros((hi - lo, 20, 3, 12), dtype=F)
            rec[..., 0:3] = nrm[:, :, None, :]
            rec[..., 4:8] = cols[None]
            w(rec.tobytes())                      # tag byte (offset 32) = 0: colour
        # attribute indices: 0 .. 60n-1
        w(hdr(ni))
        for lo in range(0, ni, 60 * CHUNK):
            w(np.arange(lo, min(ni, lo + 60 * CHUNK), dtype=np.int64).tobytes())
        if ni % 2:
            w(bytes(8))
        w(hdr(0))                                 # no textures
    return total


def write_soup(path: str, n: int, seed: int = 1) -> int:
    """The n-icosahedron scene as a triangle soup: the same triangles (geometry, normals, colours),
    but every triangle with its own three vertices (no index shared, so no mesh to find) and the
    triangles in a shuffled order (SplitMix64 keys, sorted).  Exercises the tile path's pooled,
    permuted clusters (clusters.cpp); small n only (built in memory)."""
    v, nrm = _chunk(seed, 0, n)
    f = np.array(ICOSA_FACES)
    tv = v[:, f].reshape(-1, 3, 3)                             # (20 n, 3 corners, xyz)
    cols = _colour_table()
    rec = np.zeros((n, 20, 3, 12), dtype=F)
    rec[..., 0:3] = nrm[:, :, None, :]
    rec[..., 4:8] = cols[None]
    rec = rec.reshape(-1, 3, 12)
    order = np.argsort(_splitmix(np.arange(20 * n, dtype=np.uint64) + np.uint64(seed) * GOLDEN), kind='stable')
    tv, rec = tv[order], rec[order]
    nt = 20 * n
    v4 = np.ones((nt, 3, 4), dtype=F)
    v4[..., :3] = tv
    hdr = lambda k: np.array([k, 0], dtype=np.uint64).tobytes()     # noqa: E731
    idx = np.arange(3 * nt, dtype=np.int64)
    pad = bytes(8) if (3 * nt) % 2 else b''
    data = b''.join([hdr(3 * nt), v4.tobytes(), hdr(3 * nt), idx.tobytes(), pad, hdr(3 * nt), rec.tobytes(),
                     hdr(3 * nt), idx.tobytes(), pad, hdr(0)])
    with open(path, 'wb') as fo:
        fo.write(data)
    return len(data)


_NAME = re.compile(r'^icosa-(soup-)?(stress|\d+)$')


def is_stress_name(name: str) -> bool:
    return bool(_NAME.match(name))


def count_of(name: str) -> int:
    m = _NAME.match(name)
    if not m:
        raise ValueError(name)
    return 1_000_000 if m.group(2) == 'stress' else int(m.group(2))


def write_named(name: str, path: str) -> int:
    if _NAME.match(name).group(1):
        return write_soup(path, count_of(name), seed=1)
    return write_stress(path, count_of(name), seed=1)


def expected_size(n: int) -> int:
    ni = 60 * n
    return 16 * 5 + 16 * 12 * n + 8 * (ni + ni % 2) + 48 * ni + 8 * (ni + ni % 2)


if __name__ == '__main__':
    import sys
    name = sys.argv[1] if len(sys.argv) > 1 else 'icosa-stress'
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join('/tmp', f'{name}.bin')
    print(out, write_named(name, out))
