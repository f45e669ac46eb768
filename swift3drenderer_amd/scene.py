"""Deterministic scenes in the reference's ``data.bin`` format.

The byte layout is the one written by ``/root/reference/data-generator/main.swift:381-416`` and read
by ``render-cpp/render.cpp:177-209``::

    u64 nV, u64 0;  nV x float4(x, y, z, 1)                              main.swift:387-389
    u64 nI, u64 0;  nI x i64 vertex indices;  (nI % 2) x 8 zero bytes    main.swift:390-392
    u64 nA, u64 0;  nA x 48-byte VertexAttribute                         main.swift:393-397
        [0:16)  normal float4(nx, ny, nz, 0)
        [16:32) payload: colour float3 (+4 pad) | texture i64 index, float2 uv at +24
        [32]    tag: 0 colour, 1 texture;  [33:48) zero
    u64 nAI, u64 0; nAI x i64 attribute indices; (nAI % 2) x 8 zero   main.swift:398-400
    u64 nTexels = nFiles << 18, u64 0; nTexels x u32 0x00RRGGBB      main.swift:402-416

The reference generator draws orientations from ``Float.random`` (main.swift:13-31) and colours from
AppKit, so its output is not reproducible.  This module restates its geometry recipes
(``addSimpleFloor`` :190-216, ``addTriangle`` :74-106, ``addTetrahedron`` :218-258,
``addIcosahedron`` :260-373, ``addRegularFloor`` :108-188) with a seeded SplitMix64 stream, float32
arithmetic in the Swift expression order, and procedural 512x512 *ripmap* textures in the layout
``render.cpp:124-132`` samples (level (Lx, Ly) at x in [512-2Lx, 512-Lx), y in [512-2Ly, 512-Ly)).
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field

import numpy as np

F = np.float32
TEX_SIDE = 512
TEX_TEXELS = TEX_SIDE * TEX_SIDE  # 1 << 18 per texture (render.cpp:347)

# NSColor.orange / .red / .blue as CIColor components x 255 (main.swift:5-10, :65-67).
ORANGE = (F(255.0), F(127.5), F(0.0))
RED = (F(255.0), F(0.0), F(0.0))
BLUE = (F(0.0), F(0.0), F(255.0))


class SplitMix64:
    """SplitMix64 -- the one PRNG all scene randomness comes from (seed in the scene name)."""

    MASK = (1 << 64) - 1

    def __init__(self, seed: int):
        self.state = seed & self.MASK

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & self.MASK
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.MASK
        return z ^ (z >> 31)

    def uniform(self, lo: float, hi: float) -> float:
        """Uniform float64 in [lo, hi) from the top 53 bits."""
        return lo + (hi - lo) * ((self.next_u64() >> 11) * (1.0 / (1 << 53)))


# ---------------------------------------------------------------- float32 vector helpers (Swift simd)
def v3(x, y, z):
    return (F(x), F(y), F(z))


def add(a, b):
    return (F(a[0] + b[0]), F(a[1] + b[1]), F(a[2] + b[2]))


def sub(a, b):
    return (F(a[0] - b[0]), F(a[1] - b[1]), F(a[2] - b[2]))


def smul(s, a):
    s = F(s)
    return (F(s * a[0]), F(s * a[1]), F(s * a[2]))


def neg(a):
    return (F(-a[0]), F(-a[1]), F(-a[2]))


def dot(a, b):
    return F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2]))


def cross(a, b):
    return (F(F(a[1] * b[2]) - F(a[2] * b[1])),
            F(F(a[2] * b[0]) - F(a[0] * b[2])),
            F(F(a[0] * b[1]) - F(a[1] * b[0])))


def normalize(a):
    """simd normalize: a * (1 / sqrt(dot(a, a))), every step rounded to float32."""
    r = F(F(1.0) / F(np.sqrt(dot(a, a))))
    return (F(a[0] * r), F(a[1] * r), F(a[2] * r))


def random_unit_sphere_point(rng: SplitMix64):
    """main.swift:15-21 (cz uniform in [-1,1], angle uniform in [0, 2pi))."""
    cz = F(rng.uniform(-1.0, 1.0))
    angle = F(rng.uniform(0.0, 2.0 * math.pi))
    s = F(np.sqrt(F(F(1.0) - F(cz * cz))))
    cx = F(F(math.cos(float(angle))) * s)
    cy = F(F(math.sin(float(angle))) * s)
    return (cx, cy, cz)


def random_unit_axis(rng: SplitMix64):
    """main.swift:23-32."""
    x = random_unit_sphere_point(rng)
    while True:
        q = random_unit_sphere_point(rng)
        if q != x and q != neg(x):
            break
    y = normalize(cross(x, q))
    z = cross(x, y)
    return x, y, z


# ---------------------------------------------------------------- scene container
@dataclass
class Scene:
    vertices: list = field(default_factory=list)          # float3 tuples
    vertex_indexes: list = field(default_factory=list)
    attributes: list = field(default_factory=list)        # (normal3, ('c', rgb3) | ('t', idx, uv2))
    attribute_indexes: list = field(default_factory=list)
    textures: list = field(default_factory=list)          # np.uint32 arrays of 512*512

    @property
    def triangle_count(self) -> int:
        return len(self.vertex_indexes) // 3


def tri_normal(v, a, b, c):
    """main.swift:69-72: normalize(cross(v[c] - v[a], v[b] - v[a]))."""
    return normalize(cross(sub(v[c], v[a]), sub(v[b], v[a])))


def add_simple_floor(sc: Scene, colour: bool = False):
    """main.swift:190-216 (textured with texture 0, uv 0..15).  ``colour`` = the flat variant."""
    a = 30
    i = len(sc.vertices)
    sc.vertices += [v3(-a / 2.0, -0.5, -a - 2.0), v3(a / 2.0, -0.5, -a - 2.0),
                    v3(-a / 2.0, -0.5, -2.0), v3(a / 2.0, -0.5, -2.0)]
    scale = F(F(15) / F(a))
    sc.vertex_indexes += [i, i + 1, i + 2, i + 2, i + 1, i + 3]
    t1 = (F(0), F(0))
    t2 = (F(F(a) * scale), F(0))
    t3 = (F(0), F(F(a) * scale))
    t4 = (F(F(a) * scale), F(F(a) * scale))
    up = v3(0, 1, 0)
    j = len(sc.attributes)
    if colour:
        cols = [RED, ORANGE, BLUE, BLUE, ORANGE, RED]
        sc.attributes += [(up, ('c', c)) for c in cols]
    else:
        sc.attributes += [(up, ('t', 0, t)) for t in (t1, t2, t3, t3, t2, t4)]
    sc.attribute_indexes += list(range(j, j + 6))


def add_triangle(sc: Scene, colour: bool = False):
    """main.swift:74-106: unit triangle at z = -10, texture 1 (colour variant: :98-100)."""
    s3 = F(np.sqrt(F(3)))
    v = [v3(F(-s3 / F(2)), -0.5, 0), v3(0, 1, 0), v3(F(s3 / F(2)), -0.5, 0)]
    r = F(1.0)
    p = v3(0, 0, -10)
    v = [add(smul(r, q), p) for q in v]
    i = len(sc.vertices)
    sc.vertices += v
    sc.vertex_indexes += [i, i + 1, i + 2]
    n = tri_normal(v, 0, 1, 2)
    j = len(sc.attributes)
    if colour:
        sc.attributes += [(n, ('c', RED)), (n, ('c', ORANGE)), (n, ('c', BLUE))]
    else:
        h = F(s3 / F(2))
        sc.attributes += [(n, ('t', 1, (F(0), h))), (n, ('t', 1, (F(0.5), F(0)))),
                          (n, ('t', 1, (F(1), h)))]
    sc.attribute_indexes += list(range(j, j + 3))


def add_tetrahedron(sc: Scene, rng: SplitMix64, centre=(-10, 5, -10), radius=2.0):
    """main.swift:218-258."""
    x, y, z = random_unit_axis(rng)
    k1, k2, k3 = F(np.sqrt(F(8.0 / 9.0))), F(np.sqrt(F(2.0 / 9.0))), F(np.sqrt(F(2.0 / 3.0)))
    z3 = (F(z[0] / F(3)), F(z[1] / F(3)), F(z[2] / F(3)))
    v = [z,
         sub(smul(k1, x), z3),
         sub(add(smul(-k2, x), smul(k3, y)), z3),
         sub(sub(smul(-k2, x), smul(k3, y)), z3)]
    r = F(radius)
    p = v3(*centre)
    v = [add(smul(r, q), p) for q in v]
    i = len(sc.vertices)
    sc.vertices += v
    sc.vertex_indexes += [i, i + 2, i + 1, i, i + 3, i + 2, i, i + 1, i + 3, i + 1, i + 2, i + 3]
    faces = [((0, 2, 1), (ORANGE, ORANGE, ORANGE)), ((0, 3, 2), (RED, ORANGE, ORANGE)),
             ((0, 1, 3), (ORANGE, ORANGE, BLUE)), ((1, 2, 3), (ORANGE, ORANGE, ORANGE))]
    j = len(sc.attributes)
    for (a, b, c), cols in faces:
        n = tri_normal(v, a, b, c)
        sc.attributes += [(n, ('c', col)) for col in cols]
    sc.attribute_indexes += list(range(j, j + 12))


ICOSA_FACES = [(0, 1, 4), (4, 8, 0), (0, 8, 9), (9, 6, 0), (0, 6, 1), (1, 10, 4), (4, 10, 5),
               (5, 8, 4), (5, 2, 8), (8, 2, 9), (9, 2, 7), (7, 6, 9), (7, 11, 6), (6, 11, 1),
               (1, 11, 10), (3, 5, 10), (10, 11, 3), (3, 11, 7), (7, 2, 3), (3, 2, 5)]
# main.swift:310-371: face 3 has (red, orange, orange), face 8 (blue, orange, red), face 15 (red, ...)
ICOSA_COLOURS = {3: (RED, ORANGE, ORANGE), 8: (BLUE, ORANGE, RED), 15: (RED, ORANGE, ORANGE)}


def icosa_unit_vertices(x, y, z):
    phi = F(F(np.sqrt(F(5)) + F(1)) / F(2))
    l_ = F(F(1) / F(np.sqrt(F(phi + F(2)))))
    k = F(phi * l_)
    return [add(smul(k, x), smul(l_, y)), sub(smul(k, x), smul(l_, y)),
            add(smul(-k, x), smul(l_, y)), sub(smul(-k, x), smul(l_, y)),
            add(smul(l_, x), smul(k, z)), add(smul(-l_, x), smul(k, z)),
            sub(smul(l_, x), smul(k, z)), sub(smul(-l_, x), smul(k, z)),
            add(smul(k, y), smul(l_, z)), sub(smul(k, y), smul(l_, z)),
            add(smul(-k, y), smul(l_, z)), sub(smul(-k, y), smul(l_, z))]


def add_icosahedron(sc: Scene, rng: SplitMix64, centre=(10, 5, -10), radius=2.0):
    """main.swift:260-373."""
    x, y, z = random_unit_axis(rng)
    v = icosa_unit_vertices(x, y, z)
    r = F(radius)
    p = v3(*centre)
    v = [add(smul(r, q), p) for q in v]
    i = len(sc.vertices)
    sc.vertices += v
    for a, b, c in ICOSA_FACES:
        sc.vertex_indexes += [i + a, i + b, i + c]
    j = len(sc.attributes)
    for f, (a, b, c) in enumerate(ICOSA_FACES):
        n = tri_normal(v, a, b, c)
        cols = ICOSA_COLOURS.get(f, (ORANGE, ORANGE, ORANGE))
        sc.attributes += [(n, ('c', col)) for col in cols]
    sc.attribute_indexes += list(range(j, j + 60))


def add_regular_floor(sc: Scene, a: int = 30):
    """main.swift:108-188: a x a quads = 2a^2 textured triangles (texture 1), staggered rows."""
    i = len(sc.vertices)
    for z in range(a + 1):
        for x in range(a + 1):
            extra = F(F(0.5) * F(z % 2))
            sc.vertices.append(v3(F(F(F(x) - F(F(a) / F(2))) + extra), -0.5, F(F(-F(z)) - F(2))))
    ppm, scale = 1, F(1)
    up = v3(0, 1, 0)
    for z in range(a):
        a1 = i + z * (a + 1)
        a2 = i + (z + 1) * (a + 1)
        for x in range(a):
            j = len(sc.attributes)
            xs = F(math.fmod(float(F(F(x) * scale)), 1.0))
            ys = F(math.fmod(float(F(F(a - z - 1) * scale)), 1.0))

            def uv(du, dv):
                return (F(xs + F(F(du) * scale)), F(ys + F(F(dv) * scale)))

            if z % 2 == 0:
                sc.vertex_indexes += [a1 + x, a2 + x, a1 + 1 + x, a1 + 1 + x, a2 + x, a2 + 1 + x]
                uvs = [uv(0, 1), uv(0.5, 0), uv(1, 1), uv(1, 1), uv(0.5, 0), uv(1.5, 0)]
            else:
                sc.vertex_indexes += [a1 + x, a2 + x, a2 + 1 + x, a2 + 1 + x, a1 + 1 + x, a1 + x]
                uvs = [uv(0.5, 1), uv(0, 0), uv(1, 0), uv(1, 0), uv(1.5, 1), uv(0.5, 1)]
            sc.attributes += [(up, ('t', ppm, t)) for t in uvs]
            sc.attribute_indexes += list(range(j, j + 6))


# ---------------------------------------------------------------- procedural ripmap textures
def _base_image(kind: int) -> np.ndarray:
    """A deterministic 256x256 RGB (uint8) base image; integer arithmetic only."""
    yy, xx = np.mgrid[0:256, 0:256].astype(np.int64)
    if kind % 2 == 0:
        # checkerboard of 32-px tiles with a colour ramp and fine 4-px stripes (stresses mip choice)
        chk = ((xx >> 5) + (yy >> 5)) & 1
        r = np.where(chk == 1, 200 - (xx >> 2), 40 + (yy >> 1))
        g = np.where(chk == 1, 90 + (yy >> 2), 160 - (xx >> 2))
        b = ((xx >> 2) & 1) * 120 + 60 + ((xx * yy) >> 12)
    else:
        # concentric rings + diagonal bands
        d2 = (xx - 128) ** 2 + (yy - 128) ** 2
        ring = (d2 >> 7) & 15
        r = 30 + ring * 14
        g = (xx + yy) & 255
        b = 255 - ((xx * 3 + yy) & 255)
    img = np.stack([r, g, b], axis=-1) & 255
    return img.astype(np.uint8)


def make_ripmap(kind: int) -> np.ndarray:
    """512x512 u32 ripmap: level (Lx, Ly) = box filter of the 256x256 base at
    x in [512-2Lx, 512-Lx), y in [512-2Ly, 512-Ly); unused texels white."""
    base = _base_image(kind).astype(np.int64)
    out = np.full((TEX_SIDE, TEX_SIDE, 3), 255, dtype=np.int64)
    levels = [1 << k for k in range(9)]  # 1..256
    for ly in levels:
        fy = 256 // ly
        by = base.reshape(ly, fy, 256, 3).sum(axis=1)
        for lx in levels:
            fx = 256 // lx
            blk = by.reshape(ly, lx, fx, 3).sum(axis=2) // (fx * fy)
            y0, x0 = TEX_SIDE - 2 * ly, TEX_SIDE - 2 * lx
            out[y0:y0 + ly, x0:x0 + lx] = blk
    rgb = (out[..., 0] << 16) | (out[..., 1] << 8) | out[..., 2]
    return rgb.astype(np.uint32).reshape(-1)


def ripmap_from_ppm(path: str) -> np.ndarray:
    """Pack a 512x512 binary PPM (P6) the way main.swift:405-414 does (skip a 15-byte header)."""
    with open(path, 'rb') as f:
        data = f.read()[15:]
    px = np.frombuffer(data, dtype=np.uint8).reshape(-1, 3).astype(np.uint32)
    return ((px[:, 0] << 16) | (px[:, 1] << 8) | px[:, 2]).astype(np.uint32)


# ---------------------------------------------------------------- named scenes
def build_scene(name: str) -> Scene:
    """Named deterministic scenes:
    full      floor(tex0) + triangle(tex1) + 2 tetrahedra + 2 icosahedra   (the packaged scene)
    flat      the same with the floor and triangle in flat colour (config 2)
    tetra     one tetrahedron, seed 0 (config 1)
    regular   addRegularFloor (1800 textured triangles) + the full scene's objects
    """
    sc = Scene()
    if name in ('full', 'flat'):
        rng = SplitMix64(0x5EED0001)
        colour = name == 'flat'
        add_simple_floor(sc, colour=colour)
        add_triangle(sc, colour=colour)
        for _ in range(2):
            add_tetrahedron(sc, rng)
        for _ in range(2):
            add_icosahedron(sc, rng)
        sc.textures = [make_ripmap(0), make_ripmap(1)]
    elif name == 'tetra':
        rng = SplitMix64(0)
        add_tetrahedron(sc, rng)
        sc.textures = []
    elif name == 'regular':
        rng = SplitMix64(0x5EED0003)
        add_regular_floor(sc)
        add_triangle(sc)
        for _ in range(2):
            add_tetrahedron(sc, rng)
        for _ in range(2):
            add_icosahedron(sc, rng)
        sc.textures = [make_ripmap(0), make_ripmap(1)]
    else:
        raise ValueError(f'unknown scene {name!r}')
    return sc


# ---------------------------------------------------------------- data.bin writer / reader
def _attr_bytes(attr) -> bytes:
    normal, ca = attr
    b = struct.pack('<4f', float(normal[0]), float(normal[1]), float(normal[2]), 0.0)
    if ca[0] == 'c':
        b += struct.pack('<4f', float(ca[1][0]), float(ca[1][1]), float(ca[1][2]), 0.0)
        b += bytes([0]) + bytes(15)
    else:
        b += struct.pack('<q2f', int(ca[1]), float(ca[2][0]), float(ca[2][1]))
        b += bytes([1]) + bytes(15)
    assert len(b) == 48
    return b


def encode(sc: Scene) -> bytes:
    """Serialize in the data.bin layout of main.swift:387-416."""
    out = bytearray()
    out += struct.pack('<2Q', len(sc.vertices), 0)
    v = np.array([[x, y, z, 1.0] for (x, y, z) in sc.vertices], dtype=np.float32).reshape(-1, 4)
    out += v.tobytes()
    for idx in (sc.vertex_indexes, None, sc.attribute_indexes):
        if idx is None:
            out += struct.pack('<2Q', len(sc.attributes), 0)
            out += b''.join(_attr_bytes(a) for a in sc.attributes)
            continue
        out += struct.pack('<2Q', len(idx), 0)
        out += np.asarray(idx, dtype=np.int64).tobytes()
        out += bytes(8 * (len(idx) % 2))
    out += struct.pack('<2Q', len(sc.textures) << 18, 0)
    for t in sc.textures:
        assert t.dtype == np.uint32 and t.size == TEX_TEXELS
        out += t.tobytes()
    return bytes(out)


def write_scene(sc: Scene, path: str) -> int:
    data = encode(sc)
    with open(path, 'wb') as f:
        f.write(data)
    return len(data)


@dataclass
class SceneArrays:
    vertices: np.ndarray            # (nV, 4) float32
    vertex_indices: np.ndarray      # (nI,) int64
    attributes: np.ndarray          # (nA, 48) uint8
    attribute_indices: np.ndarray   # (nAI,) int64
    texels: np.ndarray              # (nT,) uint32


def decode(data: bytes) -> SceneArrays:
    """Parse data.bin exactly like render.cpp:177-209 (including the nI % 2 padding)."""
    off = 0

    def hdr():
        nonlocal off
        n, z = struct.unpack_from('<2Q', data, off)
        off += 16
        return n

    nv = hdr()
    vert = np.frombuffer(data, dtype=np.float32, count=4 * nv, offset=off).reshape(nv, 4)
    off += 16 * nv
    ni = hdr()
    vi = np.frombuffer(data, dtype=np.int64, count=ni, offset=off)
    off += 8 * (ni + ni % 2)
    na = hdr()
    attrs = np.frombuffer(data, dtype=np.uint8, count=48 * na, offset=off).reshape(na, 48)
    off += 48 * na
    nai = hdr()
    ai = np.frombuffer(data, dtype=np.int64, count=nai, offset=off)
    off += 8 * (nai + nai % 2)
    nt = hdr()
    tex = np.frombuffer(data, dtype=np.uint32, count=nt, offset=off)
    off += 4 * nt
    if off != len(data):
        raise ValueError(f'data.bin: {len(data) - off} trailing bytes')
    return SceneArrays(vert, vi, attrs, ai, tex)


def read_scene(path: str) -> SceneArrays:
    with open(path, 'rb') as f:
        return decode(f.read())


def write_named(name: str, path: str) -> int:
    from . import stress
    if stress.is_stress_name(name):       # icosa-stress (config 5) / icosa-<n>: streamed, vectorized
        return stress.write_named(name, path)
    return write_scene(build_scene(name), path)
