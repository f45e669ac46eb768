"""data.bin format (main.swift:381-416 writer, render.cpp:177-209 reader) and the
deterministic scene generator."""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from swift3drenderer_amd import scene

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden', 'scenes.json')


def test_packaged_scene_size_and_counts():
    data = scene.encode(scene.build_scene('full'))
    # nV=39, nI=153, nA=153, nAI=153, 2 textures -> 2 107 664 bytes
    assert len(data) == 2_107_664
    a = scene.decode(data)
    assert a.vertices.shape == (39, 4)
    assert len(a.vertex_indices) == 153 and len(a.attribute_indices) == 153
    assert a.attributes.shape == (153, 48)
    assert len(a.texels) == 2 << 18


def test_header_layout_and_padding():
    data = scene.encode(scene.build_scene('full'))
    nv, z = struct.unpack_from('<2Q', data, 0)
    assert (nv, z) == (39, 0)
    off = 16 + 16 * nv
    ni, z = struct.unpack_from('<2Q', data, off)
    assert (ni, z) == (153, 0)
    off += 16 + 8 * ni
    assert data[off:off + 8] == bytes(8)          # nI odd -> one 8-byte pad (main.swift:392)
    off += 8
    na, _ = struct.unpack_from('<2Q', data, off)
    assert na == 153


def test_vertex_w_is_one_and_attribute_layout():
    a = scene.decode(scene.encode(scene.build_scene('full')))
    assert np.all(a.vertices[:, 3] == 1.0)
    tags = a.attributes[:, 32]
    assert set(np.unique(tags)) <= {0, 1}
    assert np.all(a.attributes[:, 33:] == 0)       # 15 zero bytes after the 33-byte struct
    normals = a.attributes[:, :16].view(np.float32).reshape(-1, 4)
    assert np.all(normals[:, 3] == 0.0)            # simd_make_float4(float3) zero-fills w
    tex = a.attributes[tags == 1]
    idx = tex[:, 16:24].view(np.int64).ravel()
    assert set(idx) <= {0, 1}
    assert (tags == 1).sum() == 9                  # floor 6 + triangle 3 textured


def test_round_trip_all_scenes():
    for name in ('full', 'flat', 'tetra', 'regular'):
        sc = scene.build_scene(name)
        a = scene.decode(scene.encode(sc))
        assert len(a.vertices) == len(sc.vertices)
        assert np.array_equal(a.vertex_indices, np.asarray(sc.vertex_indexes))
        assert np.array_equal(a.attribute_indices, np.asarray(sc.attribute_indexes))


def test_flat_scene_has_no_texture_path():
    a = scene.decode(scene.encode(scene.build_scene('flat')))
    assert np.all(a.attributes[:, 32] == 0)


def test_trailing_bytes_rejected():
    data = scene.encode(scene.build_scene('tetra'))
    with pytest.raises(ValueError):
        scene.decode(data + b'\0')


def test_ripmap_levels_are_box_filters():
    t = scene.make_ripmap(0).reshape(512, 512)
    rgb = np.stack([(t >> 16) & 255, (t >> 8) & 255, t & 255], -1).astype(np.int64)
    base = rgb[:256, :256]
    # level (Lx=128, Ly=256) at x in [256, 384): 2x horizontal box downsample
    half = (base[:, 0::2] + base[:, 1::2]) // 2
    assert np.array_equal(rgb[:256, 256:384], half)
    # level (1, 1) at (510, 510) = mean of the base
    assert np.array_equal(rgb[510, 510], base.reshape(-1, 3).sum(0) // (256 * 256))
    # column 511 and row 511 unused (white)
    assert np.all(t[:, 511] == 0xFFFFFF) and np.all(t[511, :] == 0xFFFFFF)


def test_ppm_packing(tmp_path):
    """main.swift:405-414: skip a 15-byte header, pack (r<<16)|(g<<8)|b."""
    px = np.arange(512 * 512 * 3, dtype=np.uint32) % 251
    p = tmp_path / 'x.ppm'
    p.write_bytes(b'P6\n512 512\n255\n' + px.astype(np.uint8).tobytes())
    t = scene.ripmap_from_ppm(str(p))
    assert t[1] == (px[3] << 16) | (px[4] << 8) | px[5]


def test_generator_is_deterministic():
    """SHA-256 of every named scene is pinned (tests/golden/scenes.json)."""
    with open(GOLDEN) as f:
        want = json.load(f)
    for name, h in want.items():
        got = hashlib.sha256(scene.encode(scene.build_scene(name))).hexdigest()
        assert got == h, name


def test_splitmix_known_answer():
    # SplitMix64 reference values for seed 1234567 (Vigna's splitmix64.c)
    r = scene.SplitMix64(1234567)
    assert [r.next_u64() for _ in range(3)] == [6457827717110365317, 3203168211198807973, 9817491932198370423]


def test_stress_scene_layout_and_determinism(tmp_path):
    """The icosahedron stress generator (config 5): data.bin layout, size formula, cross-check of
    one icosahedron against the scalar addIcosahedron restatement, and a pinned digest."""
    from swift3drenderer_amd import stress
    p = str(tmp_path / 'i500.bin')
    n = stress.write_stress(p, 500, seed=1)
    assert n == stress.expected_size(500) == len(open(p, 'rb').read())
    s = scene.read_scene(p)
    assert s.vertices.shape == (6000, 4) and np.all(s.vertices[:, 3] == 1)
    assert np.array_equal(s.attribute_indices, np.arange(30000))
    assert s.vertex_indices[:60].tolist() == [v for f in scene.ICOSA_FACES for v in f]
    assert s.vertex_indices.max() == 5999 and s.texels.size == 0
    assert np.all(s.attributes[:, 32] == 0)                       # colour tag
    z = s.vertices[:, 2]
    assert z.max() < -4.9 and z.min() > -60.5
    with open(p, 'rb') as f:
        assert hashlib.sha256(f.read()).hexdigest() == \
            '1edf44cfbed40516b3ae72494776ec0c455f489db36f58552ba8d007048b7ef6'
    assert stress.is_stress_name('icosa-stress') and stress.count_of('icosa-stress') == 1_000_000
    assert stress.count_of('icosa-2000') == 2000 and not stress.is_stress_name('full')


def test_stress_matches_scalar_icosahedron():
    from swift3drenderer_amd import stress
    ids = np.arange(7, 8, dtype=np.uint64)
    x, y, z = stress._frames(1, ids)
    v, nrm = stress._chunk(1, 7, 8)
    uv = scene.icosa_unit_vertices(*[tuple(np.float32(c) for c in a[0]) for a in (x, y, z)])
    depth = stress._uniform(1, 4, ids, *stress.DEPTH)
    cx = stress._uniform(1, 5, ids, -1.05, 1.05) * stress.HALF_X * depth
    cy = stress._uniform(1, 6, ids, -1.05, 1.05) * stress.HALF_Y * depth
    r = depth * stress._uniform(1, 7, ids, *stress.RADIUS_PER_DEPTH)
    vv = [scene.add(scene.smul(r[0], q), (cx[0], cy[0], -depth[0])) for q in uv]
    assert np.array_equal(np.array(vv, dtype=np.float32), v[0])
    nn = [scene.tri_normal(vv, a, b, c) for a, b, c in scene.ICOSA_FACES]
    assert np.array_equal(np.array(nn, dtype=np.float32), nrm[0])
