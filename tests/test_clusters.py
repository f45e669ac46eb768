"""Init-time clusters of the tile path (csrc/clusters.cpp, include/render.h s3r_build_clusters), on
the CPU: every triangle in exactly one cluster, clusters of at most 32 triangles, bounding spheres
that hold every corner, meshes kept whole, loose triangles pooled into compact clusters.  The
per-frame cull on the GPU is checked against the oracle in tests/test_tiles.py."""
import ctypes

import numpy as np
import pytest

from swift3drenderer_amd import scene, stress
from swift3drenderer_amd.renderer import load_library


def clusters_of(vtx: np.ndarray, vidx: np.ndarray):
    lib = load_library()
    f = lib.s3r_build_clusters
    f.restype = ctypes.c_uint32
    P = ctypes.POINTER
    f.argtypes = [P(ctypes.c_float), ctypes.c_uint32, P(ctypes.c_uint32), ctypes.c_uint32, P(ctypes.c_uint32),
                  P(ctypes.c_float), ctypes.c_uint32, P(ctypes.c_uint32)]
    vtx = np.ascontiguousarray(vtx, dtype=np.float32)
    vidx = np.ascontiguousarray(vidx, dtype=np.uint32)
    ntri = vidx.size // 3
    cap = ntri + 1
    first = np.zeros(cap, dtype=np.uint32)
    sphere = np.zeros((cap, 4), dtype=np.float32)
    perm = np.zeros(max(ntri, 1), dtype=np.uint32)
    n = f(vtx.ctypes.data_as(P(ctypes.c_float)), vtx.shape[0], vidx.ctypes.data_as(P(ctypes.c_uint32)), ntri,
          first.ctypes.data_as(P(ctypes.c_uint32)), sphere.ctypes.data_as(P(ctypes.c_float)), cap,
          perm.ctypes.data_as(P(ctypes.c_uint32)))
    return first[:n + 1].astype(np.int64), sphere[:n], perm[:ntri]


def check_invariants(vtx, vidx, first, sphere, perm):
    ntri = vidx.size // 3
    assert first[0] == 0 and first[-1] == ntri
    sizes = np.diff(first)
    assert (sizes >= 1).all() and (sizes <= 32).all()
    assert np.array_equal(np.sort(perm), np.arange(ntri))          # a permutation of the slots
    corners = vtx[vidx.reshape(-1, 3)[perm], :3].astype(np.float64)  # (ntri, 3, 3) in cluster order
    cl = np.repeat(np.arange(len(sizes)), sizes)
    d = np.linalg.norm(corners - sphere[cl, None, :3].astype(np.float64), axis=2)
    assert (d <= sphere[cl, None, 3]).all()                        # every corner inside its sphere
    return sizes


def test_icosahedra_are_one_cluster_each(tmp_path):
    p = str(tmp_path / 'i.bin')
    stress.write_stress(p, 500, seed=1)
    a = scene.read_scene(p)
    vidx = a.vertex_indices.astype(np.uint32)
    first, sphere, perm = clusters_of(a.vertices, vidx)
    sizes = check_invariants(a.vertices, vidx, first, sphere, perm)
    assert len(sizes) == 500 and (sizes == 20).all()
    assert np.array_equal(perm, np.arange(vidx.size // 3))         # file order kept: no permutation
    # the sphere of an icosahedron is its circumsphere: radius = the icosahedron's own radius
    v = a.vertices[:12, :3].astype(np.float64)
    r = np.linalg.norm(v - v.mean(axis=0), axis=1).max()
    assert sphere[0, 3] == pytest.approx(r, rel=1e-5)


def test_soup_is_pooled_into_compact_clusters(tmp_path):
    p = str(tmp_path / 's.bin')
    stress.write_soup(p, 400, seed=1)
    a = scene.read_scene(p)
    vidx = a.vertex_indices.astype(np.uint32)
    first, sphere, perm = clusters_of(a.vertices, vidx)
    sizes = check_invariants(a.vertices, vidx, first, sphere, perm)
    assert not np.array_equal(perm, np.arange(vidx.size // 3))     # shuffled loose triangles: reordered
    assert sizes.mean() > 24                                       # pooled up to 32
    # Morton-ordered pools: a cluster spans a few neighbouring icosahedra, not the scene
    scene_ext = np.ptp(a.vertices[:, :3], axis=0).max()
    assert np.median(sphere[:, 3]) < 0.1 * scene_ext


def test_large_mesh_is_cut(tmp_path):
    sc = scene.build_scene('regular')                              # addRegularFloor: 1 800 triangles, one mesh
    p = str(tmp_path / 'r.bin')
    scene.write_scene(sc, p)
    a = scene.read_scene(p)
    vidx = a.vertex_indices.astype(np.uint32)
    first, sphere, perm = clusters_of(a.vertices, vidx)
    sizes = check_invariants(a.vertices, vidx, first, sphere, perm)
    assert len(sizes) >= 1800 // 32


def test_tiny_and_degenerate_inputs():
    vtx = np.array([[0, 0, -1, 1], [1, 0, -1, 1], [0, 1, -1, 1]], dtype=np.float32)
    first, sphere, perm = clusters_of(vtx, np.array([0, 1, 2], dtype=np.uint32))
    assert list(first) == [0, 1] and list(perm) == [0]
    assert sphere[0, 3] >= np.sqrt(0.5) * 0.999
    # a non-finite corner: radius +inf (the cull keeps that cluster)
    vtx[2, 0] = np.inf
    first, sphere, perm = clusters_of(vtx, np.array([0, 1, 2], dtype=np.uint32))
    assert np.isinf(sphere[0, 3])
    first, sphere, perm = clusters_of(vtx, np.zeros(0, dtype=np.uint32))
    assert list(first) == [0] and len(sphere) == 0
