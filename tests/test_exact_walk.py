"""The O(binades) walker that replaces render.cpp's per-pixel `w += dx` loop (render.cpp:374-379)
must equal n sequential float32 additions bit-for-bit.  CPU: the library's host build against the
oracle's sequential loop; GPU: the device build (rcp-based jump) against the same loop."""
import ctypes

import numpy as np
import pytest

from oracle.oracle import lib as oracle_lib
from swift3drenderer_amd.renderer import load_library


def sequential(s, d, n):
    """n sequential float32 adds, vectorised over cases (numpy float32 adds are IEEE binary32)."""
    s = s.astype(np.float32).copy()
    d = d.astype(np.float32)
    out = s.copy()
    nmax = int(n.max()) if len(n) else 0
    for k in range(nmax):
        act = n > k
        s[act] = (s[act] + d[act]).astype(np.float32)
    out[:] = s
    return out


def linear_truth(s, d, n):
    """Whether S(s, d, k) == s + k*del for k < n, with del = S(s,d,1) - s (checked sequentially)."""
    ok = np.ones(len(s), dtype=bool)
    cur = s.astype(np.float32).copy()
    step = (cur + d).astype(np.float32) - cur
    for k in range(1, int(n.max())):
        act = n > k
        cur[act] = (cur[act] + d[act]).astype(np.float32)
        pred = (s + np.float32(k) * step).astype(np.float32)
        ok &= ~act | (cur == pred)
    return ok, step


def cases(seed, count=20000, nmax=4000):
    rng = np.random.default_rng(seed)
    s = rng.uniform(-3, 3, count).astype(np.float32)
    mag = 10.0 ** rng.uniform(-7, -0.5, count)
    d = (mag * rng.choice([-1, 1], count)).astype(np.float32)
    n = rng.integers(0, nmax, count).astype(np.uint32)
    # edge cases: zeros, signed zeros, zero step, exact halves (tie-to-even), binade edges
    s[:8] = [0.0, -0.0, 1.0, -1.0, 0.5, 2.0 ** -20, 1.0 - 2 ** -24, -2.0]
    d[:8] = [0.0, 0.0, -2 ** -25, 2 ** -25, -2 ** -26 * 3, 2 ** -30, 2 ** -24, 1e-3]
    s[8:16] = 1.0
    d[8:16] = np.float32(2 ** -24) * np.array([0.5, 1.5, 2.5, -0.5, -1.5, 3.5, 0.25, 1.0], dtype=np.float32)
    return s, d, n


def run_host(s, d, n):
    lib = load_library()
    c = len(s)
    out = np.empty(c, np.float32)
    lin = np.empty(c, np.uint32)
    dl = np.empty(c, np.float32)
    P = ctypes.POINTER
    lib.s3r_selftest_walk_host(s.ctypes.data_as(P(ctypes.c_float)), d.ctypes.data_as(P(ctypes.c_float)),
                               n.ctypes.data_as(P(ctypes.c_uint32)), out.ctypes.data_as(P(ctypes.c_float)),
                               lin.ctypes.data_as(P(ctypes.c_uint32)), dl.ctypes.data_as(P(ctypes.c_float)),
                               ctypes.c_uint64(c))
    return out, lin, dl


def run_device(s, d, n):
    lib = load_library()
    c = len(s)
    out = np.empty(c, np.float32)
    lin = np.empty(c, np.uint32)
    dl = np.empty(c, np.float32)
    P = ctypes.POINTER
    rc = lib.s3r_selftest_walk_device(s.ctypes.data_as(P(ctypes.c_float)), d.ctypes.data_as(P(ctypes.c_float)),
                                      n.ctypes.data_as(P(ctypes.c_uint32)), out.ctypes.data_as(P(ctypes.c_float)),
                                      lin.ctypes.data_as(P(ctypes.c_uint32)), dl.ctypes.data_as(P(ctypes.c_float)),
                                      ctypes.c_uint32(c))
    assert rc == 0
    return out, lin, dl


def bits(x):
    return np.asarray(x, np.float32).view(np.uint32)


def test_sequential_helper_matches_oracle_loop():
    s, d, n = cases(1, count=200, nmax=300)
    want = sequential(s, d, n)
    got = np.array([oracle_lib().oracle_repeat_add(float(a), float(b), int(k)) for a, b, k in zip(s, d, n)],
                   dtype=np.float32)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize('seed', [1, 2, 3])
def test_host_walk_exact(seed):
    s, d, n = cases(seed)
    want = sequential(s, d, n)
    got, _, _ = run_host(s, d, n)
    bad = np.nonzero(bits(got) != bits(want))[0]
    assert bad.size == 0, f'{bad.size} mismatches, first s={s[bad[0]]!r} d={d[bad[0]]!r} n={n[bad[0]]}'


def test_host_walk_pixel_scale():
    """Realistic raster ranges: |w| <= 1.5, |dx| in [1e-4, 3e-2], n up to 7680 (8K rows)."""
    rng = np.random.default_rng(11)
    c = 20000
    s = rng.uniform(-1.5, 1.5, c).astype(np.float32)
    d = (10.0 ** rng.uniform(-4, -1.5, c) * rng.choice([-1, 1], c)).astype(np.float32)
    n = rng.integers(0, 7680, c).astype(np.uint32)
    want = sequential(s, d, n)
    got, _, _ = run_host(s, d, n)
    assert np.array_equal(bits(got), bits(want))


def adversarial_cases(seed, count=20000):
    """Steps that are exact half-ulps (tie-to-even), starts just below/above binade edges, both
    directions, and long runs across many binades."""
    rng = np.random.default_rng(seed)
    e = rng.integers(-12, 3, count)
    s = (2.0 ** e * rng.choice([1.0, 1.0 - 2 ** -23, 1.0 + 2 ** -23, 1.5], count)).astype(np.float32)
    s *= rng.choice([-1, 1], count).astype(np.float32)
    u = 2.0 ** (e - 23)
    k = rng.integers(1, 4000, count)
    half = rng.random(count) < 0.5
    d = np.where(half, (k + 0.5) * u, k * u * rng.uniform(0.9, 1.1, count)) * rng.choice([-1, 1], count)
    d = d.astype(np.float32)
    n = rng.integers(1, 12000, count).astype(np.uint32)
    return s, d, n


@pytest.mark.parametrize('seed', [21, 22])
def test_host_walk_adversarial(seed):
    s, d, n = adversarial_cases(seed)
    want = sequential(s, d, n)
    got, _, _ = run_host(s, d, n)
    bad = np.nonzero(bits(got) != bits(want))[0]
    assert bad.size == 0, f'{bad.size} mismatches, first s={s[bad[0]]!r} d={d[bad[0]]!r} n={n[bad[0]]}'


def test_chunk_linear_is_sound():
    """Whenever chunk_linear says 'linear', every k < m is exactly s + k*delta."""
    s, d, _ = cases(5, count=20000)
    m = np.random.default_rng(5).integers(1, 65, len(s)).astype(np.uint32)
    _, lin, dl = run_host(s, d, m)
    truth, _ = linear_truth(s, d, m)
    claimed = lin.astype(bool)
    assert not np.any(claimed & ~truth), 'chunk_linear claimed a non-linear chunk'
    # and it is not uselessly conservative at raster scales
    assert claimed.mean() > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize('seed', [1, 4])
def test_device_walk_exact(seed):
    from conftest import gpu_available
    if not gpu_available():
        pytest.skip('no GPU')
    import torch
    torch.cuda.init()
    s, d, n = cases(seed, count=50000)
    s2, d2, n2 = adversarial_cases(seed + 100, count=20000)
    s, d, n = np.concatenate([s, s2]), np.concatenate([d, d2]), np.concatenate([n, n2])
    want = sequential(s, d, n)
    got, _, _ = run_device(s, d, n)
    assert np.array_equal(bits(got), bits(want))
    # the device's chunk_linear (chunks of <= 64 pixels) is sound too
    m = np.minimum(n, 64).astype(np.uint32)
    _, lin, _ = run_device(s, d, m)
    truth, _ = linear_truth(s, d, m)
    assert not np.any(lin.astype(bool) & ~truth)


@pytest.mark.gpu
@pytest.mark.parametrize('mode,count', [(0, 0), (1, 0), (2, 1 << 30), (3, 1 << 26)])
def test_fast_div_sqrt_device(mode, count):
    """The shading stage's trimmed exact sequences (s3r_common.h: div_recip / div_with_recip /
    sqrt_in_range, used only inside their range checks) return the IEEE operators' bits: sqrt over
    every input of its range, 1/s over every divisor the normalisation can see, and 2^30 hashed
    in-range quotients (plus 2^26 whole normalisations)."""
    from conftest import gpu_available
    if not gpu_available():
        pytest.skip('no GPU')
    import torch
    torch.cuda.init()
    lib = load_library()
    lib.s3r_selftest_fastmath_device.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    out = (ctypes.c_uint64 * 2)()
    assert lib.s3r_selftest_fastmath_device(mode, count, out) == 0
    assert out[0] == 0, f'mode {mode}: {out[0]} mismatches, first at index {out[1]}'
