"""The RNG substitution, checked as distributions (CPU; oracle primitives).

The reference draws from rand::thread_rng() (unseedable ChaCha12) and rand_distr's Normal, so
its streams cannot be reproduced (parity unpinned at the RNG boundary, oracle/oracle.h).  What the
substitution must preserve is each draw's DISTRIBUTION:
  * gen_range(0.0..1.0) (ray_tracing.rs:78-79, materials.rs:137)    -> u01: uniform on [0, 1)
  * Vec3::random_unit_vector (geometry.rs:139-152): a normalised 3-D standard normal, i.e.
    uniform on S^2                                                   -> unit_vec(u1, u2)
  * Vec3::random_in_unit_disk (geometry.rs:154-168): rejection on [-1,1]^2 -> uniform on the disk
These tests draw from the same Philox4x32-10 words (fp64) and Philox2x32-10 words (fp32) and the same
polynomial sin/cos as the oracle and the kernel, and compare moments and histograms with the exact
distributions.
"""
import ctypes
import math

import numpy as np

from oracle_bind import load_oracle

SEED = 0x5EED0001
N = 60000


def _blocks(n, stream, bounce=0):
    lib = load_oracle()
    out = np.zeros((n, 4), np.uint64)
    o = (ctypes.c_uint32 * 4)()
    key = (ctypes.c_uint32 * 2)(SEED & 0xFFFFFFFF, SEED >> 32)
    for s in range(n):
        lib.oracle_philox4x32_10((ctypes.c_uint32 * 4)(s, 12345, bounce, stream), key, o)
        out[s] = list(o)
    return out


def _u01_f64(b, hi, lo):
    return (((b[:, hi] << np.uint64(32)) | b[:, lo]) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def _unit_vec(u1, u2):
    lib = load_oracle()
    z = 1.0 - 2.0 * u1
    r = np.sqrt(1.0 - z * z)
    s, c = ctypes.c_double(), ctypes.c_double()
    sc = np.zeros((len(u2), 2))
    for i, u in enumerate(u2):
        lib.oracle_sincos2pi_f64(float(u), ctypes.byref(s), ctypes.byref(c))
        sc[i] = (s.value, c.value)
    return np.stack([r * sc[:, 1], r * sc[:, 0], z], axis=1)


def test_uniform_draws():
    b = _blocks(N, 2)
    for u in (_u01_f64(b, 0, 1), _u01_f64(b, 2, 3), (b[:, 0] >> np.uint64(8)).astype(np.float64) * 2.0 ** -24):
        assert u.min() >= 0.0 and u.max() < 1.0
        assert abs(u.mean() - 0.5) < 4 * math.sqrt(1 / 12 / N)
        hist = np.histogram(u, bins=20, range=(0, 1))[0]
        chi2 = ((hist - N / 20) ** 2 / (N / 20)).sum()
        assert chi2 < 45.0          # 19 dof, p ~ 1e-3
    # the two uniforms of one block are independent
    u1, u2 = _u01_f64(b, 0, 1), _u01_f64(b, 2, 3)
    assert abs(np.corrcoef(u1, u2)[0, 1]) < 4 / math.sqrt(N)


def test_unit_vector_is_uniform_on_sphere():
    """Same law as normalize(N(0,1)^3): unit length, zero mean, covariance I/3, and by Archimedes'
    theorem every coordinate is uniform on [-1, 1]; octants equally likely."""
    b = _blocks(N, 2, bounce=3)
    v = _unit_vec(_u01_f64(b, 0, 1), _u01_f64(b, 2, 3))
    np.testing.assert_allclose(np.linalg.norm(v, axis=1), 1.0, atol=1e-14)
    se = math.sqrt(1 / 3 / N)
    assert np.all(np.abs(v.mean(axis=0)) < 4 * se)
    cov = v.T @ v / N
    np.testing.assert_allclose(np.diag(cov), 1 / 3, atol=4 * math.sqrt(4 / 45 / N))
    assert np.all(np.abs(cov - np.diag(np.diag(cov))) < 4 * math.sqrt(1 / 15 / N))
    for k in range(3):
        hist = np.histogram(v[:, k], bins=20, range=(-1, 1))[0]
        assert ((hist - N / 20) ** 2 / (N / 20)).sum() < 45.0
    octant = (v[:, 0] > 0) * 4 + (v[:, 1] > 0) * 2 + (v[:, 2] > 0)
    hist = np.bincount(octant, minlength=8)
    assert ((hist - N / 8) ** 2 / (N / 8)).sum() < 25.0     # 7 dof


def test_unit_vector_matches_normalised_gaussian_in_distribution():
    """Two-sample Kolmogorov-Smirnov on the polar angle of our unit_vec against numpy's
    normalised Gaussians (what rand_distr's Normal + normalize produces)."""
    b = _blocks(N, 2, bounce=5)
    ours = _unit_vec(_u01_f64(b, 0, 1), _u01_f64(b, 2, 3))
    g = np.random.default_rng(7).standard_normal((N, 3))
    ref = g / np.linalg.norm(g, axis=1, keepdims=True)
    for f in (lambda v: v[:, 2], lambda v: np.arctan2(v[:, 1], v[:, 0])):
        a, c = np.sort(f(ours)), np.sort(f(ref))
        grid = np.concatenate([a, c])
        d = np.max(np.abs(np.searchsorted(a, grid, side="right") / N - np.searchsorted(c, grid, side="right") / N))
        assert d < 1.95 * math.sqrt(2 / N)       # KS critical value, alpha ~ 0.001


def test_disk_rejection_is_uniform_on_disk():
    """random_in_unit_disk: first accepted draw of stream 1 — uniform on the unit disk, so the
    radius^2 is uniform on [0,1) and the angle uniform; about pi/4 of draws accepted."""
    lib = load_oracle()
    key = (ctypes.c_uint32 * 2)(SEED & 0xFFFFFFFF, SEED >> 32)
    o = (ctypes.c_uint32 * 4)()
    pts, tries = [], 0
    for s in range(20000):
        for i in range(256):
            lib.oracle_philox4x32_10((ctypes.c_uint32 * 4)(s, 777, i, 1), key, o)
            w = list(o)
            x = 2.0 * ((((w[0] << 32) | w[1]) >> 11) * 2.0 ** -53) - 1.0
            y = 2.0 * ((((w[2] << 32) | w[3]) >> 11) * 2.0 ** -53) - 1.0
            tries += 1
            if x * x + y * y <= 1.0:
                pts.append((x, y))
                break
    p = np.array(pts)
    n = len(p)
    assert abs(n / tries - math.pi / 4) < 0.01
    r2 = (p ** 2).sum(axis=1)
    hist = np.histogram(r2, bins=10, range=(0, 1))[0]
    assert ((hist - n / 10) ** 2 / (n / 10)).sum() < 30.0
    ang = np.histogram(np.arctan2(p[:, 1], p[:, 0]), bins=12, range=(-math.pi, math.pi))[0]
    assert ((ang - n / 12) ** 2 / (n / 12)).sum() < 35.0


def _blocks2(n, code, pix=12345):
    """fp32 draws: Philox2x32-10 at counter (pixel, sample | code << 20), key seed lo ^ fmix32(seed hi)."""
    lib = load_oracle()
    out = np.zeros((n, 2), np.uint64)
    o = (ctypes.c_uint32 * 2)()
    lib.oracle_fmix32.restype = ctypes.c_uint32
    key = ctypes.c_uint32((SEED & 0xFFFFFFFF) ^ lib.oracle_fmix32(ctypes.c_uint32(SEED >> 32)))
    for s in range(n):
        lib.oracle_philox2x32_10((ctypes.c_uint32 * 2)(pix, s | (code << 20)), key, o)
        out[s] = list(o)
    return out


def test_f32_uniform_draws():
    """The fp32 build's two 24-bit uniforms per block (camera, scatter at bounces 0 and 49): uniform, and
    independent of each other and of the neighbouring streams."""
    bs = [_blocks2(N, code) for code in (0, 257, 257 + 49)]
    us = []
    for b in bs:
        for w in (0, 1):
            u = (b[:, w] >> np.uint64(8)).astype(np.float64) * 2.0 ** -24
            assert u.min() >= 0.0 and u.max() < 1.0
            assert abs(u.mean() - 0.5) < 4 * math.sqrt(1 / 12 / N)
            hist = np.histogram(u, bins=20, range=(0, 1))[0]
            assert ((hist - N / 20) ** 2 / (N / 20)).sum() < 45.0
            us.append(u)
    c = np.corrcoef(np.stack(us))
    assert np.all(np.abs(c - np.eye(len(us))) < 4 / math.sqrt(N))
    # the unit vector from an fp32 block: every coordinate uniform on [-1, 1]
    b = bs[1]
    v = _unit_vec((b[:, 0] >> np.uint64(8)).astype(np.float64) * 2.0 ** -24,
                  (b[:, 1] >> np.uint64(8)).astype(np.float64) * 2.0 ** -24)
    for k in range(3):
        hist = np.histogram(v[:, k], bins=20, range=(-1, 1))[0]
        assert ((hist - N / 20) ** 2 / (N / 20)).sum() < 45.0
