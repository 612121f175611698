"""The kernel's div_dim (rt_kernel.hip): for the camera's pixel coordinate x = col + u (u a 24-bit
uniform, ray_tracing.rs:78-79) and an image dimension W < 2^20, float32(float64(x) * RN64(1/W))
equals the correctly rounded float32 x / W.  Proof in the kernel comment; here checked for every
W <= 4096 on a sample of x per W (256 random col + u, plus the integer and just-below-integer
boundaries), and for the BASELINE dimensions and large W on 200 000 random x each (numpy's float32
division is IEEE correctly rounded).  A sampled check, not an exhaustive one: the proof covers the rest."""
import numpy as np


def _check(W, x):
    x = x.astype(np.float32)
    want = x / np.float32(W)
    got = (x.astype(np.float64) * (1.0 / float(W))).astype(np.float32)
    bad = np.flatnonzero(want != got)
    assert bad.size == 0, (W, x[bad[:4]], want[bad[:4]], got[bad[:4]])


def test_div_dim_every_small_dimension():
    rng = np.random.default_rng(0x5EED0001)
    for W in range(1, 4097):
        col = rng.integers(0, W, 256)
        u = rng.integers(0, 1 << 24, 256) * 2.0 ** -24
        x = np.concatenate([col + u, np.arange(min(W, 64)), np.arange(min(W, 64)) + (1 - 2.0 ** -24)])
        _check(W, x)


def test_div_dim_large_dimensions():
    rng = np.random.default_rng(7)
    for W in (3840, 2160, 1920, 1080, 1280, 720, 400, 225, 8191, 65535, 65536, 99991, (1 << 20) - 1):
        col = rng.integers(0, W, 200000)
        u = rng.integers(0, 1 << 24, 200000) * 2.0 ** -24
        _check(W, col + u)
