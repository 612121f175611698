"""trace_vectorized3's in-place swap partition (/root/reference/src/ray_tracing.rs:561-607, CombinedIndex
:113-214) and the closed form the kernel's finish_pixel replays it with (rt_kernel.hip, "vectorized3"):

  after bounce k the slots q < 4 L hold enabled rays iff their sample has e > k (e: the bounce at which
  the sample's ray missed, or depth); D = disabled slots ascending, E = enabled slots descending;
  the literal loop swaps D[j] <-> E[j] for j < J = max over chunk boundaries c of
  min(#D below 4c, #E at or above 4c) and stops with num_active = chunk(max(E[J], D[J-1])) + 1
  (no disabled slot: C; no enabled slot: 0).

Both are run on random termination patterns and must leave the same slot -> sample map and the same
num_active after every bounce.  Plus CPU oracle checks of the mode itself (oracle/, trace_pixel_v3)."""
import numpy as np
import pytest

import rt_mi355x as rt
from rt_mi355x import abi
from oracle_bind import oracle_render


def literal(sig, en, C, na):
    """The reference loop on slot arrays (sig: sample per slot, en: enabled per slot); in place."""
    P = 4 * C

    def inc(i):   # CombinedIndex::increment on a flat slot index; -1 = before_first
        return i + 1 if i + 1 < P else None

    def dec(i):
        return i - 1 if i - 1 >= 0 else None

    front, back = -1, 4 * na
    while True:
        i = inc(front)
        while i is not None and en[i]:
            i = inc(i)
        if i is None:
            return C
        front = i
        i = dec(back)
        while i is not None and not en[i]:
            i = dec(i)
        if i is None:
            return 0
        back = i
        if front // 4 >= back // 4:
            return back // 4 + 1
        sig[front], sig[back] = sig[back], sig[front]
        en[front], en[back] = True, False


def closed_form(sig, en, C):
    """The kernel's replay: J from chunk-boundary counts, swaps by rank, num_active from E[J] / D[J-1]."""
    P = 4 * C
    D = [q for q in range(P) if not en[q]]
    E = [q for q in range(P) if en[q]][::-1]
    if not D:
        return C
    if not E:
        return 0
    J = 0
    for c in range(C + 1):
        d = sum(1 for q in D if q < 4 * c)
        e = sum(1 for q in E if q >= 4 * c)
        J = max(J, min(d, e))
    new = list(sig)
    for j in range(J):
        new[D[j]], new[E[j]] = sig[E[j]], sig[D[j]]
    back = max(E[J] if J < len(E) else -1, D[J - 1] if J >= 1 else -1)
    sig[:] = new
    return back // 4 + 1


@pytest.mark.parametrize("seed", range(6))
def test_closed_form_matches_literal_loop(seed):
    rng = np.random.default_rng(seed)
    for _ in range(150):
        spp = int(rng.integers(1, 90))
        C = (spp + 3) // 4
        depth = int(rng.integers(1, 9))
        p_miss = rng.uniform(0.05, 0.9)
        e = np.minimum(rng.geometric(p_miss, spp) - 1, depth)   # bounce of the miss, depth = survived
        sa, sb = list(range(4 * C)), list(range(4 * C))
        la = lb = C
        K = min(depth, int(e.max()) + 1)
        for k in range(K):
            # enabled after bounce k: traced slots (< 4 L) whose real sample has not missed yet
            en_a = [q < 4 * la and sa[q] < spp and e[sa[q]] > k for q in range(4 * C)]
            en_b = [q < 4 * lb and sb[q] < spp and e[sb[q]] > k for q in range(4 * C)]
            assert en_a == en_b
            la = literal(sa, list(en_a), C, la)
            lb = closed_form(sb, list(en_b), C)
            assert (la, sa) == (lb, sb), (spp, k, la, lb)
            if la == 0:
                break


# ---- the oracle's vectorized3 mode (CPU) ----
V1, V3 = abi.RT_FLAG_MODE_VECTORIZED, abi.RT_FLAG_MODE_VECTORIZED3


@pytest.fixture(scope="module")
def scene_100():
    return rt.scenes.random_spheres(100).flatten()


def cam_for(w, h):
    return rt.camera_new_py(w, h, **rt.MAIN_CAMERA)


def test_v3_equals_v1_with_one_chunk(scene_100):
    """spp = 4: one chunk, nothing can be swapped across chunks, so trace_vectorized3 sums the same
    values as trace_vectorized in the same order: bit-identical."""
    cam = cam_for(24, 14)
    for prec in ("f64", "f32"):
        a = oracle_render(scene_100, cam, 50, 4, 0x5EED0001, V1, precision=prec)
        b = oracle_render(scene_100, cam, 50, 4, 0x5EED0001, V3, precision=prec)
        np.testing.assert_array_equal(a[1], b[1])
        assert a[2] == b[2]


@pytest.mark.parametrize("spp", [8, 64, 100])
def test_v3_same_values_as_v1_other_order(scene_100, spp):
    """Whole chunks: the same per-sample values as trace_vectorized, summed in the swap partition's
    order -- equal to rounding (and the same ray segments)."""
    cam = cam_for(24, 14)
    a = oracle_render(scene_100, cam, 50, spp, 0x5EED0001, V1)
    b = oracle_render(scene_100, cam, 50, spp, 0x5EED0001, V3)
    assert a[2] == b[2]
    np.testing.assert_allclose(b[1], a[1], rtol=1e-12, atol=1e-15)
    assert not np.array_equal(a[1], b[1]) or spp == 8   # the order really differs somewhere


@pytest.mark.parametrize("spp,depth", [(6, 50), (33, 50), (6, 0)])
def test_v3_missing_lanes_add_sky0(scene_100, spp, depth):
    """A partial last chunk: trace_vectorized3 starts every lane white (:515), its missing lanes are
    disabled and marked hit_sky at bounce 0 with a zero direction, so each adds sky(0) = (0.75, 0.85,
    1.0) where trace_vectorized adds black; with no bounce at all they stay white."""
    cam = cam_for(16, 9)
    a = oracle_render(scene_100, cam, depth, spp, 0x5EED0001, V1)[1]
    b = oracle_render(scene_100, cam, depth, spp, 0x5EED0001, V3)[1]
    miss = 4 * ((spp + 3) // 4) - spp
    add = np.array([0.75, 0.85, 1.0]) if depth > 0 else np.ones(3)
    np.testing.assert_allclose(b, a + miss * add / spp, rtol=1e-12, atol=1e-14)
