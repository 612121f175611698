"""CPU checks of two bit-level encodings in the fp32 kernel (round 6), against the plain rules they replace:

* hit_update's 64-bit best-hit key (csrc/rt_sweep.hpp, HitBest<float>): key(t, i) = (bits(t) - bits(0.001f)) << 32 | ~i,
  the high half wrapping mod 2^32.  "key(r, i) < state" must equal PackedHitRecords::update's rule (objects.rs:140-155,
  valid root :272): 0.001 <= r < inf and (r < best_t or (r == best_t and i > best)), for every root the kernel can form
  (negative, -0, subnormal, below 0.001, the boundary itself, large, +inf, NaN) and every reachable state (no hit yet:
  +inf and -1; a valid best).
* sincos2pi's branch-free quadrant selection (csrc/rt_device.hpp): two selects and two sign-bit xors must give the
  bits of the switch it replaced for every quadrant, octant swap and sign of zero.
"""
import numpy as np

KT001 = np.float32(0.001).view(np.uint32)


def key(r, i):
    hi = (np.asarray(r, np.float32).view(np.uint32).astype(np.uint64) - np.uint64(KT001)) & np.uint64(0xFFFFFFFF)
    return (hi << np.uint64(32)) | (~np.asarray(i, np.uint32)).astype(np.uint64)


def state(t, i):
    """HitBest<float>'s k for best (t, i); (inf, -1) is the initial state."""
    return key(np.float32(t), np.uint32(i & 0xFFFFFFFF))


def test_kt001_is_the_float_threshold():
    assert KT001 == 0x3A83126F
    assert np.float32(0.001) == np.float32(np.uint32(0x3A83126F).view(np.float32))


def test_hit_key_compare_equals_reference_rule():
    rng = np.random.default_rng(0x5EED)
    t001 = np.float32(0.001)
    special = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-38, 5e-4, np.nextafter(t001, np.float32(0)), t001,
                        np.nextafter(t001, np.float32(1)), 0.5, 1.0, 1e30, 3.4e38, np.inf, -np.inf, np.nan, -1.0, -np.nan],
                       dtype=np.float32)
    roots = np.concatenate([special, rng.uniform(-2, 50, 4000).astype(np.float32),
                            rng.integers(0, 2 ** 32, 4000, dtype=np.uint64).astype(np.uint32).view(np.float32)])
    bests = [(np.float32(np.inf), -1)]
    for t in np.concatenate([special[(special >= t001) & np.isfinite(special)], rng.uniform(0.001, 50, 60).astype(np.float32)]):
        for b in (0, 7, 499, 2 ** 31 - 2):
            bests.append((np.float32(t), b))
    idx = np.array([0, 1, 6, 7, 8, 498, 499, 500, 2 ** 31 - 1], dtype=np.int64)
    for bt, bi in bests:
        st = state(bt, bi)
        for i in idx:
            # ties need r == bt: test the best's own t with every index as well
            rr = np.concatenate([roots, np.array([bt, np.nextafter(bt, np.float32(0)), np.nextafter(bt, np.float32(np.inf))],
                                                 dtype=np.float32)])
            with np.errstate(invalid="ignore"):
                valid = (rr >= t001) & (rr < np.float32(np.inf))
                ref = valid & ((rr < bt) | ((rr == bt) & (i > bi)))
            got = key(rr, np.full(rr.shape, i, np.uint32)) < st
            assert np.array_equal(got, ref), (bt, bi, i, rr[got != ref][:5])


def test_hit_key_decodes():
    for t, i in ((np.float32(np.inf), -1), (np.float32(0.001), 0), (np.float32(3.25), 499), (np.float32(1e30), 2 ** 31 - 1)):
        k = int(state(t, i))
        assert np.uint32(((k >> 32) + int(KT001)) & 0xFFFFFFFF).view(np.float32) == t          # bt()
        assert np.int32(np.uint32(~k & 0xFFFFFFFF).view(np.int32)) == i                          # bi()


def _switch(s, c, q, sw):
    if sw:
        s, c = c, s
    q &= 3
    if q == 0:
        return s, c
    if q == 1:
        return c, -s
    if q == 2:
        return -s, -c
    return -c, s


def _bits(s, c, q, sw):
    qs = (q << 30) & 0xFFFFFFFF
    swp = sw != ((qs & 0x40000000) != 0)
    sm, cm = (c, s) if swp else (s, c)
    so = np.uint32(np.float32(sm).view(np.uint32) ^ np.uint32(qs & 0x80000000)).view(np.float32)
    co = np.uint32(np.float32(cm).view(np.uint32) ^ np.uint32((qs + 0x40000000) & 0x80000000)).view(np.float32)
    return so, co


def test_sincos_quadrant_bits_equal_switch():
    rng = np.random.default_rng(7)
    vals = np.concatenate([np.array([0.0, -0.0, 1.0, 0.70710677, 1e-30], np.float32), rng.uniform(-1, 1, 200).astype(np.float32)])
    for q in range(4):
        for sw in (False, True):
            for s in vals[:40]:
                for c in vals[::7]:
                    a = _switch(np.float32(s), np.float32(c), q, sw)
                    b = _bits(np.float32(s), np.float32(c), q, sw)
                    assert np.float32(a[0]).view(np.uint32) == b[0].view(np.uint32)
                    assert np.float32(a[1]).view(np.uint32) == b[1].view(np.uint32)
