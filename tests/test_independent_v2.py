"""The oracle's second pin: the independent pure-Python restatement of the live packed
path (tests/independent_v2.py, written from the reference source without the C oracle) against the
C oracle's f64 build, bit for bit, and both against the committed golden vectors the restatement
produced (tests/golden/independent_v2.npz, tests/golden/make_independent_golden.py).

Parity with the real reference binary stays unpinned: it cannot be built here, it ships no tests or
fixtures, and its RNG (thread_rng) cannot be seeded.  This pins the oracle's
READING of trace_vectorized2 against a second, independently written reading."""
import ctypes
import json
import math
import os
import random
from fractions import Fraction

import numpy as np
import pytest

import independent_v2 as iv
import rt_mi355x as rt
from oracle_bind import load_oracle, oracle_render

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "independent_v2.npz")
SEED = 0x5EED0001


def _golden():
    z = np.load(GOLDEN, allow_pickle=False)
    return z, json.loads(str(z["meta"]))


def _flat(tag):
    import importlib.util
    spec = importlib.util.spec_from_file_location("mig", os.path.join(HERE, "golden", "make_independent_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.SCENES[tag]().flatten()


def test_philox_published_kats():
    """Random123 kat_vectors, philox4x32 R=10 (restated from the spec, not from the oracle)."""
    assert iv.philox4x32_10((0, 0, 0, 0), (0, 0)) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert iv.philox4x32_10((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2) == (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)
    assert iv.philox4x32_10((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)) == \
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)


def test_philox2x32_published_kats():
    """Random123 kat_vectors, philox2x32 R=10 (the fp32 draws; restated from the spec, not from the oracle)."""
    assert iv.philox2x32_10((0, 0), 0) == (0xFF1DAE59, 0x6CD10DF2)
    assert iv.philox2x32_10((0xFFFFFFFF, 0xFFFFFFFF), 0xFFFFFFFF) == (0x2C3F628B, 0xAB4FD7AD)
    assert iv.philox2x32_10((0x243F6A88, 0x85A308D3), 0x13198A2E) == (0xDD7CE038, 0xF62A4C12)


def test_exact_fma():
    """iv.fma is the correctly rounded a*b+c (checked against Fraction arithmetic)."""
    rng = random.Random(7)
    for _ in range(20000):
        a, b = rng.uniform(-4, 4) * 2.0 ** rng.randint(-30, 30), rng.uniform(-4, 4) * 2.0 ** rng.randint(-30, 30)
        c = -a * b * (1 + rng.uniform(-1e-9, 1e-9)) if rng.random() < 0.5 else rng.uniform(-4, 4) * 2.0 ** rng.randint(-40, 40)
        assert iv.fma(a, b, c) == float(Fraction(a) * Fraction(b) + Fraction(c))
    assert math.copysign(1.0, iv.fma(-0.0, 1.0, -0.0)) < 0 and math.copysign(1.0, iv.fma(2.0, 3.0, -6.0)) > 0


def test_sincos_and_camera_match_the_oracle():
    lib = load_oracle()
    s, c = ctypes.c_double(), ctypes.c_double()
    rng = random.Random(3)
    for u in [0.0, 0.125, 0.25, 0.5, 0.75, 1 - 2 ** -53] + [rng.random() for _ in range(2000)]:
        lib.oracle_sincos2pi_f64(u, ctypes.byref(s), ctypes.byref(c))
        assert iv.sincos2pi(u) == (s.value, c.value), u
    for (W, H, dfa) in [(400, 225, 0.0), (16, 9, 0.0), (8, 5, 2.0), (1920, 1080, 0.0)]:
        p = dict(rt.MAIN_CAMERA)
        p["defocus_angle"] = dfa
        a = rt.camera_new_py(W, H, **p)
        b = iv.camera_new(W, H, p["focal_length"], p["view_angle"], p["center"], p["look_at"], p["up"], dfa)
        for k in ("center", "ulc", "vu", "vv", "du", "dv"):
            assert tuple(getattr(a, k)) == tuple(b[k]), (k, W, H)
        o, d = (ctypes.c_double * 3)(), (ctypes.c_double * 3)()
        for (col, row, smp) in [(0, 0, 0), (W - 1, H - 1, 7), (W // 2, H // 3, 99)]:
            lib.oracle_get_ray_f64(ctypes.byref(a), col, row, smp, SEED, o, d)
            ro, rd = iv.get_ray(b, col, row, smp, row * W + col, SEED)
            assert ro == tuple(o) and rd == tuple(d), (W, H, col, row, smp)


@pytest.mark.parametrize("tag,W,H,spp,depth", [("A", 8, 5, 6, 8), ("A", 6, 4, 33, 50), ("S100", 4, 3, 12, 50),
                                               ("Q", 6, 4, 9, 50)])
def test_restatement_matches_oracle(tag, W, H, spp, depth):
    """Fresh (uncommitted) cases: the Python restatement and the C oracle agree bit for bit."""
    flat = _flat(tag)
    p = dict(rt.MAIN_CAMERA)
    cam_abi = rt.camera_new_py(W, H, **p)
    cam = iv.camera_new(W, H, p["focal_length"], p["view_angle"], p["center"], p["look_at"], p["up"], p["defocus_angle"])
    lin, rgb, segs = iv.render(flat, cam, spp, depth, SEED)
    rgb_o, lin_o, segs_o, rc = oracle_render(flat, cam_abi, depth, spp, SEED)
    assert rc == 0 and segs == segs_o
    assert np.array_equal(np.array(lin), lin_o)
    assert np.array_equal(np.array(rgb, dtype=np.uint8), rgb_o)


def test_oracle_matches_independent_goldens():
    """Every committed case of the independent restatement, against the C oracle's f64 build."""
    z, meta = _golden()
    assert len(meta) >= 15
    for name, m in meta.items():
        flat = _flat(m["scene"])
        cam = rt.camera_new_py(m["W"], m["H"], **m["camera"])
        rgb_o, lin_o, segs_o, rc = oracle_render(flat, cam, m["depth"], m["spp"], m["seed"])
        assert rc == 0, name
        assert segs_o == m["segments"], name
        assert np.array_equal(lin_o, z[f"{name}_lin"]), name
        assert np.array_equal(rgb_o, z[f"{name}_rgb"]), name


def test_goldens_regenerate():
    """The restatement still produces the committed vectors (a cheap subset of the cases)."""
    z, meta = _golden()
    for name in ("a_spp6_d8", "q_defocus_spp10_d20"):
        m = meta[name]
        cam = iv.camera_new(m["W"], m["H"], m["camera"]["focal_length"], m["camera"]["view_angle"],
                            m["camera"]["center"], m["camera"]["look_at"], m["camera"]["up"],
                            m["camera"]["defocus_angle"])
        lin, rgb, segs = iv.render(_flat(m["scene"]), cam, m["spp"], m["depth"], m["seed"])
        assert segs == m["segments"]
        assert np.array_equal(np.array(lin), z[f"{name}_lin"]), name


# ---- round 4: the BASELINE configs at their real sizes, f64 and fp32 ---------------------------------
GOLDEN_BASELINE = os.path.join(HERE, "golden", "independent_baseline.npz")


def _baseline():
    z = np.load(GOLDEN_BASELINE, allow_pickle=False)
    return z, json.loads(str(z["meta"]))


def test_exact_fma32():
    """iv.fma32 is the correctly rounded fp32 a*b+c (against Fraction arithmetic rounded to 24 bits by
    numpy's own conversion of the exact value's nearest doubles, checked two-sided)."""
    rng = random.Random(11)
    F = np.float32
    for _ in range(20000):
        a = F(rng.uniform(-4, 4) * 2.0 ** rng.randint(-20, 20))
        b = F(rng.uniform(-4, 4) * 2.0 ** rng.randint(-20, 20))
        c = F(-float(a) * float(b) * (1 + rng.uniform(-1e-5, 1e-5))) if rng.random() < 0.5 else \
            F(rng.uniform(-4, 4) * 2.0 ** rng.randint(-30, 30))
        r = iv.fma32(a, b, c)
        exact = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
        if exact == 0:
            assert r == 0
            continue
        # r is the fp32 nearest to exact: both neighbours are at least as far
        lo, hi = np.nextafter(r, F(-np.inf)), np.nextafter(r, F(np.inf))
        d = abs(Fraction(float(r)) - exact)
        assert d <= abs(Fraction(float(lo)) - exact) and d <= abs(Fraction(float(hi)) - exact), (a, b, c)
        if d == abs(Fraction(float(lo)) - exact) or d == abs(Fraction(float(hi)) - exact):   # a tie: even
            assert (int(np.float32(r).view(np.uint32)) & 1) == 0


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_estimate_is_invisible(prec):
    """hit_scene's numpy estimate (skipping spheres with a hopelessly negative discriminant) changes no
    bit: the literal restatement (every sphere through the mul_add sequence) gives the same pixels."""
    flat = rt.scenes.config_scene("C").flatten()
    p = dict(rt.MAIN_CAMERA)
    cam = iv.camera_new(24, 14, p["focal_length"], p["view_angle"], p["center"], p["look_at"], p["up"], 0.0)
    px = [0, 5, 77, 150, 200, 321, 335]
    a = iv.render(flat, cam, 8, 50, SEED, pixels=px, prec=prec)
    b = iv.render(flat, cam, 8, 50, SEED, pixels=px, prec=prec, literal=True)
    assert a[2] == b[2] and np.array_equal(np.array(a[0], dtype=np.float64), np.array(b[0], dtype=np.float64))
    assert a[1] == b[1]


@pytest.mark.parametrize("tag,W,H,spp,depth", [("A", 8, 5, 6, 8), ("S100", 4, 3, 12, 50), ("Q", 6, 4, 9, 50)])
def test_fp32_restatement_matches_oracle(tag, W, H, spp, depth):
    """The fp32 reading (every value a numpy float32, exact fp32 mul_add) against the C oracle's f32
    build, bit for bit: the headline path's second pin."""
    flat = _flat(tag)
    p = dict(rt.MAIN_CAMERA)
    cam_abi = rt.camera_new_py(W, H, **p)
    cam = iv.camera_new(W, H, p["focal_length"], p["view_angle"], p["center"], p["look_at"], p["up"], p["defocus_angle"])
    lin, rgb, segs = iv.render(flat, cam, spp, depth, SEED, prec="f32")
    rgb_o, lin_o, segs_o, rc = oracle_render(flat, cam_abi, depth, spp, SEED, precision="f32")
    assert rc == 0 and segs == segs_o
    assert np.array_equal(np.array(lin, dtype=np.float64), lin_o)
    assert np.array_equal(np.array(rgb, dtype=np.uint8), rgb_o)


def test_oracle_matches_baseline_goldens():
    """The C oracle (f64 and f32 builds) against the independent restatement's vectors at every BASELINE
    config's real image size, sphere count, spp and depth (tests/golden/independent_baseline.npz)."""
    z, meta = _baseline()
    assert {m["config"] for m in meta.values()} >= {"B", "C", "D", "E"}
    assert {m["precision"] for m in meta.values()} == {"f64", "f32"}
    for name, m in meta.items():
        flat = rt.scenes.config_scene(m["config"]).flatten()
        cam = rt.camera_new_py(m["W"], m["H"], **m["camera"])
        px = z[f"{name}_pix"]
        rgb_o, lin_o, segs_o, rc = oracle_render(flat, cam, m["depth"], m["spp"], m["seed"],
                                                 pixels=px.astype(np.uint32), precision=m["precision"])
        assert rc == 0, name
        assert segs_o == int(z[f"{name}_segs"].sum()), name
        assert np.array_equal(lin_o, z[f"{name}_lin"]), name
        assert np.array_equal(rgb_o, z[f"{name}_rgb"]), name
        assert 1.0 < segs_o / (len(px) * m["spp"]) < 4.0, name   # not all sky


def test_baseline_goldens_regenerate():
    """The restatement still produces the committed baseline vectors (two pixels per precision)."""
    z, meta = _baseline()
    for name in ("C_f32", "B_f64"):
        m = meta[name]
        c = m["camera"]
        cam = iv.camera_new(m["W"], m["H"], c["focal_length"], c["view_angle"], c["center"], c["look_at"], c["up"],
                            c["defocus_angle"])
        flat = rt.scenes.config_scene(m["config"]).flatten()
        for k in (1, 2):
            q = int(z[f"{name}_pix"][k])
            lin, rgb, segs = iv.render(flat, cam, m["spp"], m["depth"], m["seed"], pixels=[q], prec=m["precision"])
            assert segs == int(z[f"{name}_segs"][k]), name
            assert np.array_equal(np.array(lin, dtype=np.float64), z[f"{name}_lin"][k:k + 1]), name
            assert np.array_equal(np.array(rgb, dtype=np.uint8), z[f"{name}_rgb"][k:k + 1]), name
