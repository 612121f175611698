"""The reference's other renderers as semantics modes of the oracle (CPU, test infrastructure).

  RT_FLAG_MODE_VECTORIZED  render_vectorized -> Scene::trace_vectorized (renderer.rs:102-139,
                           ray_tracing.rs:312-373): per chunk, every sample keeps its own value,
                           sky from its own final direction; hit_packed (so Q1 unless ROOT2).
  RT_FLAG_MODE_SCALAR      render -> Scene::trace_rays (renderer.rs:68-100, ray_tracing.rs:264-306):
                           scalar Sphere::hit (objects.rs:216-247), Scene::hit's min_by_key
                           (first minimum wins), Color::average in sample order.

Pins: the scalar mode is checked bit-for-bit against a pure-Python restatement of trace_rays
written from the reference source (below), sharing only the already-pinned primitives (Philox
KATs, the camera, the sincos polynomial); the vectorized mode against the default mode where
the two are provably equal (empty scene; one bounce with an odd chunk count).
"""
import ctypes
import math

import numpy as np
import pytest

import rt_mi355x as rt
from rt_mi355x import abi
from oracle_bind import load_oracle, oracle_render

SEED = 0x5EED0001
V1, SCALAR = abi.RT_FLAG_MODE_VECTORIZED, abi.RT_FLAG_MODE_SCALAR
INF = float("inf")


# ---------------- pure-Python restatement of the scalar path (f64) ----------------
def _philox(ctr, seed):
    out = (ctypes.c_uint32 * 4)()
    load_oracle().oracle_philox4x32_10((ctypes.c_uint32 * 4)(*ctr),
                                       (ctypes.c_uint32 * 2)(seed & 0xFFFFFFFF, seed >> 32), out)
    return list(out)


def _sqrt(x):          # C sqrt: NaN for negative inputs (math.sqrt raises)
    return math.sqrt(x) if (x >= 0.0 or x != x) else float("nan")


def _fmin(a, b):       # C fmin: the non-NaN operand
    if a != a:
        return b
    if b != b:
        return a
    return a if a < b else b


def add(a, b): return (a[0] + b[0], a[1] + b[1], a[2] + b[2])
def sub(a, b): return (a[0] - b[0], a[1] - b[1], a[2] - b[2])
def mul(a, s): return (a[0] * s, a[1] * s, a[2] * s)
def dvs(a, s): return (a[0] / s, a[1] / s, a[2] / s)
def neg(a): return (-a[0], -a[1], -a[2])
def dot(a, b): return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]          # geometry.rs:122-124
def len2(a): return a[0] * a[0] + a[1] * a[1] + a[2] * a[2]            # geometry.rs:106-108


def _unit_vec(u1, u2):
    z = 1.0 - 2.0 * u1
    r = _sqrt(1.0 - z * z)
    s, c = ctypes.c_double(), ctypes.c_double()
    load_oracle().oracle_sincos2pi_f64(u2, ctypes.byref(s), ctypes.byref(c))
    return (r * c.value, r * s.value, z)


def _reflect(v, n): return sub(v, mul(n, 2.0 * dot(v, n)))              # geometry.rs:179-181


def _refract(v, n, ratio):                                               # geometry.rs:183-188
    ct = _fmin(dot(neg(v), n), 1.0)
    rperp = mul(add(v, mul(n, ct)), ratio)
    rpar = mul(n, -_sqrt(abs(1.0 - len2(rperp))))
    return add(rperp, rpar)


def _scatter(m, d, p, n, front, pix, sid, k, seed):                     # materials.rs:54-147
    r = _philox([sid, pix, k, 2], seed)
    u1 = (((r[0] << 32) | r[1]) >> 11) * 2.0 ** -53
    u2 = (((r[2] << 32) | r[3]) >> 11) * 2.0 ** -53
    if m.kind == abi.RT_LAMBERTIAN:
        sd = add(_unit_vec(u1, u2), n)
        if abs(sd[0]) < 1e-8 and abs(sd[1]) < 1e-8 and abs(sd[2]) < 1e-8:
            sd = n
        return sd, tuple(m.albedo)
    if m.kind == abi.RT_METAL:
        return add(_reflect(d, n), mul(_unit_vec(u1, u2), m.fuzz)), tuple(m.albedo)
    ratio = 1.0 / m.ior if front else m.ior
    nn = neg(n) if m.hollow else n
    ct = _fmin(dot(neg(d), nn), 1.0)
    st = _sqrt(1.0 - ct * ct)
    refl = ratio * st > 1.0
    if not refl:
        q = (1.0 - ratio) / (1.0 + ratio)
        r0 = q * q
        m1 = 1.0 - ct
        m2 = m1 * m1
        refl = r0 + (1.0 - r0) * (m1 * (m2 * m2)) > u1
    return (_reflect(d, nn) if refl else _refract(d, nn, ratio)), (1.0, 1.0, 1.0)


def _scene_hit(spheres, o, d):
    """Scene::hit (ray_tracing.rs:231-235) over Sphere::hit (objects.rs:216-247)."""
    best = None
    for i, (c, rad, _) in enumerate(spheres):
        oc = sub(o, c)
        a = len2(d)
        hb = dot(oc, d)
        cc = len2(oc) - rad * rad
        disc = hb * hb - a * cc
        if disc < 0.0:
            continue
        sd = _sqrt(disc)
        root = (-hb - sd) / a
        if not (0.001 <= root < INF):
            root = (-hb + sd) / a
            if not (0.001 <= root < INF):
                continue
        if best is None or root < best[0]:        # min_by_key keeps the first minimum
            best = (root, i)
    return best


def _sky(y):
    a = 0.5 * (y + 1.0)
    return ((1.0 - a) + a * 0.5, (1.0 - a) + a * 0.7, (1.0 - a) + a * 1.0)


def trace_rays_py(flat, cam, depth, spp, seed, col, row):
    """TileRenderTask::render's per-pixel body (renderer.rs:80-86) in Python doubles."""
    lib = load_oracle()
    mats = [m.to_abi() for m in flat.materials]
    spheres = [(tuple(float(x) for x in flat.center[i]), float(flat.radius[i]), mats[int(flat.material[i])])
               for i in range(flat.n_spheres)]
    pix = row * cam.image_width + col
    ob, db = (ctypes.c_double * 3)(), (ctypes.c_double * 3)()
    tot = [0.0, 0.0, 0.0]
    for s in range(spp):
        lib.oracle_get_ray_f64(ctypes.addressof(cam), col, row, s, seed, ob, db)
        o, d = tuple(ob), tuple(db)
        color, alive = (1.0, 1.0, 1.0), True
        for k in range(depth):                                             # ray_tracing.rs:272-302
            h = _scene_hit(spheres, o, d)
            if h is None:
                sk = _sky(d[1])
                color = (color[0] * sk[0], color[1] * sk[1], color[2] * sk[2])
                alive = False
                break
            t, i = h
            c, rad, m = spheres[i]
            p = add(o, mul(d, t))
            outward = dvs(sub(p, c), rad)
            front = dot(d, outward) < 0.0
            n = outward if front else neg(outward)
            nd, att = _scatter(m, d, p, n, front, pix, s, k, seed)
            color = (color[0] * att[0], color[1] * att[1], color[2] * att[2])
            o, d = p, nd
        if alive:
            color = (0.0, 0.0, 0.0)
        tot = [tot[0] + color[0], tot[1] + color[1], tot[2] + color[2]]   # Color::average
    return [t / spp for t in tot]


@pytest.mark.parametrize("scene,depth,spp", [("B", 6, 5), ("A", 8, 4)])
def test_scalar_mode_matches_python_restatement(scene, depth, spp):
    flat = rt.scenes.config_scene(scene).flatten()
    w, h = 4, 3
    cam = rt.camera_new_py(w, h, **rt.MAIN_CAMERA)
    _, lin, segs, rc = oracle_render(flat, cam, depth, spp, SEED, flags=SCALAR)
    assert rc == 0
    for row in range(h):
        for col in range(w):
            assert trace_rays_py(flat, cam, depth, spp, SEED, col, row) == list(lin[row * w + col]), (row, col)


def _empty():
    return rt.FlatScene(np.zeros((0, 3)), np.zeros(0), np.zeros(0, np.uint32), [rt.Lambertian((1, 1, 1))])


def _one(center, radius, mat):
    return rt.FlatScene(np.array([center], float), np.array([radius], float), np.array([0], np.uint32), [mat])


def test_empty_scene_all_modes():
    """No objects: every sample escapes at bounce 0 with its primary ray, so Q2/Q3 cannot act and
    the vectorized mode equals the default bit for bit; the scalar mode is Color::average."""
    cam = rt.camera_new_py(10, 6, **rt.MAIN_CAMERA)
    _, v2, _, _ = oracle_render(_empty(), cam, 8, 12, SEED)
    _, v1, _, _ = oracle_render(_empty(), cam, 8, 12, SEED, flags=V1)
    np.testing.assert_array_equal(v1, v2)
    # A partial last chunk differs: trace_vectorized starts its disabled lanes black (:319-320),
    # trace_vectorized2 marks them hit_sky at bounce 0 so they add sky(y = 0) (:421-424).
    _, v2p, _, _ = oracle_render(_empty(), cam, 8, 10, SEED)
    _, v1p, _, _ = oracle_render(_empty(), cam, 8, 10, SEED, flags=V1)
    np.testing.assert_allclose(v2p - v1p, np.broadcast_to(2 * np.array(_sky(0.0)) / 10, v1p.shape), rtol=0, atol=1e-15)
    _, sc, _, _ = oracle_render(_empty(), cam, 8, 10, SEED, flags=SCALAR)
    lib = load_oracle()
    o, d = (ctypes.c_double * 3)(), (ctypes.c_double * 3)()
    for pix in (0, 17, 59):
        col, row = pix % 10, pix // 10
        tot = [0.0, 0.0, 0.0]
        for s in range(10):
            lib.oracle_get_ray_f64(ctypes.addressof(cam), col, row, s, SEED, o, d)
            sk = _sky(d[1])
            tot = [tot[i] + 1.0 * sk[i] for i in range(3)]
        assert [t / 10 for t in tot] == list(sc[pix])


@pytest.mark.parametrize("spp", [4, 12, 20])
def test_vectorized_equals_default_for_one_bounce_odd_chunks(spp):
    """depth 1, full chunks and C = spp/4 odd: S = (C-1)%2 = 0, the final read is bounce 0's
    unsorted buffer, every slot keeps its own ray and the primary ray IS the escaping ray."""
    flat = rt.scenes.config_scene("B").flatten()
    cam = rt.camera_new_py(16, 9, **rt.MAIN_CAMERA)
    for flags in (0, abi.RT_FLAG_ROOT2):
        _, v2, s2, _ = oracle_render(flat, cam, 1, spp, SEED, flags=flags)
        _, v1, s1, _ = oracle_render(flat, cam, 1, spp, SEED, flags=flags | V1)
        np.testing.assert_array_equal(v1, v2)
        assert s1 == s2


def test_modes_differ_where_the_quirks_act():
    flat = rt.scenes.config_scene("B").flatten()
    cam = rt.camera_new_py(16, 9, **rt.MAIN_CAMERA)
    _, v2, s2, _ = oracle_render(flat, cam, 8, 8, SEED)
    _, v1, s1, _ = oracle_render(flat, cam, 8, 8, SEED, flags=V1)
    assert s1 == s2                       # same rays traced: only the read-out differs
    assert not np.array_equal(v1, v2)


def test_scalar_tie_first_sphere_wins():
    """Scene::hit's min_by_key returns the FIRST of equal minima; the packed paths' t <= best
    (objects.rs:141) keeps the LAST."""
    red, blue = rt.Lambertian((0.9, 0.1, 0.1)), rt.Lambertian((0.1, 0.1, 0.9))
    both = rt.FlatScene(np.array([[0, 0, 0], [0, 0, 0]], float), np.array([4.0, 4.0]), np.array([0, 1], np.uint32),
                        [red, blue])
    cam = rt.camera_new_py(16, 9, **rt.MAIN_CAMERA)
    _, sc, _, _ = oracle_render(both, cam, 8, 8, SEED, flags=SCALAR)
    _, sc_red, _, _ = oracle_render(_one((0, 0, 0), 4.0, red), cam, 8, 8, SEED, flags=SCALAR)
    _, v1, _, _ = oracle_render(both, cam, 8, 8, SEED, flags=V1)
    _, v1_blue, _, _ = oracle_render(_one((0, 0, 0), 4.0, blue), cam, 8, 8, SEED, flags=V1)
    np.testing.assert_array_equal(sc, sc_red)
    np.testing.assert_array_equal(v1, v1_blue)


def test_scalar_sees_far_side_from_inside():
    """Scalar Sphere::hit tries root2 (objects.rs:228-234): from inside a sphere the far side is hit."""
    inside = _one((0, 0, 0), 1000.0, rt.Lambertian((0.5, 0.5, 0.5)))
    cam = rt.camera_new_py(16, 9, **rt.MAIN_CAMERA)
    _, e, _, _ = oracle_render(_empty(), cam, 8, 8, SEED, flags=SCALAR)
    _, s, _, _ = oracle_render(inside, cam, 8, 8, SEED, flags=SCALAR)
    _, q1, _, _ = oracle_render(inside, cam, 8, 8, SEED, flags=V1)      # hit_packed: Q1 applies
    assert s.mean() < 0.8 * e.mean()
    _, v1e, _, _ = oracle_render(_empty(), cam, 8, 8, SEED, flags=V1)
    np.testing.assert_array_equal(q1, v1e)


def test_vectorized_root2_tracks_scalar_statistically():
    """Vectorized + ROOT2 and scalar are both unbiased estimates of the same image (they differ
    only in rounding: FMA, 1/a, unit normals); their means agree to within Monte-Carlo noise."""
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(32, 18, **rt.MAIN_CAMERA)
    _, v1, _, _ = oracle_render(flat, cam, 50, 64, SEED, flags=V1 | abi.RT_FLAG_ROOT2)
    _, sc, _, _ = oracle_render(flat, cam, 50, 64, SEED, flags=SCALAR)
    _, v2, _, _ = oracle_render(flat, cam, 50, 64, SEED)
    for ch in range(3):
        assert abs(v1[:, ch].mean() - sc[:, ch].mean()) < 0.01 * sc[:, ch].mean()
    # the live path's Q2/Q3 read-out estimates a different image: here it is
    # brighter (Q2 shades with the primary ray's y), by far more than the noise between v1 and scalar
    assert abs(v2.mean() - v1.mean()) > 0.03 * v1.mean() > abs(v1.mean() - sc.mean())


def test_mode_bits_are_exclusive():
    cam = rt.camera_new_py(4, 3, **rt.MAIN_CAMERA)
    assert oracle_render(_empty(), cam, 8, 4, SEED, flags=V1 | SCALAR)[3] == 1
