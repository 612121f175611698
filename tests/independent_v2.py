"""Independent pure-Python restatement of the reference's LIVE packed path — TEST INFRASTRUCTURE.

Second pin of the oracle (VERDICT r02 "next round" item 1): written directly from the
reference source (/root/reference/src/*.rs, read as text), without reading oracle/oracle_impl.h, so a
misreading of trace_vectorized2 that the C oracle and the HIP kernel shared would show up here as a
mismatch.  Only tests/ import it; it never runs on the product path.

What it restates, literally and in the reference's operation order (f64, the reference's arithmetic;
and, round 4, the same algorithm in fp32 -- every value a numpy.float32 scalar, IEEE single rounding
per operation, an exact single-rounding fp32 mul_add -- the headline path's precision):
  * Camera::new / Camera::get_ray                          ray_tracing.rs:27-62, 77-89
  * renderer: spp camera rays chunked by 4 -> PackedRays<4>, partial chunk lanes disabled,
    / spp, Color::to_u8_array                               renderer.rs:155-163, ray.rs:136-153, color.rs:54-64
  * Scene::trace_vectorized2: two ray/colour/hit_sky buffers, bounce loop over the active chunks,
    per-lane scatter, the stable two-pass shuffle into the other buffer, the final read of buffer
    (C-1)%2 with the sky from the ORIGINAL primary rays      ray_tracing.rs:375-505
  * Sphere::hit_packed (root1 tested twice: root2 never valid; masked_select -> root1 when valid)
    + PackedHitRecords::update (t <= best: the later sphere wins ties) / finalize / at
                                                            objects.rs:121-176, 249-290
  * Lambertian / Metal / Dielectric::get_hit_result         materials.rs:54-63, 92-97, 121-147
  * Vec3 ops without FMA (left-to-right sums), PackedVec3::length_squared / dot with mul_add,
    reflect / refract / near_zero                           geometry.rs:37-188, 434-468

mul_add is computed exactly (Python 3.10 has no math.fma): the exact product plus addend as an
integer at a common binary exponent, rounded once (f64: Python's correctly rounded int -> float
conversion; fp32: an explicit round-to-nearest-even to 24 bits).  powi(2) is x*x, powi(5) LLVM's
binary expansion x*((x*x)*(x*x)).

Speed (round 4): hit_scene first evaluates every sphere's discriminant for the ray at once in numpy
f64, without FMA, and runs the literal test only on the spheres whose estimate is not hopelessly
negative: disc_est < -tol (hb^2 + a (|oc|^2 + r^2)) with tol = 1e-9 (f64) / 1e-4 (fp32), far above
the few-ulp rounding difference between the estimate and the literal mul_add sequence (~10 u of those
magnitudes, u = 2^-53 / 2^-24).  A skipped sphere has a literal disc < 0: no root, no update.  The
visiting order stays the scene order.  literal=True switches the estimate off (test_independent_v2.py
checks both agree).

The RNG is the declared substitution (rt_device.hpp): the reference's thread_rng()
cannot be seeded, so every build keys Philox4x32-10 (fp32: Philox2x32-10, see uniforms) by (sample,
pixel, bounce, stream): stream 0 (s, pix, 0, 0) camera jitter, stream 1 (s, pix, i, 1) disk try i,
stream 2 (s, pix, k, 2) the scatter at bounce k (random_unit_vector from (u1, u2) as z = 1-2 u1, phi = 2 pi u2 with the
fixed fma-Horner sin/cos; the Dielectric draw is u1).  Philox itself is restated from Random123's
spec and checked against its published KAT vectors (tests/test_independent_v2.py).
"""
import math

import numpy as np

F32 = np.float32
# The fp32 reading relies on NumPy 2's scalar promotion (NEP 50): float32 combined with a Python float
# stays float32.  Under NumPy 1.x expressions such as 2.0*ux-1.0 or t*4.0 would silently turn float64,
# and the committed fp32 goldens would disagree in ways that look like kernel bugs.
if type(F32(1) * 1.0) is not F32:
    raise ImportError(f"tests/independent_v2.py needs NumPy >= 2 scalar promotion (NEP 50); numpy {np.__version__} "
                      "promotes float32 * float to float64")

# ---------------------------------------------------------------- exact fused multiply-add (f64)
_TWO53 = float(1 << 53)


def _split(x):
    """x (finite) == m * 2**e with m an int."""
    m, e = math.frexp(x)
    return int(m * _TWO53), e - 53


def fma(a, b, c):
    """Correctly rounded a*b + c (IEEE fusedMultiplyAdd, round to nearest even); fp32 operands: fma32."""
    if isinstance(a, F32):
        return fma32(a, b, c)
    if not (math.isfinite(a) and math.isfinite(b) and math.isfinite(c)):
        return a * b + c   # inf / nan propagate the same way
    ma, ea = _split(a)
    mb, eb = _split(b)
    mc, ec = _split(c)
    mp, ep = ma * mb, ea + eb
    e = min(ep, ec)
    s = (mp << (ep - e)) + (mc << (ec - e))
    if s == 0:
        # exact zero: -0 only if both the product and c are -0 (or the product is -0 and c == -0)
        pneg = (math.copysign(1.0, a) * math.copysign(1.0, b)) < 0
        return -0.0 if (pneg and math.copysign(1.0, c) < 0) else 0.0
    r = (s / (1 << -e)) if e < 0 else float(s << e)   # int / int and int -> float round correctly
    assert r == 0.0 or abs(r) >= 2.2250738585072014e-308, "subnormal fma result: not modelled"
    return r


def _round_f32(s, e):
    """The float32 nearest to the nonzero exact value s * 2**e (s an int; ties to even; normal range)."""
    neg = s < 0
    s = -s if neg else s
    sh = s.bit_length() - 24
    if sh > 0:
        q, r = s >> sh, s & ((1 << sh) - 1)
        half = 1 << (sh - 1)
        if r > half or (r == half and (q & 1)):
            q += 1
        s, e = q, e + sh
    v = math.ldexp(float(s), e)   # s < 2**25: exact
    assert v == 0.0 or 1.1754943508222875e-38 <= v < 3.4028234663852886e+38, "fp32 fma outside the normal range"
    return F32(-v if neg else v)


def fma32(a, b, c):
    """Correctly rounded fp32 a*b + c: the exact value from the f64 splits, rounded once to 24 bits."""
    a, b, c = float(a), float(b), float(c)
    if not (math.isfinite(a) and math.isfinite(b) and math.isfinite(c)):
        return F32(F32(a) * F32(b) + F32(c))
    ma, ea = _split(a)
    mb, eb = _split(b)
    mc, ec = _split(c)
    mp, ep = ma * mb, ea + eb
    e = min(ep, ec)
    s = (mp << (ep - e)) + (mc << (ec - e))
    if s == 0:
        pneg = (math.copysign(1.0, a) * math.copysign(1.0, b)) < 0
        return F32(-0.0) if (pneg and math.copysign(1.0, c) < 0) else F32(0.0)
    return _round_f32(s, e)


def sqrt(x):
    """f64::sqrt (fp32: sqrtf): NaN for a negative argument (Python's math.sqrt raises)."""
    if isinstance(x, F32):
        return np.sqrt(x) if x >= 0.0 else F32(math.nan)
    return math.sqrt(x) if x >= 0.0 else math.nan


def fmin(x, y):
    """f64::min: the other operand when one is NaN."""
    if x != x:
        return y
    if y != y:
        return x
    return x if x < y else y


# ---------------------------------------------------------------- Vec3 (geometry.rs:9-188)
def v_add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def v_sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def v_mul(a, s):   # Vec3 * f64 (and f64 * Vec3 = rhs * self, :70-74)
    return (a[0] * s, a[1] * s, a[2] * s)


def v_div(a, s):
    return (a[0] / s, a[1] / s, a[2] / s)


def v_neg(a):
    return (-a[0], -a[1], -a[2])


def v_dot(a, b):   # :122-124, no FMA
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def v_len2(a):     # :106-108, powi(2) = x*x
    return a[0] * a[0] + a[1] * a[1] + a[2] * a[2]


def v_unit(a):     # :118-120
    return v_div(a, sqrt(v_len2(a)))


def v_cross(a, b):  # :126-132
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def near_zero(v):  # :134-137
    e = 1e-8
    return abs(v[0]) < e and abs(v[1]) < e and abs(v[2]) < e


def reflect(v, n):  # :179-181: v - (2.0 * v.dot(n)) * n
    return v_sub(v, v_mul(n, 2.0 * v_dot(v, n)))


def refract(v, n, ratio):  # :183-188
    cos_theta = fmin(v_dot(v_neg(v), n), 1.0)
    r_perp = v_mul(v_add(v, v_mul(n, cos_theta)), ratio)
    r_par = v_mul(n, -(sqrt(abs(1.0 - v_len2(r_perp)))))
    return v_add(r_perp, r_par)


# PackedVec3 (per lane): length_squared / dot with mul_add (:434-436, :466-468)
def pk_len2(a):
    return fma(a[2], a[2], fma(a[1], a[1], a[0] * a[0]))


def pk_dot(a, b):
    return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0]))


# ---------------------------------------------------------------- RNG substitution
_M = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Random123 Philox4x32 with 10 rounds: round(ctr, key), then bump the key (Weyl constants)."""
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & _M, p1 & _M, ((p0 >> 32) ^ c3 ^ k1) & _M, p0 & _M
        k0 = (k0 + 0x9E3779B9) & _M
        k1 = (k1 + 0xBB67AE85) & _M
    return (c0, c1, c2, c3)


def philox2x32_10(ctr, key):
    """Random123 Philox2x32 with 10 rounds: hi:lo = 0xD256D193 * c0, (c0, c1) <- (hi ^ key ^ c1, lo), then
    bump the key by the Weyl constant 0x9E3779B9."""
    c0, c1 = ctr
    for _ in range(10):
        p = 0xD256D193 * c0
        c0, c1 = ((p >> 32) ^ key ^ c1) & _M, p & _M
        key = (key + 0x9E3779B9) & _M
    return (c0, c1)


def fmix32(h):
    """murmur3's 32-bit finaliser; the fp32 key is seed lo ^ fmix32(seed hi) (fmix32(0) = 0)."""
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M
    return h ^ (h >> 16)


def uniforms(sid, pix, k, stream, seed, prec="f64"):
    """Two uniforms in [0, 1): f64 from 53 bits of (r0, r1) and of (r2, r3) of Philox4x32-10 at counter
    (sid, pix, k, stream), key (seed lo, seed hi); fp32 from 24 bits of each word of Philox2x32-10 at
    counter (pix, sid | code << 20), code 0 camera / 1 + k disk try / 257 + k scatter, key
    seed lo ^ fmix32(seed hi)."""
    if prec == "f32":
        code = 0 if stream == 0 else (1 + k if stream == 1 else 257 + k)
        assert sid < (1 << 20) and code < (1 << 12)
        r = philox2x32_10((pix, sid | (code << 20)), (seed & _M) ^ fmix32((seed >> 32) & _M))
        return F32((r[0] >> 8) * 2.0 ** -24), F32((r[1] >> 8) * 2.0 ** -24)
    r = philox4x32_10((sid, pix, k, stream), (seed & _M, (seed >> 32) & _M))
    ua = (((r[0] << 32) | r[1]) >> 11) * 2.0 ** -53
    ub = (((r[2] << 32) | r[3]) >> 11) * 2.0 ** -53
    return ua, ub


def sincos2pi(u):
    """sin and cos of 2 pi u: exact quadrant split in u, Taylor by fma-Horner on [0, pi/4] (fp32: the
    shorter polynomials, coefficients rounded to fp32)."""
    f32 = isinstance(u, F32)
    t = u * 4.0
    q = int(t)
    f = t - (F32(q) if f32 else q)
    sw = f > 0.5
    g = 1.0 - f if sw else f
    x = g * 1.5707963267948966
    x2 = x * x
    if f32:
        ps = F32(1.0 / 362880.0)
        for cst in (-1.0 / 5040.0, 1.0 / 120.0, -1.0 / 6.0):
            ps = fma(ps, x2, F32(cst))
        pc = F32(-1.0 / 3628800.0)
        for cst in (1.0 / 40320.0, -1.0 / 720.0, 1.0 / 24.0, -1.0 / 2.0):
            pc = fma(pc, x2, F32(cst))
    else:
        ps = 1.0 / 355687428096000.0
        for cst in (-1.0 / 1307674368000.0, 1.0 / 6227020800.0, -1.0 / 39916800.0, 1.0 / 362880.0, -1.0 / 5040.0,
                    1.0 / 120.0, -1.0 / 6.0):
            ps = fma(ps, x2, cst)
        pc = -1.0 / 6402373705728000.0
        for cst in (1.0 / 20922789888000.0, -1.0 / 87178291200.0, 1.0 / 479001600.0, -1.0 / 3628800.0, 1.0 / 40320.0,
                    -1.0 / 720.0, 1.0 / 24.0, -1.0 / 2.0):
            pc = fma(pc, x2, cst)
    s = fma(x * x2, ps, x)
    c = fma(x2, pc, F32(1.0) if f32 else 1.0)
    if sw:
        s, c = c, s
    qq = q & 3
    if qq == 0:
        return s, c
    if qq == 1:
        return c, -s
    if qq == 2:
        return -s, -c
    return -c, s


def random_unit_vector(u1, u2):
    """The distribution of Vec3::random_unit_vector (geometry.rs:139-152): uniform on S^2."""
    z = 1.0 - 2.0 * u1
    r = sqrt(1.0 - z * z)
    s, c = sincos2pi(u2)
    return (r * c, r * s, z)


# ---------------------------------------------------------------- Camera (ray_tracing.rs:27-89)
def camera_new(w, h, focal_length, view_angle, center, look_at, up, defocus_angle):
    rad = math.pi / 180.0                                    # f64::to_radians
    aspect = w / h                                           # :28
    vh = math.tan((view_angle * rad) / 2.0) * focal_length * 2.0   # :29
    vw = vh * aspect                                         # :32
    direction = v_unit(v_sub(look_at, center))               # :34
    wv = v_neg(direction)                                    # :35
    u = v_unit(v_cross(up, wv))                              # :36
    v = v_cross(wv, u)                                       # :37
    vu = v_mul(u, vw)                                        # :39
    vv = v_mul(v_neg(v), vh)                                 # :40
    ulc = v_sub(v_sub(v_sub(center, v_mul(wv, focal_length)), v_div(vu, 2.0)), v_div(vv, 2.0))   # :41
    dr = focal_length * math.tan((defocus_angle / 2.0) * rad)   # :43
    return {"W": w, "H": h, "center": tuple(center), "ulc": ulc, "vu": vu, "vv": vv,
            "du": v_mul(u, dr), "dv": v_mul(v, dr)}           # :44-45 (f64 * Vec3 = Vec3 * f64)


def camera_in(cam, prec):
    """The camera's constants in the precision of the arithmetic (fp32: each rounded from f64)."""
    if prec != "f32":
        return cam
    out = dict(cam)
    for k in ("center", "ulc", "vu", "vv", "du", "dv"):
        out[k] = tuple(F32(x) for x in cam[k])
    return out


def get_ray(cam, col, row, sid, pix, seed, prec="f64"):
    """Camera::get_ray (:77-89): (origin, unit direction).  cam: camera_in(.., prec)."""
    T = F32 if prec == "f32" else float
    xo, yo = uniforms(sid, pix, 0, 0, seed, prec)                                 # :78-79
    off = v_add(v_mul(cam["vu"], (T(col) + xo) / T(cam["W"])), v_mul(cam["vv"], (T(row) + yo) / T(cam["H"])))   # :80
    pc = v_add(cam["ulc"], off)                                                    # :81
    i = 0
    while True:                                                                    # geometry.rs:154-168
        ux, uy = uniforms(sid, pix, i, 1, seed, prec)
        x, y = 2.0 * ux - 1.0, 2.0 * uy - 1.0
        if x * x + y * y <= 1.0:
            break
        i += 1
    origin = v_add(v_add(v_mul(cam["du"], x), v_mul(cam["dv"], y)), cam["center"])   # :83
    return origin, v_unit(v_sub(pc, origin))                                       # :84


# ---------------------------------------------------------------- the packed path
N = 4   # renderer.rs:142


class Material:
    """rt_material: kind 0 lambertian, 1 metal, 2 dielectric (parameters in the arithmetic's precision)."""

    def __init__(self, kind, albedo, fuzz, ior, hollow, prec="f64"):
        T = F32 if prec == "f32" else float
        self.kind, self.albedo, self.ior, self.hollow = kind, tuple(T(a) for a in albedo), T(ior), bool(hollow)
        self.fuzz = T(fuzz if fuzz < 1.0 else 1.0)   # Metal::new clamp (materials.rs:79-88)


def get_hit_result(mat, d, loc, normal, front, u1, u2):
    """Material::get_hit_result (materials.rs): (attenuation, scattered direction); origin = loc."""
    if mat.kind == 0:   # Lambertian :54-63
        sd = v_add(random_unit_vector(u1, u2), normal)
        if near_zero(sd):
            sd = normal
        return mat.albedo, sd
    if mat.kind == 1:   # Metal :92-97
        return mat.albedo, v_add(reflect(d, normal), v_mul(random_unit_vector(u1, u2), mat.fuzz))
    ratio = 1.0 / mat.ior if front else mat.ior               # Dielectric :129
    n = v_neg(normal) if mat.hollow else normal               # :131
    cos_theta = fmin(v_dot(v_neg(d), n), 1.0)                 # :132
    sin_theta = sqrt(1.0 - cos_theta * cos_theta)             # :133 (NaN past |cos| > 1: d is not unit)
    cannot = ratio * sin_theta > 1.0                          # :135
    if not cannot:                                            # :137, the draw only when it can refract
        q = (1.0 - ratio) / (1.0 + ratio)
        r0 = q * q                                            # :122
        m = 1.0 - cos_theta
        refl = r0 + (1.0 - r0) * (m * ((m * m) * (m * m))) > u1   # :123, powi(5)
    else:
        refl = True
    one = F32(1.0) if isinstance(ratio, F32) else 1.0
    return (one, one, one), (reflect(d, n) if refl else refract(d, n, ratio))


class Packet:
    """PackedRays<4> (ray.rs:36-153) plus, per lane, the sample id the RNG substitution keys on."""

    def __init__(self, zero=0.0):
        self.o = [(zero, zero, zero)] * N
        self.d = [(zero, zero, zero)] * N
        self.en = [True] * N        # PackedRays::new: all enabled (:49-55)
        self.sid = [-1] * N

    def copy(self):
        p = Packet(self.o[0][0] * 0)
        p.o, p.d, p.en, p.sid = list(self.o), list(self.d), list(self.en), list(self.sid)
        return p


class Spheres(list):
    """[(centre, r^2)] in the arithmetic's precision, plus f64 arrays for hit_scene's estimate."""

    def __init__(self, items, tol, literal=False):
        super().__init__(items)
        self.C = np.array([[float(x) for x in c] for c, _ in items], dtype=np.float64).reshape(-1, 3)
        self.R2 = np.array([float(r2) for _, r2 in items], dtype=np.float64)
        self.tol, self.literal = tol, literal

    def candidates(self, o, d):
        """Scene indices whose discriminant may be >= 0 (all of them when literal)."""
        if self.literal or len(self) == 0:
            return range(len(self))
        with np.errstate(all="ignore"):
            dd = np.array([float(x) for x in d])
            oc = np.array([float(x) for x in o]) - self.C
            a = dd @ dd
            hb = oc @ dd
            l2 = np.einsum("ij,ij->i", oc, oc)
            disc = hb * hb - a * (l2 - self.R2)
            keep = ~(disc < -self.tol * (hb * hb + a * (l2 + np.abs(self.R2))))   # NaN / inf: kept
        return np.flatnonzero(keep).tolist()


def hit_scene(spheres, o, d):
    """Per lane of an ENABLED ray: the object loop (ray_tracing.rs:399-401) with Sphere::hit_packed
    (objects.rs:249-290) and PackedHitRecords::update / finalize (:140-162).  Returns None (no hit) or
    (t, location, unit normal against the ray, front_face, sphere index).  spheres: Spheres; only the
    spheres its estimate cannot rule out run the literal test, in scene order (module docstring)."""
    best_t, best_n, best_i = math.inf, None, -1
    a = pk_len2(d)                                   # :253
    inv_a = 1.0 / a                                  # :254
    for i in spheres.candidates(o, d):
        c, r2 = spheres[i]
        oc = v_sub(o, c)                             # :252
        hb = pk_dot(oc, d)                           # :255
        cc = pk_len2(oc) - r2                        # :256, Simd::splat(radius.powi(2))
        disc = fma(hb, hb, (-a) * cc)                # :257
        if not disc >= 0.0:                          # :259 (the lane's part of the any() gate)
            continue
        sd = sqrt(disc)                              # :263
        root1 = (-hb - sd) * inv_a                   # :270
        root1_valid = root1 >= 0.001 and root1 < math.inf   # :272, simd_inside(0.001..inf)
        root2_valid = root1_valid                    # :273 tests root1 again (quirk Q1)
        if not (root1_valid or root2_valid):         # :277
            continue
        root = root1                                 # :275 masked_select(root2, root1, root1_valid)
        loc = v_add(o, v_mul(d, root))               # :279 at_t (no FMA)
        normal = v_sub(loc, c)                       # :280
        if root <= best_t:                           # update :141 (t <= best: later sphere wins)
            best_t, best_n, best_i = root, normal, i
    if best_i < 0:
        return None
    n = v_div(best_n, sqrt(pk_len2(best_n)))         # finalize :158 unit_vector (packed length)
    loc = v_add(o, v_mul(d, best_t))                 # :159 at_t(self.t)
    front = pk_dot(d, n) < 0.0                       # :160
    if not front:
        n = v_neg(n)                                 # :161
    return best_t, loc, n, front, best_i


def trace_vectorized2(spheres, smat, mats, rays, depth_limit, pix, seed, stats=None, prec="f64"):
    """ray_tracing.rs:375-505, literally.  rays: list of Packet (the primary rays)."""
    T = F32 if prec == "f32" else float
    C = len(rays)
    buf = [[p.copy() for p in rays], [Packet(T(0.0)) for _ in range(C)]]               # :382
    col = [[[(T(1.0), T(1.0), T(1.0))] * N for _ in range(C)] for _ in range(2)]         # :383
    sky = [[[False] * N for _ in range(C)] for _ in range(2)]                            # :384
    last = C                                                                             # :386
    for k in range(depth_limit):                                                         # :388
        if last == 0:
            break
        sel = k % 2
        for j in range(last):                                                            # :396
            pk = buf[sel][j]
            for i in range(N):                                                           # :406
                rec = hit_scene(spheres, pk.o[i], pk.d[i]) if pk.en[i] else None         # at(i): enabled only
                if stats is not None and pk.en[i]:
                    stats["segments"] += 1
                if rec is not None:
                    t, loc, n, front, si = rec
                    u1, u2 = uniforms(pk.sid[i], pix, k, 2, seed, prec)
                    att, sd = get_hit_result(mats[smat[si]], pk.d[i], loc, n, front, u1, u2)
                    c0 = col[sel][j][i]
                    col[sel][j][i] = (c0[0] * att[0], c0[1] * att[1], c0[2] * att[2])    # :410-411
                    pk.o[i], pk.d[i], pk.en[i] = loc, sd, True                           # update :414
                else:
                    pk.en[i] = False                                                     # :422
                    sky[sel][j][i] = True                                                # :423
        nxt = 1 - sel                                                                    # :433
        oc_, os_ = 0, 0

        def put(src_j, src_i, en):
            nonlocal oc_, os_
            s, d = buf[sel][src_j], buf[nxt][oc_]
            d.o[os_], d.d[os_], d.en[os_], d.sid[os_] = s.o[src_i], s.d[src_i], en, s.sid[src_i]
            col[nxt][oc_][os_] = col[sel][src_j][src_i]
            sky[nxt][oc_][os_] = sky[sel][src_j][src_i]
            os_ += 1
            if os_ >= N:
                os_, oc_ = 0, oc_ + 1

        for i in range(last):                                                            # :435-458
            for j in range(N):
                if buf[sel][i].en[j]:
                    put(i, j, True)
        new_last = oc_ if os_ == 0 else oc_ + 1                                          # :461
        for i in range(last):                                                            # :463-481
            for j in range(N):
                if not buf[sel][i].en[j]:
                    put(i, j, False)
        last = new_last                                                                  # :483
    S = (C - 1) % 2                                                                      # :486
    acc = [[T(0.0)] * N for _ in range(3)]                                               # :499 black
    for j in range(C):                                                                   # :488-502
        for i in range(N):
            a = (rays[j].d[i][1] + 1.0) * 0.5                                            # :490 the ORIGINAL rays
            skyc = (1.0 * (-a + 1.0) + 0.5 * a, 1.0 * (-a + 1.0) + 0.7 * a, 1.0 * (-a + 1.0) + 1.0 * a)
            c = col[S][j][i]
            if sky[S][j][i]:
                c = (c[0] * skyc[0], c[1] * skyc[1], c[2] * skyc[2])                      # :494-495
            if buf[S][j].en[i]:
                c = (T(0.0), T(0.0), T(0.0))                                             # :496
            for ch in range(3):
                acc[ch][i] = acc[ch][i] + c[ch]                                          # :501
    return tuple(((acc[ch][0] + acc[ch][1]) + acc[ch][2]) + acc[ch][3] for ch in range(3))   # PackedColor::sum


def to_u8(v):
    """Color::to_u8_array (color.rs:54-64) for one channel; raises where the reference panics."""
    if not v <= 2.0:
        raise ValueError("channel > 2.0: Color::to_u8_array panics")
    x = sqrt(v) * 255.999
    if not x > 0.0:
        return 0      # `as u8` saturates; NaN -> 0
    return 255 if x >= 255.0 else int(x)


def render_pixel(scene, cam, col_, row_, spp, depth, seed, stats=None, prec="f64"):
    """TileRenderTask::render_vectorized2's pixel body (renderer.rs:152-163): (linear, rgb8).
    cam: camera_in(.., prec)."""
    spheres, smat, mats = scene
    T = F32 if prec == "f32" else float
    pix = row_ * cam["W"] + col_
    chunks = []
    for s in range(spp):                                                  # :157 .chunks(4)
        if s % N == 0:
            p = Packet(T(0.0))
            p.en = [False] * N                                            # FromIterator: lanes start disabled
            chunks.append(p)
        o, d = get_ray(cam, col_, row_, s, pix, seed, prec)
        p.o[s % N], p.d[s % N], p.en[s % N], p.sid[s % N] = o, d, True, s   # update (:148)
    tot = trace_vectorized2(spheres, smat, mats, chunks, depth, pix, seed, stats, prec)
    lin = tuple(t / spp for t in tot)                                     # :161
    return lin, tuple(to_u8(v) for v in lin)


def scene_from_flat(flat, prec="f64", literal=False):
    """(Spheres [(centre, r*r)], material index per sphere, materials) from an rt_mi355x.FlatScene, in the
    arithmetic's precision (fp32: centre and radius rounded to fp32, r*r in fp32)."""
    T = F32 if prec == "f32" else float
    spheres = [((T(c[0]), T(c[1]), T(c[2])), T(r) * T(r)) for c, r in zip(flat.center, flat.radius)]
    mats = []
    for m in flat.materials:
        a = m.to_abi()
        mats.append(Material(a.kind, tuple(a.albedo), a.fuzz, a.ior, a.hollow, prec))
    tol = 1e-4 if prec == "f32" else 1e-9
    return Spheres(spheres, tol, literal), [int(x) for x in flat.material], mats


def render(flat, cam, spp, depth, seed, pixels=None, prec="f64", literal=False):
    """Every pixel (row-major) or the listed pixel indices: (linear [n][3], rgb [n][3], segments).
    prec: "f64" (the reference's arithmetic) or "f32"; literal: no estimate in hit_scene."""
    scene = scene_from_flat(flat, prec, literal)
    camp = camera_in(cam, prec)
    W, H = cam["W"], cam["H"]
    pixels = range(W * H) if pixels is None else pixels
    lin, rgb, stats = [], [], {"segments": 0}
    for p in pixels:
        l, c = render_pixel(scene, camp, p % W, p // W, spp, depth, seed, stats, prec)
        lin.append(l)
        rgb.append(c)
    return lin, rgb, stats["segments"]
