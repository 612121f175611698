/*
 * oracle_impl.h — TEST INFRASTRUCTURE ONLY (see oracle.h for parity status).
 *
 * Precision-generic body of the oracle.  Included twice by oracle.c with
 *   REAL = double, SFX(x) = x##_f64   (reference arithmetic: all f64)
 *   REAL = float,  SFX(x) = x##_f32   (same algorithm, every op in f32)
 * Compiled with -ffp-contract=off: an FMA appears exactly where the reference
 * writes mul_add (PackedVec3::length_squared/dot, geometry.rs:434-436,466-468;
 * the discriminant, objects.rs:257) and nowhere else (scalar Vec3 ops,
 * geometry.rs:105-188, have none).
 *
 * RNG boundary (parity unpinned, see oracle.h):  every random draw is a pure
 * function of (seed, pixel, sample, bounce, stream) through Philox4x32-10 (f64; f32: Philox2x32-10, SFX(draw) below), so
 * results do not depend on threading, compaction order or GPU count.
 *   stream 0, ctr (s, pix, 0, 0): Camera::get_ray jitter      (ray_tracing.rs:78-79)
 *   stream 1, ctr (s, pix, i, 1): random_in_unit_disk try i  (geometry.rs:154-168)
 *   stream 2, ctr (s, pix, k, 2): scatter draw at bounce k    (materials.rs:56,93,137)
 * Vec3::random_unit_vector (geometry.rs:139-152) normalises 3 N(0,1) draws, i.e.
 * it is uniform on S^2; we draw the same distribution directly
 * (z = 1-2u1, phi = 2*pi*u2) with a fixed fma-Horner sin/cos so CPU and GPU
 * evaluate bit-identical arithmetic.
 */

#define V3 SFX(v3)
typedef struct { REAL x, y, z; } V3;

static inline V3 SFX(mk)(REAL x, REAL y, REAL z) { V3 r = {x, y, z}; return r; }
/* Scalar Vec3 ops: geometry.rs:37-132 (no FMA, left-to-right sums). */
static inline V3 SFX(add)(V3 a, V3 b) { return SFX(mk)(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 SFX(sub)(V3 a, V3 b) { return SFX(mk)(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 SFX(mul)(V3 a, REAL s) { return SFX(mk)(a.x * s, a.y * s, a.z * s); }
static inline V3 SFX(dvs)(V3 a, REAL s) { return SFX(mk)(a.x / s, a.y / s, a.z / s); }
static inline V3 SFX(neg)(V3 a) { return SFX(mk)(-a.x, -a.y, -a.z); }
static inline REAL SFX(dot)(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline REAL SFX(len2)(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }   /* powi(2) == x*x */
static inline V3 SFX(unit)(V3 a) { return SFX(dvs)(a, SQRT(SFX(len2)(a))); }        /* geometry.rs:118-120 */
/* Packed ops with the reference's explicit FMA (geometry.rs:434-436, 466-468). */
static inline REAL SFX(pk_len2)(V3 a) { return FMA(a.z, a.z, FMA(a.y, a.y, a.x * a.x)); }
static inline REAL SFX(pk_dot)(V3 a, V3 b) { return FMA(a.z, b.z, FMA(a.y, b.y, a.x * b.x)); }

/* geometry.rs:134-137 */
static inline int SFX(near_zero)(V3 v) {
    const REAL e = (REAL)1e-8;
    return FABS(v.x) < e && FABS(v.y) < e && FABS(v.z) < e;
}
/* geometry.rs:179-181: v - 2*(v.n)*n */
static inline V3 SFX(reflect)(V3 v, V3 n) { return SFX(sub)(v, SFX(mul)(n, (REAL)2.0 * SFX(dot)(v, n))); }
/* geometry.rs:183-188 (note .abs(): never NaN) */
static inline V3 SFX(refract)(V3 v, V3 n, REAL ratio) {
    REAL ct = FMIN(SFX(dot)(SFX(neg)(v), n), (REAL)1.0);
    V3 rperp = SFX(mul)(SFX(add)(v, SFX(mul)(n, ct)), ratio);
    V3 rpar = SFX(mul)(n, -(SQRT(FABS((REAL)1.0 - SFX(len2)(rperp)))));
    return SFX(add)(rperp, rpar);
}

/* ---- RNG transforms ---- */
static inline REAL SFX(u01)(const uint32_t* r) {   /* uniform [0,1): f64 53 bits of (r0,r1); f32 24 bits of r0 */
#if ORACLE_IS_F64
    return (double)((((uint64_t)r[0] << 32) | r[1]) >> 11) * 0x1.0p-53;
#else
    return (float)(r[0] >> 8) * 0x1.0p-24f;
#endif
}
static inline REAL SFX(u01b)(const uint32_t* r) {  /* second independent uniform of the block */
#if ORACLE_IS_F64
    return (double)((((uint64_t)r[2] << 32) | r[3]) >> 11) * 0x1.0p-53;
#else
    return (float)(r[1] >> 8) * 0x1.0p-24f;
#endif
}

/* One draw block for (sample, pixel, k, stream) (the kernel's rng<T>, rt_device.hpp): stream 0 the camera
 * jitter (k = 0), 1 disk try k, 2 the scatter at bounce k.  f64: Philox4x32-10, counter (sid, pix, k,
 * stream), key (seed lo, seed hi).  f32 uses two 24-bit words only: Philox2x32-10, counter
 * (pix, sid | code << 20) with code 0 / 1 + k / 257 + k, key seed lo ^ fmix32(seed hi) (murmur3's
 * finaliser, oracle_fmix32; r[2], r[3] unused). */
static inline void SFX(draw)(uint32_t sid, uint32_t pix, uint32_t k, uint32_t stream, uint32_t k0, uint32_t k1,
                             uint32_t r[4]) {
#if ORACLE_IS_F64
    const uint32_t ctr[4] = {sid, pix, k, stream}, key[2] = {k0, k1};
    oracle_philox4x32_10(ctr, key, r);
#else
    const uint32_t code = stream == 0u ? 0u : (stream == 1u ? 1u + k : 257u + k);
    const uint32_t ctr[2] = {pix, sid | (code << 20)};
    oracle_philox2x32_10(ctr, k0 ^ oracle_fmix32(k1), r);
    r[2] = 0u; r[3] = 0u;
#endif
}

/* sin(2*pi*u), cos(2*pi*u) for u in [0,1): exact quadrant/octant reduction in u-space, then
 * Taylor polynomials on [0, pi/4] evaluated by fma-Horner (bit-identical on CPU and GPU). */
static inline void SFX(sincos2pi)(REAL u, REAL* so, REAL* co) {
    REAL t = u * (REAL)4.0;
    int q = (int)t;
    REAL f = t - (REAL)q;
    int sw = f > (REAL)0.5;
    REAL g = sw ? (REAL)1.0 - f : f;
    REAL x = g * (REAL)1.5707963267948966;
    REAL x2 = x * x;
    REAL ps, pc;
#if ORACLE_IS_F64
    ps = 1.0 / 355687428096000.0;
    ps = FMA(ps, x2, -1.0 / 1307674368000.0);
    ps = FMA(ps, x2, 1.0 / 6227020800.0);
    ps = FMA(ps, x2, -1.0 / 39916800.0);
    ps = FMA(ps, x2, 1.0 / 362880.0);
    ps = FMA(ps, x2, -1.0 / 5040.0);
    ps = FMA(ps, x2, 1.0 / 120.0);
    ps = FMA(ps, x2, -1.0 / 6.0);
    pc = -1.0 / 6402373705728000.0;
    pc = FMA(pc, x2, 1.0 / 20922789888000.0);
    pc = FMA(pc, x2, -1.0 / 87178291200.0);
    pc = FMA(pc, x2, 1.0 / 479001600.0);
    pc = FMA(pc, x2, -1.0 / 3628800.0);
    pc = FMA(pc, x2, 1.0 / 40320.0);
    pc = FMA(pc, x2, -1.0 / 720.0);
    pc = FMA(pc, x2, 1.0 / 24.0);
    pc = FMA(pc, x2, -1.0 / 2.0);
#else
    ps = (float)(1.0 / 362880.0);
    ps = FMA(ps, x2, (float)(-1.0 / 5040.0));
    ps = FMA(ps, x2, (float)(1.0 / 120.0));
    ps = FMA(ps, x2, (float)(-1.0 / 6.0));
    pc = (float)(-1.0 / 3628800.0);
    pc = FMA(pc, x2, (float)(1.0 / 40320.0));
    pc = FMA(pc, x2, (float)(-1.0 / 720.0));
    pc = FMA(pc, x2, (float)(1.0 / 24.0));
    pc = FMA(pc, x2, (float)(-1.0 / 2.0));
#endif
    REAL s = FMA(x * x2, ps, x);
    REAL c = FMA(x2, pc, (REAL)1.0);
    if (sw) { REAL tmp = s; s = c; c = tmp; }
    switch (q & 3) {
        case 0: *so = s; *co = c; break;
        case 1: *so = c; *co = -s; break;
        case 2: *so = -s; *co = -c; break;
        default: *so = -c; *co = s; break;
    }
}

/* Uniform direction on S^2 (distribution of Vec3::random_unit_vector, geometry.rs:139-152). */
static inline V3 SFX(unit_vec)(REAL u1, REAL u2) {
    REAL z = (REAL)1.0 - (REAL)2.0 * u1;
    REAL r = SQRT((REAL)1.0 - z * z);
    REAL s, c;
    SFX(sincos2pi)(u2, &s, &c);
    return SFX(mk)(r * c, r * s, z);
}

/* ---- scene / camera in REAL ---- */
typedef struct {
    uint32_t kind, hollow;
    REAL ar, ag, ab, fuzz, ior;
} SFX(mat_r);

typedef struct {
    uint32_t n;
    REAL* cx; REAL* cy; REAL* cz; REAL* r;
    const uint32_t* mat;
    SFX(mat_r)* mats;
} SFX(scene_r);

typedef struct {
    uint32_t W, H;
    V3 center, ulc, vu, vv, du, dv;
} SFX(cam_r);

/* Camera::get_ray, ray_tracing.rs:77-89 */
static void SFX(get_ray)(const SFX(cam_r)* c, uint32_t col, uint32_t row, uint32_t pix, uint32_t s,
                         uint32_t k0, uint32_t k1, V3* o, V3* d) {
    uint32_t r[4];
    SFX(draw)(s, pix, 0u, 0u, k0, k1, r);
    REAL xo = SFX(u01)(r), yo = SFX(u01b)(r);
    REAL s1 = ((REAL)col + xo) / (REAL)c->W;
    REAL s2 = ((REAL)row + yo) / (REAL)c->H;
    V3 po = SFX(add)(SFX(mul)(c->vu, s1), SFX(mul)(c->vv, s2));
    V3 pc = SFX(add)(c->ulc, po);
    /* random_in_unit_disk: rejection on [-1,1]^2 (geometry.rs:154-168) */
    REAL dx = 0, dy = 0;
    for (uint32_t i = 0; i < 256u; ++i) {
        SFX(draw)(s, pix, i, 1u, k0, k1, r);
        REAL x = (REAL)2.0 * SFX(u01)(r) - (REAL)1.0;
        REAL y = (REAL)2.0 * SFX(u01b)(r) - (REAL)1.0;
        if (x * x + y * y <= (REAL)1.0) { dx = x; dy = y; break; }
    }
    V3 orig = SFX(add)(SFX(add)(SFX(mul)(c->du, dx), SFX(mul)(c->dv, dy)), c->center);
    *o = orig;
    *d = SFX(unit)(SFX(sub)(pc, orig));
}

/* PackedRays<4> (ray.rs:36-43) + sample id carried for RNG keying. */
typedef struct {
    REAL ox[4], oy[4], oz[4], dx[4], dy[4], dz[4];
    int en[4];
    uint32_t sid[4];
} SFX(prays);
typedef struct { REAL r[4], g[4], b[4]; } SFX(pcol);   /* PackedColor<4> (color.rs:176-182) */

/* PackedHitRecords<4> (objects.rs:109-119); material stored as sphere material index. */
typedef struct {
    REAL nx[4], ny[4], nz[4], t[4], px[4], py[4], pz[4];
    int front[4], hit[4];
    uint32_t mat[4];
} SFX(phit);

/* Sphere::hit_packed, objects.rs:249-290, folded into PackedHitRecords::update (objects.rs:140-155). */
static inline void SFX(hit_packed)(const SFX(prays)* R, REAL cx, REAL cy, REAL cz, REAL rad, uint32_t mat,
                                   SFX(phit)* H, uint32_t flags) {
    REAL a[4], inv_a[4], hb[4], disc[4];
    int any = 0;
    for (int l = 0; l < 4; ++l) {
        V3 oc = SFX(mk)(R->ox[l] - cx, R->oy[l] - cy, R->oz[l] - cz);               /* :252 */
        V3 d = SFX(mk)(R->dx[l], R->dy[l], R->dz[l]);
        a[l] = SFX(pk_len2)(d);                                                        /* :253 */
        inv_a[l] = (REAL)1.0 / a[l];                                                   /* :254 */
        hb[l] = SFX(pk_dot)(oc, d);                                                    /* :255 */
        REAL c = SFX(pk_len2)(oc) - rad * rad;                                         /* :256 */
        disc[l] = FMA(hb[l], hb[l], -a[l] * c);                                        /* :257 */
        any |= (disc[l] >= (REAL)0.0) & R->en[l];                                      /* :259-261 */
    }
    if (!any) return;
    for (int l = 0; l < 4; ++l) {
        REAL nhb = -hb[l];                                                             /* :262 */
        REAL sd = SQRT(disc[l]);                                                       /* :263 */
        REAL r1 = (nhb - sd) * inv_a[l];                                               /* :270 */
        REAL r2 = (nhb + sd) * inv_a[l];                                               /* :271 */
        int r1v = r1 >= (REAL)0.001 && r1 < (REAL)INFINITY;                            /* :272 simd_inside */
        /* Q1: the reference tests root1 twice (:273); ROOT2 flag restores the scalar semantics. */
        int r2v = (flags & OR_FLAG_ROOT2) ? (r2 >= (REAL)0.001 && r2 < (REAL)INFINITY) : r1v;
        REAL root = r1v ? r1 : r2;                                                     /* :275 */
        int valid = (r1v | r2v) & R->en[l];                                            /* :277 */
        /* update: ties -> later sphere wins (t <= best), objects.rs:141 */
        if (valid && root <= H->t[l]) {
            REAL lx = R->ox[l] + R->dx[l] * root;                                      /* at_t, ray.rs:102-104 */
            REAL ly = R->oy[l] + R->dy[l] * root;
            REAL lz = R->oz[l] + R->dz[l] * root;
            H->nx[l] = lx - cx; H->ny[l] = ly - cy; H->nz[l] = lz - cz;                /* :280 */
            H->t[l] = root;
            H->hit[l] = 1;
            H->mat[l] = mat;
        }
    }
}

/* PackedHitRecords::finalize, objects.rs:157-162 */
static inline void SFX(finalize)(const SFX(prays)* R, SFX(phit)* H) {
    for (int l = 0; l < 4; ++l) {
        V3 n = SFX(mk)(H->nx[l], H->ny[l], H->nz[l]);
        REAL len = SQRT(SFX(pk_len2)(n));
        n = SFX(mk)(n.x / len, n.y / len, n.z / len);
        H->px[l] = R->ox[l] + R->dx[l] * H->t[l];
        H->py[l] = R->oy[l] + R->dy[l] * H->t[l];
        H->pz[l] = R->oz[l] + R->dz[l] * H->t[l];
        V3 d = SFX(mk)(R->dx[l], R->dy[l], R->dz[l]);
        int front = SFX(pk_dot)(d, n) < (REAL)0.0;
        H->front[l] = front;
        if (!front) n = SFX(neg)(n);
        H->nx[l] = n.x; H->ny[l] = n.y; H->nz[l] = n.z;
    }
}

/* Material::get_hit_result for one lane: materials.rs:54-63 (lambertian), 92-97 (metal),
 * 128-147 (dielectric).  Writes the scattered ray; returns attenuation. */
static inline void SFX(scatter)(const SFX(mat_r)* m, V3 d, V3 p, V3 n, int front, uint32_t pix, uint32_t sid,
                                uint32_t k, uint32_t k0, uint32_t k1, V3* od, REAL att[3]) {
    uint32_t r[4];
    SFX(draw)(sid, pix, k, 2u, k0, k1, r);
    (void)p;
    if (m->kind == 0u) {
        V3 sd = SFX(add)(SFX(unit_vec)(SFX(u01)(r), SFX(u01b)(r)), n);
        if (SFX(near_zero)(sd)) sd = n;
        *od = sd;
        att[0] = m->ar; att[1] = m->ag; att[2] = m->ab;
    } else if (m->kind == 1u) {
        V3 rv = SFX(add)(SFX(reflect)(d, n), SFX(mul)(SFX(unit_vec)(SFX(u01)(r), SFX(u01b)(r)), m->fuzz));
        *od = rv;
        att[0] = m->ar; att[1] = m->ag; att[2] = m->ab;
    } else {
        REAL ratio = front ? (REAL)1.0 / m->ior : m->ior;
        V3 nn = m->hollow ? SFX(neg)(n) : n;
        REAL ct = FMIN(SFX(dot)(SFX(neg)(d), nn), (REAL)1.0);
        REAL st = SQRT((REAL)1.0 - ct * ct);
        int cannot = ratio * st > (REAL)1.0;
        int refl = cannot;
        if (!refl) {
            /* Dielectric::reflectance, materials.rs:121-124; powi(5) = x*((x*x)*(x*x)) */
            REAL q = ((REAL)1.0 - ratio) / ((REAL)1.0 + ratio);
            REAL r0 = q * q;
            REAL m1 = (REAL)1.0 - ct;
            REAL m2 = m1 * m1;
            REAL m5 = m1 * (m2 * m2);
            REAL refl_p = r0 + ((REAL)1.0 - r0) * m5;
            refl = refl_p > SFX(u01)(r);
        }
        *od = refl ? SFX(reflect)(d, nn) : SFX(refract)(d, nn, ratio);
        att[0] = (REAL)1.0; att[1] = (REAL)1.0; att[2] = (REAL)1.0;
    }
}

/* sky gradient of trace_vectorized2's final pass, ray_tracing.rs:490-494 */
static inline void SFX(sky)(REAL y, REAL s[3]) {
    REAL a = (y + (REAL)1.0) * (REAL)0.5;
    REAL oma = -a + (REAL)1.0;
    s[0] = (REAL)1.0 * oma + (REAL)0.5 * a;
    s[1] = (REAL)1.0 * oma + (REAL)0.7 * a;
    s[2] = (REAL)1.0 * oma + (REAL)1.0 * a;
}

typedef struct {
    uint32_t C;
    SFX(prays)* rays0;     /* the caller's primary chunks (`rays`) */
    SFX(prays)* buf[2];
    SFX(pcol)* col[2];
    int* sky[2];           /* [C][4] */
} SFX(ws);

static int SFX(ws_init)(SFX(ws)* w, uint32_t C) {
    w->C = C;
    w->rays0 = (SFX(prays)*)calloc(C, sizeof(SFX(prays)));
    for (int i = 0; i < 2; ++i) {
        w->buf[i] = (SFX(prays)*)calloc(C, sizeof(SFX(prays)));
        w->col[i] = (SFX(pcol)*)calloc(C, sizeof(SFX(pcol)));
        w->sky[i] = (int*)calloc((size_t)C * 4, sizeof(int));
    }
    return w->rays0 && w->buf[0] && w->buf[1] && w->col[0] && w->col[1] && w->sky[0] && w->sky[1];
}
static void SFX(ws_free)(SFX(ws)* w) {
    free(w->rays0);
    for (int i = 0; i < 2; ++i) { free(w->buf[i]); free(w->col[i]); free(w->sky[i]); }
}

static inline void SFX(copy_slot)(SFX(ws)* w, int from_sel, uint32_t fc, int fl, int to_sel, uint32_t tc, int tl, int en) {
    SFX(prays)* a = &w->buf[from_sel][fc];
    SFX(prays)* b = &w->buf[to_sel][tc];
    b->ox[tl] = a->ox[fl]; b->oy[tl] = a->oy[fl]; b->oz[tl] = a->oz[fl];
    b->dx[tl] = a->dx[fl]; b->dy[tl] = a->dy[fl]; b->dz[tl] = a->dz[fl];
    b->en[tl] = en; b->sid[tl] = a->sid[fl];
    w->col[to_sel][tc].r[tl] = w->col[from_sel][fc].r[fl];
    w->col[to_sel][tc].g[tl] = w->col[from_sel][fc].g[fl];
    w->col[to_sel][tc].b[tl] = w->col[from_sel][fc].b[fl];
    w->sky[to_sel][tc * 4 + tl] = w->sky[from_sel][fc * 4 + fl];
}

/* Scene::trace_vectorized2, ray_tracing.rs:375-505 (N = 4), literal two-buffer form. */
static void SFX(trace_pixel)(const SFX(scene_r)* S, SFX(ws)* w, uint32_t depth, uint32_t pix,
                             uint32_t k0, uint32_t k1, uint32_t flags, REAL out[3], uint64_t* segs) {
    const uint32_t C = w->C;
    /* :382-384 init: buffer0 = rays, buffer1 = zero rays with enabled=true (PackedRays::new); colours white */
    for (uint32_t j = 0; j < C; ++j) {
        w->buf[0][j] = w->rays0[j];
        memset(&w->buf[1][j], 0, sizeof(SFX(prays)));
        for (int l = 0; l < 4; ++l) {
            w->buf[1][j].en[l] = 1;
            for (int s = 0; s < 2; ++s) {
                w->col[s][j].r[l] = 1; w->col[s][j].g[l] = 1; w->col[s][j].b[l] = 1;
                w->sky[s][j * 4 + l] = 0;
            }
        }
    }
    uint32_t last_active = C;                                                         /* :386 */
    uint64_t nseg = 0;
    for (uint32_t k = 0; k < depth; ++k) {                                            /* :388 */
        if (last_active == 0) break;                                                  /* :389-392 */
        int sel = (int)(k % 2);                                                       /* :394 */
        for (uint32_t j = 0; j < last_active; ++j) {                                  /* :396 */
            SFX(prays)* R = &w->buf[sel][j];
            SFX(phit) H;
            for (int l = 0; l < 4; ++l) {                                             /* default(), objects.rs:124-133 */
                H.t[l] = (REAL)INFINITY; H.hit[l] = 0; H.front[l] = 0; H.mat[l] = 0;
                H.nx[l] = H.ny[l] = H.nz[l] = 0;
                nseg += (uint64_t)R->en[l];
            }
            for (uint32_t i = 0; i < S->n; ++i)                                      /* :399-401 */
                SFX(hit_packed)(R, S->cx[i], S->cy[i], S->cz[i], S->r[i], S->mat[i], &H, flags);
            SFX(finalize)(R, &H);                                                     /* :403 */
            for (int l = 0; l < 4; ++l) {                                             /* :406-426 */
                if (H.hit[l]) {
                    V3 d = SFX(mk)(R->dx[l], R->dy[l], R->dz[l]);
                    V3 p = SFX(mk)(H.px[l], H.py[l], H.pz[l]);
                    V3 n = SFX(mk)(H.nx[l], H.ny[l], H.nz[l]);
                    V3 nd;
                    REAL att[3];
                    SFX(scatter)(&S->mats[H.mat[l]], d, p, n, H.front[l], pix, R->sid[l], k, k0, k1, &nd, att);
                    SFX(pcol)* cc = &w->col[sel][j];
                    cc->r[l] = cc->r[l] * att[0];                                     /* :410 */
                    cc->g[l] = cc->g[l] * att[1];
                    cc->b[l] = cc->b[l] * att[2];
                    R->ox[l] = p.x; R->oy[l] = p.y; R->oz[l] = p.z;                  /* :414 update() */
                    R->dx[l] = nd.x; R->dy[l] = nd.y; R->dz[l] = nd.z;
                    R->en[l] = 1;
                } else {
                    R->en[l] = 0;                                                     /* :422 */
                    w->sky[sel][j * 4 + l] = 1;                                       /* :423 */
                }
            }
        }
        /* shuffle, :430-481: enabled lanes first (stable), then disabled lanes (stable) */
        int ns = 1 - sel;
        uint32_t oc = 0; int os = 0;
        for (uint32_t i = 0; i < last_active; ++i)
            for (int l = 0; l < 4; ++l)
                if (w->buf[sel][i].en[l]) {
                    SFX(copy_slot)(w, sel, i, l, ns, oc, os, 1);
                    if (++os >= 4) { os = 0; ++oc; }
                }
        uint32_t new_last = os == 0 ? oc : oc + 1;                                    /* :461 */
        for (uint32_t i = 0; i < last_active; ++i)
            for (int l = 0; l < 4; ++l)
                if (!w->buf[sel][i].en[l]) {
                    SFX(copy_slot)(w, sel, i, l, ns, oc, os, 0);
                    if (++os >= 4) { os = 0; ++oc; }
                }
        last_active = new_last;                                                       /* :483 */
    }
    /* :486-504 — Q3: read buffer (C-1)%2; Q2: sky from the ORIGINAL primary ray at each slot */
    int sel = (int)((C - 1) % 2);
    REAL acc[3][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    for (uint32_t j = 0; j < C; ++j) {
        for (int l = 0; l < 4; ++l) {
            REAL sk[3];
            SFX(sky)(w->rays0[j].dy[l], sk);
            REAL cr = w->col[sel][j].r[l], cg = w->col[sel][j].g[l], cb = w->col[sel][j].b[l];
            if (w->sky[sel][j * 4 + l]) { cr = cr * sk[0]; cg = cg * sk[1]; cb = cb * sk[2]; }
            if (w->buf[sel][j].en[l]) { cr = 0; cg = 0; cb = 0; }
            acc[0][l] = acc[0][l] + cr;                                               /* :500-502 */
            acc[1][l] = acc[1][l] + cg;
            acc[2][l] = acc[2][l] + cb;
        }
    }
    for (int ch = 0; ch < 3; ++ch)                                                    /* PackedColor::sum, color.rs:226-232 */
        out[ch] = (((REAL)0.0 + acc[ch][0]) + acc[ch][1] + acc[ch][2]) + acc[ch][3];
    *segs += nseg;
}

/* ---- "vectorized3" mode: Scene::trace_vectorized3, ray_tracing.rs:508-628 (N = 4), as called by
 * render_vectorized3 (renderer.rs:178-213).  Literal: one buffer, colours start white for every lane
 * (:515), the chunks [0, num_active) are traced, then an in-place swap partition with CombinedIndex
 * (:113-214, :561-607): the next disabled slot from the front (over ALL chunks) swaps with the previous
 * enabled slot from the back (below num_active) while the front's chunk is below the back's; the final
 * sky uses each slot's own (final) direction and the sum is per lane over chunks (:611-627). ---- */
/* CombinedIndex::increment / decrement (:129-171); slot 4 = before_first (:121-123) */
static inline int SFX(ci_inc)(uint32_t C, uint32_t* c, uint32_t* l) {
    if (*l >= 4u) { if (C > 0) { *c = 0; *l = 0; return 1; } return 0; }
    if (*l < 3u) { *l += 1; return 1; }
    if (*c + 1 < C) { *c += 1; *l = 0; return 1; }
    return 0;
}
static inline int SFX(ci_dec)(uint32_t* c, uint32_t* l) {
    if (*l > 0) { *l -= 1; return 1; }
    if (*c > 0) { *c -= 1; *l = 3; return 1; }
    return 0;
}
static void SFX(trace_pixel_v3)(const SFX(scene_r)* S, SFX(ws)* w, uint32_t depth, uint32_t pix,
                                uint32_t k0, uint32_t k1, uint32_t flags, REAL out[3], uint64_t* segs) {
    const uint32_t C = w->C;
    SFX(prays)* R = w->buf[0];
    SFX(pcol)* col = w->col[0];
    int* sky = w->sky[0];
    for (uint32_t j = 0; j < C; ++j) {                                                /* :515-516 */
        R[j] = w->rays0[j];
        for (int l = 0; l < 4; ++l) { col[j].r[l] = 1; col[j].g[l] = 1; col[j].b[l] = 1; sky[j * 4 + l] = 0; }
    }
    uint32_t na = C;                                                                  /* :518 */
    uint64_t nseg = 0;
    for (uint32_t k = 0; k < depth; ++k) {                                            /* :520 */
        if (na == 0) break;                                                           /* :521-524 */
        for (uint32_t j = 0; j < na; ++j) {                                           /* :526-559 */
            SFX(phit) H;
            for (int l = 0; l < 4; ++l) {
                H.t[l] = (REAL)INFINITY; H.hit[l] = 0; H.front[l] = 0; H.mat[l] = 0;
                H.nx[l] = H.ny[l] = H.nz[l] = 0;
                nseg += (uint64_t)R[j].en[l];
            }
            for (uint32_t i = 0; i < S->n; ++i)
                SFX(hit_packed)(&R[j], S->cx[i], S->cy[i], S->cz[i], S->r[i], S->mat[i], &H, flags);
            SFX(finalize)(&R[j], &H);
            for (int l = 0; l < 4; ++l) {
                if (H.hit[l]) {
                    V3 d = SFX(mk)(R[j].dx[l], R[j].dy[l], R[j].dz[l]);
                    V3 p = SFX(mk)(H.px[l], H.py[l], H.pz[l]);
                    V3 n = SFX(mk)(H.nx[l], H.ny[l], H.nz[l]);
                    V3 nd;
                    REAL att[3];
                    SFX(scatter)(&S->mats[H.mat[l]], d, p, n, H.front[l], pix, R[j].sid[l], k, k0, k1, &nd, att);
                    col[j].r[l] = col[j].r[l] * att[0];                               /* :542-543 */
                    col[j].g[l] = col[j].g[l] * att[1];
                    col[j].b[l] = col[j].b[l] * att[2];
                    R[j].ox[l] = p.x; R[j].oy[l] = p.y; R[j].oz[l] = p.z;             /* :546 update() */
                    R[j].dx[l] = nd.x; R[j].dy[l] = nd.y; R[j].dz[l] = nd.z;
                    R[j].en[l] = 1;
                } else {                                                              /* :553-556 */
                    R[j].en[l] = 0;
                    sky[j * 4 + l] = 1;
                }
            }
        }
        /* :563-607 swap partition */
        uint32_t fc = 0, fl = 4, bc = na, bl = 0;                                     /* before_first; (na, 0) */
        for (;;) {
            int found = 0;                                                            /* next_disabled */
            while (SFX(ci_inc)(C, &fc, &fl)) if (!R[fc].en[fl]) { found = 1; break; }
            if (!found) { na = C; break; }                                            /* :573 */
            found = 0;                                                                /* previous_enabled */
            while (SFX(ci_dec)(&bc, &bl)) if (R[bc].en[bl]) { found = 1; break; }
            if (!found) { na = 0; break; }                                            /* :581 */
            if (fc >= bc) { na = bc + 1; break; }                                     /* :586-589 */
            /* :592-605: front takes back's ray (enabled), back takes front's (disabled); colours and
             * hit_sky swap with them; the sample id travels with its ray (RNG key) */
            SFX(prays) t = R[fc];
            R[fc].ox[fl] = R[bc].ox[bl]; R[fc].oy[fl] = R[bc].oy[bl]; R[fc].oz[fl] = R[bc].oz[bl];
            R[fc].dx[fl] = R[bc].dx[bl]; R[fc].dy[fl] = R[bc].dy[bl]; R[fc].dz[fl] = R[bc].dz[bl];
            R[fc].sid[fl] = R[bc].sid[bl]; R[fc].en[fl] = 1;
            R[bc].ox[bl] = t.ox[fl]; R[bc].oy[bl] = t.oy[fl]; R[bc].oz[bl] = t.oz[fl];
            R[bc].dx[bl] = t.dx[fl]; R[bc].dy[bl] = t.dy[fl]; R[bc].dz[bl] = t.dz[fl];
            R[bc].sid[bl] = t.sid[fl]; R[bc].en[bl] = 0;
            REAL cr = col[fc].r[fl], cg = col[fc].g[fl], cb = col[fc].b[fl];
            col[fc].r[fl] = col[bc].r[bl]; col[fc].g[fl] = col[bc].g[bl]; col[fc].b[fl] = col[bc].b[bl];
            col[bc].r[bl] = cr; col[bc].g[bl] = cg; col[bc].b[bl] = cb;
            int hs = sky[fc * 4 + fl];
            sky[fc * 4 + fl] = sky[bc * 4 + bl];
            sky[bc * 4 + bl] = hs;
        }
    }
    REAL acc[3][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    for (uint32_t j = 0; j < C; ++j) {                                                /* :611-625 */
        for (int l = 0; l < 4; ++l) {
            REAL sk[3];
            SFX(sky)(R[j].dy[l], sk);                                                 /* its own direction */
            REAL cr = col[j].r[l], cg = col[j].g[l], cb = col[j].b[l];
            if (sky[j * 4 + l]) { cr = cr * sk[0]; cg = cg * sk[1]; cb = cb * sk[2]; }
            if (R[j].en[l]) { cr = 0; cg = 0; cb = 0; }
            acc[0][l] = acc[0][l] + cr; acc[1][l] = acc[1][l] + cg; acc[2][l] = acc[2][l] + cb;
        }
    }
    for (int ch = 0; ch < 3; ++ch)                                                    /* :627 PackedColor::sum */
        out[ch] = (((REAL)0.0 + acc[ch][0]) + acc[ch][1] + acc[ch][2]) + acc[ch][3];
    *segs += nseg;
}

/* ---- "vectorized" mode: Scene::trace_vectorized, ray_tracing.rs:312-373 (one PackedRays<4>
 * chunk, no shuffle), as called by render_vectorized (renderer.rs:102-139). ---- */
static void SFX(trace_chunk_v1)(const SFX(scene_r)* S, SFX(prays) R, uint32_t depth, uint32_t pix,
                                uint32_t k0, uint32_t k1, uint32_t flags, SFX(pcol)* out, uint64_t* segs) {
    SFX(pcol) col;
    int sky[4] = {0, 0, 0, 0};
    for (int l = 0; l < 4; ++l) {                                                      /* :319-320 */
        REAL w = R.en[l] ? (REAL)1.0 : (REAL)0.0;
        col.r[l] = w; col.g[l] = w; col.b[l] = w;
    }
    for (uint32_t k = 0; k < depth; ++k) {                                            /* :323 */
        if (!(R.en[0] | R.en[1] | R.en[2] | R.en[3])) break;                          /* :324-327 */
        SFX(phit) H;
        for (int l = 0; l < 4; ++l) {
            H.t[l] = (REAL)INFINITY; H.hit[l] = 0; H.front[l] = 0; H.mat[l] = 0;
            H.nx[l] = H.ny[l] = H.nz[l] = 0;
            *segs += (uint64_t)R.en[l];
        }
        for (uint32_t i = 0; i < S->n; ++i)                                          /* :331-333 */
            SFX(hit_packed)(&R, S->cx[i], S->cy[i], S->cz[i], S->r[i], S->mat[i], &H, flags);
        SFX(finalize)(&R, &H);                                                        /* :335 */
        for (int l = 0; l < 4; ++l) {                                                 /* :339-360 */
            if (H.hit[l]) {
                V3 d = SFX(mk)(R.dx[l], R.dy[l], R.dz[l]);
                V3 p = SFX(mk)(H.px[l], H.py[l], H.pz[l]);
                V3 n = SFX(mk)(H.nx[l], H.ny[l], H.nz[l]);
                V3 nd;
                REAL att[3];
                SFX(scatter)(&S->mats[H.mat[l]], d, p, n, H.front[l], pix, R.sid[l], k, k0, k1, &nd, att);
                col.r[l] = col.r[l] * att[0]; col.g[l] = col.g[l] * att[1]; col.b[l] = col.b[l] * att[2];
                R.ox[l] = p.x; R.oy[l] = p.y; R.oz[l] = p.z;
                R.dx[l] = nd.x; R.dy[l] = nd.y; R.dz[l] = nd.z;
            } else {                                                                  /* :355-358 */
                R.en[l] = 0;
                sky[l] = 1;
            }
        }
    }
    for (int l = 0; l < 4; ++l) {   /* :365-370: sky from the FINAL direction of each lane */
        REAL sk[3];
        SFX(sky)(R.dy[l], sk);
        REAL cr = col.r[l], cg = col.g[l], cb = col.b[l];
        if (sky[l]) { cr = cr * sk[0]; cg = cg * sk[1]; cb = cb * sk[2]; }
        if (R.en[l]) { cr = 0; cg = 0; cb = 0; }
        out->r[l] = cr; out->g[l] = cg; out->b[l] = cb;
    }
}

/* ---- "scalar" mode: Sphere::hit (objects.rs:216-247), Scene::hit (ray_tracing.rs:231-235),
 * Scene::trace_rays (ray_tracing.rs:264-306) as called by TileRenderTask::render
 * (renderer.rs:68-100).  Scalar Vec3 arithmetic (no FMA), both roots, true division by a,
 * normal divided by the signed radius, the first minimum wins ties (min_by_key). ---- */
static int SFX(scene_hit_scalar)(const SFX(scene_r)* S, V3 o, V3 d, REAL* t_out, uint32_t* i_out) {
    int found = 0;
    REAL best = 0;
    for (uint32_t i = 0; i < S->n; ++i) {
        V3 oc = SFX(sub)(o, SFX(mk)(S->cx[i], S->cy[i], S->cz[i]));                   /* :217 */
        REAL a = SFX(len2)(d);                                                         /* :219 */
        REAL hb = SFX(dot)(oc, d);                                                     /* :220 */
        REAL c = SFX(len2)(oc) - S->r[i] * S->r[i];                                    /* :221 */
        REAL disc = hb * hb - a * c;                                                   /* :222 */
        if (disc < (REAL)0.0) continue;                                                /* :223-225 */
        REAL sd = SQRT(disc);
        REAL root = (-hb - sd) / a;                                                    /* :228 */
        if (!(root >= (REAL)0.001 && root < (REAL)INFINITY)) {                         /* :229-234 */
            root = (-hb + sd) / a;
            if (!(root >= (REAL)0.001 && root < (REAL)INFINITY)) continue;
        }
        if (!found || root < best) { best = root; *i_out = i; found = 1; }            /* min_by_key: first min */
    }
    *t_out = best;
    return found;
}

static void SFX(trace_ray_scalar)(const SFX(scene_r)* S, V3 o, V3 d, uint32_t depth, uint32_t pix, uint32_t sid,
                                  uint32_t k0, uint32_t k1, REAL out[3], uint64_t* segs) {
    REAL cr = 1, cg = 1, cb = 1;                                                       /* :266-269 */
    int alive = 1;
    for (uint32_t k = 0; k < depth && alive; ++k) {                                   /* :272-302 */
        *segs += 1;
        REAL t;
        uint32_t i;
        if (SFX(scene_hit_scalar)(S, o, d, &t, &i)) {
            V3 p = SFX(add)(o, SFX(mul)(d, t));                                        /* Ray::at, ray.rs:28-30 */
            V3 outw = SFX(dvs)(SFX(sub)(p, SFX(mk)(S->cx[i], S->cy[i], S->cz[i])), S->r[i]);   /* objects.rs:242 */
            int front = SFX(dot)(d, outw) < (REAL)0.0;                                /* HitRecord::new, objects.rs:69-73 */
            V3 n = front ? outw : SFX(neg)(outw);
            V3 nd;
            REAL att[3];
            SFX(scatter)(&S->mats[S->mat[i]], d, p, n, front, pix, sid, k, k0, k1, &nd, att);
            cr = cr * att[0]; cg = cg * att[1]; cb = cb * att[2];                      /* :280 */
            o = p; d = nd;
        } else {                                                                       /* :283-292 */
            REAL sk[3];
            SFX(sky)(d.y, sk);   /* 0.5*(y+1), (1-a)+a*k: the same values as the packed gradient */
            cr = cr * sk[0]; cg = cg * sk[1]; cb = cb * sk[2];
            alive = 0;
        }
    }
    if (alive) { cr = 0; cg = 0; cb = 0; }                                             /* :300-305 */
    out[0] = cr; out[1] = cg; out[2] = cb;
}

/* Color::to_u8_array (color.rs:54-64): sqrt gamma, *255.999, saturating `as u8`, NaN -> 0. */
static inline uint8_t SFX(q8)(REAL v) {
    REAL x = SQRT(v) * (REAL)255.999;
    if (!(x > (REAL)0.0)) return 0;      /* NaN and negatives */
    if (x >= (REAL)255.0) return 255;
    return (uint8_t)x;                    /* truncation toward zero */
}

typedef struct {
    const SFX(scene_r)* S;
    const SFX(cam_r)* cam;
    uint32_t depth, spp, flags, k0, k1;
    const uint32_t* pixels;
    uint32_t n_pixels;
    uint8_t* rgb; double* lin;
    volatile uint32_t next;   /* MPMC work counter (renderer.rs:251 tile queue) */
    uint64_t segs;
    int panic;
    pthread_mutex_t mu;
} SFX(job);

#define ORACLE_BLOCK 64u

static void* SFX(worker)(void* arg) {
    SFX(job)* J = (SFX(job)*)arg;
    const uint32_t C = (J->spp + 3u) / 4u;
    SFX(ws) w;
    if (!SFX(ws_init)(&w, C)) { SFX(ws_free)(&w); return NULL; }
    uint64_t segs = 0;
    int panic = 0;
    for (;;) {
        uint32_t b = __atomic_fetch_add(&J->next, ORACLE_BLOCK, __ATOMIC_RELAXED);
        if (b >= J->n_pixels) break;
        uint32_t e = b + ORACLE_BLOCK < J->n_pixels ? b + ORACLE_BLOCK : J->n_pixels;
        for (uint32_t idx = b; idx < e; ++idx) {
            uint32_t pix = J->pixels ? J->pixels[idx] : idx;
            uint32_t col = pix % J->cam->W, row = pix / J->cam->W;
            /* render_vectorized2, renderer.rs:155-159: spp camera rays chunked by 4; a partial
             * last chunk has its missing lanes disabled with zero origin/direction (ray.rs:136-153) */
            for (uint32_t j = 0; j < C; ++j) {
                SFX(prays)* P = &w.rays0[j];
                memset(P, 0, sizeof(*P));
                for (int l = 0; l < 4; ++l) {
                    uint32_t s = j * 4u + (uint32_t)l;
                    P->sid[l] = s;
                    if (s < J->spp) {
                        V3 o, d;
                        SFX(get_ray)(J->cam, col, row, pix, s, J->k0, J->k1, &o, &d);
                        P->ox[l] = o.x; P->oy[l] = o.y; P->oz[l] = o.z;
                        P->dx[l] = d.x; P->dy[l] = d.y; P->dz[l] = d.z;
                        P->en[l] = 1;
                    }
                }
            }
            REAL sum[3];
            if (J->flags & OR_FLAG_MODE_SCALAR) {
                /* render (renderer.rs:80-86): trace_rays then Color::average, summed in sample order */
                REAL acc[3] = {0, 0, 0};
                for (uint32_t s = 0; s < J->spp; ++s) {
                    const SFX(prays)* P = &w.rays0[s / 4u];
                    const int l = (int)(s % 4u);
                    REAL v[3];
                    SFX(trace_ray_scalar)(J->S, SFX(mk)(P->ox[l], P->oy[l], P->oz[l]), SFX(mk)(P->dx[l], P->dy[l], P->dz[l]),
                                          J->depth, pix, s, J->k0, J->k1, v, &segs);
                    acc[0] = acc[0] + v[0]; acc[1] = acc[1] + v[1]; acc[2] = acc[2] + v[2];   /* color.rs:74-79 */
                }
                sum[0] = acc[0]; sum[1] = acc[1]; sum[2] = acc[2];
            } else if (J->flags & OR_FLAG_MODE_VECTORIZED) {
                /* render_vectorized (renderer.rs:116-124): per-lane sum over chunks, then PackedColor::sum */
                REAL acc[3][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
                for (uint32_t j = 0; j < C; ++j) {
                    SFX(pcol) pc;
                    SFX(trace_chunk_v1)(J->S, w.rays0[j], J->depth, pix, J->k0, J->k1, J->flags, &pc, &segs);
                    for (int l = 0; l < 4; ++l) {
                        acc[0][l] = acc[0][l] + pc.r[l]; acc[1][l] = acc[1][l] + pc.g[l]; acc[2][l] = acc[2][l] + pc.b[l];
                    }
                }
                for (int ch = 0; ch < 3; ++ch)
                    sum[ch] = (((REAL)0.0 + acc[ch][0]) + acc[ch][1] + acc[ch][2]) + acc[ch][3];
            } else if (J->flags & OR_FLAG_MODE_VECTORIZED3) {
                SFX(trace_pixel_v3)(J->S, &w, J->depth, pix, J->k0, J->k1, J->flags, sum, &segs);
            } else {
                SFX(trace_pixel)(J->S, &w, J->depth, pix, J->k0, J->k1, J->flags, sum, &segs);
            }
            for (int ch = 0; ch < 3; ++ch) {
                REAL v = sum[ch] / (REAL)J->spp;                                      /* renderer.rs:161 */
                if (!(v <= (REAL)2.0)) panic = 1;                                     /* color.rs:55-57 */
                if (J->rgb) J->rgb[(size_t)idx * 3 + ch] = SFX(q8)(v);
                if (J->lin) J->lin[(size_t)idx * 3 + ch] = (double)v;
            }
        }
    }
    SFX(ws_free)(&w);
    pthread_mutex_lock(&J->mu);
    J->segs += segs;
    J->panic |= panic;
    pthread_mutex_unlock(&J->mu);
    return NULL;
}

int SFX(oracle_render)(const or_scene* sc, const or_camera* cam, uint32_t max_bounces,
                       uint32_t spp, uint64_t seed, uint32_t flags,
                       const uint32_t* pixels, uint32_t n_pixels,
                       uint8_t* rgb_out, double* lin_out, uint64_t* segments, int n_threads) {
    if (!sc || !cam || spp == 0 || cam->image_width == 0 || cam->image_height == 0) return 1;
    if (spp > (1u << 20)) return 4;                   /* SFX(draw)'s counters */
#if !ORACLE_IS_F64
    if (max_bounces > 3839u) return 4;                /* 257 + bounce < 2^12 (RT_MAX_BOUNCES_F32) */
#endif
    {
        const uint32_t modes = flags & (OR_FLAG_MODE_VECTORIZED | OR_FLAG_MODE_SCALAR | OR_FLAG_MODE_VECTORIZED3);
        if (modes & (modes - 1u)) return 1;   /* at most one mode */
    }
    if (sc->n_spheres && (!sc->center || !sc->radius || !sc->material || !sc->materials)) return 1;
    for (uint32_t i = 0; i < sc->n_spheres; ++i)
        if (sc->material[i] >= sc->n_materials) return 1;
    if (!pixels) n_pixels = cam->image_width * cam->image_height;
    SFX(scene_r) S;
    S.n = sc->n_spheres;
    S.cx = (REAL*)malloc(sizeof(REAL) * (S.n + 1));
    S.cy = (REAL*)malloc(sizeof(REAL) * (S.n + 1));
    S.cz = (REAL*)malloc(sizeof(REAL) * (S.n + 1));
    S.r = (REAL*)malloc(sizeof(REAL) * (S.n + 1));
    S.mat = sc->material;
    S.mats = (SFX(mat_r)*)malloc(sizeof(SFX(mat_r)) * (sc->n_materials + 1));
    for (uint32_t i = 0; i < S.n; ++i) {
        S.cx[i] = (REAL)sc->center[3 * i]; S.cy[i] = (REAL)sc->center[3 * i + 1];
        S.cz[i] = (REAL)sc->center[3 * i + 2]; S.r[i] = (REAL)sc->radius[i];
    }
    for (uint32_t i = 0; i < sc->n_materials; ++i) {
        const or_material* m = &sc->materials[i];
        SFX(mat_r)* o = &S.mats[i];
        o->kind = m->kind; o->hollow = m->hollow;
        o->ar = (REAL)m->albedo[0]; o->ag = (REAL)m->albedo[1]; o->ab = (REAL)m->albedo[2];
        o->fuzz = (REAL)m->fuzz; o->ior = (REAL)m->ior;
    }
    SFX(cam_r) C;
    C.W = cam->image_width; C.H = cam->image_height;
    C.center = SFX(mk)((REAL)cam->center[0], (REAL)cam->center[1], (REAL)cam->center[2]);
    C.ulc = SFX(mk)((REAL)cam->ulc[0], (REAL)cam->ulc[1], (REAL)cam->ulc[2]);
    C.vu = SFX(mk)((REAL)cam->vu[0], (REAL)cam->vu[1], (REAL)cam->vu[2]);
    C.vv = SFX(mk)((REAL)cam->vv[0], (REAL)cam->vv[1], (REAL)cam->vv[2]);
    C.du = SFX(mk)((REAL)cam->du[0], (REAL)cam->du[1], (REAL)cam->du[2]);
    C.dv = SFX(mk)((REAL)cam->dv[0], (REAL)cam->dv[1], (REAL)cam->dv[2]);

    SFX(job) J;
    memset(&J, 0, sizeof(J));
    J.S = &S; J.cam = &C; J.depth = max_bounces; J.spp = spp; J.flags = flags;
    J.k0 = (uint32_t)seed; J.k1 = (uint32_t)(seed >> 32);
    J.pixels = pixels; J.n_pixels = n_pixels; J.rgb = rgb_out; J.lin = lin_out;
    pthread_mutex_init(&J.mu, NULL);
    if (n_threads < 1) n_threads = 1;
    if (n_threads == 1) {
        SFX(worker)(&J);
    } else {
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
        for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, SFX(worker), &J);
        for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
        free(th);
    }
    pthread_mutex_destroy(&J.mu);
    free(S.cx); free(S.cy); free(S.cz); free(S.r); free(S.mats);
    if (segments) *segments = J.segs;
    return J.panic ? 3 : 0;
}
