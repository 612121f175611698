/*
 * oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's live
 * packed path, the parity checker and timed CPU baseline.  See oracle.h for the
 * parity status ("parity unpinned" w.r.t. the real Rust binary) and
 * oracle_impl.h for the per-function file:line citations.
 *
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off -fno-math-errno).
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
 * SC'11; Random123 philox4x32 with R = 10): multipliers 0xD2511F53/0xCD9E8D57,
 * Weyl key bumps 0x9E3779B9/0xBB67AE85. */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int i = 0; i < 10; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Philox2x32-10 (Random123 philox2x32 with R = 10): multiplier 0xD256D193, Weyl key bump 0x9E3779B9;
 * round: hi:lo = M * c0, (c0, c1) <- (hi ^ key ^ c1, lo).  The fp32 build's draws (oracle_impl.h SFX(draw),
 * rt_device.hpp rng<float>). */
void oracle_philox2x32_10(const uint32_t ctr[2], uint32_t key, uint32_t out[2]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], k = key;
    for (int i = 0; i < 10; ++i) {
        uint64_t p = (uint64_t)0xD256D193u * c0;
        uint32_t n0 = (uint32_t)(p >> 32) ^ k ^ c1;
        c1 = (uint32_t)p;
        c0 = n0;
        k += 0x9E3779B9u;
    }
    out[0] = c0; out[1] = c1;
}

/* murmur3's 32-bit finaliser (a bijection, fmix32(0) = 0): the fp32 build keys Philox2x32-10 with
 * seed lo ^ fmix32(seed hi) (rt_device.hpp fmix32), so that the 64-bit seed is not folded by a plain xor. */
uint32_t oracle_fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}

/* ---------------- f64 instantiation (the reference's arithmetic) ---------------- */
#define REAL double
#define SFX(x) x##_f64
#define FMA fma
#define SQRT sqrt
#define FABS fabs
#define FMIN fmin
#define ORACLE_IS_F64 1
#include "oracle_impl.h"
#undef REAL
#undef SFX
#undef FMA
#undef SQRT
#undef FABS
#undef FMIN
#undef ORACLE_IS_F64
#undef V3

/* ---------------- f32 instantiation (same algorithm in float) ---------------- */
#define REAL float
#define SFX(x) x##_f32
#define FMA fmaf
#define SQRT sqrtf
#define FABS fabsf
#define FMIN fminf
#define ORACLE_IS_F64 0
#include "oracle_impl.h"

/* ---------------- probes for known-answer tests ---------------- */
void oracle_sincos2pi_f64(double u, double* s, double* c) { sincos2pi_f64(u, s, c); }

void oracle_to_u8(const double rgb[3], uint8_t out[3], int* panics) {
    *panics = 0;
    for (int i = 0; i < 3; ++i) {
        if (!(rgb[i] <= 2.0)) *panics = 1;   /* color.rs:55-57 assert */
        out[i] = q8_f64(rgb[i]);
    }
}

static cam_r_f64 cam_to_r64(const or_camera* cam) {
    cam_r_f64 C;
    C.W = cam->image_width; C.H = cam->image_height;
    C.center = mk_f64(cam->center[0], cam->center[1], cam->center[2]);
    C.ulc = mk_f64(cam->ulc[0], cam->ulc[1], cam->ulc[2]);
    C.vu = mk_f64(cam->vu[0], cam->vu[1], cam->vu[2]);
    C.vv = mk_f64(cam->vv[0], cam->vv[1], cam->vv[2]);
    C.du = mk_f64(cam->du[0], cam->du[1], cam->du[2]);
    C.dv = mk_f64(cam->dv[0], cam->dv[1], cam->dv[2]);
    return C;
}

void oracle_get_ray_f64(const or_camera* cam, uint32_t col, uint32_t row, uint32_t sample,
                        uint64_t seed, double origin[3], double dir[3]) {
    cam_r_f64 C = cam_to_r64(cam);
    v3_f64 o, d;
    get_ray_f64(&C, col, row, row * cam->image_width + col, sample, (uint32_t)seed,
                (uint32_t)(seed >> 32), &o, &d);
    origin[0] = o.x; origin[1] = o.y; origin[2] = o.z;
    dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
}

/* Camera::new, ray_tracing.rs:27-62 (f64; Vec3 ops without FMA). */
int oracle_camera_new(or_camera* out, uint32_t w, uint32_t h, double focal_length,
                      double view_angle_deg, const double center[3], const double look_at[3],
                      const double up[3], double defocus_angle_deg) {
    if (!out || w == 0 || h == 0) return 1;
    const double deg = 3.141592653589793 / 180.0;                      /* f64::to_radians */
    double aspect = (double)w / (double)h;                              /* :28 */
    double vh = tan((view_angle_deg * deg) / 2.0) * focal_length * 2.0; /* :29 */
    double vw = vh * aspect;                                            /* :32 */
    v3_f64 C = mk_f64(center[0], center[1], center[2]);
    v3_f64 L = mk_f64(look_at[0], look_at[1], look_at[2]);
    v3_f64 U = mk_f64(up[0], up[1], up[2]);
    v3_f64 dir = unit_f64(sub_f64(L, C));                               /* :34 */
    v3_f64 wv = neg_f64(dir);                                           /* :35 */
    v3_f64 cr = mk_f64(U.y * wv.z - U.z * wv.y, U.z * wv.x - U.x * wv.z, U.x * wv.y - U.y * wv.x);
    v3_f64 u = unit_f64(cr);                                            /* :36 */
    v3_f64 v = mk_f64(wv.y * u.z - wv.z * u.y, wv.z * u.x - wv.x * u.z, wv.x * u.y - wv.y * u.x); /* :37 */
    v3_f64 vu = mul_f64(u, vw);                                         /* :39 */
    v3_f64 vv = mul_f64(neg_f64(v), vh);                                /* :40 */
    v3_f64 ulc = sub_f64(sub_f64(sub_f64(C, mul_f64(wv, focal_length)), dvs_f64(vu, 2.0)), dvs_f64(vv, 2.0)); /* :41 */
    double dr = focal_length * tan((defocus_angle_deg / 2.0) * deg);    /* :43 */
    v3_f64 du = mul_f64(u, dr);                                         /* :44 */
    v3_f64 dv = mul_f64(v, dr);                                         /* :45 */
    out->image_width = w; out->image_height = h;
    out->center[0] = C.x; out->center[1] = C.y; out->center[2] = C.z;
    out->ulc[0] = ulc.x; out->ulc[1] = ulc.y; out->ulc[2] = ulc.z;
    out->vu[0] = vu.x; out->vu[1] = vu.y; out->vu[2] = vu.z;
    out->vv[0] = vv.x; out->vv[1] = vv.y; out->vv[2] = vv.z;
    out->du[0] = du.x; out->du[1] = du.y; out->du[2] = du.z;
    out->dv[0] = dv.x; out->dv[1] = dv.y; out->dv[2] = dv.z;
    return 0;
}

/* ---------------- the reference-shaped packed CPU baseline (explicit AVX2, 128x128 tiles) ---------------- */
#include "packed_avx2.h"
