// rt_device.hpp — device-side scalar math of the sample loop, generic over T = float | double.
//
// Every formula restates the reference's arithmetic (file:line cited) and must be compiled
// with -ffp-contract=off: an fma appears exactly where the reference writes mul_add
// (PackedVec3::length_squared / dot, geometry.rs:434-436,466-468; discriminant,
// objects.rs:257).  Division and sqrt are the correctly-rounded IEEE ops (hipcc default for
// f64; -fhip-fp32-correctly-rounded-divide-sqrt for f32), so the kernel computes the same
// bits as the CPU restatement in oracle/ for the same (seed, pixel, sample).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rt {

template <typename T> struct V3 { T x, y, z; };

template <typename T> __device__ __forceinline__ V3<T> mk(T x, T y, T z) { return V3<T>{x, y, z}; }
// Scalar Vec3 ops (geometry.rs:37-132): no FMA, sums left to right.
template <typename T> __device__ __forceinline__ V3<T> add(V3<T> a, V3<T> b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
template <typename T> __device__ __forceinline__ V3<T> sub(V3<T> a, V3<T> b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
template <typename T> __device__ __forceinline__ V3<T> mul(V3<T> a, T s) { return mk(a.x * s, a.y * s, a.z * s); }
template <typename T> __device__ __forceinline__ V3<T> dvs(V3<T> a, T s) { return mk(a.x / s, a.y / s, a.z / s); }
// a / |a| for fp32 (unit(), next_ray's normal): the compiler's correctly rounded division is
// div_scale x2, rcp, 6 FMAs, div_fmas, div_fixup per component; when v_div_scale would scale nothing and
// div_fixup has no special case to fix (every lane: 2^-20 <= len <= 2^20 and every |component| >= 2^-100,
// which bounds |a_i / len| by ~1 since |a_i| <= len), the same sequence without them gives the same bits,
// with the denominator's refined reciprocal shared by the three components.  Otherwise the full division.
template <> __device__ __forceinline__ V3<float> dvs(V3<float> a, float s) {
    const float mn = fminf(fminf(fabsf(a.x), fabsf(a.y)), fabsf(a.z));
    const bool ok = s >= 0x1.0p-20f && s <= 0x1.0p20f && mn >= 0x1.0p-100f;
    if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
        const float r0 = __builtin_amdgcn_rcpf(s);
        const float r1 = __builtin_fmaf(__builtin_fmaf(-s, r0, 1.0f), r0, r0);
        auto q = [&](float x) {
            const float m = x * r1;
            const float f3 = __builtin_fmaf(__builtin_fmaf(-s, m, x), r1, m);
            return __builtin_fmaf(__builtin_fmaf(-s, f3, x), r1, f3);
        };
        return mk(q(a.x), q(a.y), q(a.z));
    }
    return mk(a.x / s, a.y / s, a.z / s);
}
// sqrt, correctly rounded, of an argument known to be +-0, >= 2^-96, +inf, negative or NaN (never a tiny
// positive one): v_sqrt_f32 (within 1 ulp) and the compiler's own correction by the residuals of the two
// neighbours, without its scaling for arguments below 2^-96 and its special-value select (both no-ops
// here: 0, +inf and NaN come through the correction unchanged).  fp64: the library sqrt.
__device__ __forceinline__ float sqrt_nd(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __int_as_float(__float_as_int(s) - 1), sup = __int_as_float(__float_as_int(s) + 1);
    float r = __builtin_fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
    r = __builtin_fmaf(-sup, s, x) > 0.0f ? sup : r;
    return r;
}
__device__ __forceinline__ double sqrt_nd(double x) { return sqrt(x); }
// fp64 a / s, s > 0, for three components: the compiler's f64 division (div_scale x2, rcp, two Newton steps,
// the residual FMA, div_fmas, div_fixup) where div_scale scales nothing and div_fixup has nothing to fix
// (every lane: 2^-20 <= s <= 2^20 and every |a_i| >= 2^-100): the same operations, the reciprocal shared.
template <> __device__ __forceinline__ V3<double> dvs(V3<double> a, double s) {
    const double mn = fmin(fmin(fabs(a.x), fabs(a.y)), fabs(a.z));
    const bool ok = s >= 0x1.0p-20 && s <= 0x1.0p20 && mn >= 0x1.0p-100;
    if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
        double r = __builtin_amdgcn_rcp(s);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
        auto q = [&](double x) {
            const double m = x * r;
            return __builtin_fma(__builtin_fma(-s, m, x), r, m);
        };
        return mk(q(a.x), q(a.y), q(a.z));
    }
    return mk(a.x / s, a.y / s, a.z / s);
}
// sqrt(x), x = |v|^2 of a direction: the compiler's f64 sqrt (rsq, then Goldschmidt/Newton refinement) without
// its ldexp scaling for x < 2^-767 and its select for zero / inf, when every lane has 2^-100 <= x <= 2^100.
__device__ __forceinline__ double sqrt_len(double x) {
    if (__builtin_expect(__ballot(!(x >= 0x1.0p-100 && x <= 0x1.0p100)) == 0ull, 1)) {
        const double g0 = __builtin_amdgcn_rsq(x);
        double sq = x * g0, h = g0 * 0.5;
        const double r = __builtin_fma(-h, sq, 0.5);
        sq = __builtin_fma(sq, r, sq);
        const double d0 = __builtin_fma(-sq, sq, x);
        h = __builtin_fma(h, r, h);
        sq = __builtin_fma(d0, h, sq);
        const double d1 = __builtin_fma(-sq, sq, x);
        return __builtin_fma(d1, h, sq);
    }
    return sqrt(x);
}
// fp32: sqrt_nd when no lane holds a tiny positive argument (a wave ballot), else the library sqrtf -- the same
// correctly rounded value.  The library sequence is ~16 VALU ops, most of them single-issue (compares, selects,
// constant operands): unit() of every camera ray, the scatter's normal length and the hit test's sqrt(disc) take
// the short form (round 6, same-box C fp32 +1.2 %, E +0.4 %: profiles/r06/sqrt_len_nd_ab.txt).
__device__ __forceinline__ float sqrt_len(float x) {
    if (__builtin_expect(__ballot(x > 0.0f && x < 0x1.0p-96f) == 0ull, 1)) return sqrt_nd(x);
    return sqrtf(x);
}
template <typename T> __device__ __forceinline__ V3<T> neg(V3<T> a) { return mk(-a.x, -a.y, -a.z); }
template <typename T> __device__ __forceinline__ T dot(V3<T> a, V3<T> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename T> __device__ __forceinline__ T len2(V3<T> a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
template <typename T> __device__ __forceinline__ V3<T> unit(V3<T> a) { return dvs(a, sqrt_len(len2(a))); }
// Packed ops keep the reference's explicit FMA.
template <typename T> __device__ __forceinline__ T pk_len2(V3<T> a) { return fma(a.z, a.z, fma(a.y, a.y, a.x * a.x)); }
template <typename T> __device__ __forceinline__ T pk_dot(V3<T> a, V3<T> b) { return fma(a.z, b.z, fma(a.y, b.y, a.x * b.x)); }

// geometry.rs:134-137
template <typename T> __device__ __forceinline__ bool near_zero(V3<T> v) {
    const T e = T(1e-8);
    return fabs(v.x) < e && fabs(v.y) < e && fabs(v.z) < e;
}
// geometry.rs:179-181
template <typename T> __device__ __forceinline__ V3<T> reflect(V3<T> v, V3<T> n) { return sub(v, mul(n, T(2.0) * dot(v, n))); }
// geometry.rs:183-188
template <typename T> __device__ __forceinline__ V3<T> refract(V3<T> v, V3<T> n, T ratio) {
    T ct = fmin(dot(neg(v), n), T(1.0));
    V3<T> rperp = mul(add(v, mul(n, ct)), ratio);
    V3<T> rpar = mul(n, -(sqrt_nd(fabs(T(1.0) - len2(rperp)))));   // |1 - x| is 0 or >= 2^-24
    return add(rperp, rpar);
}

// ---- counter-based RNG: Philox4x32-10 keyed by (sample, pixel, bounce, stream) ----
struct U4 { uint32_t a, b, c, d; };
__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        // one v_mad_u64_u32 per 32x32->64 product (hi and lo together)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        // each three-way xor as one v_bitop3_b32 (gfx950 has no v_xor3_b32; the backend emits two v_xor)
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return U4{c0, c1, c2, c3};
}
// Philox2x32-10 (Random123's philox2x32, R = 10): one 32x32->64 product and one three-way xor per round.
__device__ __forceinline__ U4 philox2(uint32_t c0, uint32_t c1, uint32_t k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p = (uint64_t)0xD256D193u * c0;
        c0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p >> 32), c1, k, 0x96);
        c1 = (uint32_t)p;
        k += 0x9E3779B9u;
    }
    return U4{c0, c1, 0u, 0u};
}
// murmur3's 32-bit finaliser (a bijection with fmix32(0) = 0): folds the seed's high word into the fp32 key.
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
// One draw block for (sample, pixel, k, stream): stream 0 the camera jitter (k = 0), 1 disk try k, 2 the
// scatter at bounce k.  fp64 takes two 53-bit uniforms from Philox4x32-10, counter (sample, pixel, k,
// stream), key (k0, k1) = (seed lo, seed hi).  fp32 needs only two 24-bit uniforms, so it draws
// Philox2x32-10 with counter (pixel, sample | code << 20), code = 0 / 1 + k / 257 + k, and the 32-bit key
// k0 = seed lo ^ fmix32(seed hi), folded by the host (launch_t; k1 = 0 unused): half the multiplies (round 5,
// same-box C fp32 +1.9 %).  The host keeps the counter injective: spp <= 2^20 and, in fp32,
// max_bounces <= RT_MAX_BOUNCES_F32 (257 + k < 2^12).
template <typename T>
__device__ __forceinline__ U4 rng(uint32_t sid, uint32_t pix, uint32_t k, uint32_t stream, uint32_t k0, uint32_t k1) {
    if constexpr (sizeof(T) == 4) {
        const uint32_t code = stream == 0u ? 0u : (stream == 1u ? 1u + k : 257u + k);
        return philox2(pix, sid | (code << 20), k0);
    } else {
        return philox(sid, pix, k, stream, k0, k1);
    }
}
// Uniform [0,1): f64 from 53 bits of (a,b) / (c,d); f32 from 24 bits of a / b.
__device__ __forceinline__ double u01a(const U4& r, double) { return (double)((((uint64_t)r.a << 32) | r.b) >> 11) * 0x1.0p-53; }
__device__ __forceinline__ double u01b(const U4& r, double) { return (double)((((uint64_t)r.c << 32) | r.d) >> 11) * 0x1.0p-53; }
__device__ __forceinline__ float u01a(const U4& r, float) { return (float)(r.a >> 8) * 0x1.0p-24f; }
__device__ __forceinline__ float u01b(const U4& r, float) { return (float)(r.b >> 8) * 0x1.0p-24f; }

// sin/cos(2*pi*u): exact quadrant reduction in u-space + Taylor on [0, pi/4] by fma-Horner.
__device__ __forceinline__ void poly_sincos(double x2, double& ps, double& pc) {
    ps = 1.0 / 355687428096000.0;
    ps = fma(ps, x2, -1.0 / 1307674368000.0);
    ps = fma(ps, x2, 1.0 / 6227020800.0);
    ps = fma(ps, x2, -1.0 / 39916800.0);
    ps = fma(ps, x2, 1.0 / 362880.0);
    ps = fma(ps, x2, -1.0 / 5040.0);
    ps = fma(ps, x2, 1.0 / 120.0);
    ps = fma(ps, x2, -1.0 / 6.0);
    pc = -1.0 / 6402373705728000.0;
    pc = fma(pc, x2, 1.0 / 20922789888000.0);
    pc = fma(pc, x2, -1.0 / 87178291200.0);
    pc = fma(pc, x2, 1.0 / 479001600.0);
    pc = fma(pc, x2, -1.0 / 3628800.0);
    pc = fma(pc, x2, 1.0 / 40320.0);
    pc = fma(pc, x2, -1.0 / 720.0);
    pc = fma(pc, x2, 1.0 / 24.0);
    pc = fma(pc, x2, -1.0 / 2.0);
}
__device__ __forceinline__ void poly_sincos(float x2, float& ps, float& pc) {
    ps = (float)(1.0 / 362880.0);
    ps = fmaf(ps, x2, (float)(-1.0 / 5040.0));
    ps = fmaf(ps, x2, (float)(1.0 / 120.0));
    ps = fmaf(ps, x2, (float)(-1.0 / 6.0));
    pc = (float)(-1.0 / 3628800.0);
    pc = fmaf(pc, x2, (float)(1.0 / 40320.0));
    pc = fmaf(pc, x2, (float)(-1.0 / 720.0));
    pc = fmaf(pc, x2, (float)(1.0 / 24.0));
    pc = fmaf(pc, x2, (float)(-1.0 / 2.0));
}
template <typename T> __device__ __forceinline__ void sincos2pi(T u, T& so, T& co) {
    const T t = u * T(4.0);
    const int q = (int)t;
    const T f = t - (T)q;
    const bool sw = f > T(0.5);
    const T g = sw ? T(1.0) - f : f;
    const T x = g * T(1.5707963267948966);
    const T x2 = x * x;
    T ps, pc;
    poly_sincos(x2, ps, pc);
    const T s = fma(x * x2, ps, x);
    const T c = fma(x2, pc, T(1.0));
    // quadrant q (0..3) of the un-swapped (s, c): sin = q odd ? c : s, negated for q & 2; cos = q odd ? s : c,
    // negated for (q + 1) & 2 -- the octant swap sw toggles the choice.  Branch-free: two selects, two sign xors.
    const uint32_t qs = (uint32_t)q << 30;                  // bit 31: q & 2, bit 30: q & 1
    const bool swp = sw != ((qs & 0x40000000u) != 0u);
    const T sm = swp ? c : s, cm = swp ? s : c;
    if constexpr (sizeof(T) == 4) {
        so = __uint_as_float(__float_as_uint(sm) ^ (qs & 0x80000000u));
        co = __uint_as_float(__float_as_uint(cm) ^ ((qs + 0x40000000u) & 0x80000000u));
    } else {
        so = __longlong_as_double(__double_as_longlong(sm) ^ ((long long)(qs & 0x80000000u) << 32));
        co = __longlong_as_double(__double_as_longlong(cm) ^ ((long long)((qs + 0x40000000u) & 0x80000000u) << 32));
    }
}
// Uniform direction on S^2: the distribution of Vec3::random_unit_vector (geometry.rs:139-152).
template <typename T> __device__ __forceinline__ V3<T> unit_vec(T u1, T u2) {
    const T z = T(1.0) - T(2.0) * u1;
    const T r = sqrt_nd(T(1.0) - z * z);   // z = 1 - 2 u1: 1 - z^2 is 0 or >= 2^-24
    T s, c;
    sincos2pi(u2, s, c);
    return mk(r * c, r * s, z);
}

// Sky gradient of trace_vectorized2's final pass (ray_tracing.rs:490-494).
template <typename T> __device__ __forceinline__ V3<T> sky(T y) {
    const T a = (y + T(1.0)) * T(0.5);
    const T oma = -a + T(1.0);
    return mk(T(1.0) * oma + T(0.5) * a, T(1.0) * oma + T(0.7) * a, T(1.0) * oma + T(1.0) * a);
}

// Color::to_u8_array (color.rs:54-64): sqrt gamma, *255.999, saturating `as u8` (NaN -> 0).
template <typename T> __device__ __forceinline__ uint8_t q8(T v) {
    const T x = sqrt(v) * T(255.999);
    if (!(x > T(0.0))) return 0;
    if (x >= T(255.0)) return 255;
    return (uint8_t)x;
}

}  // namespace rt
