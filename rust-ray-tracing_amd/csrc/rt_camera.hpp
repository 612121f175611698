// rt_camera.hpp — primary rays: the wave-level cone cull of camera batches, the per-pixel camera
// candidate lists, the per-launch camera-origin tables, and next_ray (Camera::get_ray,
// ray_tracing.rs:77-89; PackedHitRecords::finalize + Material::get_hit_result, objects.rs:157-162,
// materials.rs:54-147).
#pragma once
#include "rt_common.hpp"

namespace rt {

// Camera-batch sweep with a wave-level cone cull (pinhole cameras; called by the whole wave, lanes
// `v` carry a primary ray d from the camera centre).  The batch's rays all start at the centre O, so
// they lie in the cone with apex O, axis a (the first ray's direction) and half-angle theta, where
// sin(theta) = max over the batch of |d^ x a| (fp32, inflated by 8 u + 4 u relative).  A sphere can
// only be hit by a ray of the batch if it meets that cone: with w = c - O, t = w.a and p = |w x a|,
// the signed distance from the centre to the cone's generator line in the plane of a and w is
// p cos(theta) - t sin(theta) (<= the distance to the cone), so the cull passes the sphere unless it
// exceeds rp.  rp (build_cam_table) = sqrt(r^2 (1 + 2^-20) + 64 u |w|^2) + 32 u |w|: the first term
// covers the reference's own rounding of the discriminant (a sphere whose computed disc >= 0 lies
// at most sqrt(r^2 + ~10 u |w|^2) from the ray's line, the same bound as the per-lane filters'), the
// second the fp32 rounding of w, t, p, a and theta (~10 u |w|).  Lanes as spheres: one coalesced
// 16-byte load and ~16 VALU per 64 spheres, then the exact test (objects.rs:252-257 on the
// camera-origin table, bit-identical to the per-ray values) for the passing spheres only, in scene
// order, so ties and the nearest hit are the reference's.  A batch whose rays spread over more than
// ~30 degrees (tiny images) skips the cull and tests every sphere exactly.
// Two levels over the sweep layout (build_layout): the always-exact spheres lane by lane, then the
// clusters lane by lane against cluster records whose rp bounds every member's (the cone distance is
// 1-Lipschitz in the centre, and rp_k >= rp_i + |c_i - C| for every member, build_cam_table), then
// the members of the passing clusters.
__device__ __forceinline__ float ufl(float x) { return __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(x))); }

// Wave-wide max of a uint32 through DPP (row_shr scans within each row of 16, then row_bcast:15 and
// row_bcast:31 carry the row maxima to lane 63): six v_max_u32 with DPP sources, no LDS round trips.
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));   // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

// Wave-wide inclusive prefix sum of a uint32 through DPP (Hillis-Steele within each row of 16 with
// zero fill, then row_bcast:15 / row_bcast:31 carry the row totals upwards).
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

// The cone cull over the sweep layout (whole wave, wave-uniform control flow): calls pass(sl) for every
// sphere slot whose cone-cull record {w = c - O, rp} the cone with axis a, sin S and cos Cc does not
// cull (all: every record passes).  Returns the wave-level cone tests run.  xw0, kw0: the first
// records of both levels, loaded by the caller before the cone's setup.
template <bool MEGA, typename KP, typename F>
__device__ __forceinline__ uint32_t cone_walk(const KP& q, float ax, float ay, float az, float S, float Cc, bool all,
                                              const float4& xw0, const float4& kw0, F&& pass) {
    const uint32_t lane = threadIdx.x & 63u;
    const float4* cs = (const float4*)__builtin_assume_aligned(q.cull, 16);    // per slot (sweep layout)
    const float4* cc = (const float4*)__builtin_assume_aligned(q.cullc, 16);   // per cluster
    const uint32_t nx = 4u * q.n_xg, ncl = 4u * q.n_top;
    // cone test of a record {w = c - O, rp}; padding records (rp = -inf) never pass
    auto cone = [&](const float4& wc) -> bool {
        const float t = __builtin_fmaf(wc.z, az, __builtin_fmaf(wc.y, ay, wc.x * ax));
        const float px = __builtin_fmaf(wc.y, az, -(wc.z * ay)), py = __builtin_fmaf(wc.z, ax, -(wc.x * az)),
                    pz = __builtin_fmaf(wc.x, ay, -(wc.y * ax));
        const float pp = __builtin_amdgcn_sqrtf(__builtin_fmaf(pz, pz, __builtin_fmaf(py, py, px * px)));
        const float f = __builtin_fmaf(pp, Cc, -(t * S));
        // NaN f passes.  Bitwise, so the record is one 16-byte load: `&&` loaded w, waited and branched before
        // loading x, y, z (C fp32 +0.25 %, fp64 +0.4 %, E +0.35 %: profiles/r05/cone_load_ab.txt)
        return (wc.w > -INFINITY) & (all | !(f > wc.w));
    };
    uint32_t n_cone = 0;
    // 1. the always-exact spheres (build_layout's leading slots), lanes as spheres
    for (uint32_t base = 0; base < nx; base += 64u) {
        ++n_cone;
        unsigned long long m = __ballot(base + lane < nx && cone(base == 0 ? xw0 : cs[base + lane]));
        while (m != 0ull) {
            const uint32_t sl = base + (uint32_t)__builtin_ctzll(m);
            m &= m - 1ull;
            pass(sl);
        }
    }
    // 2. clusters: lanes as clusters (records bound every member's record), then the members of up
    // to 4 passing clusters per pass, 16 lanes each.  M: ballot of a cluster test in which lane L
    // tested cluster klane(L).
    auto members = [&](unsigned long long M, uint32_t klane) {
        while (M != 0ull) {
            ++n_cone;
            uint32_t k[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {   // empty quarters take the padding cluster ncl (all dummies)
                k[j] = M != 0ull ? (uint32_t)__builtin_amdgcn_readlane(klane, (int)__builtin_ctzll(M)) : ncl;
                M &= M - 1ull;
            }
            const uint32_t qd = lane >> 4;
            const uint32_t kl = qd == 0 ? k[0] : qd == 1 ? k[1] : qd == 2 ? k[2] : k[3];
            unsigned long long m = __ballot(cone(cs[nx + 16u * kl + (lane & 15u)]));
            while (m != 0ull) {
                const uint32_t b = (uint32_t)__builtin_ctzll(m);
                m &= m - 1ull;
                const uint32_t kb = (b >> 4) == 0 ? k[0] : (b >> 4) == 1 ? k[1] : (b >> 4) == 2 ? k[2] : k[3];
                pass(nx + 16u * kb + (b & 15u));
            }
        }
    };
    const uint32_t nsu = MEGA ? q.n_supc : 0u;   // the super level exists only in the MEGA kernels
    if (nsu == 0u) {
        for (uint32_t cb = 0; cb < ncl; cb += 64u) {
            ++n_cone;
            members(__ballot(cone(cb == 0 ? kw0 : cc[cb + lane])), cb + lane);   // padded to whole 64s
        }
    } else {
        // big scenes: lanes as supers first (their records, after the clusters', bound every member
        // sphere's record the same way), then the 4 clusters of up to 16 passing supers per pass
        const float4* csu = cc + q.n_clp;
        for (uint32_t sb = 0; sb < nsu; sb += 64u) {
            ++n_cone;
            unsigned long long SM = __ballot(cone(csu[sb + lane]));   // padded to whole 64s (rp = -inf)
            while (SM != 0ull) {
                uint32_t mys = 0xFFFFFFFFu;
                for (uint32_t j = 0; j < 16u && SM != 0ull; ++j) {
                    const uint32_t sj = sb + (uint32_t)__builtin_ctzll(SM);
                    SM &= SM - 1ull;
                    if ((lane >> 2) == j) mys = sj;
                }
                const bool have = mys != 0xFFFFFFFFu;
                const uint32_t kl = have ? 4u * mys + (lane & 3u) : ncl;
                ++n_cone;
                members(__ballot(have && cone(cc[kl])), kl);
            }
        }
    }
    return n_cone;
}

// The reference's exact test (objects.rs:252-257 on the camera-origin table) of sphere slot sl for the
// camera rays of lanes v; the scene index (hit_update's tie rule and the result) comes with it.
template <typename T, bool root2, bool SCALAR, typename KP>
__device__ __forceinline__ void camera_exact(const KP& q, uint32_t sl, bool v, const V3<T>& d, T a, T inv_a,
                                             HitBest<T>& bh) {
    KSTAT(2);
    constexpr bool kBothRoots = root2 || SCALAR;
    cptr<T> cxt = (cptr<T>)__builtin_assume_aligned(q.camx, 16);
    cptr<uint32_t> ri = (cptr<uint32_t>)q.ridx;
    const uint32_t i = ri[sl];
    const T ocx = cxt[4 * sl], ocy = cxt[4 * sl + 1], ocz = cxt[4 * sl + 2], c = cxt[4 * sl + 3];
    if (v) {
        T hb, disc;
        if constexpr (SCALAR) {   // objects.rs:217-222
            hb = (ocx * d.x + ocy * d.y) + ocz * d.z;
            disc = hb * hb - a * c;
        } else {                  // objects.rs:255, 257
            hb = fma(ocz, d.z, fma(ocy, d.y, ocx * d.x));
            disc = fma(hb, hb, (-a) * c);
        }
        if (kBothRoots ? disc >= T(0.0) : (disc >= T(0.0) && hb <= T(0.0)))
            hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, bh);
    }
}

template <typename T, bool root2, bool SCALAR, bool MEGA = false>
__device__ __forceinline__ int camera_sweep(bool v, const V3<T>& d, T& t_out) {
    const uint32_t lane = threadIdx.x & 63u;
    const unsigned long long vm = __ballot(v);
    // the first records of both levels do not depend on the cone: request them before its setup
    const auto& q = *cold_args<T>();
    const float4* cs = (const float4*)__builtin_assume_aligned(q.cull, 16);    // per slot (sweep layout)
    const float4* cc = (const float4*)__builtin_assume_aligned(q.cullc, 16);   // per cluster
    const uint32_t nx = 4u * q.n_xg, ncl = 4u * q.n_top;
    const float4 kPad = {0.0f, 0.0f, 0.0f, -INFINITY};
    const float4 xw0 = lane < nx ? cs[lane] : kPad, kw0 = lane < ncl ? cc[lane] : kPad;
    const float fdx = v ? (float)d.x : 0.0f, fdy = v ? (float)d.y : 0.0f, fdz = v ? (float)d.z : 0.0f;
    const int l0 = (int)__builtin_ctzll(vm);
    float ax = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(fdx), l0));
    float ay = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(fdy), l0));
    float az = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(fdz), l0));
    // v_rsq / v_rcp (1 ulp) below: the cone's sin is inflated by 4 u relative + 8 u, and a's length
    // error scales t and p alike (covered by rp's 32 u |w|)
    const float ia = __builtin_amdgcn_rsqf(__builtin_fmaf(az, az, __builtin_fmaf(ay, ay, ax * ax)));
    // wave-uniform: keep the axis and the cone's (cos, sin) in SGPRs
    ax = ufl(ax * ia);
    ay = ufl(ay * ia);
    az = ufl(az * ia);
    // sin^2 of each ray's angle to the axis: |d^ x a|^2 / |d^|^2 (0 for idle lanes)
    const float cx = __builtin_fmaf(fdy, az, -(fdz * ay)), cy = __builtin_fmaf(fdz, ax, -(fdx * az)),
                cz = __builtin_fmaf(fdx, ay, -(fdy * ax));
    const float dn2 = __builtin_fmaf(fdz, fdz, __builtin_fmaf(fdy, fdy, fdx * fdx));
    const float s2 = v ? __builtin_fmaf(cz, cz, __builtin_fmaf(cy, cy, cx * cx)) * __builtin_amdgcn_rcpf(dn2) * (1.0f + 0x1.0p-22f) : 0.0f;
    const float dt = __builtin_fmaf(fdz, az, __builtin_fmaf(fdy, ay, fdx * ax));
    bool all = __ballot(v && !(dt > 0.5f)) != 0ull;   // some ray > 60 deg off the axis (or NaN)
    // non-negative floats (and NaN above +inf) order as integers
    const uint32_t sm = wave_max_dpp(__float_as_uint(s2));
    // v_sqrt_f32 (1 ulp) for the cone's sin, cos and each record's p: 2 u relative each, inside the
    // 4 u inflation of sin and rp's 32 u |w| (tests/cone_cull_fuzz.c models them as +-1 ulp)
    const float S = ufl(__builtin_fmaf(__builtin_amdgcn_sqrtf(__uint_as_float(sm)), 1.0f + 0x1.0p-22f, 0x1.0p-21f));
    if (!(S < 0.5f)) all = true;
    const float Cc = ufl(__builtin_amdgcn_sqrtf(__builtin_fmaf(-S, S, 1.0f)));
    const T a = SCALAR ? len2(d) : pk_len2(d);       // objects.rs:219 / :253
    const T inv_a = SCALAR ? T(0) : T(1.0) / a;      // objects.rs:254
    HitBest<T> bh;
    KSTAT(3);
    uint32_t n_cx = 0;   // executed-work counts (work_add below)
    const uint32_t n_cone = cone_walk<MEGA>(q, ax, ay, az, S, Cc, all, xw0, kw0, [&](uint32_t sl) {
        ++n_cx;
        camera_exact<T, root2, SCALAR>(q, sl, v, d, a, inv_a, bh);
    });
    work_add(kWCone, n_cone);
    work_add(kWCExact, n_cx);
    t_out = bh.bt();
    return bh.bi();
}

// Per-pixel camera candidate lists (camera batches): every primary ray of pixel (col, row) starts at
// the camera centre O and points into the pixel's footprint, the parallelogram ulc + vu (col + x) / W
// + vv (row + y) / H, x, y in [0, 1] (ray_tracing.rs:80-84).  Its directions form a convex set whose
// largest angle from the axis (the direction to the footprint's centre) is taken at a corner, so the
// cone with that axis and sin S = max over the 4 corners of |D x a| / |D| (fp32, inflated like the
// batch cone: 4 u relative + 8 u) contains every exactly computed ray.  The pixel margin 2^-20 M / |Dc|
// (M = |ulc|_1 + |vu|_1 + |vv|_1 + |centre|_1, Dc the centre's direction) covers the rounding of the
// corners here and of the rays themselves in T, which grows with the coordinates' magnitudes over the
// focal distance (tests/pixel_cone_fuzz.c: every computed ray inside, worst case 7 % of the margin).
// The cone walk runs ONCE per pixel, when its slot opens, and records the passing sphere slots (at most
// kCList - 1; more, a cone over 60 degrees, or a slot index past u16: list[0] = 0xFFFF, and the
// pixel's batches run the per-batch camera_sweep instead).  A batch then runs the exact test of the
// listed spheres of its pixels only: for a lane, the union of its batch's lists holds every sphere its
// ray can hit, and extra exact tests never change a result.
constexpr uint32_t kCList = 8;
template <typename T, bool MEGA>
__device__ __forceinline__ uint32_t pixel_list(uint32_t col, uint32_t row, uint16_t* list) {
    const uint32_t lane = threadIdx.x & 63u;
    const auto& q = *cold_args<T>();
    const float4* cs = (const float4*)__builtin_assume_aligned(q.cull, 16);
    const float4* cc = (const float4*)__builtin_assume_aligned(q.cullc, 16);
    const uint32_t nx = 4u * q.n_xg, ncl = 4u * q.n_top;
    const float4 kPad = {0.0f, 0.0f, 0.0f, -INFINITY};
    const float4 xw0 = lane < nx ? cs[lane] : kPad, kw0 = lane < ncl ? cc[lane] : kPad;
    // lanes 0..3: the footprint's corners, lane 4 its centre (fp32)
    const float fx = lane < 4u ? (float)(lane & 1u) : 0.5f, fy = lane < 4u ? (float)(lane >> 1) : 0.5f;
    const float s1 = ((float)col + fx) / (float)q.W, s2 = ((float)row + fy) / (float)q.H;
    const float Dx = ((float)q.ulc[0] + ((float)q.vu[0] * s1 + (float)q.vv[0] * s2)) - (float)q.center[0];
    const float Dy = ((float)q.ulc[1] + ((float)q.vu[1] * s1 + (float)q.vv[1] * s2)) - (float)q.center[1];
    const float Dz = ((float)q.ulc[2] + ((float)q.vu[2] * s1 + (float)q.vv[2] * s2)) - (float)q.center[2];
    float ax = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(Dx), 4));
    float ay = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(Dy), 4));
    float az = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(Dz), 4));
    const float ia = __builtin_amdgcn_rsqf(__builtin_fmaf(az, az, __builtin_fmaf(ay, ay, ax * ax)));
    ax = ufl(ax * ia);
    ay = ufl(ay * ia);
    az = ufl(az * ia);
    const float cx = __builtin_fmaf(Dy, az, -(Dz * ay)), cy = __builtin_fmaf(Dz, ax, -(Dx * az)),
                cz = __builtin_fmaf(Dx, ay, -(Dy * ax));
    const float dn2 = __builtin_fmaf(Dz, Dz, __builtin_fmaf(Dy, Dy, Dx * Dx));
    const bool corner = lane < 4u;
    const float s2c = corner ? __builtin_fmaf(cz, cz, __builtin_fmaf(cy, cy, cx * cx)) * __builtin_amdgcn_rcpf(dn2) * (1.0f + 0x1.0p-22f) : 0.0f;
    const float dt = (__builtin_fmaf(Dz, az, __builtin_fmaf(Dy, ay, Dx * ax))) * __builtin_amdgcn_rsqf(dn2);
    bool over = __ballot(corner && !(dt > 0.5f)) != 0ull;   // a corner > 60 deg off the axis (or NaN)
    const uint32_t sm = wave_max_dpp(__float_as_uint(s2c));
    float M = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        M += ((fabsf((float)q.ulc[k]) + fabsf((float)q.vu[k])) + fabsf((float)q.vv[k])) + fabsf((float)q.center[k]);
    const float dnc = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(dn2), 4));
    const float margin = (M * 0x1.0p-20f) * __builtin_amdgcn_rsqf(dnc);
    const float S = ufl(__builtin_fmaf(__builtin_amdgcn_sqrtf(__uint_as_float(sm)), 1.0f + 0x1.0p-22f, 0x1.0p-21f + margin));
    if (!(S < 0.5f)) over = true;
    const float Cc = ufl(__builtin_amdgcn_sqrtf(__builtin_fmaf(-S, S, 1.0f)));
    uint32_t n = 0;
    uint32_t n_cone = 0;
    if (!over) {
        n_cone = cone_walk<MEGA>(q, ax, ay, az, S, Cc, false, xw0, kw0, [&](uint32_t sl) {
            if (sl >= 0xFFFFu) over = true;
            else if (n + 1u < kCList && lane == 0) list[1u + n] = (uint16_t)sl;
            ++n;
        });
    }
    if (over || n + 1u > kCList) n = 0xFFFFu;
    if (lane == 0) list[0] = (uint16_t)n;
    work_add(kWCone, n_cone);
    return n;
}

// A camera batch against its pixels' candidate lists (slots in smask): the exact test of every listed
// sphere for every lane (a lane of one pixel also tests the other pixel's spheres: extra exact tests
// never change a result).
template <typename T, bool root2, bool SCALAR>
__device__ __forceinline__ int camera_listed(bool v, const V3<T>& d, T& t_out, const uint16_t (*lists)[kCList],
                                             uint32_t smask) {
    const auto& q = *cold_args<T>();
    const T a = SCALAR ? len2(d) : pk_len2(d);       // objects.rs:219 / :253
    const T inv_a = SCALAR ? T(0) : T(1.0) / a;      // objects.rs:254
    HitBest<T> bh;
    uint32_t n_cx = 0;
    // fp64: the whole list in one 16-byte LDS read (entries unpacked from SGPRs), and the next listed
    // sphere's camera-origin record and scene index requested while the current one is tested (C fp64
    // +0.5 %).  fp32 keeps one LDS read and one record load per entry (the pipeline's SGPRs cost its W6
    // kernel 0.4 %: profiles/r05/clist_pipe_ab.txt).
    if constexpr (sizeof(T) == 8) {
        cptr<T> cxt = (cptr<T>)__builtin_assume_aligned(q.camx, 16);
        cptr<uint32_t> ri = (cptr<uint32_t>)q.ridx;
        struct CX { uint32_t i; T ox, oy, oz, c; };
        auto fetch = [&](uint32_t sl) -> CX { return CX{ri[sl], cxt[4 * sl], cxt[4 * sl + 1], cxt[4 * sl + 2], cxt[4 * sl + 3]}; };
        constexpr bool kBothRoots = root2 || SCALAR;
        for (; smask != 0u; smask &= smask - 1u) {
            uint4 w;   // the whole list: n, then up to 7 slots (memcpy: no type-punned read of the u16 entries)
            __builtin_memcpy(&w, __builtin_assume_aligned(lists[__builtin_ctz(smask)], 16), sizeof(w));
            const uint32_t w0 = __builtin_amdgcn_readfirstlane(w.x), w1 = __builtin_amdgcn_readfirstlane(w.y),
                           w2 = __builtin_amdgcn_readfirstlane(w.z), w3 = __builtin_amdgcn_readfirstlane(w.w);
            const uint32_t n = w0 & 0xFFFFu;
            auto entry = [&](uint32_t j) -> uint32_t {   // list[j], 1 <= j < kCList
                const uint32_t ww = j < 2u ? w0 : (j < 4u ? w1 : (j < 6u ? w2 : w3));
                return (ww >> (16u * (j & 1u))) & 0xFFFFu;
            };
            if (n == 0u) continue;
            CX cur = fetch(entry(1u));
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_sched_barrier(0);
            for (uint32_t j = 0; j < n; ++j) {
                ++n_cx;
                // the next listed sphere's record (this one's again past the end: never unused entries)
                const CX nxt = fetch(j + 1u < n ? entry(j + 2u) : entry(j + 1u));
                __builtin_amdgcn_sched_barrier(0);
                KSTAT(2);
                if (v) {
                    T hb, disc;
                    if constexpr (SCALAR) {   // objects.rs:217-222
                        hb = (cur.ox * d.x + cur.oy * d.y) + cur.oz * d.z;
                        disc = hb * hb - a * cur.c;
                    } else {                  // objects.rs:255, 257
                        hb = fma(cur.oz, d.z, fma(cur.oy, d.y, cur.ox * d.x));
                        disc = fma(hb, hb, (-a) * cur.c);
                    }
                    if (kBothRoots ? disc >= T(0.0) : (disc >= T(0.0) && hb <= T(0.0)))
                        hit_update<T, root2, SCALAR>(hb, disc, cur.i, a, inv_a, bh);
                }
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_sched_barrier(0);
                cur = nxt;
            }
        }
    } else {
        for (; smask != 0u; smask &= smask - 1u) {
            const uint16_t* l = lists[__builtin_ctz(smask)];
            const uint32_t n = __builtin_amdgcn_readfirstlane(l[0]);
            for (uint32_t j = 0; j < n; ++j) {
                ++n_cx;
                camera_exact<T, root2, SCALAR>(q, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, bh);
            }
        }
    }
    work_add(kWCExact, n_cx);
    t_out = bh.bt();
    return bh.bi();
}

// The per-lane "next ray" stage.  Fresh lanes run Camera::get_ray (ray_tracing.rs:77-89; jitter
// stream 0, disk stream 1); lanes that hit at bounce k run PackedHitRecords::finalize
// (objects.rs:157-162) and Material::get_hit_result (materials.rs:54-147; stream 2).  Both draw one
// Philox block and normalise one vector (v / sqrt(|v|^2): unit() for the camera direction, the
// finalize normal), so the wave issues those once per iteration, not once per role.
// SCALAR: HitRecord::new's normal is (p - c) / radius (objects.rs:242, 65-73).
template <typename T, bool SCALAR>
__device__ __forceinline__ void next_ray(bool cam, uint32_t colx, uint32_t rowy, uint32_t pix, uint32_t sid,
                                         uint32_t k, int hit_i, T hit_t, V3<T>& o, V3<T>& d, V3<T>& c) {
    // the hit sphere's centre and material, requested before the draw (scatter lanes; a camera lane reads
    // record 0, unused)
    const int hg = cam ? 0 : hit_i;
    const auto& qg = *cold_args<T>();
    const T* sgp = qg.cen + 4 * hg;
    const V3<T> hcen = mk(sgp[0], sgp[1], sgp[2]);
    const T hrad = sgp[3];
    const MatT<T> m = qg.mats[hg];                       // = materials[material[hit_i]] (objects.rs:296)
    const U4 r = [&] {
        const auto& q0 = *cold_args<T>();
        return rng<T>(sid, pix, cam ? 0u : k, cam ? 0u : 2u, q0.k0, q0.k1);
    }();
    const auto& q = *cold_args_after<T>(r.a ^ r.b);
    const T ua = u01a(r, T(0)), ub = u01b(r, T(0));
    V3<T> vec, base;
    T l2, rad = T(1.0);
    if (cam) {
        const T s1 = div_dim((T)colx + ua, q.W, q.rW);
        const T s2 = div_dim((T)rowy + ub, q.H, q.rH);
        const V3<T> vu = mk(q.vu[0], q.vu[1], q.vu[2]), vv = mk(q.vv[0], q.vv[1], q.vv[2]);
        const V3<T> pc = add(mk(q.ulc[0], q.ulc[1], q.ulc[2]), add(mul(vu, s1), mul(vv, s2)));
        const V3<T> center = mk(q.center[0], q.center[1], q.center[2]);
        if (q.flags & kFlagPinholeInternal) {
            // Zero defocus vectors and no -0.0 in the centre (checked on the host): du*dx + dv*dy
            // + center == center for every disk sample, so the draw cannot change a bit.
            base = center;
        } else {
            T dx = 0, dy = 0;   // random_in_unit_disk (geometry.rs:154-168): rejection on [-1,1]^2
            for (uint32_t i = 0; i < 256u; ++i) {
                // Only cameras with defocus get here.  Re-launder the key each draw: hoisted, its
                // 20-word round-key schedule held SGPRs across the whole camera stage and spilled
                // the camera constants on every iteration, pinhole or not.
                uint32_t k0 = q.k0, k1 = q.k1;
                asm volatile("" : "+s"(k0), "+s"(k1));
                const U4 qq = rng<T>(sid, pix, i, 1u, k0, k1);
                const T x = T(2.0) * u01a(qq, T(0)) - T(1.0);
                const T y = T(2.0) * u01b(qq, T(0)) - T(1.0);
                if (x * x + y * y <= T(1.0)) { dx = x; dy = y; break; }
            }
            base = add(add(mul(mk(q.du[0], q.du[1], q.du[2]), dx), mul(mk(q.dv[0], q.dv[1], q.dv[2]), dy)), center);
        }
        vec = sub(pc, base);
        l2 = len2(vec);                                   // unit(): Vec3::length (geometry.rs:106-112)
    } else {
        base = mk(o.x + d.x * hit_t, o.y + d.y * hit_t, o.z + d.z * hit_t);   // at_t
        vec = sub(base, hcen);                           // normal = at_t(t) - center (objects.rs:279-280)
        if constexpr (SCALAR) rad = hrad;
        l2 = pk_len2(vec);
    }
    const T len = (SCALAR && !cam) ? rad : sqrt_len(l2);
    const V3<T> u = dvs(vec, len);
    if (cam) {
        o = base;
        d = u;
        c = mk(T(1.0), T(1.0), T(1.0));
        return;
    }
    V3<T> nrm = u;
    const bool front = (SCALAR ? dot(d, nrm) : pk_dot(d, nrm)) < T(0.0);
    if (!front) nrm = neg(nrm);
    V3<T> nd;
    if (m.kind != RT_DIELECTRIC) {
        // One random_unit_vector for both kinds (a wave usually holds both: one evaluation, not two).
        const V3<T> rv = unit_vec(ua, ub);
        if (m.kind == RT_LAMBERTIAN) {
            nd = add(rv, nrm);
            if (near_zero(nd)) nd = nrm;
        } else {
            nd = add(reflect(d, nrm), mul(rv, m.p[3]));   // fuzz
        }
        c = mk(c.x * m.p[0], c.y * m.p[1], c.z * m.p[2]);   // albedo
    } else {
        const T ratio = front ? m.p[1] : m.p[0];   // 1/ior : ior
        const V3<T> nn = m.hollow ? neg(nrm) : nrm;
        const T ct = fmin(dot(neg(d), nn), T(1.0));
        const T st = sqrt_nd(T(1.0) - ct * ct);   // ct <= 1: 0, >= 2^-24 or negative
        bool refl = ratio * st > T(1.0);
        if (!refl) {   // Dielectric::reflectance (materials.rs:121-124), powi(5) = x*((x*x)*(x*x))
            const T r0 = front ? m.p[2] : m.p[3];   // r0_front : r0_back
            const T m1 = T(1.0) - ct;
            const T m2 = m1 * m1;
            const T m5 = m1 * (m2 * m2);
            refl = r0 + (T(1.0) - r0) * m5 > ua;
        }
        nd = refl ? reflect(d, nn) : refract(d, nn, ratio);
        c = mk(c.x * T(1.0), c.y * T(1.0), c.z * T(1.0));
    }
    o = base;
    d = nd;
}

// Camera-origin sphere table for pinhole launches.  Every primary ray starts at the camera centre
// (the host checked that the origin is the centre bit for bit), so oc = o - c and c = |oc|^2 - r^2
// (objects.rs:252, 256; scalar: 217, 221) are the same for all of them.  Computed once per launch
// with the same operations, in the sph group layout with {cx, cy, cz, r^2} -> {ocx, ocy, ocz, c};
// a dummy (r^2 = -inf) gets c = +inf, so its discriminant is still -inf.
// Also the camera filter table (fp32, groups of 4 spheres), used by the camera-batch sweep under Q1.
template <typename T, bool SCALAR>
__global__ void build_cam_table(const T* sph, T* cam, uint32_t n_slots, float* camf, uint32_t n_fslots, T ox, T oy,
                                T oz, uint32_t pass_all, T* camx, float* cull, uint32_t n_cull, uint32_t n_real,
                                const uint32_t* ridx, uint32_t n_cslots, const double* clus, float* cullc,
                                uint32_t n_clp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slots && i >= n_fslots && i >= n_cull && i >= n_cslots && i >= n_clp) return;
    constexpr uint32_t G = kGroup<T>, NE = 64 / sizeof(T);
    const uint32_t g = i / G, j = i % G;
    auto at = [&](uint32_t f) -> uint32_t {
        return sizeof(T) == 4 ? g * NE + 8 * (j / 2) + 2 * f + (j % 2) : g * NE + 4 * j + f;
    };
    T ocx = T(0), ocy = T(0), ocz = T(0), c = T(INFINITY);   // slots past the exact table: dummies
    if (i < n_slots) {
        const T cx = sph[at(0)], cy = sph[at(1)], cz = sph[at(2)], r2 = sph[at(3)];
        ocx = ox - cx; ocy = oy - cy; ocz = oz - cz;
        c = SCALAR ? ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2 : fma(ocz, ocz, fma(ocy, ocy, ocx * ocx)) - r2;
        cam[at(0)] = ocx;
        cam[at(1)] = ocy;
        cam[at(2)] = ocz;
        cam[at(3)] = c;
    }
    if (i < n_fslots) {
        // Camera filter record (fp32 layout, nearest_hit CAMT + Q1): {ocx, ocy, ocz} in fp32 and
        // sc = sqrt(c) - 24 u |oc| - 1e-20 rounded down (u = 2^-24), or +inf when c <= 0 (the
        // camera is inside or on the sphere: under Q1 root1 <= 0, never a hit) or NaN.
        const double cd = (double)c;
        const double ocn = sqrt((double)ocx * (double)ocx + (double)ocy * (double)ocy + (double)ocz * (double)ocz);
        float sc = pass_all ? -INFINITY : INFINITY;   // pass_all: RT_FILTER_OFF (every group exact)
        if (cd > 0.0 && !pass_all) {
            const double v = sqrt(cd) - 0x1.8p-20 * ocn - 1e-20;   // 24 u = 1.5 * 2^-20
            sc = (float)v;
            if ((double)sc > v) sc = nextafterf(sc, -INFINITY);
        }
        const uint32_t fg = i / 4, fj = i % 4;
        float* out = camf + 16 * fg + 8 * (fj / 2) + (fj % 2);
        out[0] = (float)ocx; out[2] = (float)ocy; out[4] = (float)ocz; out[6] = sc;
    }
    auto rup = [](double v) -> float {   // fp32 >= v; +inf past 1e30 (and for NaN)
        if (!(v < 1e30)) return INFINITY;
        float f = (float)v;
        if ((double)f < v) f = nextafterf(f, INFINITY);
        return f;
    };
    if (i < n_cslots) {
        // Cone-cull record of slot i of the sweep layout (camera_sweep): w = c - O in fp32 and
        // rp = sqrt(r^2 (1 + 2^-20) + 64 u |w|^2) + 32 u |w| rounded up (u = 2^-24); +inf (always tested)
        // for non-finite values and under RT_FILTER_OFF, -inf for dummy slots (never pass).
        // Also the slot's camera-origin record {ocx, ocy, ocz, c} (the exact test of camera_sweep),
        // computed with the reference's operations as above; a dummy slot gets c = +inf.
        const uint32_t sj = ridx[i];
        float w[3] = {0.0f, 0.0f, 0.0f}, rp = -INFINITY;
        T ex = T(0), ey = T(0), ez = T(0), ec = T(INFINITY);
        if (sj != 0xFFFFFFFFu) {
            const uint32_t gj = sj / G, jj = sj % G;
            auto atj = [&](uint32_t f) -> uint32_t {
                return sizeof(T) == 4 ? gj * NE + 8 * (jj / 2) + 2 * f + (jj % 2) : gj * NE + 4 * jj + f;
            };
            const T cx = sph[atj(0)], cy = sph[atj(1)], cz = sph[atj(2)], r2 = sph[atj(3)];
            ex = ox - cx; ey = oy - cy; ez = oz - cz;
            ec = SCALAR ? ((ex * ex + ey * ey) + ez * ez) - r2 : fma(ez, ez, fma(ey, ey, ex * ex)) - r2;
            const double wn2 = (double)ex * (double)ex + (double)ey * (double)ey + (double)ez * (double)ez;
            rp = pass_all ? INFINITY
                          : rup(sqrt((double)r2 * (1.0 + 0x1.0p-20) + 0x1.0p-18 * wn2) + 0x1.0p-19 * sqrt(wn2) + 1e-30);
            w[0] = -(float)ex; w[1] = -(float)ey; w[2] = -(float)ez;   // c - O = -(O - c) exactly
        }
        cull[4 * i] = w[0]; cull[4 * i + 1] = w[1]; cull[4 * i + 2] = w[2]; cull[4 * i + 3] = rp;
        camx[4 * i] = ex; camx[4 * i + 1] = ey; camx[4 * i + 2] = ez; camx[4 * i + 3] = ec;
    }
    if (i < n_clp) {
        // Cluster record: W = C - O and rp_k = R (1 + 2^-20) + (2^-9 + 2^-16) (|W| + R) (C, R: the
        // cluster's bounding sphere, set_scene; R = -inf: padding, never passes).  A member's rp_i <=
        // r_i (1 + 2^-21) + (2^-9 + 2^-19) |w_i| (sqrt(64 u) = 2^-9) and |w_i| <= |W| + R, so rp_k >=
        // rp_i + |c_i - C| plus the fp32 evaluation errors of both records (camera_sweep).
        const double R = clus[4 * i + 3];
        float w[3] = {0.0f, 0.0f, 0.0f}, rp = -INFINITY;
        if (R > -INFINITY) {
            const double wx = clus[4 * i] - (double)ox, wy = clus[4 * i + 1] - (double)oy, wz = clus[4 * i + 2] - (double)oz;
            const double wn = sqrt(wx * wx + wy * wy + wz * wz);
            rp = pass_all ? INFINITY : rup(R * (1.0 + 0x1.0p-20) + (0x1.0p-9 + 0x1.0p-16) * (wn + R) + 1e-30);
            w[0] = (float)wx; w[1] = (float)wy; w[2] = (float)wz;
        }
        cullc[4 * i] = w[0]; cullc[4 * i + 1] = w[1]; cullc[4 * i + 2] = w[2]; cullc[4 * i + 3] = rp;
    }
}

}  // namespace rt
