// rt_sweep.hpp — the general sweep (bounced rays and defocus cameras) and the camera-origin sweep:
// conservative fp32 culls (box slab tests, sphere distance filters) in front of the reference's
// exact test (Sphere::hit_packed, objects.rs:249-290) and PackedHitRecords::update (objects.rs:121-155).
#pragma once
#include "rt_common.hpp"

namespace rt {

// The general-sweep filter for one 4-sphere group (nearest_hit): per sphere pair
//   x = cx*e1x + (cz*e1z - oe1),  y = cx*e2x + (cy*e2y + (cz*e2z - oe2)),  D = (r2f - y^2) - x^2
// in packed FP32 (two spheres per op), then acc = ~(D0 & D1 & D2 & D3) on the sign bits.  The
// per-lane constants (the basis already scaled by the margin, nearest_hit) come two to a VGPR
// pair, K0 = {e1x, e1z}, K1 = {e2x, e2y}, K2 = {e2z, -}, K3 = {-oe1, -oe2}, and each use
// broadcasts one half with op_sel / op_sel_hi (the compiler materialises such splats as extra VGPR
// pairs).  The two pairs are interleaved so that no packed result is read by the next instruction
// (the one-wait-state packed-FP32 read hazard the compiler pads with s_nop).  14 packed ops, then
// v_and3 + v_bitop3 on the sign bits.
__device__ __forceinline__ uint32_t filter_group(const SphGroup<float>& cur, f2 K0, f2 K1, f2 K2, f2 K3, uint32_t& s0,
                                                 uint32_t& s1, f2* D = nullptr) {
    const f2 cx0 = {cur.v[0], cur.v[1]}, cy0 = {cur.v[2], cur.v[3]}, cz0 = {cur.v[4], cur.v[5]}, rr0 = {cur.v[6], cur.v[7]};
    const f2 cx1 = {cur.v[8], cur.v[9]}, cy1 = {cur.v[10], cur.v[11]}, cz1 = {cur.v[12], cur.v[13]}, rr1 = {cur.v[14], cur.v[15]};
    f2 a0, b0, a1, b1, r0, r1;
    asm volatile(
        "v_pk_fma_f32 %[a0], %[cz0], %[K0], %[K3] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"   // cz*e1z - oe1
        "v_pk_fma_f32 %[b0], %[cz0], %[K2], %[K3] op_sel:[0,0,1] op_sel_hi:[1,0,1]\n\t"   // cz*e2z - oe2
        "v_pk_fma_f32 %[a1], %[cz1], %[K0], %[K3] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
        "v_pk_fma_f32 %[b1], %[cz1], %[K2], %[K3] op_sel:[0,0,1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[a0], %[cx0], %[K0], %[a0] op_sel_hi:[1,0,1]\n\t"                  // x = cx*e1x + .
        "v_pk_fma_f32 %[b0], %[cy0], %[K1], %[b0] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"   // cy*e2y + .
        "v_pk_fma_f32 %[a1], %[cx1], %[K0], %[a1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[b1], %[cy1], %[K1], %[b1] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[b0], %[cx0], %[K1], %[b0] op_sel_hi:[1,0,1]\n\t"                  // y = cx*e2x + .
        "v_pk_fma_f32 %[b1], %[cx1], %[K1], %[b1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[r0], %[b0], %[b0], %[rr0] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"      // r2f - y^2
        "v_pk_fma_f32 %[r1], %[b1], %[b1], %[rr1] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
        "v_pk_fma_f32 %[r0], %[a0], %[a0], %[r0] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"       // D = . - x^2
        "v_pk_fma_f32 %[r1], %[a1], %[a1], %[r1] neg_lo:[1,0,0] neg_hi:[1,0,0]"
        : [a0] "=&v"(a0), [b0] "=&v"(b0), [a1] "=&v"(a1), [b1] "=&v"(b1), [r0] "=&v"(r0), [r1] "=&v"(r1)
        : [cx0] "s"(cx0), [cy0] "s"(cy0), [cz0] "s"(cz0), [rr0] "s"(rr0), [cx1] "s"(cx1), [cy1] "s"(cy1),
          [cz1] "s"(cz1), [rr1] "s"(rr1), [K0] "v"(K0), [K1] "v"(K1), [K2] "v"(K2), [K3] "v"(K3));
    // ~(D0 & D1 & D2 & D3): sign set iff some sphere of the group passes (D >= +0); s0, s1: the
    // same per sphere pair, un-negated (sign clear iff a sphere of the pair passes)
    s0 = __float_as_uint(r0.x) & __float_as_uint(r0.y);
    s1 = __float_as_uint(r1.x) & __float_as_uint(r1.y);
    if (D) { D[0] = r0; D[1] = r1; }   // per sphere (fp64 rays: exact tests per sphere)
    return ~(s0 & s1);
}

// The camera-batch filter for one 4-sphere group (nearest_hit, CAMT under Q1): per sphere pair
// hb' = ocx*dx^ + ocy*dy^ + ocz*dz^ and t = hb' + sc; returns t0 | t1 | t2 | t3, whose sign bit
// is set iff some sphere passes (t < 0).  K0 = {dx^, dy^}, K1 = {dz^, -} broadcast with op_sel;
// the two pairs are interleaved so no packed result is read by the next instruction.
__device__ __forceinline__ uint32_t cam_filter_group(const SphGroup<float>& cur, f2 K0, f2 K1) {
    const f2 ox0 = {cur.v[0], cur.v[1]}, oy0 = {cur.v[2], cur.v[3]}, oz0 = {cur.v[4], cur.v[5]}, sc0 = {cur.v[6], cur.v[7]};
    const f2 ox1 = {cur.v[8], cur.v[9]}, oy1 = {cur.v[10], cur.v[11]}, oz1 = {cur.v[12], cur.v[13]}, sc1 = {cur.v[14], cur.v[15]};
    f2 t0, t1;
    asm volatile(
        "v_pk_mul_f32 %[t0], %[ox0], %[K0] op_sel_hi:[1,0]\n\t"                         // ocx*dx^
        "v_pk_mul_f32 %[t1], %[ox1], %[K0] op_sel_hi:[1,0]\n\t"
        "v_pk_fma_f32 %[t0], %[oy0], %[K0], %[t0] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"   // + ocy*dy^
        "v_pk_fma_f32 %[t1], %[oy1], %[K0], %[t1] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[t0], %[oz0], %[K1], %[t0] op_sel_hi:[1,0,1]\n\t"                  // + ocz*dz^
        "v_pk_fma_f32 %[t1], %[oz1], %[K1], %[t1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_add_f32 %[t0], %[t0], %[sc0]\n\t"                                           // + sc
        "v_pk_add_f32 %[t1], %[t1], %[sc1]"
        : [t0] "=&v"(t0), [t1] "=&v"(t1)
        : [ox0] "s"(ox0), [oy0] "s"(oy0), [oz0] "s"(oz0), [sc0] "s"(sc0), [ox1] "s"(ox1), [oy1] "s"(oy1),
          [oz1] "s"(oz1), [sc1] "s"(sc1), [K0] "v"(K0), [K1] "v"(K1));
    return (__float_as_uint(t0.x) | __float_as_uint(t0.y) | __float_as_uint(t1.x)) | __float_as_uint(t1.y);
}

// The general sweep's cluster test for one top group of 4 cluster boxes: a slab test of the ray
// against each box widened by the lane's margin.  Per axis a: u = C.i + A (i = 1/d, A = -o.i), near
// t = u - h J and far t = u + h J with J = |i| (1 + kappa) (nearest_hit), tn = max over axes of
// near, tf = min of far; a cluster is culled for the lane iff tf < tn or tf < 0 (NaN: kept).
// B0 = {ix, iy}, B1 = {iz, Az}, B2 = {Ax, Ay}, B3 = {Jx, Jy}, B4 = {Jz, -}, broadcast with op_sel;
// 9 packed FMAs per box pair, then max3/min3 per box.  Returns the 4-bit wave mask of clusters
// that pass for some lane.
// bt (>= the lane's best hit t so far, +inf before any hit) also culls a box the ray enters only past
// its best hit: tn > bt.  The widened box holds every point o + t* d of a root t* the reference could
// report for a member, and the computed near time is <= t* (the margin covers its rounding;
// tests/box_cull_fuzz.c checks tn <= t* directly), so such a box holds no hit with t* <= bt: none that
// could replace the best (ties need t* == best).  The test is tn0 = max(tn, 0) <= min(tf, bt).
__device__ __forceinline__ uint32_t box_pair(const float* v, f2 B0, f2 B1, f2 B2, f2 B3, f2 B4, float bt) {
    f2 ux, uy, uz, nx, ny, nz;
    const f2 cx = {v[0], v[1]}, cy = {v[2], v[3]}, cz = {v[4], v[5]}, hx = {v[6], v[7]}, hy = {v[8], v[9]},
             hz = {v[10], v[11]};
    // one pair at a time (12 temporaries); each packed result is read 3 instructions after its write
    asm volatile(
        "v_pk_fma_f32 %[ux], %[cx], %[B0], %[B2] op_sel_hi:[1,0,0]\n\t"                         // u = c i + A
        "v_pk_fma_f32 %[uy], %[cy], %[B0], %[B2] op_sel:[0,1,1] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[uz], %[cz], %[B1], %[B1] op_sel:[0,0,1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[nx], %[hx], %[B3], %[ux] op_sel_hi:[1,0,1] neg_lo:[0,1,0] neg_hi:[0,1,0]\n\t"   // near = u - h J
        "v_pk_fma_f32 %[ny], %[hy], %[B3], %[uy] op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_lo:[0,1,0] neg_hi:[0,1,0]\n\t"
        "v_pk_fma_f32 %[nz], %[hz], %[B4], %[uz] op_sel_hi:[1,0,1] neg_lo:[0,1,0] neg_hi:[0,1,0]\n\t"
        "v_pk_fma_f32 %[ux], %[hx], %[B3], %[ux] op_sel_hi:[1,0,1]\n\t"                        // far = u + h J
        "v_pk_fma_f32 %[uy], %[hy], %[B3], %[uy] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[uz], %[hz], %[B4], %[uz] op_sel_hi:[1,0,1]"
        : [ux] "=&v"(ux), [uy] "=&v"(uy), [uz] "=&v"(uz), [nx] "=&v"(nx), [ny] "=&v"(ny), [nz] "=&v"(nz)
        : [cx] "s"(cx), [cy] "s"(cy), [cz] "s"(cz), [hx] "s"(hx), [hy] "s"(hy), [hz] "s"(hz), [B0] "v"(B0),
          [B1] "v"(B1), [B2] "v"(B2), [B3] "v"(B3), [B4] "v"(B4));
    // Culled iff tf < tn or tf < 0, i.e. iff tf < max(tn, 0) (NaN: kept).  Inline asm down to the
    // wave mask: fmaxf / fminf on the asm's outputs made the compiler canonicalise each input first
    // (two v_max_f32 x, x per box; these values come from FMAs, never signalling NaNs), and the
    // ballot's bool took a round trip through a VGPR.  v_cmp_e64 writes 0 for inactive lanes, as a
    // ballot does.
    auto pass = [bt](float nx, float ny, float nz, float fx, float fy, float fz, auto bitc) -> uint32_t {
        constexpr uint32_t bit = decltype(bitc)::value;
        float tn, tf;
        unsigned long long m;
        uint32_t r;
        asm volatile(
            "v_max3_f32 %[tn], %[nx], %[ny], %[nz]\n\t"
            "v_min3_f32 %[tf], %[fx], %[fy], %[fz]\n\t"
            "v_max_f32 %[tn], 0, %[tn]\n\t"
            "v_min_f32 %[tf], %[tf], %[bt]\n\t"
            "v_cmp_nlt_f32_e64 %[m], %[tf], %[tn]\n\t"
            "s_cmp_lg_u64 %[m], 0\n\t"
            "s_cselect_b32 %[r], %[bit], 0"
            : [tn] "=&v"(tn), [tf] "=&v"(tf), [m] "=&s"(m), [r] "=s"(r)
            : [nx] "v"(nx), [ny] "v"(ny), [nz] "v"(nz), [fx] "v"(fx), [fy] "v"(fy), [fz] "v"(fz), [bt] "v"(bt),
              [bit] "n"(bit)
            : "scc");
        return r;
    };
    // readfirstlane: the mask is wave-uniform (the compiler cannot see that through the asm)
    return __builtin_amdgcn_readfirstlane(pass(nx.x, ny.x, nz.x, ux.x, uy.x, uz.x, std::integral_constant<uint32_t, 1>{}) |
                                          pass(nx.y, ny.y, nz.y, ux.y, uy.y, uz.y, std::integral_constant<uint32_t, 2>{}));
}
__device__ __forceinline__ uint32_t box_mask(const BoxGroup& cur, f2 B0, f2 B1, f2 B2, f2 B3, f2 B4, float bt) {
    return box_pair(&cur.v[0], B0, B1, B2, B3, B4, bt) | (box_pair(&cur.v[12], B0, B1, B2, B3, B4, bt) << 2);
}
__device__ __forceinline__ uint32_t box_mask(const LBoxGroup& cur, f2 B0, f2 B1, f2 B2, f2 B3, f2 B4, float bt) {
    return box_pair(&cur.v[0], B0, B1, B2, B3, B4, bt) | (box_pair(&cur.v[12], B0, B1, B2, B3, B4, bt) << 2);
}

// The object loop of trace_vectorized2 for one enabled ray (ray_tracing.rs:399-403): returns the
// index of the nearest valid hit (-1: the sky, :421-424) and its t.
// SCALAR selects Sphere::hit + Scene::hit (objects.rs:216-247, ray_tracing.rs:231-235): no FMA,
// both roots, root = (-hb -/+ sd) / a, the first minimum wins ties.  Otherwise hit_packed +
// PackedHitRecords::update (objects.rs:249-290, 140-155).
// CAMT: the ray starts at the camera centre and the sweep reads the camera-origin table
// (build_cam_table): oc and c come precomputed, bit-identical to the per-ray values.
// Sphere::hit_packed's root and PackedHitRecords::update (objects.rs:263-290, 140-155) for a
// candidate whose discriminant is non-negative; SCALAR: Sphere::hit + Scene::hit's min_by_key
// (objects.rs:227-234, ray_tracing.rs:231-235: the first minimum wins).  i is the scene index; ties
// are broken by it (later wins, scalar: earlier wins), so the result does not depend on the order
// in which spheres are visited (the general sweep visits them cluster by cluster).
// The best hit so far (PackedHitRecords' t and sphere, objects.rs:121-155).  fp32: one 64-bit key
// (bits(t) - bits(0.001f)) << 32 | ~index, the high half wrapping mod 2^32.  Non-negative floats order as their bits,
// so "a smaller t, or the same t and a later sphere" (:141) is one unsigned 64-bit compare, and with the offset the
// compare also holds the validity test (:272): a root below 0.001, -0, negative or NaN lands above every valid key,
// and +inf meets the initial key (+inf, ~(-1) = 0) with ~index >= 1.  Round 6, same-box C fp32 +0.4 %, E +0.5 %
// (profiles/r06/hit_key64_ab.txt): 5 compares, 4 SALU mask ops, a move and two selects became a subtract, a move,
// one compare and two selects per candidate.
template <typename T> struct HitBest {
    T t = T(INFINITY);
    int i = -1;
    __device__ __forceinline__ T bt() const { return t; }
    __device__ __forceinline__ int bi() const { return i; }
    __device__ __forceinline__ void set(T r, uint32_t j) { t = r; i = (int)j; }
};
constexpr uint32_t kT001 = 0x3A83126Fu;   // bits of 0.001f (RN), the smallest valid root
__device__ __forceinline__ uint64_t hit_key(float r, uint32_t j) {
    return ((uint64_t)(__float_as_uint(r) - kT001) << 32) | (uint64_t)~j;
}
template <> struct HitBest<float> {
    uint64_t k = (uint64_t)(0x7F800000u - kT001) << 32;
    __device__ __forceinline__ float bt() const { return __uint_as_float((uint32_t)(k >> 32) + kT001); }
    __device__ __forceinline__ int bi() const { return (int)~(uint32_t)k; }
    __device__ __forceinline__ void set(float r, uint32_t j) { k = hit_key(r, j); }
};
template <typename T, bool root2, bool SCALAR>
__device__ __forceinline__ void hit_update(T hb, T disc, uint32_t i, T a, T inv_a, HitBest<T>& bh) {
    if constexpr (SCALAR) {
        const T sd = sqrt(disc);
        T root = (-hb - sd) / a;
        if (!(root >= T(0.001) && root < T(INFINITY))) {
            root = (-hb + sd) / a;
            if (!(root >= T(0.001) && root < T(INFINITY))) return;
        }
        if (root < bh.bt() || (root == bh.bt() && (int)i < bh.bi())) bh.set(root, i);   // first wins
        return;
    }
    // sqrt_len: the library sqrt's sequence without its range scaling when every candidate lane is in range
    // (fp64: E +0.6 %; fp32: round 6, with the other sqrt_len calls C +1.2 %)
    const T sd = sqrt_len(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270
    if constexpr (sizeof(T) == 4 && !root2) {
        // valid (:272) && better (:141) in one compare (HitBest<float>)
        const uint64_t key = hit_key(r1, i);
        bh.k = key < bh.k ? key : bh.k;
        return;
    }
    bool valid = r1 >= T(0.001) && r1 < T(INFINITY);       // :272
    T root = r1;
    if (root2 && !valid) {                                 // Q1 off: scalar semantics
        root = (-hb + sd) * inv_a;                         // :271
        valid = root >= T(0.001) && root < T(INFINITY);
    }
    // ties: later wins (:141); bitwise, so the update is two selects, not nested exec-mask branches (C fp32
    // +0.2 %, fp64 +1.3 %, E +0.4 % / +0.7 %: profiles/r05/hit_select_ab.txt)
    if constexpr (sizeof(T) == 4) {
        const uint64_t key = hit_key(root, i);
        const bool take = valid & (key < bh.k);
        bh.k = take ? key : bh.k;
    } else {
        const bool take = valid & ((root < bh.t) | ((root == bh.t) & ((int)i > bh.i)));
        bh.t = take ? root : bh.t;
        bh.i = take ? (int)i : bh.i;
    }
}

template <typename T, bool root2, bool SCALAR = false, bool CAMT = false, bool MEGA = false>
__device__ __forceinline__ int nearest_hit(const KParams<T>& p, const V3<T>& o, const V3<T>& d, T& t_out) {
    const T a = SCALAR ? len2(d) : pk_len2(d);       // objects.rs:219 / :253
    const T inv_a = SCALAR ? T(0) : T(1.0) / a;      // objects.rs:254 (loop-invariant)
    HitBest<T> bh;                   // PackedHitRecords::default, objects.rs:128
    // Sphere::hit_packed (objects.rs:249-290) + PackedHitRecords::update (objects.rs:140-155)
    // for a candidate whose discriminant is non-negative.  Exact pre-filter: with hb >= 0,
    // root1 = (-hb - sd)*inv_a <= 0 can never be valid, so only Q1-off (root2) mode needs it.
    KSTAT(CAMT ? 3 : 1);   // sweeps (one per wave)
    auto hit = [&](T hb, T disc, uint32_t i) { hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, bh); };
    // Spheres stream through the scalar cache in 64-byte groups; group g+1 is requested before
    // group g is tested so the K$ latency hides behind the group's VALU work.
    // The buffer holds one extra dummy group, so the prefetch of group g+1 is always in bounds.
    // Read through the laundered kernarg pointer at each sweep, so the sphere pointer and count do
    // not hold SGPRs across the persistent loop (they were spilled to VGPR lanes, 2 VALU a group).
    auto sbits = [](T x) -> uint32_t {
        if constexpr (sizeof(T) == 4) return __float_as_uint(x);
        else return (uint32_t)__double2hiint(x);
    };
    constexpr bool kBothRoots = root2 || SCALAR;
    auto is_cand = [](uint32_t m) -> bool { return (int32_t)m < 0; };
    // Per-sphere test inside a taken group: a float superset of cand (hb == +0 passes too).
    auto cand_f = [&](T hb, T disc) -> bool { return kBothRoots ? disc >= T(0.0) : (disc >= T(0.0) && hb <= T(0.0)); };
    if constexpr (CAMT && !kBothRoots) {
        // Camera batches under Q1 (hit_packed; root1 only).  A valid hit needs hb < 0 (root1 =
        // (-hb - sd)/a > 0) and disc >= 0, i.e. -hb >= sqrt(a c): with d^ = d / |d| (fp32) and
        // hb' = oc.d^, the filter passes a sphere iff hb' + sc < 0, where the camera filter table
        // holds sc = sqrt(c) - 24 u |oc| - 1e-20 (build_cam_table; +inf for c <= 0: a camera inside
        // or on the sphere never hits it under Q1).  The 24 u covers the reference's rounding of
        // hb and disc, d^'s and hb''s rounding and the fp32 conversion of fp64 rays (a first-order
        // bound is ~13 u; fuzzed worst case 3.7 u, tests/test_filter_margin.py).  4 packed ops per
        // sphere pair against the exact 5 (fp32) or 10 fp64 ops; taken groups rerun the exact
        // test from the camera-origin table.
        const auto& qa = *cold_args<T>();
        cptr<float> ff = (cptr<float>)__builtin_assume_aligned(qa.camf, 64);
        cptr<T> fe = (cptr<T>)__builtin_assume_aligned(qa.camsph, 64);
        const uint32_t ngf = qa.n_fgroups;
        const float fdx = (float)d.x, fdy = (float)d.y, fdz = (float)d.z;
        const float inv = 1.0f / sqrtf(__builtin_fmaf(fdz, fdz, __builtin_fmaf(fdy, fdy, fdx * fdx)));
        const f2 K0 = {fdx * inv, fdy * inv}, K1 = {fdz * inv, 0.0f};
        auto exact4 = [&](uint32_t g) {
            KSTAT(2);
            if constexpr (sizeof(T) == 4) {
                const SphGroup<T> cur = load_group(fe, g);
                const f2 dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z};
                const f2 na = {-a, -a};
                f2 hb[2], disc[2];
#pragma unroll
                for (uint32_t q = 0; q < 2; ++q) {
                    const T* v = &cur.v[8 * q];
                    const f2 ocx = {v[0], v[1]}, ocy = {v[2], v[3]}, ocz = {v[4], v[5]}, c = {v[6], v[7]};
                    hb[q] = fma2(ocz, dz, fma2(ocy, dy, ocx * dx));
                    disc[q] = fma2(hb[q], hb[q], na * c);
                }
                const uint32_t i0 = 4 * g;
                if (cand_f(hb[0].x, disc[0].x)) hit(hb[0].x, disc[0].x, i0);
                if (cand_f(hb[0].y, disc[0].y)) hit(hb[0].y, disc[0].y, i0 + 1);
                if (cand_f(hb[1].x, disc[1].x)) hit(hb[1].x, disc[1].x, i0 + 2);
                if (cand_f(hb[1].y, disc[1].y)) hit(hb[1].y, disc[1].y, i0 + 3);
            } else {
                const SphGroup<T> c0 = load_group(fe, 2 * g), c1 = load_group(fe, 2 * g + 1);
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const T* v = j < 2 ? &c0.v[4 * j] : &c1.v[4 * (j - 2)];
                    hb[j] = pk_dot(mk(v[0], v[1], v[2]), d);
                    disc[j] = fma(hb[j], hb[j], -a * v[3]);
                }
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (cand_f(hb[j], disc[j])) hit(hb[j], disc[j], 4 * g + j);
            }
        };
        auto group = [&](const SphGroup<float>& cur, uint32_t g) {
            if (is_cand(cam_filter_group(cur, K0, K1))) exact4(g);
        };
        sphere_loop(ff, ngf, group);
    } else if constexpr (CAMT) {
        // Camera batches: {ocx, ocy, ocz, c} from the camera-origin table, so the exact test is
        // hb (3 ops) and disc (2).  Filter on the exact sign bits: a sphere can only be hit if
        // disc >= +0 (disc is never -0: fma(hb, hb, -(a*c)) and hb*hb - a*c round an exact zero
        // to +0; NaNs never give a valid root), so ~(bits(d0) & bits(d1) & ...) has its sign set
        // iff some sphere of the group may be a candidate (v_and3 + v_bitop3 + one compare).
        const auto& qa = *cold_args<T>();
        cptr<T> f = (cptr<T>)__builtin_assume_aligned(qa.camsph, 64);
        const uint32_t ng = qa.n_groups;
        if constexpr (sizeof(T) == 4) {
            const f2 dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z};
            const f2 na = {-a, -a};
            auto group = [&](const SphGroup<T>& cur, uint32_t g) {
                f2 hb[2], disc[2];
#pragma unroll
                for (uint32_t q = 0; q < 2; ++q) {
                    const T* v = &cur.v[8 * q];
                    const f2 ocx = {v[0], v[1]}, ocy = {v[2], v[3]}, ocz = {v[4], v[5]}, c = {v[6], v[7]};
                    if constexpr (SCALAR) {
                        hb[q] = (ocx * dx + ocy * dy) + ocz * dz;
                        disc[q] = hb[q] * hb[q] - (-na) * c;
                    } else {
                        hb[q] = fma2(ocz, dz, fma2(ocy, dy, ocx * dx));
                        disc[q] = fma2(hb[q], hb[q], na * c);
                    }
                }
                const uint32_t t = sbits(disc[0].x) & sbits(disc[0].y) & sbits(disc[1].x);   // v_and3_b32
                const uint32_t acc = __builtin_amdgcn_bitop3_b32(t, sbits(disc[1].y), 0u, 0x3F);   // ~(S0 & S1)
                if (is_cand(acc)) {
                    KSTAT(2);
                    const uint32_t i0 = 4 * g;
                    if (cand_f(hb[0].x, disc[0].x)) hit(hb[0].x, disc[0].x, i0);
                    if (cand_f(hb[0].y, disc[0].y)) hit(hb[0].y, disc[0].y, i0 + 1);
                    if (cand_f(hb[1].x, disc[1].x)) hit(hb[1].x, disc[1].x, i0 + 2);
                    if (cand_f(hb[1].y, disc[1].y)) hit(hb[1].y, disc[1].y, i0 + 3);
                }
            };
            sphere_loop(f, ng, group);
        } else {
            auto group = [&](const SphGroup<T>& cur, uint32_t g) {
                T hb[2], disc[2];
#pragma unroll
                for (uint32_t j = 0; j < 2; ++j) {
                    const T* v = &cur.v[4 * j];
                    const V3<T> oc = mk(v[0], v[1], v[2]);
                    hb[j] = SCALAR ? dot(oc, d) : pk_dot(oc, d);
                    disc[j] = SCALAR ? hb[j] * hb[j] - a * v[3] : fma(hb[j], hb[j], -a * v[3]);
                }
                const uint32_t acc = __builtin_amdgcn_bitop3_b32(sbits(disc[0]), sbits(disc[1]), 0u, 0x3F);   // ~(d0 & d1)
                if (is_cand(acc)) {
                    KSTAT(2);
                    if (cand_f(hb[0], disc[0])) hit(hb[0], disc[0], 2 * g);
                    if (cand_f(hb[1], disc[1])) hit(hb[1], disc[1], 2 * g + 1);
                }
            };
            sphere_loop(f, ng, group);
        }
    } else {
        // General sweep: a conservative fp32 distance filter, then the exact test for taken groups.
        //
        // Filter: with e1, e2 an orthonormal basis of the plane perpendicular to d (e1 has no y
        // component), x = (c - o).e1 and y = (c - o).e2 are the centre's offset from the ray's
        // line, so the line meets the sphere iff x^2 + y^2 <= r^2.  The margin
        // m = 48 u ((max|c|_1 + |o|_1)^2 + max r2f), u = 2^-24, covers the reference's own rounding
        // of disc (a sphere it computes disc >= 0 for may lie slightly outside), the filter's basis
        // and rounding errors, and for fp64 rays the conversion to fp32: a first-order bound is
        // ~30 u, 80M adversarial near-tangent cases need at most 5 u
        // (tests/test_filter_margin.py).  It is applied by scaling the basis by
        // 1/sqrt(1 + m/r2min) (r2min: the smallest filtered r2f): the test x'^2 + y'^2 <= r2f is then
        // x^2 + y^2 <= r2f (1 + m/r2min) >= r2f + m.  Per sphere pair: x 2 packed FMAs, y 3,
        // D = r2f - y^2 - x^2 2 -- 7 ops against the exact test's 12.  So every sphere the reference
        // could hit passes; a group with any passing sphere recomputes all four exactly from the
        // exact stream, and only the exact values ever reach hit().
        // Spheres far outside the scene (|c|_1 + r > 8x the median, e.g. a ground sphere) would
        // inflate the margin for all: the host gives them r2f = +inf, "always exact".  Lanes whose
        // basis degenerates (d nearly parallel to y) or whose origin is huge get a zero basis, so
        // every real sphere passes for them (D = r2f; a -inf dummy never does).  RT_FILTER_OFF=1
        // (host, diagnostics and tests) sets f_cmax = +inf (every lane degenerate, every group
        // exact) and sc = -inf in the camera filter table.
        const auto& qa = *cold_args<T>();
        cptr<float> ff = (cptr<float>)__builtin_assume_aligned(qa.rfsph, 64);
        cptr<T> fe = (cptr<T>)__builtin_assume_aligned(qa.rsph, 64);
        // scene indices of slot group g: from the inline record ip (a walked cluster's group) or the slot table
        auto sidx = [&](uint32_t g, cptr<float> ip) -> Q4 {
            if (ip != nullptr) {
                cptr<uint32_t> r = (cptr<uint32_t>)ip;
                return Q4{r[0], r[1], r[2], r[3]};
            }
            const auto& qi = *cold_args<T>();
            cptr<uint32_t> ri = (cptr<uint32_t>)__builtin_assume_aligned(qi.ridx, 16);
            return Q4{ri[4 * g], ri[4 * g + 1], ri[4 * g + 2], ri[4 * g + 3]};
        };
        const float fdx = (float)d.x, fdy = (float)d.y, fdz = (float)d.z;
        const float fox = (float)o.x, foy = (float)o.y, foz = (float)o.z;
        const float L = __builtin_fmaf(fdz, fdz, fdx * fdx);
        const float af = __builtin_fmaf(fdz, fdz, __builtin_fmaf(fdy, fdy, fdx * fdx));
        const float on = fabsf(fox) + fabsf(foy) + fabsf(foz);
        const float pm = qa.f_cmax + on;
        const float m = kFilterMargin * __builtin_fmaf(pm, pm, qa.f_r2max);
        // Basis scaled by sg = 1/sqrt(1 + m/r2min): x'^2 + y'^2 <= r2f is x^2 + y^2 <= r2f (1 + m/r2min)
        // >= r2f + m for every sphere (r2f >= r2min), so the margin needs no per-pair add.
        // The filter constants need no correctly rounded division or square root: v_rsq_f32 and
        // v_rcp_f32 (1 ulp) add a few u to the basis error, well inside the margin (the fuzz tests
        // model them as +-1 ulp).  1/r2min, 0.5/r2min and 8u/sqrt(r2min) come from the host.
        // MEGA: the basis stays unscaled here; each walked cluster scales it by its own local margin.
        const float sg = MEGA ? 1.0f : __builtin_amdgcn_rsqf(__builtin_fmaf(m, qa.f_ir2, 1.0f));
        const float s1 = __builtin_amdgcn_rsqf(L) * sg, s2 = __builtin_amdgcn_rsqf(L * af) * sg;
        float e1x = fdz * s1, e1z = -fdx * s1;
        float e2x = -(fdx * fdy) * s2, e2y = L * s2, e2z = -(fdy * fdz) * s2;
        float oe1 = __builtin_fmaf(foz, e1z, fox * e1x);
        float oe2 = __builtin_fmaf(foz, e2z, __builtin_fmaf(foy, e2y, fox * e2x));
        // Degenerate lanes: L*af must not underflow (L >= 1e-15: d within ~3e-8 of the y axis), and
        // x^2, y^2 must stay finite (|c|_1 + |o|_1 <= 1e15), so D is never inf - inf.
        // Cluster boxes (box_mask): i = 1/d per axis (|d_a| clamped to >= 1e-20, keeping its sign: a
        // ray parallel to a slab then has near/far times of ~1e20 and the slab test stays exact in
        // effect), A = -o.i, and J = |i| (1 + kappa).  kappa widens every box by kappa h >= kappa
        // sqrt(r2min) (h >= sqrt(r2min), pack_sweep): m / (2 sqrt(r2min)) covers the reference's own
        // rounding (a hit point lies within sqrt(r2f + m) <= sqrt(r2f) + m / (2 sqrt(r2min)) of its
        // sphere's centre, m as for the sphere filter), 8 u pm the fp32 rounding of u, near and far.
        auto inv_ax = [](float v) -> float {
            return __builtin_amdgcn_rcpf(fabsf(v) >= 1e-20f ? v : copysignf(1e-20f, v));
        };
        float ix = inv_ax(fdx), iy = inv_ax(fdy), iz = inv_ax(fdz);
        const float kap = 1.0f + __builtin_fmaf(m, qa.f_hir2, pm * qa.f_isr);   // m / (2 r2min) + 8 u pm / sqrt(r2min)
        float Jx = fabsf(ix) * kap, Jy = fabsf(iy) * kap, Jz = fabsf(iz) * kap;
        float Ax = -(fox * ix), Ay = -(foy * iy), Az = -(foz * iz);
        if (!(L >= 1e-15f) || !(pm <= 1e15f)) {   // zero basis: x = y = 0, every real sphere passes
            e1x = e1z = e2x = e2y = e2z = 0.0f;
            oe1 = oe2 = 0.0f;
            ix = iy = iz = Jx = Jy = Jz = Ax = Ay = Az = 0.0f;   // box times all 0 (or NaN): every box passes
        }
        // Two per-lane constants per VGPR pair; every use broadcasts one half through the packed
        // op's op_sel (filter_group), so the filter state is 8 VGPRs, not 16.
        const f2 K0 = {e1x, e1z}, K1 = {e2x, e2y}, K2 = {e2z, 0.0f}, K3 = {-oe1, -oe2};
        const f2 B0 = {ix, iy}, B1 = {iz, Az}, B2 = {Ax, Ay}, B3 = {Jx, Jy}, B4 = {Jz, 0.0f};
        // MEGA: a box group in its own frame S (pack_local_boxes): o' = o - S (fp64 rays: in double,
        // then rounded), the margin from pm = |o'|_1 + Rg, A = -o'.i, J = |i| (1 + kappa).
        // Packed where two axes take the same op: o'xy, A'xy = -(o'xy ixy), J'xy = |ixy| kp.  kp =
        // 1 + m / (2 r2min) + 8 u pm / sqrt(r2min) as fma(pm^2 + r2max, 48 u 0.5 / r2min, fma(pm, 8 u /
        // sqrt(r2min), 1)): the margin factor folded into the host constant (box_cull_fuzz models this).
        // The best hit so far as a box-time bound (box_pair): fp64 rounds it up to a float.
        auto btf = [&]() -> float {
            if constexpr (sizeof(T) == 4) return bh.bt();
            else return (float)bh.bt() * (1.0f + 0x1.0p-22f);   // RN(RN(b) (1 + 2^-22)) > b (b > 0)
        };
        const f2 nixy = {-ix, -iy}, aixy = {fabsf(ix), fabsf(iy)};
        const float aiz = fabsf(iz);
        auto lmask = [&](const LBoxGroup& g) -> uint32_t {
            const auto& ql = *cold_args<T>();
            const f2 Sxy = {g.v[24], g.v[25]};
            const float Sz = g.v[26], Rg = g.v[27];
            f2 opxy;
            float opz;
            if constexpr (sizeof(T) == 4) {
                opxy = f2{o.x, o.y} - Sxy;
                opz = o.z - Sz;
            } else {
                opxy = f2{(float)(o.x - (double)Sxy.x), (float)(o.y - (double)Sxy.y)};
                opz = (float)(o.z - (double)Sz);
            }
            const float pmg = ((fabsf(opxy.x) + fabsf(opxy.y)) + fabsf(opz)) + Rg;
            const float kp = __builtin_fmaf(__builtin_fmaf(pmg, pmg, ql.l_r2max), ql.l_hir2,
                                            __builtin_fmaf(pmg, ql.l_isr, 1.0f));
            const f2 C1 = {iz, -(opz * iz)}, C2 = opxy * nixy;
            const f2 C3 = aixy * f2{kp, kp}, C4 = {aiz * kp, 0.0f};
            return box_mask(g, B0, C1, C2, C3, C4, btf());
        };
        // The exact test of spheres 4g..4g+3 (objects.rs:252-257; SCALAR: Sphere::hit :217-222), of
        // the sphere pairs set in `pairs` (fp32, bit q: spheres 4g+2q, 4g+2q+1; fp64, bit j: sphere
        // 4g+j; wave-uniform).
        auto exact4 = [&](uint32_t g, uint32_t pairs = sizeof(T) == 4 ? 3u : 15u, cptr<float> ip = nullptr) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                // Packed FP32: each v_pk_{add,mul,fma}_f32 evaluates the same IEEE op for two
                // spheres, so the results are bit-identical to the scalar sequence (:252-257).
                const SphGroup<T> cur = load_group(fe, g);
                const f2 ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
                const f2 dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z};
                const f2 na = {-a, -a};
                const Q4 si = sidx(g, ip);
#pragma unroll
                for (uint32_t q = 0; q < 2; ++q) {
                    if (!((pairs >> q) & 1u)) continue;
                    f2 hb, disc;
                    const T* v = &cur.v[8 * q];
                    const f2 cx = {v[0], v[1]}, cy = {v[2], v[3]}, cz = {v[4], v[5]}, r2 = {v[6], v[7]};
                    const f2 ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;             // :252
                    if constexpr (SCALAR) {                                           // objects.rs:217-222
                        hb = (ocx * dx + ocy * dy) + ocz * dz;
                        const f2 c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2;
                        disc = hb * hb - (-na) * c;
                    } else {
                        hb = fma2(ocz, dz, fma2(ocy, dy, ocx * dx));                  // :255
                        const f2 c = fma2(ocz, ocz, fma2(ocy, ocy, ocx * ocx)) - r2;  // :256
                        disc = fma2(hb, hb, na * c);                                  // :257
                    }
                    if (cand_f(hb.x, disc.x)) hit(hb.x, disc.x, q ? si.z : si.x);
                    if (cand_f(hb.y, disc.y)) hit(hb.y, disc.y, q ? si.w : si.y);
                }
            } else {
                const SphGroup<T> c0 = load_group(fe, 2 * g), c1 = load_group(fe, 2 * g + 1);
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (!((pairs >> j) & 1u)) continue;
                    const T* v = j < 2 ? &c0.v[4 * j] : &c1.v[4 * (j - 2)];
                    const V3<T> oc = mk(o.x - v[0], o.y - v[1], o.z - v[2]);   // :252
                    if constexpr (SCALAR) {                                    // objects.rs:217-222
                        hb[j] = dot(oc, d);
                        disc[j] = hb[j] * hb[j] - a * (len2(oc) - v[3]);
                    } else {
                        hb[j] = pk_dot(oc, d);                                 // :255
                        const T c = pk_len2(oc) - v[3];                        // :256
                        disc[j] = fma(hb[j], hb[j], -a * c);                   // :257
                    }
                }
                const Q4 si = sidx(g, ip);
                const uint32_t sv[4] = {si.x, si.y, si.z, si.w};
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (((pairs >> j) & 1u) && cand_f(hb[j], disc[j])) hit(hb[j], disc[j], sv[j]);
            }
        };
        // fp32, scene-frame filter groups (not MEGA): the exact test of a taken group takes the centres
        // from its filter group, already in SGPRs (the same fp32 values, pack_filter / pack_sweep), and
        // loads only the group's r² and scene indices: one s_load_dwordx8 from its record, which follows the
        // cluster's filter groups in the same stream (round 6: a separate table behind a kernel-argument load
        // cost two dependent scalar round trips per taken group; C fp32 +1.1 %, profiles/r06/xrec_inline_ab.txt)
        auto exact4f = [&](const SphGroup<float>& cur, cptr<float> recp, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                cptr<uint32_t> xr = (cptr<uint32_t>)recp;
                uint32_t rec[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) rec[j] = xr[(uint32_t)j];
                const f2 ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
                const f2 dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z};
                const f2 na = {-a, -a};
#pragma unroll
                for (uint32_t q = 0; q < 2; ++q) {
                    if (!((pairs >> q) & 1u)) continue;
                    f2 hb, disc;
                    const float* v = &cur.v[8 * q];
                    const f2 cx = {v[0], v[1]}, cy = {v[2], v[3]}, cz = {v[4], v[5]};
                    const f2 r2 = {__uint_as_float(rec[2 * q]), __uint_as_float(rec[2 * q + 1])};
                    const f2 ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;             // :252
                    if constexpr (SCALAR) {                                           // objects.rs:217-222
                        hb = (ocx * dx + ocy * dy) + ocz * dz;
                        const f2 c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2;
                        disc = hb * hb - (-na) * c;
                    } else {
                        hb = fma2(ocz, dz, fma2(ocy, dy, ocx * dx));                  // :255
                        const f2 c = fma2(ocz, ocz, fma2(ocy, ocy, ocx * ocx)) - r2;  // :256
                        disc = fma2(hb, hb, na * c);                                  // :257
                    }
                    if (cand_f(hb.x, disc.x)) hit(hb.x, disc.x, rec[4 + 2 * q]);
                    if (cand_f(hb.y, disc.y)) hit(hb.y, disc.y, rec[5 + 2 * q]);
                }
            }
        };
        // Two levels (build_layout): the always-exact spheres first, then spatial clusters of 16
        // spheres (4 groups each) with bounding spheres, 4 bounds per top group.  Per chunk of 32
        // clusters: phase 1 tests the bounds with the lanes' filter (a cluster bound contains its
        // members, so it passes whenever a member's filter would) into a 32-bit wave mask; phase 2
        // walks the set clusters' groups with the per-sphere filter and, where it passes, the exact
        // test.  The phases never hold both SGPR pipelines at once (no SGPR spills).
        const uint32_t nxg = qa.n_xg, ntop = qa.n_top;
        // executed-work counts of this sweep (wave-uniform; work_add below)
        uint32_t n_box = 0, n_filt = 0, n_exact = 0;
        // the always-exact groups; fp32 skips a pair of dummies at the end (the ground sphere's group
        // at config C: ground + 3 dummies); in fp64 the variable pair mask costs VGPR spills at W4
        for (uint32_t g = 0; g < nxg; ++g) {
            const uint32_t pr = sizeof(T) == 4 ? (4u * g + 2u >= qa.n_xs ? 1u : 3u) : 15u;
            n_exact += pr == 1u ? 2u : 4u;
            exact4(g, pr);
        }
        // Three levels: super boxes (4 clusters each, 4 per group) per chunk of 32 supers, then the
        // passing supers' cluster boxes (one group each), then the passing clusters' sphere groups.
        // Scenes with more than 32 supers (config E: 157) test mega boxes (4 supers each) first, per
        // chunk of 32, and only the passing megas' super groups.
        cptr<float> ft = (cptr<float>)__builtin_assume_aligned(qa.ftop, 32);
        cptr<float> fs = (cptr<float>)__builtin_assume_aligned(qa.fsup, 32);
        const uint32_t nsg = (ntop + 3u) / 4u;   // super groups (ntop supers, one per cluster top group)
        // the clusters of one passing super: its group of 4 cluster boxes, then their sphere groups
        auto walk_super = [&](uint32_t sup) {
            KSTAT(5);
            ++n_box;
            uint32_t mask;
            if constexpr (MEGA) {
                mask = lmask(load_lbox((cptr<float>)__builtin_assume_aligned(qa.lclb, 64), sup));
            }
            else mask = box_mask(load_box(ft, sup), B0, B1, B2, B3, B4, btf());
            while (mask != 0u) {
                const uint32_t kc = 4u * sup + (uint32_t)__builtin_ctz(mask);   // cluster
                const uint32_t g0 = nxg + 4u * kc;
                mask &= mask - 1u;
                KSTAT(4);
                n_filt += 4u;
                f2 L0 = K0, L1 = K1, L2 = K2, L3 = K3;
                cptr<float> fg = ff;
                if constexpr (MEGA) {
                    // The cluster's frame (pack_local): o' = o - C_k (fp64 rays: in double, then
                    // rounded), the margin from |o'|_1 and the cluster's Rc, r2max and 1/r2min, the
                    // basis scaled by it, and o' projected on the scaled basis.
                    const auto& ql = *cold_args<T>();
                    // the cluster's block in the local stream: 4 groups, then 4 records whose unused r^2 words
                    // hold the frame {C_k, Rc} (record 0) and {r2max, 1/r2min} (record 1)
                    fg = (cptr<float>)__builtin_assume_aligned(ql.lfsph, 64) + 16u * nxg + 96u * kc;
                    const f2 Ckxy = {fg[64], fg[65]};
                    const float Ckz = fg[66];
                    const float Rc = fg[67], r2x = fg[72], ir2 = fg[73];
                    f2 opxy;
                    float opz;
                    if constexpr (sizeof(T) == 4) {
                        opxy = f2{o.x, o.y} - Ckxy;
                        opz = o.z - Ckz;
                    } else {
                        opxy = f2{(float)(o.x - (double)Ckxy.x), (float)(o.y - (double)Ckxy.y)};
                        opz = (float)(o.z - (double)Ckz);
                    }
                    const float opx = opxy.x, opy = opxy.y;
                    const float pmk = ((fabsf(opx) + fabsf(opy)) + fabsf(opz)) + Rc;
                    const float mk = kFilterMargin * __builtin_fmaf(pmk, pmk, r2x);
                    const float sgk = __builtin_amdgcn_rsqf(__builtin_fmaf(mk, ir2, 1.0f));
                    L0 = K0 * sgk; L1 = K1 * sgk; L2 = K2 * sgk;
                    const float oe1l = __builtin_fmaf(opz, L0.y, opx * L0.x);
                    const float oe2l = __builtin_fmaf(opz, L2.x, __builtin_fmaf(opy, L1.y, opx * L1.x));
                    L3 = f2{-oe1l, -oe2l};
                }
                // cluster kc's block in the filter stream: its 4 groups, then their 4 records (r^2 for the fp32
                // scene-frame stream, the scene indices), then (mega streams) the frame record (inline_stream)
                constexpr bool kInl = sizeof(T) == 4 && !MEGA && !CAMT;
                const cptr<float> fgb = MEGA ? fg : ff + 16u * nxg + 96u * kc;
                sphere_loop(fgb, 4u, [&](const SphGroup<float>& cur, uint32_t g) {
                    uint32_t s0, s1;
                    // A wave-uniform branch: lanes the filter rejects run the exact test too, and it
                    // rejects them as well (the filter passes every sphere the reference can hit).
                    f2 Dv[2];
                    const unsigned long long fpass = __ballot(is_cand(filter_group(cur, L0, L1, L2, L3, s0, s1, sizeof(T) == 8 ? Dv : nullptr)));
                    KSTAT(7, (uint32_t)__popcll(fpass));   // lanes with a candidate in this group
                    if (fpass != 0ull) {
                        // only the sphere pairs some lane passes (one compare each, taken groups
                        // only; fp64 too since the ray left scratch memory: +1.0 % at C).  fp64 rays
                        // (no packed ops): only the spheres some lane passes.
                        uint32_t pairs;
                        if constexpr (sizeof(T) == 4) {
                            pairs = (__ballot(!is_cand(s0)) != 0ull ? 1u : 0u) | (__ballot(!is_cand(s1)) != 0ull ? 2u : 0u);
                            n_exact += 2u * (uint32_t)__builtin_popcount(pairs);
                        } else {
                            auto ps = [](float D) -> bool { return (int32_t)__float_as_uint(D) >= 0; };   // D >= +0
                            pairs = (__ballot(ps(Dv[0].x)) != 0ull ? 1u : 0u) | (__ballot(ps(Dv[0].y)) != 0ull ? 2u : 0u) |
                                    (__ballot(ps(Dv[1].x)) != 0ull ? 4u : 0u) | (__ballot(ps(Dv[1].y)) != 0ull ? 8u : 0u);
                            n_exact += (uint32_t)__builtin_popcount(pairs);
                        }
                        if constexpr (kInl) exact4f(cur, fgb + 64u + 8u * g, pairs);
                        else
                            exact4(g0 + g, pairs, fgb + 68u + 8u * g);
                    }
                });
            }
        };
        // The top level is the super boxes, or (MEGA: scenes with more than 8 super groups, config E)
        // the mega boxes; chunks of 8 top groups (32 boxes) give a 32-bit wave mask of the passing
        // top boxes.  A mega box nd covers super group nd.  MEGA kernels test every level in
        // group-local frames (lmask).
        if constexpr (MEGA) {
            cptr<float> lm = (cptr<float>)__builtin_assume_aligned(qa.lmeg, 64);
            cptr<float> ls = (cptr<float>)__builtin_assume_aligned(qa.lsup, 64);
            const uint32_t ntg = qa.n_mg;
            // the supers of one passing mega
            auto walk_mega = [&](uint32_t nd) {
                ++n_box;
                uint32_t smask = lmask(load_lbox(ls, nd));
                if (4u * nd + 4u > ntop) smask &= (1u << (ntop - 4u * nd)) - 1u;   // padding supers
                while (smask != 0u) {
                    const uint32_t sup = 4u * nd + (uint32_t)__builtin_ctz(smask);
                    smask &= smask - 1u;
                    walk_super(sup);
                }
            };
            // Up to 64 megas (16 groups) at once: test them all, then walk the passing ones in tiers
            // of distance from the reference point's grid cell (the host's mega tier table: the megas
            // whose box touches the cell, then those within a quarter and a half of a mega's size,
            // then the rest), index order inside a tier.  More megas: chunks of 32 in index order.
            const uint32_t span = ntg <= 16u ? 16u : 8u;
            constexpr uint32_t kTest = 1;   // the tiers below kTest are walked before the top-level tests
            for (uint32_t t0 = 0; t0 < ntg; t0 += span) {
                const uint32_t nt = min(span, ntg - t0);
                // padding megas (empty boxes) past the last
                const uint64_t valid = 4u * (t0 + nt) > nsg ? (1ull << (nsg - 4u * t0)) - 1ull : ~0ull;
                // Tiers (span 16, up to 64 megas): T0 = the megas whose box touches the reference point's
                // grid cell (the first active lane's origin), T1 = those within a quarter of a mega's
                // size (the host's table, pack_mega_tiers); the tier-0 megas are walked first without
                // a top-level test (a mega the rays miss has no passing supers either), then all mega
                // boxes are tested, with the best hits found so far culling far ones, and the rest are
                // walked tier by tier, index order inside a tier.  Same-box E fp32: 9328 in index order,
                // 9819 with the tiers (profiles/r02/experiments/tiers.txt, tiers_t0.txt)
                uint64_t T0 = 0, T1 = 0;
                if (span == 16u) {
                    const auto& qt = *cold_args<T>();
                    auto cell = [](float v, float lo, float inv, uint32_t n) -> uint32_t {
                        const float c = fminf(fmaxf((v - lo) * inv, 0.0f), (float)(n - 1u));   // NaN -> 0
                        return __builtin_amdgcn_readfirstlane((uint32_t)c);
                    };
                    const uint32_t cx = cell((float)o.x, qt.mt_lo[0], qt.mt_inv, qt.mt_n[0]);
                    const uint32_t cy = cell((float)o.y, qt.mt_lo[1], qt.mt_inv, qt.mt_n[1]);
                    const uint32_t cz = cell((float)o.z, qt.mt_lo[2], qt.mt_inv, qt.mt_n[2]);
                    const uint32_t ci = 4u * (cx + qt.mt_n[0] * (cy + qt.mt_n[1] * cz));
                    cptr<uint64_t> tt = (cptr<uint64_t>)__builtin_assume_aligned(qt.mtiers, 32);
                    T0 = tt[ci] & valid;
                    T1 = tt[ci + 1u] & valid;
                }
                uint64_t tm = 0;
#pragma unroll 1
                for (uint32_t k = 0; k < 3u; ++k) {
                    if (k == kTest) {
                        const uint32_t ngg = span == 16u ? qa.n_gg : 0u;
                        if (ngg != 0u) {
                            // Gigas (one mega group's 4 megas each, k-d subtrees): the giga boxes first, then
                            // the mega groups of the passing gigas only.  A giga box holds its megas' boxes,
                            // so a mega of a culled giga would fail its own test: tm is unchanged.
                            uint32_t gm = 0;
                            n_box += ngg;
                            lbox_loop((cptr<float>)__builtin_assume_aligned(qa.lgig, 64), ngg,
                                      [&](const LBoxGroup& cur, uint32_t t) { gm |= lmask(cur) << (4u * t); });
                            gm &= (1u << nt) - 1u;
                            while (gm != 0u) {
                                const uint32_t gg = (uint32_t)__builtin_ctz(gm);
                                gm &= gm - 1u;
                                ++n_box;
                                tm |= (uint64_t)lmask(load_lbox(lm, gg)) << (4u * gg);
                            }
                        } else {
                            n_box += nt;
                            for (uint32_t t1 = 0; t1 < nt; t1 += 8u)
                                lbox_loop(lm + 32u * (t0 + t1), min(8u, nt - t1), [&](const LBoxGroup& cur, uint32_t t) {
                                    KSTAT(5);
                                    tm |= (uint64_t)lmask(cur) << (4u * (t1 + t));
                                });
                        }
                        tm &= valid;
                    }
                    uint64_t w = k == 0u ? (kTest == 0u ? tm & T0 : T0)
                                         : (k == 1u ? (kTest <= 1u ? tm & T1 : T1) & ~T0 : tm & ~T1);
                    while (w != 0ull) {
                        const uint32_t nd = 4u * t0 + (uint32_t)__builtin_ctzll(w);
                        w &= w - 1ull;
                        walk_mega(nd);
                    }
                }
            }
        } else {
            for (uint32_t t0 = 0; t0 < nsg; t0 += 8u) {
                uint32_t tmask = 0;
                n_box += min(8u, nsg - t0);
                box_loop(fs + kBoxFloats * t0, min(8u, nsg - t0), [&](const BoxGroup& cur, uint32_t t) {
                    KSTAT(5);
                    tmask |= box_mask(cur, B0, B1, B2, B3, B4, btf()) << (4u * t);
                });
                while (tmask != 0u) {
                    const uint32_t nd = 4u * t0 + (uint32_t)__builtin_ctz(tmask);
                    tmask &= tmask - 1u;
                    // padding supers past the last one are empty boxes; a degenerate lane (all box
                    // times NaN) passes them, and nothing lies behind them
                    if (nd >= ntop) break;
                    walk_super(nd);
                }
            }
        }
        work_add(kWBox, n_box);
        work_add(kWFilt, n_filt);
        work_add(kWExact, n_exact);
    }
    t_out = bh.bt();
    return bh.bi();
}

}  // namespace rt
