// rt_common.hpp — device-side building blocks shared by every stage of the megakernel: the scene's
// group layouts (scalar-cache loads), the kernel arguments, the executed-work counters and the
// two-deep scalar-load pipelines.  Part of the single translation unit rt_kernel.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <array>
#include <initializer_list>
#include <chrono>
#include <cmath>
#include <limits>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "rt_device.hpp"
#include "rt_experiments.hpp"

namespace rt {

template <typename T> struct MatT {
    uint32_t kind, hollow;
    // Lambertian / metal: {albedo r, g, b, fuzz}; dielectric: {ior, 1/ior, r0_front, r0_back} -- the constants
    // precomputed on the host in T with the reference's operations (IEEE, no contraction, so the bits equal the
    // per-ray device computation): 1/ior (materials.rs:131) and Schlick's r0 = ((1-ratio)/(1+ratio))^2
    // (materials.rs:122) for ratio = 1/ior and ior.  Only the fields of the record's kind: fp64 40 bytes, fp32 24.
    T p[4];
};

// Device sphere layout (rt_context_set_scene): 64-byte groups, one s_load_dwordx16 each, padded
// with never-hit dummies (r^2 = -inf makes the discriminant -inf) to whole groups.
//   fp32: 4 spheres per group as 2 pair-interleaved records {cx0,cx1, cy0,cy1, cz0,cz1, r0,r1}
//         so each quantity of a sphere pair is an adjacent SGPR pair for packed-FP32 VALU ops;
//   fp64: 2 spheres per group as {cx, cy, cz, r^2}.
// A separate AoS table {cx, cy, cz, r^2} per sphere serves the per-lane finalize gather.
// The filter stream (both precisions) is fp32 in the fp32 layout, with r^2 replaced by the filter's
// r2f: r^2 rounded up to fp32, +inf for "always exact" spheres, -inf for dummies (see
// general_sweep).
template <typename T> constexpr uint32_t kGroup = 64 / (4 * sizeof(T));
template <typename T> struct alignas(64) SphGroup { T v[64 / sizeof(T)]; };

// One 64-byte scalar load worth of spheres (s_load_dwordx16 into SGPRs).
template <typename T>
__device__ __forceinline__ SphGroup<T> load_group(const __attribute__((address_space(4))) T* f, uint32_t g) {
    constexpr int NE = 64 / sizeof(T);
    SphGroup<T> r;
#pragma unroll
    for (int e = 0; e < NE; ++e) r.v[e] = f[g * NE + e];
    return r;
}

typedef float f2 __attribute__((ext_vector_type(2)));
struct Q4 { uint32_t x, y, z, w; };

// One top group of the general sweep: 4 cluster boxes {centre, half-extent} (pack_sweep), 96 bytes,
// pair-interleaved like SphGroup: pair q at 12 q, {cx0,cx1, cy0,cy1, cz0,cz1, hx0,hx1, hy0,hy1, hz0,hz1}.
constexpr uint32_t kBoxFloats = 24;
struct alignas(32) BoxGroup { float v[kBoxFloats]; };
__device__ __forceinline__ BoxGroup load_box(const __attribute__((address_space(4))) float* f, uint32_t g) {
    BoxGroup r;
#pragma unroll
    for (uint32_t e = 0; e < kBoxFloats; ++e) r.v[e] = f[g * kBoxFloats + e];
    return r;
}
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <typename T> struct KParams {
    const T* sph;              // grouped sphere records (layout above); r^2 = r.powi(2) in T (objects.rs:256)
    const T* cen;              // [n][4] = cx, cy, cz, r^2 (AoS, finalize gather)
    uint32_t n_groups;
    const MatT<T>* mats;       // [n] each sphere's material record, materials[material[i]] (one gather)
    uint32_t n_spheres;
    uint32_t W, H;
    double rW, rH;             // RN(1/W), RN(1/H) for div_dim (0: divide)
    T center[3], ulc[3], vu[3], vv[3], du[3], dv[3];
    uint32_t spp, P, C, depth, flags, s_sel, k0, k1;
    uint32_t row_begin, row_step, col_begin, col_count;
    uint8_t* rgb;
    double* lin;
    unsigned long long* segs;  // kSegShards shards of kSegStride counters (256 B per shard; direct_sky_samples at slot 16)
    uint32_t* err;
    uint32_t* counter;         // next block of work items (guided_block)
    uint32_t blk_g;            // largest block (a power of two <= kMaxBlock; launch_t)
    uint32_t n_items;
    char* scratch;             // per-wave scratch regions
    size_t scratch_stride;
    uint32_t vbytes, sbytes;   // trace_paths: position-map bytes, per-slot record bytes (PScratch)
    uint32_t swide;            // PScratch::wide
    const T* camsph;           // camera-origin table {oc, c} in the sph layout (pinhole launches)
    const float* fsph;         // filter stream: fp32 groups of 4 {cx, cy, cz, r2f} (layout above)
    const float* camf;         // camera filter table: fp32 groups of 4 {ocx, ocy, ocz, sc} (build_cam_table)
    uint32_t n_fgroups;
    float f_cmax, f_r2max;     // filter margin bounds: max |c|_1 and max r2f over non-exact spheres
    float f_r2min;             // min r2f over non-exact spheres (after the host's floor)
    float f_ir2, f_hir2, f_isr; // 1/r2min, 0.5/r2min and 8 u/sqrt(r2min), rounded up (launch_t)
    const float* cull;         // camera cone-cull records {wx, wy, wz, rp} per slot of the sweep layout
    const float* cullc;        // ... and per cluster, then per super (build_cam_table)
    uint32_t n_clp, n_supc;    // cluster records (x64), super records after them (x64; 0: none)
    const T* camx;             // camera-origin table per sphere {ocx, ocy, ocz, c} (AoS; build_cam_table)
    // general sweep, two-level (build_layout / pack_sweep): slot-order exact and filter streams,
    // cluster bounds (fp32 groups of 4 {cx, cy, cz, R2}), slot -> scene index; n_top top groups,
    // n_xg leading groups of always-exact spheres, then cluster k at groups n_xg + 4k .. + 3
    const T* rsph;
    const float* rfsph;        // its fp32 filter groups, inline: cluster k's 4 groups at 16 n_xg + 96 k, then
                               // their 4 records {r^2 of the pairs (fp32 rays), 4 scene indices} (inline_stream)
    const float* ftop;
    const float* fsup;         // super boxes (4 clusters each), 4 per group
    const float* fmeg;         // mega boxes (4 supers each), 4 per group; n_mg groups, 0: no mega level
    uint32_t n_mg;
    // MEGA kernels: the sphere filter in cluster-local frames (pack_local): filter groups with centres
    // relative to their cluster's centre, inline with each cluster's records (set_scene's inline_stream: the
    // scene indices, and the frame {Cx, Cy, Cz, Rc} / {r2max, 1/r2min} in the r^2 words of records 0 / 1)
    const float* lfsph;
    const float* lclb;         // ... the box levels in group-local frames (pack_local_boxes): per super its
    const float* lsup;         //     4 cluster boxes, per mega its 4 supers, per mega group its 4 megas
    const float* lmeg;
    const float* lgig;         //     and per giga group its 4 gigas (a giga: one mega group, 4 megas)
    uint32_t n_gg;             // giga groups (0: the megas are tested without the giga pre-test)
    float l_r2max, l_hir2, l_isr;   // their margin constants: max local r2f, 48 u 0.5 / min, 8 u / sqrt(min)
    // ... and the mega walk's order (<= 64 megas): a grid over the megas' union, per cell 4 u64 words
    // {touching, within 1/4 of a mega's size, within 1/2, 0} (pack_mega_tiers)
    const uint64_t* mtiers;
    float mt_lo[3], mt_inv;
    uint32_t mt_n[3];
    const uint32_t* ridx;
    uint32_t n_top, n_xg, n_xs;   // n_xs: always-exact spheres (the rest of their last group are dummies)
};

constexpr int kSegShards = 256;
constexpr uint32_t kFlagPinholeInternal = 0x80000000u;   // set by the host: defocus vectors are +-0
constexpr int kWavesF32 = 6;   // default min-waves-per-SIMD targets (measured sweep);
constexpr int kWavesF64 = 4;   // RT_WAVES (read per launch) selects another for the live-path kernels
constexpr int kWavesMegaF32 = 6;   // the mega-level kernels (config E; RT_WAVES=5 selects the W5 build)
// fp32 launches with fewer pixels than this per resident W6 wave run at W5: W6's extra waves then split
// the pixels thinner and the tail costs more than the occupancy gains.  tools/waves_ab.py with the claim
// streams (rt_trace.hpp), W6/W5 speed: C whole 1.058, 8-way shards (42 px per W6 wave) 1.032, 16-way
// (21) 0.971; B 4-way (37.5) 1.056, 8-way (18.8) 0.966.  (Round 3's one claim counter put the 8-way
// C shard on the other side.)
constexpr uint64_t kW6PixelsPerWave = 24;
// RT_WAVES=7 selects a 7-waves-per-SIMD fp32 live-path build (72 VGPRs; the LDS of 7 workgroups
// just fits): +2 % on C and D, but it spills ~7 VGPRs around every sweep, and the scratch lines
// (4 MB per XCD) push HBM writes from 23 to 41 B/sample, so the default stays at 6
template <typename T> constexpr int kWavesModes = sizeof(T) == 4 ? 6 : 4;   // ROOT2 and semantics modes
constexpr int kSegStride = 32;  // u64 per shard (256 B)
constexpr float kFilterMargin = 48.0f * 0x1.0p-24f;   // general-sweep filter margin factor (nearest_hit)
constexpr double kExactRatio = 8.0;  // spheres with |c|_1 + r > kExactRatio x the median are "always exact"

// Executed-work counters (product build): per wave, the wave-level tests the culls and
// exact tests actually run, one LDS add per sweep or camera batch, flushed to shard slots
// kWorkSlot.. at the end.  The host turns them into executed FLOP (rt_work_stats).
enum WorkCounter : uint32_t {
    kWBox = 0,      // general sweep: box groups tested (4 boxes, 18 v_pk_fma_f32)
    kWFilt = 1,     // general sweep: filter groups tested (4 spheres, 14 v_pk_fma_f32)
    kWExact = 2,    // general sweep: spheres through the reference's exact test (17 FLOP in T each)
    kWCone = 3,     // camera sweep: cone tests (64 records per wave test, 23 fp32 FLOP)
    kWCExact = 4,   // camera sweep: exact tests from the camera-origin table (8 FLOP in T each)
    kNWork = 5,
};
constexpr int kWorkSlot = 11;   // shard slots 11..15 (kstats uses 3..10)
constexpr int kDirectSkySlot = 16;   // samples of pixels finished at claim time (rt_stats.direct_sky_samples)
static_assert(kWorkSlot + kNWork <= kDirectSkySlot && kDirectSkySlot < kSegStride, "counters past the shard's slots");
// u64: a wave of a persistent launch can run billions of tests (config E: ~1.3M filter groups per
// wave; spp up to 2^20 on a 4K frame is ~3000x that), past a u32.
__shared__ unsigned long long g_work[4][kNWork];
// Add wave-uniform counts from the first active lane (the caller may be inside a divergent branch).
__device__ __forceinline__ void work_add(uint32_t i, uint32_t n) {
    const uint32_t first = (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
    if ((threadIdx.x & 63u) == first) atomicAdd(&g_work[threadIdx.x >> 6][i], (unsigned long long)n);
}


// #{set bits of m in the lanes below this one}: v_mbcnt_lo/hi, no lane mask held in VGPRs
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Uniform (scalar-cache) view of a read-only kernel buffer: the sphere loop index is
// wave-uniform, so these become s_load into SGPRs — a free broadcast to all 64 lanes.
template <typename T> using cptr = const __attribute__((address_space(4))) T*;

// Cold kernel arguments (the camera) are read through an opaque pointer to the kernarg segment
// at their point of use: otherwise the backend hoists every kernarg load to the kernel entry and
// keeps ~40 camera SGPRs live across the whole persistent loop (SGPR spills into VGPR lanes).
template <typename T> __device__ __forceinline__ cptr<KParams<T>> cold_args() {
    cptr<KParams<T>> k = (cptr<KParams<T>>)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return k;
}
// Same, but ordered after `dep` is computed: loads through it cannot be hoisted above that value's
// producer (used to keep the camera constants out of SGPRs while a Philox block is in flight).
template <typename T> __device__ __forceinline__ cptr<KParams<T>> cold_args_after(uint32_t dep) {
    cptr<KParams<T>> k = (cptr<KParams<T>>)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k) : "v"(dep));
    return k;
}

// x / W for the camera's pixel coordinate (ray_tracing.rs:78-79), W the image width or height.
// fp32: RN_f(RN_d(x * RN_d(1/W))) == RN_f(x / W).  The double product is within 2^-52 relative of
// x / W; a quotient of a float by an integer W < 2^20 that is not a float midpoint lies at least
// 2^-25 / W (>= 2^-45) relative from every midpoint, and it is never one (an odd 25-bit mantissa
// times W has more than 24 significant bits).  3 ops instead of the ~10 of a correctly rounded fp32 divide.  The
// host sets r = 0 (plain division) for larger images; fp64 always divides.
template <typename T> __device__ __forceinline__ T div_dim(T x, uint32_t W, double r) {
    if constexpr (sizeof(T) == 4) {
        if (r != 0.0) return (float)((double)x * r);
    }
    return x / (T)W;
}

// Walk the sphere groups with a two-deep scalar-load pipeline over two SGPR buffers (no
// per-group SGPR copies).  Scalar loads return out of order, so any use waits lgkmcnt(0): the
// next group's load is pinned (sched_barrier) BEFORE the current group's math and waited right
// after it, so it is always one whole group of VALU work old when it is consumed.  The device
// buffer holds a dummy group past the end, so the prefetches never need clamping.
// The same two-deep pipeline over the general sweep's box groups (cluster bounds).
template <typename F>
__device__ __forceinline__ void box_loop(cptr<float> f, uint32_t ng, F&& group) {
    BoxGroup A = load_box(f, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t g = 0;
    for (; g + 1 < ng; g += 2) {
        const BoxGroup B = load_box(f, g + 1);
        __builtin_amdgcn_sched_barrier(0);
        group(A, g);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        A = load_box(f, g + 2);
        __builtin_amdgcn_sched_barrier(0);
        group(B, g + 1);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (g < ng) group(A, g);
}

// A box group in a group-local frame (MEGA kernels, pack_local_boxes): 24 floats of boxes (BoxGroup
// layout), then the frame {Sx, Sy, Sz, Rg}, padded to 128 bytes (two s_load_dwordx16).
struct alignas(64) LBoxGroup { float v[32]; };
__device__ __forceinline__ LBoxGroup load_lbox(const __attribute__((address_space(4))) float* f, uint32_t g) {
    LBoxGroup r;
#pragma unroll
    for (uint32_t e = 0; e < 28; ++e) r.v[e] = f[g * 32u + e];
    return r;
}
template <typename F>
__device__ __forceinline__ void lbox_loop(cptr<float> f, uint32_t ng, F&& group) {
    LBoxGroup A = load_lbox(f, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t g = 0;
    for (; g + 1 < ng; g += 2) {
        const LBoxGroup B = load_lbox(f, g + 1);
        __builtin_amdgcn_sched_barrier(0);
        group(A, g);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        A = load_lbox(f, g + 2);
        __builtin_amdgcn_sched_barrier(0);
        group(B, g + 1);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (g < ng) group(A, g);
}

template <typename T, typename F>
__device__ __forceinline__ void sphere_loop(cptr<T> f, uint32_t ng, F&& group) {
    SphGroup<T> A = load_group(f, 0);
    // Wait for the first group here: otherwise the loop header inherits its pending load and the
    // compiler's wait before the first use also waits for the group just prefetched in the body.
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t g = 0;
    for (; g + 1 < ng; g += 2) {
        const SphGroup<T> B = load_group(f, g + 1);
        __builtin_amdgcn_sched_barrier(0);
        group(A, g);
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): B has landed
        __builtin_amdgcn_sched_barrier(0);
        A = load_group(f, g + 2);
        __builtin_amdgcn_sched_barrier(0);
        group(B, g + 1);
        __builtin_amdgcn_s_waitcnt(0xC07F);   // A has landed
        __builtin_amdgcn_sched_barrier(0);
    }
    if (g < ng) group(A, g);
}

}  // namespace rt
