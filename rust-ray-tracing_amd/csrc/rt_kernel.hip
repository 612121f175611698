// rt_kernel.hip — MI355X (gfx950) megakernel for the reference's per-pixel sample loop.
//
// Replaces TileRenderTask::render_vectorized2 (src/renderer.rs:141-176) and everything it
// calls: Camera::get_ray (ray_tracing.rs:77-89), Scene::trace_vectorized2
// (ray_tracing.rs:375-505), Sphere::hit_packed (objects.rs:249-290), PackedHitRecords
// (objects.rs:121-176), Material::get_hit_result (materials.rs:54-147), the final sky pass and
// reduction (ray_tracing.rs:486-504), /spp and Color::to_u8_array (renderer.rs:161,
// color.rs:54-64).
//
// Mapping:
//   * path regeneration: a persistent wave keeps one ray per lane from its camera ray to its
//     termination, then takes the next sample (of this pixel or of the next one its workgroup
//     claims from an atomic block counter; up to kSlots pixels in flight).  Every ray's bounce k depends only
//     on its own state and the counter-based RNG key (sample, pixel, k, stream), so no ray waits
//     for the others; lane utilisation is ~1.0.
//   * each sweep finds every sphere the reference could hit through conservative fp32 culls and
//     runs the reference's exact test on those only: spheres stream through the scalar cache in
//     64-byte groups (s_load_dwordx16 into SGPRs, a free broadcast to all 64 lanes), two spheres
//     per packed-FP32 instruction; bounced rays first slab-test 16-sphere cluster boxes, then a
//     per-sphere distance filter on the clusters some lane may hit (nearest_hit).
//   * pinhole cameras: primary rays run in full-wave camera batches; a cone around the batch's
//     rays culls clusters and spheres with lanes as spheres (camera_sweep), survivors get the
//     exact test from a per-launch camera-origin table (oc and c are the same for every primary
//     ray); hits wait in an LDS queue for free lanes.
//   * the reference's positions (its per-bounce stable shuffle) are a function of the per-sample
//     termination bounces alone; when a pixel's last sample ends, finish_pixel replays them,
//     applies quirk Q3's buffer read ("retire rule") and sums in the reference's order, so fp64
//     and fp32 results are bit-identical to the CPU restatement in oracle/.
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

// Build kinds.  The product library (make) defines RT_PRODUCT and refuses every experiment macro
// below; the A/B builds (make exp / kstats) define RT_EXPERIMENT, and rt_version() says so, which
// rt_mi355x.load_library refuses unless RT_ALLOW_EXPERIMENT=1.  Every experiment keeps the results
// bit-identical (timing or ordering changes only); tests/test_abi.py checks that this list names
// every RT_EXP_ macro the source tests.
#if defined(RT_PRODUCT) && defined(RT_EXPERIMENT)
#error "RT_PRODUCT and RT_EXPERIMENT are exclusive"
#endif
#if defined(RT_PRODUCT) && (defined(RT_EXP_FLAT_SWEEP) || defined(RT_EXP_NO_PRUNE) || defined(RT_EXP_NO_XREC) ||   \
                            defined(RT_EXP_KTEST) || defined(RT_EXP_NO_ORDER) || defined(RT_EXP_SLOTS) ||            \
                            defined(RT_EXP_BLOCK_SAMPLES) || defined(RT_EXP_TMUL) || defined(RT_EXP_OLD_REPLAY) ||   \
                            defined(RT_EXP_NO_PARK) || defined(RT_EXP_PARKC_ALL) || defined(RT_EXP_DUP_FINISH) ||    \
                            defined(RT_EXP_DUP_CAMRAY) || defined(RT_EXP_NO_CAMCULL) || defined(RT_EXP_DUP_CAM) ||   \
                            defined(RT_EXP_DUP_SCATTER) || defined(RT_EXP_DUP_SWEEP) || defined(RT_EXP_LMAP_CAP) ||   \
                            defined(RT_EXP_DUP_CLBOX) || defined(RT_EXP_DUP_FILTER) || defined(RT_EXP_DUP_SUPBOX) ||  \
                            defined(RT_EXP_DUP_MEGABOX) || defined(RT_EXP_DUP_PLIST) || defined(RT_EXP_DUP_REPLAY) || \
                            defined(RT_EXP_DUP_REDUCE) || \
                            defined(RT_KSTATS))
#error "an experiment macro in the product build"
#endif
#ifndef RT_SRC_HASH
#define RT_SRC_HASH "unknown"
#endif
#ifdef RT_EXPERIMENT
#define RT_BUILD_KIND "experiment"
#else
#define RT_BUILD_KIND "product"
#endif

namespace rt {

template <typename T> struct MatT {
    uint32_t kind, hollow;
    T ar, ag, ab, fuzz, ior;
    // Dielectric constants precomputed on the host in T with the reference's operations (IEEE,
    // no contraction, so the bits equal the per-ray device computation): 1/ior (materials.rs:131)
    // and Schlick's r0 = ((1-ratio)/(1+ratio))^2 (materials.rs:122) for ratio = 1/ior and ior.
    T inv_ior, r0_front, r0_back;
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
    unsigned long long* segs;  // kSegShards counters, one per 128-B line
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
    const float* rfsph;
    const uint32_t* xrec;      // fp32: per slot group {r² of pair 0, r² of pair 1, 4 scene indices} (32 B)
    const float* ftop;
    const float* fsup;         // super boxes (4 clusters each), 4 per group
    const float* fmeg;         // mega boxes (4 supers each), 4 per group; n_mg groups, 0: no mega level
    uint32_t n_mg;
    // MEGA kernels: the sphere filter in cluster-local frames (pack_local): filter groups with centres
    // relative to their cluster's centre, and per cluster {Cx, Cy, Cz, Rc, r2max, 1/r2min, 0, 0}
    const float* lfsph;
    const float* lclu;
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
// fp32 launches below this many samples per resident W6 wave run at W5: W6's extra waves then split
// the pixels thinner and the tail costs more than the occupancy gains (tools/waves_ab.py: an 8-way
// shard of C, 21 600 samples per wave, is 6 % slower at W6; the 4-way shard, 43 200, 5.6 % faster)
constexpr uint64_t kW6SamplesPerWave = 32768;
// RT_WAVES=7 selects a 7-waves-per-SIMD fp32 live-path build (72 VGPRs; the LDS of 7 workgroups
// just fits): +2 % on C and D, but it spills ~7 VGPRs around every sweep, and the scratch lines
// (4 MB per XCD) push HBM writes from 23 to 41 B/sample, so the default stays at 6
template <typename T> constexpr int kWavesModes = sizeof(T) == 4 ? 6 : 4;   // ROOT2 and semantics modes
constexpr int kSegStride = 16;  // u64 per shard (128 B)
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
static_assert(kWorkSlot + kNWork <= kSegStride, "work counters past the shard's line");
// u64: a wave of a persistent launch can run billions of tests (config E: ~1.3M filter groups per
// wave; spp up to 2^20 on a 4K frame is ~3000x that), past a u32.
__shared__ unsigned long long g_work[4][kNWork];
// Add wave-uniform counts from the first active lane (the caller may be inside a divergent branch).
__device__ __forceinline__ void work_add(uint32_t i, uint32_t n) {
    const uint32_t first = (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
    if ((threadIdx.x & 63u) == first) atomicAdd(&g_work[threadIdx.x >> 6][i], (unsigned long long)n);
}

// Instrumented build only (make kstats): wave-level event counters, written to shard slots 3..10.
#ifdef RT_KSTATS
__shared__ unsigned long long g_kst[4][8];
__device__ __forceinline__ void kstat(uint32_t i, uint32_t n = 1) {
    const unsigned long long ex = __builtin_amdgcn_read_exec();
    if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(ex)) atomicAdd(&g_kst[threadIdx.x >> 6][i], (unsigned long long)n);
}
#define KSTAT(...) kstat(__VA_ARGS__)
#else
#define KSTAT(...) ((void)0)
#endif

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
template <typename T, bool root2, bool SCALAR>
__device__ __forceinline__ void hit_update(T hb, T disc, uint32_t i, T a, T inv_a, T& best_t, int& best) {
    if constexpr (SCALAR) {
        const T sd = sqrt(disc);
        T root = (-hb - sd) / a;
        if (!(root >= T(0.001) && root < T(INFINITY))) {
            root = (-hb + sd) / a;
            if (!(root >= T(0.001) && root < T(INFINITY))) return;
        }
        if (root < best_t || (root == best_t && (int)i < best)) { best_t = root; best = (int)i; }   // first wins
        return;
    }
    const T sd = sqrt(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270
    bool valid = r1 >= T(0.001) && r1 < T(INFINITY);       // :272
    T root = r1;
    if (root2 && !valid) {                                 // Q1 off: scalar semantics
        root = (-hb + sd) * inv_a;                         // :271
        valid = root >= T(0.001) && root < T(INFINITY);
    }
    if (valid && (root < best_t || (root == best_t && (int)i > best))) { best_t = root; best = (int)i; }   // ties: later wins (:141)
}

template <typename T, bool root2, bool SCALAR = false, bool CAMT = false, bool MEGA = false>
__device__ __forceinline__ int nearest_hit(const KParams<T>& p, const V3<T>& o, const V3<T>& d, T& t_out) {
    const T a = SCALAR ? len2(d) : pk_len2(d);       // objects.rs:219 / :253
    const T inv_a = SCALAR ? T(0) : T(1.0) / a;      // objects.rs:254 (loop-invariant)
    T best_t = T(INFINITY);          // PackedHitRecords::default, objects.rs:128
    int best = -1;
    // Sphere::hit_packed (objects.rs:249-290) + PackedHitRecords::update (objects.rs:140-155)
    // for a candidate whose discriminant is non-negative.  Exact pre-filter: with hb >= 0,
    // root1 = (-hb - sd)*inv_a <= 0 can never be valid, so only Q1-off (root2) mode needs it.
    KSTAT(CAMT ? 3 : 1);   // sweeps (one per wave)
    auto hit = [&](T hb, T disc, uint32_t i) { hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, best_t, best); };
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
#ifdef RT_EXP_FLAT_SWEEP
        cptr<float> ff = (cptr<float>)__builtin_assume_aligned(qa.fsph, 64);
        cptr<T> fe = (cptr<T>)__builtin_assume_aligned(qa.sph, 64);
        const uint32_t ngf = qa.n_fgroups;
        auto sidx = [&](uint32_t g) -> Q4 { return Q4{4 * g, 4 * g + 1, 4 * g + 2, 4 * g + 3}; };
#else
        cptr<float> ff = (cptr<float>)__builtin_assume_aligned(qa.rfsph, 64);
        cptr<T> fe = (cptr<T>)__builtin_assume_aligned(qa.rsph, 64);
        auto sidx = [&](uint32_t g) -> Q4 {   // scene indices of slot group g (one s_load_dwordx4)
            const auto& qi = *cold_args<T>();
            cptr<uint32_t> ri = (cptr<uint32_t>)__builtin_assume_aligned(qi.ridx, 16);
            return Q4{ri[4 * g], ri[4 * g + 1], ri[4 * g + 2], ri[4 * g + 3]};
        };
#endif
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
#ifdef RT_EXP_NO_PRUNE
            return INFINITY;
#else
            if constexpr (sizeof(T) == 4) return best_t;
            else return (float)best_t * (1.0f + 0x1.0p-22f);   // RN(RN(b) (1 + 2^-22)) > b (b > 0)
#endif
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
        auto exact4 = [&](uint32_t g, uint32_t pairs = sizeof(T) == 4 ? 3u : 15u) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                // Packed FP32: each v_pk_{add,mul,fma}_f32 evaluates the same IEEE op for two
                // spheres, so the results are bit-identical to the scalar sequence (:252-257).
                const SphGroup<T> cur = load_group(fe, g);
                const f2 ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
                const f2 dx = {d.x, d.x}, dy = {d.y, d.y}, dz = {d.z, d.z};
                const f2 na = {-a, -a};
                const Q4 si = sidx(g);
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
                const Q4 si = sidx(g);
                const uint32_t sv[4] = {si.x, si.y, si.z, si.w};
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (((pairs >> j) & 1u) && cand_f(hb[j], disc[j])) hit(hb[j], disc[j], sv[j]);
            }
        };
        // fp32, scene-frame filter groups (not MEGA): the exact test of a taken group takes the centres
        // from its filter group, already in SGPRs (the same fp32 values, pack_filter / pack_sweep), and
        // loads only the group's r² and scene indices (one s_load_dwordx8 instead of the 64-byte exact
        // group plus the index table behind a kernel-argument load)
        auto exact4f = [&](const SphGroup<float>& cur, uint32_t g, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                const auto& qx = *cold_args<T>();
                cptr<uint32_t> xr = (cptr<uint32_t>)__builtin_assume_aligned(qx.xrec, 32);
                uint32_t rec[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) rec[j] = xr[8u * g + (uint32_t)j];
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
#ifdef RT_EXP_FLAT_SWEEP
        auto group = [&](const SphGroup<float>& cur, uint32_t g) {
            uint32_t s0, s1;
            if (is_cand(filter_group(cur, K0, K1, K2, K3, s0, s1))) exact4(g);
        };
        sphere_loop(ff, ngf, group);
#else
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
#ifdef RT_EXP_DUP_CLBOX   // timing experiment: the cluster-box test twice (same result)
                { uint32_t sup2 = sup; asm volatile("" : "+s"(sup2)); const uint32_t m2 = lmask(load_lbox((cptr<float>)__builtin_assume_aligned(qa.lclb, 64), sup2)); asm volatile("" :: "s"(m2)); }
#endif
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
                    cptr<float> lr = (cptr<float>)__builtin_assume_aligned(ql.lclu, 32);
                    const f2 Ckxy = {lr[8u * kc], lr[8u * kc + 1u]};
                    const float Ckz = lr[8u * kc + 2u];
                    const float Rc = lr[8u * kc + 3u], r2x = lr[8u * kc + 4u], ir2 = lr[8u * kc + 5u];
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
                    fg = (cptr<float>)__builtin_assume_aligned(ql.lfsph, 64);
                }
                sphere_loop(fg + 16u * g0, 4u, [&](const SphGroup<float>& cur, uint32_t g) {
                    uint32_t s0, s1;
                    // A wave-uniform branch: lanes the filter rejects run the exact test too, and it
                    // rejects them as well (the filter passes every sphere the reference can hit).
#ifdef RT_EXP_DUP_FILTER   // timing experiment: the filter of each walked group twice (same result)
                    { f2 M0 = L0; asm volatile("" : "+v"(M0)); uint32_t a0, a1; const uint32_t r2 = filter_group(cur, M0, L1, L2, L3, a0, a1); asm volatile("" :: "v"(r2), "v"(a0), "v"(a1)); }
#endif
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
#ifndef RT_EXP_NO_XREC
                        if constexpr (sizeof(T) == 4 && !MEGA && !CAMT) exact4f(cur, g0 + g, pairs);
                        else
#endif
                            exact4(g0 + g, pairs);
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
#ifdef RT_EXP_DUP_SUPBOX   // timing experiment: the super-box test twice (same result)
                { uint32_t nd2 = nd; asm volatile("" : "+s"(nd2)); const uint32_t m2 = lmask(load_lbox(ls, nd2)); asm volatile("" :: "s"(m2)); }
#endif
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
#ifndef RT_EXP_KTEST
#define RT_EXP_KTEST 1
#endif
            constexpr uint32_t kTest = RT_EXP_KTEST;   // the tiers below kTest are walked before the top-level tests
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
#if !defined(RT_EXP_NO_ORDER)
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
#endif
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
#ifdef RT_EXP_DUP_MEGABOX   // timing experiment: the mega-box tests twice (same result)
                                    { LBoxGroup c2 = cur; asm volatile("" : "+s"(c2.v[0])); const uint32_t m2 = lmask(c2); asm volatile("" :: "s"(m2)); }
#endif
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
#endif
    }
    t_out = best_t;
    return best;
}

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
        return wc.w > -INFINITY && (all || !(f > wc.w));   // NaN f passes
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
__device__ __forceinline__ void camera_exact(const KP& q, uint32_t sl, bool v, const V3<T>& d, T a, T inv_a, T& best_t,
                                             int& best) {
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
            hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, best_t, best);
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
    T best_t = T(INFINITY);
    int best = -1;
    KSTAT(3);
    uint32_t n_cx = 0;   // executed-work counts (work_add below)
    const uint32_t n_cone = cone_walk<MEGA>(q, ax, ay, az, S, Cc, all, xw0, kw0, [&](uint32_t sl) {
        ++n_cx;
        camera_exact<T, root2, SCALAR>(q, sl, v, d, a, inv_a, best_t, best);
    });
    work_add(kWCone, n_cone);
    work_add(kWCExact, n_cx);
    t_out = best_t;
    return best;
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
    T best_t = T(INFINITY);
    int best = -1;
    uint32_t n_cx = 0;
    for (; smask != 0u; smask &= smask - 1u) {
        const uint16_t* l = lists[__builtin_ctz(smask)];
        const uint32_t n = __builtin_amdgcn_readfirstlane(l[0]);
        for (uint32_t j = 0; j < n; ++j) {
            ++n_cx;
            camera_exact<T, root2, SCALAR>(q, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, best_t, best);
        }
    }
    work_add(kWCExact, n_cx);
    t_out = best_t;
    return best;
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
    const U4 r = [&] {
        const auto& q0 = *cold_args<T>();
        return philox(sid, pix, cam ? 0u : k, cam ? 0u : 2u, q0.k0, q0.k1);
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
                const U4 qq = philox(sid, pix, i, 1u, k0, k1);
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
        const T* sg = q.cen + 4 * hit_i;
        vec = sub(base, mk(sg[0], sg[1], sg[2]));        // normal = at_t(t) - center (objects.rs:279-280)
        if constexpr (SCALAR) rad = sg[3];
        l2 = pk_len2(vec);
    }
    const T len = (SCALAR && !cam) ? rad : sqrt(l2);
    const V3<T> u = mk(vec.x / len, vec.y / len, vec.z / len);
    if (cam) {
        o = base;
        d = u;
        c = mk(T(1.0), T(1.0), T(1.0));
        return;
    }
    V3<T> nrm = u;
    const bool front = (SCALAR ? dot(d, nrm) : pk_dot(d, nrm)) < T(0.0);
    if (!front) nrm = neg(nrm);
    const MatT<T> m = q.mats[hit_i];                     // = materials[material[hit_i]] (objects.rs:296)
    V3<T> nd;
    if (m.kind != RT_DIELECTRIC) {
        // One random_unit_vector for both kinds (a wave usually holds both: one evaluation, not two).
        const V3<T> rv = unit_vec(ua, ub);
        if (m.kind == RT_LAMBERTIAN) {
            nd = add(rv, nrm);
            if (near_zero(nd)) nd = nrm;
        } else {
            nd = add(reflect(d, nrm), mul(rv, m.fuzz));
        }
        c = mk(c.x * m.ar, c.y * m.ag, c.z * m.ab);
    } else {
        const T ratio = front ? m.inv_ior : m.ior;
        const V3<T> nn = m.hollow ? neg(nrm) : nrm;
        const T ct = fmin(dot(neg(d), nn), T(1.0));
        const T st = sqrt(T(1.0) - ct * ct);
        bool refl = ratio * st > T(1.0);
        if (!refl) {   // Dielectric::reflectance (materials.rs:121-124), powi(5) = x*((x*x)*(x*x))
            const T r0 = front ? m.r0_front : m.r0_back;
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

// Make this wave's earlier global stores visible to its later loads (other lanes, same wave).
__device__ __forceinline__ void wave_mem_sync() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------------------------
// Path regeneration.  Each ray of a pixel evolves independently of the others: bounce k of
// sample s depends only on (origin, direction, colour, s, k).  The reference's positions are a
// function of the termination bounces alone: with e_s = the bounce at which sample s hit the sky
// (or depth if it was still enabled after the last bounce), the stable shuffle keeps sample
// order, so at bounce k sample s sits at pos_k(s) = #{s' < s : e_s' >= k}, and a ray terminated
// at bounce k moves to n_{k+1} + #{s' < s : e_s' == k}.  So each lane keeps ONE ray in registers
// from its camera ray to its termination, then takes the next sample (of this pixel or of the
// next pixel the wave pulls), and writes one record (e_s, colour, primary y) per sample.  When
// all samples of a pixel are done, the wave replays the positions from the records, applies the
// retire rule and sums in the reference's order — the same values, bit for bit,
// as the bounce-synchronous schedule, with every lane busy and no per-bounce ray-state traffic.
// ---------------------------------------------------------------------------------------------
#ifndef RT_EXP_SLOTS
#define RT_EXP_SLOTS 8
#endif
constexpr uint32_t kSlots = RT_EXP_SLOTS;   // pixels a wave may have in flight (lane s holds slot s's metadata)
static_assert(kSlots >= 1 && kSlots <= 8, "the camera-batch queue packs the slot into 3 bits (sid | slot << 29)");

// Semantics modes (RT_FLAG_MODE_*): which of the reference's renderers the kernel reproduces.
enum Mode : int {
    kModeV2 = 0,       // render_vectorized2 -> trace_vectorized2 (the live path; quirks Q2, Q3)
    kModeV1 = 1,       // render_vectorized -> trace_vectorized (ray_tracing.rs:312-373): own value, final-ray sky
    kModeScalar = 2,   // render -> trace_rays (ray_tracing.rs:264-306) + Color::average
    kModeV3 = 3,       // render_vectorized3 -> trace_vectorized3 (ray_tracing.rs:508-628): own value, swap order
};

// Per-wave scratch of trace_paths (HBM layout): the position map of the pixel being
// reduced (P entries, u16 -- u32 past 32764 positions: the sample whose value position q holds at the
// final read, all ones = none), then kSlots record regions indexed by sample: y[P] (T, the primary
// ray's y), c[P] (3 T, AoS: one dwordx3 store per termination), e[P] (u8 -- u32 when depth > 254: the
// termination bounce).  In the V1 and scalar modes c holds each sample's final value (colour x sky of
// its own escaping ray, or 0).
template <typename T> struct C3 { T x, y, z; };
template <typename T> struct PScratch {
    char* base;        // wave-uniform
    uint32_t P, vbytes, sbytes, wide;   // wide: bit 0 = u32 e, bit 1 = u32 map
    static constexpr uint32_t kNone = 0xFFFFFFFFu;
    // A map entry is a sample index, with kWhite set when that sample hit the sky at bounce 0: its
    // colour is white, so it wrote no colour record (terminate) and the reduction reads none.  u16
    // entries keep the flag in bit 15 (P <= 32764, so no flagged index is 0xFFFF).
    static constexpr uint32_t kWhite = 0x80000000u;
    __device__ __forceinline__ static uint32_t from16(uint32_t m) {
        return m == 0xFFFFu ? kNone : (m & 0x7FFFu) | ((m & 0x8000u) << 16);
    }
    __device__ __forceinline__ static uint16_t to16(uint32_t v) { return (uint16_t)((v & 0x7FFFu) | ((v >> 16) & 0x8000u)); }
    __device__ __forceinline__ uint32_t map(uint32_t q) const {
        if (wide & 2u) return *(const uint32_t*)(base + 4u * q);
        return from16(*(const uint16_t*)(base + 2u * q));
    }
    __device__ __forceinline__ void set_map(uint32_t q, uint32_t smp) const {
        if (wide & 2u) *(uint32_t*)(base + 4u * q) = smp;
        else *(uint16_t*)(base + 2u * q) = to16(smp);
    }
    __device__ __forceinline__ T& y(uint32_t s, uint32_t i) const {
        return *(T*)(base + vbytes + s * sbytes + i * (uint32_t)sizeof(T));
    }
    __device__ __forceinline__ C3<T>& c(uint32_t s, uint32_t i) const {
        return *(C3<T>*)(base + vbytes + s * sbytes + (P + 3u * i) * (uint32_t)sizeof(T));
    }
    __device__ __forceinline__ void store_c(uint32_t s, uint32_t i, T x, T y, T z) const {
        T* r = &c(s, i).x;
        r[0] = x;
        asm volatile("" ::: "memory");   // keep the three stores apart (no dwordx3 merge)
        r[1] = y;
        asm volatile("" ::: "memory");
        r[2] = z;
    }
    __device__ __forceinline__ uint32_t e(uint32_t s, uint32_t i) const {
        const char* b = base + vbytes + s * sbytes + 4u * P * (uint32_t)sizeof(T);
        return (wide & 1u) ? *(const uint32_t*)(b + 4u * i) : (uint32_t) * (const uint8_t*)(b + i);
    }
    __device__ __forceinline__ void set_e(uint32_t s, uint32_t i, uint32_t v) const {
        char* b = base + vbytes + s * sbytes + 4u * P * (uint32_t)sizeof(T);
        if (wide & 1u) *(uint32_t*)(b + 4u * i) = v;
        else *(uint8_t*)(b + i) = (uint8_t)v;
    }
};
// This wave's scratch view, re-derived from the kernel arguments where it is used (it is needed
// only at record writes and pixel completion, so it does not hold SGPRs across the sphere sweep).
template <typename T> __device__ __forceinline__ PScratch<T> wave_scratch(uint32_t wave) {
    const auto& q = *cold_args<T>();
    const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + wave;
    return PScratch<T>{q.scratch + (size_t)gw * q.scratch_stride, q.P, q.vbytes, q.sbytes, q.swide};
}

// Wave-uniform issue state, parked in LDS between refills for the same reason.
// need: slots opened since their pixel's camera candidate list was last built (camera batches)
struct IssueState { uint32_t busy, cur, cur_next, cur_pix, cur_row, cur_col, drained, qhead, qcount, blk_next, blk_end, need; };

// Work items (pixels) are claimed in blocks.  One global counter counts blocks, and block j's items
// are a fixed function of j (guided_block): sizes G, G/2, ..., 2 while more than G T, ..., 2T items
// remain after it, then single items (T = kTMul x workgroups), so blocks shrink to one item towards
// the end without any wave estimating how much is left.  The claiming wave takes the block's first
// item and offers the rest to its workgroup through an LDS pool (s_pool, a lock-free 64-bit CAS;
// if another wave refilled the pool first, the claimer keeps the rest to itself).  Waves take items
// from their private rest, then the pool, then the counter.
//   * Global atomics are the cost: the device sustained ~90 M/s on this counter (11 ns each; spread
//     over 16 counters, no faster).  One atomic per pixel held config B (921 600 pixels) at 10.6 ms
//     whatever its spp.
//   * The tail is the other cost: a block is worked off by the 4 waves of one workgroup, and a late
//     16-pixel block of long glass paths at 512 spp, claimed by one wave, ran ~15 ms past the rest.
//     G (a power of two <= kMaxBlock, chosen per launch by the host) keeps a block within
//     kBlockSamples samples and within 1/kBlockShare of a wave's share of the pixels.  The second
//     bound is for small launches: 8-way row shards of C (~50 pixels per wave) with G = 16 ended
//     with one workgroup on 16 adjacent glass pixels, 8.2 ms against 5.7 ideal; with G = 2 they
//     scale perfectly.  Scattering the claim order instead (pixels or 16-pixel tiles) cost 4-5 % at
//     config C: waves on a CU then walk different clusters, and the sphere data thrash the scalar cache.
constexpr uint32_t kMaxBlock = 16;
constexpr uint32_t kBlockShare = 24;
// The counter serves ~90 M claims/s, and the chip runs ~3e10 samples/s: a launch claims at most one
// block per kClaimSpp samples (G >= kClaimSpp / spp), so claims stay under ~half the counter's rate
// at any spp.  Without it the share bound took small launches to single pixels: a quarter of config B
// (128 spp) then made 230 k claims, 2.5 ms of atomics for 1 ms of work (tools/multirank_check.sh).
constexpr uint32_t kClaimSpp = 640;
#ifndef RT_EXP_BLOCK_SAMPLES
#define RT_EXP_BLOCK_SAMPLES 8192
#endif
#ifndef RT_EXP_TMUL
#define RT_EXP_TMUL 8
#endif
constexpr uint32_t kBlockSamples = RT_EXP_BLOCK_SAMPLES;
constexpr uint32_t kTMul = RT_EXP_TMUL;

// Block j of np items -> items [start, end); false past the last block.
__device__ __forceinline__ bool guided_block(uint32_t np, uint32_t T, uint32_t G, uint32_t j, uint32_t& start,
                                             uint32_t& end) {
    uint32_t a = 0;
#pragma unroll
    for (uint32_t sz = kMaxBlock; sz >= 1u; sz >>= 1) {
        const uint32_t r = np - a, keep = sz * T;
        const uint32_t len = sz == 1u ? r : (sz <= G && r > keep ? ((r - keep) / sz) * sz : 0u);
        const uint32_t nb = len / sz;
        if (j < nb) { start = a + j * sz; end = start + sz; return true; }
        j -= nb;
        a += len;
    }
    return false;
}

// PScratch sizes: the map (u16, u32 past 32764 positions), the records (e u8, u32 when depth > 254).
__host__ __device__ inline uint32_t paths_wide(uint32_t P, uint32_t depth) { return (depth > 254u ? 1u : 0u) | (P > 32764u ? 2u : 0u); }
__host__ __device__ inline uint32_t paths_vbytes(uint32_t P, uint32_t wide, bool v3) {
    return v3 ? (8u * P + 255u) & ~255u   // vectorized3: slot -> sample map + the swap tables (finish_pixel)
              : (P * ((wide & 2u) ? 4u : 2u) + 255u) & ~255u;
}
__host__ __device__ inline uint32_t paths_sbytes(uint32_t P, uint32_t tsz, uint32_t wide) {
    return (P * (4u * tsz + ((wide & 1u) ? 4u : 1u)) + 255u) & ~255u;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// Replay pixel slot s's positions from its records, apply the retire rule, reduce, write the
// pixel (whole wave; returns the number of bounce iterations the reference runs for the pixel).
// The position map in LDS (live-path kernels without the mega level, P <= kLMapCap positions: config C's
// 512 spp): the replay's scattered u16 writes, the map's initialisation and the reduction's reads stay
// on the CU instead of going to HBM as partial lines.  Larger P uses the global map in PScratch.
#ifndef RT_EXP_LMAP_CAP
#define RT_EXP_LMAP_CAP 512
#endif
constexpr uint32_t kLMapCap = RT_EXP_LMAP_CAP;
template <typename T, int MODE>
__device__ __forceinline__ uint32_t finish_pixel(const PScratch<T>& sc, uint32_t s, uint32_t item, uint32_t* hist,
                                                 T (*stage)[64], uint16_t* lmap) {
    const auto& q = *cold_args<T>();
    const uint32_t lane = threadIdx.x & 63u;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    const uint32_t spp = q.spp, P = q.P, C = q.C, depth = q.depth;
    constexpr uint32_t kNone = PScratch<T>::kNone;
    const bool lm = kLMapCap > 0u && lmap != nullptr && P <= kLMapCap;   // wave-uniform
    auto set_map = [&](uint32_t qq, uint32_t smp) {
        if (lm) lmap[qq] = PScratch<T>::to16(smp);
        else sc.set_map(qq, smp);
    };
    // Map init: no position holds a terminated sample's value yet (survivors and never-written
    // positions read 0; positions [spp, P), the missing lanes of a partial last chunk, get their
    // fixed value in the final reduction).  Two u16 entries per u32 store.
    if (MODE == kModeV2) {
        if (lm) {
            for (uint32_t qi = 2u * lane; qi < P; qi += 128u) *(uint32_t*)(lmap + qi) = 0xFFFFFFFFu;
        } else if (sc.wide & 2u) {
            for (uint32_t qi = lane; qi < P; qi += 64u) sc.set_map(qi, kNone);
        } else {
            for (uint32_t qi = 2u * lane; qi < P; qi += 128u) *(uint32_t*)(sc.base + 2u * qi) = 0xFFFFFFFFu;
        }
    }
    // Bounce iterations the reference runs: K = min(depth, max e + 1).  The same pass builds the
    // histogram of the termination bounces below 64 (a sample terminated iff e < depth, and then
    // e < K); it is only used when K <= 64.
    uint32_t K = 0;
    const bool hist_on = MODE == kModeV2 && depth > 0u;
    if (hist_on) {
        hist[lane] = 0u;
        __builtin_amdgcn_wave_barrier();
    }
    if (depth > 0) {
        uint32_t me = 0;
        for (uint32_t b = 0; b < spp; b += 512u) {
            uint32_t ev[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t i = b + 64u * u + lane;
                ev[u] = i < spp ? sc.e(s, i) : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                me = max(me, ev[u]);
                if (hist_on && b + 64u * u + lane < spp && ev[u] < depth && ev[u] < 64u) atomicAdd(&hist[ev[u]], 1u);
            }
        }
        K = min(depth, __builtin_amdgcn_readfirstlane(wave_max(me)) + 1u);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    wave_mem_sync();
    // One pass over the samples (K <= 64, the common case): lane k holds the per-bounce counts, so
    // every sample finds its positions from running counts and ballots over its own chunk of 64.
    // Sample s, terminated at bounce k = e_s < K, sat at pold = #{s' < s : e_s' >= k} during bounce
    // k and moves to pnew = n_{k+1} + #{s' < s : e_s' == k} in the sorted copy (n_k = #{e >= k});
    // the retire rule then picks which of the two holds its value, and the position
    // map records the sample there (the value itself is formed in the final reduction).
    bool replayed = false;
#if !defined(RT_EXP_OLD_REPLAY)
    if (MODE == kModeV2 && K > 0u && K <= 64u) {
        replayed = true;
        const uint32_t H = hist[lane];   // lane k: #{e == k} over the pixel (pass 1)
        const uint32_t nn_l = spp - wave_scan_dpp(H);   // n_{k+1} = #{e > k} for k = lane
        uint32_t cge = 0, ceq = 0;   // lane k: samples of the earlier chunks with e >= k, e == k
        // Per chunk, each retiring lane needs #{lanes below with e' >= e} and #{... e' == e}.  With the
        // values clamped to ec = min(e, K) (nb bits; survivors and e >= K compare as K), the wave
        // ballots ec's bit planes once per chunk and every lane compares itself against all lanes at
        // once, most significant bit first: gt collects the lanes found greater, eq those still equal.
        // Round 2 ran one pass per distinct bounce in the chunk (ballots, readlanes and selects each).
        const uint32_t nb = 32u - (uint32_t)__builtin_clz(K);   // ec in [0, K], K <= 64: 1..7 bits
#ifdef RT_EXP_DUP_REPLAY   // timing experiment: the replay twice (the same map writes)
        for (uint32_t rep = 0; rep < 2u; ++rep) {
            asm volatile("" ::: "memory");
            cge = 0; ceq = 0;
#endif
        for (uint32_t b = 0; b < spp; b += 512u) {   // the samples in order, 64 at a time
            uint32_t ev[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t i = b + 64u * u + lane;
                ev[u] = i < spp ? sc.e(s, i) : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (b + 64u * u >= spp) break;
                const uint32_t i = b + 64u * u + lane, e = ev[u];
                const bool in = i < spp, ret = e < K;
                const uint32_t ec = ret ? e : K;
                const unsigned long long inm = __ballot(in);
                // eq, gt: the lanes equal to / greater than this lane's ec; eqk: the lanes whose ec equals
                // this lane's index k (lane k's count of e == k).  A plane no lane sets changes neither eq
                // nor gt, and clears eqk in the lanes k with that bit (zb)
                unsigned long long eq = inm, gt = 0ull, eqk = inm;
                uint32_t zb = 0;
                for (uint32_t bb = nb; bb-- > 0u;) {
                    const unsigned long long P = __ballot(in && ((ec >> bb) & 1u));
                    if (P == 0ull) { zb |= 1u << bb; continue; }
                    const unsigned long long B = ((ec >> bb) & 1u) ? ~0ull : 0ull;     // this lane's bit
                    const unsigned long long Bk = ((lane >> bb) & 1u) ? ~0ull : 0ull;  // bit of k = lane
                    gt |= eq & P & ~B;     // equal so far, 1 where this lane has 0: greater
                    eq &= ~(P ^ B);        // still equal
                    eqk &= ~(P ^ Bk);
                }
                const uint32_t ek = ret ? e : 0u;
                // the earlier chunks' counts at this lane's bounce
                const uint32_t cg = (uint32_t)__shfl((int)cge, (int)ek), cq = (uint32_t)__shfl((int)ceq, (int)ek);
                const uint32_t nn = (uint32_t)__shfl((int)nn_l, (int)ek);
                // lane k < K: #{e == k} in this chunk (lanes k >= 2^nb or > K are never read)
                const uint32_t h = (lane & zb) != 0u ? 0u : (uint32_t)__popcll(eqk);
                // lane k <= K: #{in && e >= k} = #{in} - #{e < k}
                cge += (uint32_t)__popcll(inm) - (wave_scan_dpp(h) - h);
                ceq += h;
                if (ret) {
                    // Sample i, terminated at bounce e, sat at pold = #{s' < i : e_s' >= e} during bounce e
                    // and moves to pnew = n_{e+1} + #{s' < i : e_s' == e}
                    const uint32_t pold = cg + (uint32_t)__popcll((gt | eq) & lt_mask);
                    const uint32_t pnew = nn + cq + (uint32_t)__popcll(eq & lt_mask);
                    const uint32_t Lnext = ek + 1u == depth ? 0u : (nn + 3u) / 4u;
                    // positions [lo, 4 ceil(n_k / 4)) retire at bounce e; pold and pnew are below n_k <= 4 Lk (pold
                    // counts the earlier samples with e >= k, pnew = n_{k+1} + the earlier ones with
                    // e == k), so only lo bounds them
                    const uint32_t lo = 4u * Lnext;
                    const bool U = q.s_sel == (ek & 1u);
                    const bool w_old = U && pold >= lo;
                    const bool w_new = !U || pnew < lo;
                    const uint32_t iw = ek == 0u ? (i | PScratch<T>::kWhite) : i;
                    if (w_old || w_new) set_map(w_old ? pold : pnew, iw);
                    if (w_old && w_new) set_map(pnew, iw);
                }
            }
        }
#ifdef RT_EXP_DUP_REPLAY
        }
#endif
    }
#endif
    // vectorized3 (ray_tracing.rs:508-628): replay the in-place swap partitions.  After bounce k the
    // slots q < 4 L hold enabled rays iff their sample has e > k; with D the disabled slots ascending
    // (all chunks, the front scan) and E the enabled slots descending (the back scan from L), the
    // literal loop swaps D[j] with E[j] while chunk(D[j]) < chunk(E[j]) (monotone in j, since D rises
    // and E falls), i.e. for j < J = max over chunk boundaries c of min(#D below c, #E at or above c),
    // and stops with num_active = chunk(max(E[J], D[J-1])) + 1 (the previous enabled slot below the
    // last swap; none disabled: all C chunks, :573; none enabled: 0, :581).  sig[q] = the sample at
    // slot q (>= spp: a missing lane of a partial chunk); tabD[j], tabE[j]: the samples at D[j], E[j].
    // tests/test_v3_partition.py checks this closed form against the literal loop.
    if constexpr (MODE == kModeV3) {
        uint32_t* sig = (uint32_t*)sc.base;
        uint32_t* tabD = sig + P;
        uint32_t* tabE = tabD + P / 2u;
        for (uint32_t qi = lane; qi < P; qi += 64u) sig[qi] = qi;
        wave_mem_sync();
        uint32_t L = C;
        for (uint32_t k = 0; k < K; ++k) {
            auto enabled = [&](uint32_t qq, uint32_t smp) -> bool { return qq < 4u * L && smp < spp && sc.e(s, smp) > k; };
            uint32_t nd = 0, ne = 0;
            for (uint32_t qb = 0; qb < P; qb += 64u) {
                const uint32_t qq = qb + lane;
                const bool in = qq < P;
                const bool en = in && enabled(qq, in ? sig[qq] : 0u);
                nd += (uint32_t)__popcll(__ballot(in && !en));
                ne += (uint32_t)__popcll(__ballot(en));
            }
            if (nd == 0u) { L = C; continue; }   // no disabled slot: next_disabled is None (:573)
            if (ne == 0u) { L = 0; break; }      // no enabled slot: previous_enabled is None (:581)
            uint32_t cd = 0, ce = 0, Jl = 0;
            for (uint32_t qb = 0; qb < P; qb += 64u) {
                const uint32_t qq = qb + lane;
                const bool in = qq < P;
                const uint32_t smp = in ? sig[qq] : 0u;
                const bool en = in && enabled(qq, smp), dis = in && !en;
                const unsigned long long bd = __ballot(dis), be = __ballot(en);
                const uint32_t rd = cd + (uint32_t)__popcll(bd & lt_mask), rf = ce + (uint32_t)__popcll(be & lt_mask);
                if (in && (qq & 3u) == 0u) Jl = max(Jl, min(rd, ne - rf));   // boundary c = qq / 4
                if (dis && rd < P / 2u) tabD[rd] = smp;
                if (en && ne - 1u - rf < P / 2u) tabE[ne - 1u - rf] = smp;
                cd += (uint32_t)__popcll(bd);
                ce += (uint32_t)__popcll(be);
            }
            const uint32_t J = __builtin_amdgcn_readfirstlane(wave_max(Jl));
            wave_mem_sync();
            cd = 0; ce = 0;
            uint32_t back = 0;   // 1 + the slot the loop stops at from the back: E[J] or D[J-1]
            for (uint32_t qb = 0; qb < P; qb += 64u) {
                const uint32_t qq = qb + lane;
                const bool in = qq < P;
                const uint32_t smp = in ? sig[qq] : 0u;
                const bool en = in && enabled(qq, smp), dis = in && !en;
                const unsigned long long bd = __ballot(dis), be = __ballot(en);
                const uint32_t rd = cd + (uint32_t)__popcll(bd & lt_mask), re = ne - 1u - (ce + (uint32_t)__popcll(be & lt_mask));
                if (dis && rd < J) sig[qq] = tabE[rd];
                if (en && re < J) sig[qq] = tabD[re];
                if ((en && re == J) || (dis && rd + 1u == J)) back = max(back, qq + 1u);
                cd += (uint32_t)__popcll(bd);
                ce += (uint32_t)__popcll(be);
            }
            L = (__builtin_amdgcn_readfirstlane(wave_max(back)) - 1u) / 4u + 1u;
            wave_mem_sync();
        }
    }
    uint32_t n = spp, kb = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < (MODE == kModeV2 && !replayed ? K : 0u); ++k) {
        if (kb == 0xFFFFFFFFu || k - kb >= 64u) {   // histogram of e over [k, k+64)
            kb = k;
            hist[lane] = 0;
            __builtin_amdgcn_wave_barrier();
            for (uint32_t i = lane; i < spp; i += 64u) {
                const uint32_t e = sc.e(s, i);
                if (e >= kb && e - kb < 64u) atomicAdd(&hist[e - kb], 1u);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
        const uint32_t m = __builtin_amdgcn_readfirstlane(hist[k - kb]);   // rays hitting the sky at k
        const uint32_t n_next = n - m;
        const uint32_t Lnext = (k + 1 == depth) ? 0u : (n_next + 3u) / 4u;
        if (m > 0) {
            const uint32_t lo = 4u * Lnext;   // positions [lo, 4 ceil(n_k / 4)) retire at bounce k
            const bool U = q.s_sel == (k & 1u);                 // final read = this bounce's unsorted buffer
            uint32_t cge = 0, ceq = 0;
            for (uint32_t b = 0; b < spp && ceq < m; b += 64u) {
                const uint32_t i = b + lane;
                const uint32_t e = i < spp ? sc.e(s, i) : 0xFFFFFFFFu;
                const bool ge = i < spp && e >= k, eq = e == k;
                const unsigned long long bge = __ballot(ge), beq = __ballot(eq);
                if (eq) {
                    const uint32_t pold = cge + (uint32_t)__popcll(bge & lt_mask);
                    const uint32_t pnew = n_next + ceq + (uint32_t)__popcll(beq & lt_mask);
                    const bool w_old = U && pold >= lo;   // pold, pnew < n_k <= hi (as above)
                    const bool w_new = !U || pnew < lo;
                    // At most one position except when the old one retires now and the new one later.
                    const uint32_t iw = k == 0u ? (i | PScratch<T>::kWhite) : i;
                    if (w_old || w_new) set_map(w_old ? pold : pnew, iw);
                    if (w_old && w_new) set_map(pnew, iw);
                }
                cge += (uint32_t)__popcll(bge);
                ceq += (uint32_t)__popcll(beq);
            }
        }
        n = n_next;
    }
    wave_mem_sync();
    // Final reduction in the reference's order: per lane l, chunks j = 0..C-1 from +0.0
    // (ray_tracing.rs:499-502), then PackedColor::sum over the 4 lanes (color.rs:226-232).
    // Position q's value (ray_tracing.rs:488-497): sample m = map[q] hit the sky -> c_m x sky(y_q),
    // y_q the primary ray's y at slot q (quirk Q2); no sample -> 0 (still enabled: black); q >= spp
    // (the missing lanes of a partial chunk: disabled from the start, ray.rs:140-144, hit_sky at
    // bounce 0, ray_tracing.rs:421-424, zero direction) -> sky(0), or white at depth 0 when the final
    // read is buffer 0.  All 64 lanes form the values of 64 positions at a time into LDS; lanes
    // ch * 4 + l then add theirs in order.
    // V1: render_vectorized's packed_color + chunk (renderer.rs:120) is the same per-lane order,
    // over each sample's own value (+0 for the disabled lanes of a partial chunk: black x sky).
    // Scalar: Color::average (color.rs:66-85), one sequential sum over the samples.
    T acc = T(0.0);
    if (MODE == kModeScalar) {
        if (lane < 3u) {
            uint32_t i = 0;
            for (; i + 16 <= spp; i += 16) {
                T v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const T* cp = &sc.c(s, i + u).x;
                    v[u] = cp[lane];
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) acc = acc + v[u];
            }
            for (; i < spp; ++i) acc = acc + (&sc.c(s, i).x)[lane];
        }
    } else {
        const V3<T> s0 = sky(T(0.0));
        const bool white0 = depth == 0u && q.s_sel == 0u;
        // the 12 running sums live in LDS (the free histogram) between batches: a short live range
        // keeps this loop from raising the kernel's register peak
        T* accl = (T*)hist;
#ifdef RT_EXP_DUP_REDUCE   // timing experiment: the final reduction twice (the same sums)
        for (uint32_t rep = 0; rep < 2u; ++rep) {
            asm volatile("" ::: "memory");
#endif
        if (lane < 12u) accl[lane] = T(0.0);
        for (uint32_t qb = 0; qb < P; qb += 64u) {
            const uint32_t qq = qb + lane;
            T vr = T(0.0), vg = T(0.0), vb = T(0.0);
            if (qq < P && MODE == kModeV3) {
                // the sample at slot qq: its own value; a missing lane (white, hit_sky at bounce 0
                // with a zero direction) adds sky(0), or white when no bounce ran (:611-619)
                const uint32_t m = ((const uint32_t*)sc.base)[qq];
                if (m < spp) {
                    const C3<T> cm = sc.c(s, m);
                    vr = cm.x; vg = cm.y; vb = cm.z;
                } else if (depth > 0u) {
                    vr = s0.x; vg = s0.y; vb = s0.z;
                } else {
                    vr = T(1.0); vg = T(1.0); vb = T(1.0);
                }
            } else if (qq < P) {
                if (qq >= spp) {
                    if (MODE == kModeV2) {
                        if (depth > 0u) { vr = s0.x; vg = s0.y; vb = s0.z; }
                        else if (white0) { vr = T(1.0); vg = T(1.0); vb = T(1.0); }
                    }
                } else if constexpr (MODE == kModeV2) {
                    uint32_t m;
                    if (lm) m = PScratch<T>::from16(lmap[qq]);
                    else m = sc.map(qq);
                    if (m != kNone) {
                        // a bounce-0 sky hit (kWhite) wrote no record: white x sky.  Branch-free (the
                        // record slot is read anyway and replaced by white: a branch cost 0.8 % at C)
                        const bool wh = (m & PScratch<T>::kWhite) != 0u;
                        const C3<T> cm = sc.c(s, m & ~PScratch<T>::kWhite);
                        const V3<T> sk = sky(sc.y(s, qq));
                        vr = (wh ? T(1.0) : cm.x) * sk.x; vg = (wh ? T(1.0) : cm.y) * sk.y; vb = (wh ? T(1.0) : cm.z) * sk.z;
                    }
                } else {
                    const C3<T> cm = sc.c(s, qq);
                    vr = cm.x; vg = cm.y; vb = cm.z;
                }
            }
            // transposed: lane (ch, l) finds its 16 values (positions qb + 4u + l) contiguous
            const uint32_t si = 16u * (lane & 3u) + (lane >> 2);
            stage[0][si] = vr; stage[1][si] = vg; stage[2][si] = vb;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if (lane < 12u) {
                const uint32_t nu = min(16u, (P - qb) / 4u);   // wave-uniform; 16 except a short last batch
                const T* sv = &stage[lane >> 2][16u * (lane & 3u)];
                T a = accl[lane];
                if (nu == 16u) {   // a whole batch: plain adds (the guarded form costs a compare and a select each)
#pragma unroll
                    for (uint32_t u0 = 0; u0 < 16u; u0 += 4u) {
                        T v[4];
#pragma unroll
                        for (uint32_t u = 0; u < 4u; ++u) v[u] = sv[u0 + u];
#pragma unroll
                        for (uint32_t u = 0; u < 4u; ++u) a = a + v[u];
                    }
                } else {
                    for (uint32_t u = 0; u < nu; ++u) a = a + sv[u];
                }
                accl[lane] = a;
            }
            __builtin_amdgcn_wave_barrier();
        }
#ifdef RT_EXP_DUP_REDUCE
        }
#endif
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 12u) acc = accl[lane];
    }
    const T s1 = __shfl(acc, (int)((lane + 1) & 63u)), s2 = __shfl(acc, (int)((lane + 2) & 63u)),
            s3 = __shfl(acc, (int)((lane + 3) & 63u));
    const bool writer = MODE == kModeScalar ? lane < 3u : (lane < 12u && (lane & 3u) == 0u);
    if (writer) {
        const uint32_t ch = MODE == kModeScalar ? lane : lane >> 2;
        const T tot = MODE == kModeScalar ? acc : (((T(0.0) + acc) + s1) + s2) + s3;
        const T v = tot / (T)spp;                                   // renderer.rs:161
        if (!(v <= T(2.0))) atomicOr(q.err, 1u);                    // color.rs:55-57 assert
        if (q.rgb) q.rgb[(size_t)item * 3 + ch] = q8(v);
        if (q.lin) q.lin[(size_t)item * 3 + ch] = (double)v;
    }
    return K;
}

// Persistent path-regeneration kernel (see above).  Wave-uniform state: the slot being issued
// (cur, next sample cur_next), the busy-slot mask, and per-slot pixel/remaining-sample counts held
// in lane s of two VGPRs.  Per iteration: hand free lanes new samples, trace one bounce for every
// live ray (one sphere sweep for the whole wave), record terminations, finish completed pixels.
//
// CAMQ (pinhole cameras, depth >= 1): primary rays are not mixed into the per-lane sweep.  They are
// traced in full-wave camera batches against the camera-origin table (5 instead of 12 packed ops
// per sphere pair); misses terminate on the spot, hits wait in a per-wave LDS queue and free lanes
// pop them as rays whose bounce-0 scatter is pending.  Every ray still meets every sphere.
constexpr uint32_t kQCap = 128;   // camera-batch queue entries per wave (a batch adds at most 64)

template <typename T, int W, bool ROOT2, int MODE = kModeV2, bool CAMQ = false, bool MEGA = false>
__global__ __launch_bounds__(256, W) void trace_paths(KParams<T> p) {
    constexpr bool SC = MODE == kModeScalar;
    // fp64 at 5+ waves per SIMD: a 64-entry queue (half the LDS), so the parked ray fits in 32 KB per
    // workgroup
    constexpr bool kF64Park = sizeof(T) == 8 && W >= 5;
    constexpr uint32_t QW = CAMQ ? 4 : 1, QN = CAMQ ? (kF64Park ? 64u : kQCap) : 1;
    __shared__ unsigned long long wcount[4][3];
    // 8-byte aligned: finish_pixel keeps its 12 running sums (T, fp64 too) in this array
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[4][64];
    __shared__ __attribute__((aligned(16))) T s_stage[4][3][64];   // finish_pixel: 64 positions' values per wave
    __shared__ IssueState s_is[4];
    __shared__ unsigned long long s_pool;   // the workgroup's pool of claimed items: next << 32 | end
    __shared__ uint32_t q_sid[QW][QN];   // sid | slot << 29 (the pixel: s_slotpix[slot])
    __shared__ uint32_t s_slotpix[4][kSlots];   // the pixel of each open slot
    __shared__ int q_hit[QW][QN];
    __shared__ T q_t[QW][QN], q_d[QW][3][QN];
    // camera candidate list of each open pixel slot (pixel_list): [0] = count (0xFFFF: none, sweep per batch)
    __shared__ uint16_t s_clist[QW][CAMQ ? kSlots : 1][kCList];
    // fp32 at 6 waves per SIMD (80 VGPRs): each lane's ray origin and direction are parked in LDS
    // across the sphere sweeps and the camera batches and re-read right before the scatter, instead
    // of being held in VGPRs (the allocator otherwise spills them to scratch memory around the sweep).
#ifdef RT_EXP_NO_PARK
    constexpr bool kPark = false;
#else
    constexpr bool kPark = (sizeof(T) == 4 && W >= 6) || kF64Park;
#endif
    // the mega-level kernels park the path colour as well (their four-level sweep holds more state)
#ifdef RT_EXP_PARKC_ALL
    constexpr bool kParkC = kPark;
#else
    constexpr bool kParkC = kPark && MEGA;
#endif
    __shared__ T s_park[kPark ? 4 : 1][kParkC ? 9 : 6][64];
    // finish_pixel's position map (P <= kLMapCap) in LDS: the fp64 live-path kernels without the mega level
    // (fp64 C +1.1 % same-box).  fp32 lost 7 % with it (the extra finish_pixel code pushed 5 more spills
    // into the hot loop at 80 VGPRs); the mega kernels' LDS is full at 6 waves per SIMD.
    constexpr bool kLMap = MODE == kModeV2 && !MEGA && kLMapCap > 0u && sizeof(T) == 8 && !kF64Park;
    __shared__ __attribute__((aligned(16))) uint16_t s_lmap[kLMap ? 4 : 1][kLMap ? kLMapCap : 2];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (lane == 0) { wcount[wave][0] = 0; wcount[wave][1] = 0; wcount[wave][2] = 0; }
    if (lane < kNWork) g_work[wave][lane] = 0ull;
#ifdef RT_KSTATS
    if (lane < 8) g_kst[wave][lane] = 0;
#endif
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    if (lane == 0) s_is[wave] = IssueState{0u, 0u, cold_args<T>()->spp, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    if (threadIdx.x == 0) s_pool = 0ull;   // {next, end} = {0, 0}: empty
    __syncthreads();
    V3<T> o = mk(T(0), T(0), T(0)), d = o, c = o;
    uint32_t sid = 0, k = 0, slot = 0, pix = 0;
    bool live = false;
    bool scat = false;                 // hit at bounce k last iteration, still below depth: scatter now
    int hit_i = -1;
    T hit_t = T(0);
    uint32_t slot_item = 0, slot_left = 0;   // lane s < kSlots: pixel item and unfinished samples of slot s
    auto park = [&](const V3<T>& po, const V3<T>& pd) {
        T* r = &s_park[kPark ? wave : 0][0][lane];
        r[0] = po.x; r[64] = po.y; r[128] = po.z; r[192] = pd.x; r[256] = pd.y; r[320] = pd.z;
    };
    auto unpark = [&](V3<T>& po, V3<T>& pd) {
        asm volatile("" ::: "memory");   // re-read: the registers must not be kept across the sweep
        const T* r = &s_park[kPark ? wave : 0][0][lane];
        po = mk(r[0], r[64], r[128]);
        pd = mk(r[192], r[256], r[320]);
    };
    auto park_c = [&](const V3<T>& pc) {
        T* r = &s_park[kPark ? wave : 0][kParkC ? 6 : 0][lane];
        r[0] = pc.x; r[64] = pc.y; r[128] = pc.z;
    };
    auto unpark_c = [&]() -> V3<T> {
        asm volatile("" ::: "memory");
        const T* r = &s_park[kPark ? wave : 0][kParkC ? 6 : 0][lane];
        return mk(r[0], r[64], r[128]);
    };

    // Hand the lanes of `want` new samples in rank order, opening pixel slots as needed; returns
    // true in the lanes that got one.
    auto issue = [&](unsigned long long want, uint32_t& i_sid, uint32_t& i_slot, uint32_t& i_pix,
                     uint32_t& i_row, uint32_t& i_col) -> bool {
        const uint32_t spp = cold_args<T>()->spp;
        bool got = false;
        uint32_t busy = __builtin_amdgcn_readfirstlane(s_is[wave].busy);
        uint32_t cur = __builtin_amdgcn_readfirstlane(s_is[wave].cur);
        uint32_t cur_next = __builtin_amdgcn_readfirstlane(s_is[wave].cur_next);
        uint32_t cur_pix = __builtin_amdgcn_readfirstlane(s_is[wave].cur_pix);
        uint32_t cur_row = __builtin_amdgcn_readfirstlane(s_is[wave].cur_row);
        uint32_t cur_col = __builtin_amdgcn_readfirstlane(s_is[wave].cur_col);
        bool drained = __builtin_amdgcn_readfirstlane(s_is[wave].drained) != 0u;
        uint32_t blk_next = __builtin_amdgcn_readfirstlane(s_is[wave].blk_next);
        uint32_t blk_end = __builtin_amdgcn_readfirstlane(s_is[wave].blk_end);
        uint32_t opened = 0;
        while (want != 0ull && !drained) {
            if (cur_next == spp) {
                const uint32_t avail = ~busy & ((1u << kSlots) - 1u);
                if (avail == 0u) break;   // every slot waits for straggler rays
                const auto& q = *cold_args<T>();
                uint32_t item = blk_next;
                if (blk_next < blk_end) {   // this wave's private rest of a block
                    ++blk_next;
                } else {   // lane 0: the workgroup pool, else the next block from the counter
                    uint32_t it = 0xFFFFFFFFu, nb = 0, ne = 0;
                    if (lane == 0) {
                        unsigned long long pv = __hip_atomic_load(&s_pool, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        for (;;) {
                            if ((uint32_t)(pv >> 32) >= (uint32_t)pv) break;   // empty
                            const unsigned long long old = atomicCAS(&s_pool, pv, pv + (1ull << 32));
                            if (old == pv) { it = (uint32_t)(pv >> 32); break; }
                            pv = old;
                        }
                        if (it == 0xFFFFFFFFu) {
                            const uint32_t j = atomicAdd(q.counter, 1u);
                            uint32_t b0 = 0, b1 = 0;
                            if (guided_block(q.n_items, max(1u, kTMul * gridDim.x), q.blk_g, j, b0, b1)) {
                                it = b0;
                                if (b1 > b0 + 1u &&
                                    atomicCAS(&s_pool, pv, ((unsigned long long)(b0 + 1u) << 32) | b1) != pv) {
                                    nb = b0 + 1u;   // the pool was refilled meanwhile: keep the rest
                                    ne = b1;
                                }
                            }
                        }
                    }
                    it = __builtin_amdgcn_readfirstlane(it);
                    if (it == 0xFFFFFFFFu) { drained = true; break; }
                    item = it;
                    blk_next = __builtin_amdgcn_readfirstlane(nb);
                    blk_end = __builtin_amdgcn_readfirstlane(ne);
                }
                const uint32_t s = __builtin_ctz(avail);
                const uint32_t ri = item / q.col_count, ci = item % q.col_count;
                cur_row = q.row_begin + ri * q.row_step;
                cur_col = q.col_begin + ci;
                cur_pix = cur_row * q.W + cur_col;
                if (lane == s) { slot_item = item; slot_left = spp; }
                if (lane == 0) s_slotpix[wave][s] = cur_pix;
                busy |= 1u << s;
                opened |= 1u << s;
                cur = s;
                cur_next = 0;
            }
            const bool isw = (want >> lane) & 1ull;
            const uint32_t take = min((uint32_t)__popcll(want), spp - cur_next);
            const uint32_t r = (uint32_t)__popcll(want & lt_mask);
            const bool mine = isw && r < take;
            if (mine) { got = true; i_sid = cur_next + r; i_slot = cur; i_pix = cur_pix; i_row = cur_row; i_col = cur_col; }
            want &= ~__ballot(mine);
            cur_next += take;
        }
        if (lane == 0) {
            s_is[wave].busy = busy; s_is[wave].cur = cur; s_is[wave].cur_next = cur_next; s_is[wave].cur_pix = cur_pix;
            s_is[wave].cur_row = cur_row; s_is[wave].cur_col = cur_col; s_is[wave].drained = drained ? 1u : 0u;
            s_is[wave].blk_next = blk_next; s_is[wave].blk_end = blk_end;
            if (CAMQ) s_is[wave].need |= opened;
        }
        return got;
    };

    // Record this step's terminations (e: the bounce of a sky hit, or depth for a ray still
    // enabled) and finish every pixel whose last sample this was.
    auto terminate = [&](bool term, bool skyhit, uint32_t e, uint32_t t_slot, uint32_t t_sid, const V3<T>& tc,
                         const V3<T>& td) {
        if (term) {
            const PScratch<T> sc = wave_scratch<T>(wave);
            sc.set_e(t_slot, t_sid, e);
            if (MODE == kModeV2) {
                // three dword stores, not one dwordx3: a dwordx3 wants three consecutive VGPRs, and
                // the copies into them raised the register peak (spills in the sphere sweeps).  A sky
                // hit at bounce 0 is white: no record (its map entry carries kWhite, finish_pixel)
                if (skyhit && e != 0u) sc.store_c(t_slot, t_sid, tc.x, tc.y, tc.z);
            } else {   // own value: colour x sky of the escaping ray's direction (:365-370 / :283-292), or black
                V3<T> v = mk(T(0.0), T(0.0), T(0.0));
                if (skyhit) { const V3<T> sk = sky(td.y); v = mk(tc.x * sk.x, tc.y * sk.y, tc.z * sk.z); }
                sc.store_c(t_slot, t_sid, v.x, v.y, v.z);
            }
        }
        unsigned long long tm = __ballot(term);
        bool synced = false;
        while (tm != 0ull) {
            const uint32_t s = __builtin_amdgcn_readlane(t_slot, __builtin_ctzll(tm));
            const unsigned long long m = __ballot(term && t_slot == s);
            tm &= ~m;
            if (lane == s) slot_left -= (uint32_t)__popcll(m);
            // pixel complete: once per spp samples -- marked unlikely, so the register allocator
            // places any spill code here rather than in the sphere sweeps
            if (__builtin_expect(__builtin_amdgcn_readlane(slot_left, s) == 0u, 0)) {
                if (!synced) { wave_mem_sync(); synced = true; }
                KSTAT(6);
#ifdef RT_EXP_DUP_FINISH   // timing experiment: finish_pixel twice (idempotent)
                (void)finish_pixel<T, MODE>(wave_scratch<T>(wave), s, __builtin_amdgcn_readlane(slot_item, s), s_hist[wave],
                                            s_stage[wave], kLMap ? s_lmap[wave] : nullptr);
                wave_mem_sync();
#endif
                const uint32_t K = finish_pixel<T, MODE>(wave_scratch<T>(wave), s, __builtin_amdgcn_readlane(slot_item, s),
                                                         s_hist[wave], s_stage[wave], kLMap ? s_lmap[wave] : nullptr);
                if (lane == 0) wcount[wave][2] += K;
                const uint32_t b = __builtin_amdgcn_readfirstlane(s_is[wave].busy);
                if (lane == 0) s_is[wave].busy = b & ~(1u << s);
            }
        }
    };

    // CAMQ: one full-wave batch of primary rays.  Returns false when no sample could be issued.
    auto camera_batch = [&]() -> bool {
        uint32_t bsid = 0, bslot = 0, bpix = 0, brow = 0, bcol = 0;
        const bool v = issue(~0ull, bsid, bslot, bpix, brow, bcol);
        const unsigned long long vm = __ballot(v);
        if (vm == 0ull) return false;
        V3<T> bd = mk(T(0), T(0), T(0));
#ifdef RT_EXP_DUP_CAMRAY   // timing experiment: the camera ray twice (same result)
        if (v) {
            uint32_t bsid2 = bsid;
            asm volatile("" : "+v"(bsid2));
            const U4 r = [&] {
                const auto& q0 = *cold_args<T>();
                return philox(bsid2, bpix, 0u, 0u, q0.k0, q0.k1);
            }();
            const auto& q = *cold_args_after<T>(r.a ^ r.b);
            const T s1 = div_dim((T)bcol + u01a(r, T(0)), q.W, q.rW);
            const T s2 = div_dim((T)brow + u01b(r, T(0)), q.H, q.rH);
            const V3<T> vu = mk(q.vu[0], q.vu[1], q.vu[2]), vv = mk(q.vv[0], q.vv[1], q.vv[2]);
            const V3<T> pc = add(mk(q.ulc[0], q.ulc[1], q.ulc[2]), add(mul(vu, s1), mul(vv, s2)));
            const V3<T> bd2 = unit(sub(pc, mk(q.center[0], q.center[1], q.center[2])));
            asm volatile("" ::"v"(bd2.x), "v"(bd2.y), "v"(bd2.z));
        }
#endif
        if (v) {   // Camera::get_ray (ray_tracing.rs:77-89) with origin == centre
            const U4 r = [&] {
                const auto& q0 = *cold_args<T>();
                return philox(bsid, bpix, 0u, 0u, q0.k0, q0.k1);
            }();
            const auto& q = *cold_args_after<T>(r.a ^ r.b);
            const T s1 = div_dim((T)bcol + u01a(r, T(0)), q.W, q.rW);
            const T s2 = div_dim((T)brow + u01b(r, T(0)), q.H, q.rH);
            const V3<T> vu = mk(q.vu[0], q.vu[1], q.vu[2]), vv = mk(q.vv[0], q.vv[1], q.vv[2]);
            const V3<T> pc = add(mk(q.ulc[0], q.ulc[1], q.ulc[2]), add(mul(vu, s1), mul(vv, s2)));
            bd = unit(sub(pc, mk(q.center[0], q.center[1], q.center[2])));
            if (MODE == kModeV2) wave_scratch<T>(wave).y(bslot, bsid) = bd.y;   // primary y (quirk Q2)
        }
        T bt = T(0);
        int bi = -1;
#ifndef RT_EXP_NO_CAMCULL
        {
            // the batch's pixel slots (one, or two where a pixel's samples end inside the batch)
            uint32_t smask = 0;
            for (unsigned long long m = vm; m != 0ull;) {
                const uint32_t sl = __builtin_amdgcn_readlane(bslot, (int)__builtin_ctzll(m));
                smask |= 1u << sl;
                m &= ~__ballot(v && bslot == sl);
            }
            // each newly opened pixel's candidate list (one cone walk per pixel, not per batch)
            uint32_t need = __builtin_amdgcn_readfirstlane(s_is[wave].need) & smask;
            if (need != 0u) {
                if (lane == 0) s_is[wave].need = s_is[wave].need & ~need;
                const uint32_t iw = cold_args<T>()->W;
                while (need != 0u) {
                    const uint32_t sl = (uint32_t)__builtin_ctz(need);
                    need &= need - 1u;
                    const uint32_t pxi = __builtin_amdgcn_readfirstlane(s_slotpix[wave][sl]);
                    const uint32_t row = pxi / iw;
#ifdef RT_EXP_DUP_PLIST   // timing experiment: each pixel's candidate list built twice (same list)
                    { uint32_t r2 = row; asm volatile("" : "+s"(r2)); (void)pixel_list<T, MEGA>(pxi - r2 * iw, r2, s_clist[wave][sl]); }
#endif
                    (void)pixel_list<T, MEGA>(pxi - row * iw, row, s_clist[wave][sl]);
                }
            }
            bool listed = true;
            for (uint32_t m = smask; m != 0u; m &= m - 1u)
                if (__builtin_amdgcn_readfirstlane(s_clist[wave][__builtin_ctz(m)][0]) == 0xFFFFu) listed = false;
#ifdef RT_EXP_DUP_CAM   // timing experiment: the batch's camera stage (listed or swept) twice (same result)
            {
                V3<T> bd2 = bd;
                asm volatile("" : "+v"(bd2.x));
                T bt2;
                const int bi2 = listed ? camera_listed<T, ROOT2, SC>(v, bd2, bt2, s_clist[wave], smask)
                                       : camera_sweep<T, ROOT2, SC, MEGA>(v, bd2, bt2);
                asm volatile("" ::"v"(bi2), "v"(bt2));
            }
#endif
            if (listed) bi = camera_listed<T, ROOT2, SC>(v, bd, bt, s_clist[wave], smask);
            else bi = camera_sweep<T, ROOT2, SC, MEGA>(v, bd, bt);   // whole wave: lanes are spheres in the cull
        }
#else
        if (v) bi = nearest_hit<T, ROOT2, SC, true>(p, bd, bd, bt);
#endif
        if (lane == 0) { wcount[wave][0] += (uint32_t)__popcll(vm); wcount[wave][1] += 64u; }
        const uint32_t depth = cold_args<T>()->depth;
        const bool skyhit = v && bi < 0;
        const bool term = v && (skyhit || depth == 1u);
        const bool push = v && !term;
        const unsigned long long pm = __ballot(push);
        const uint32_t qhead = __builtin_amdgcn_readfirstlane(s_is[wave].qhead);
        const uint32_t qcount = __builtin_amdgcn_readfirstlane(s_is[wave].qcount);
        if (push) {
            const uint32_t e = (qhead + qcount + (uint32_t)__popcll(pm & lt_mask)) % QN;
            q_sid[wave][e] = bsid | (bslot << 29);
            q_hit[wave][e] = bi;
            q_t[wave][e] = bt;
            q_d[wave][0][e] = bd.x; q_d[wave][1][e] = bd.y; q_d[wave][2][e] = bd.z;
        }
        if (lane == 0) s_is[wave].qcount = qcount + (uint32_t)__popcll(pm);
        terminate(term, skyhit, skyhit ? 0u : depth, bslot, bsid, mk(T(1.0), T(1.0), T(1.0)), bd);
        return true;
    };

    for (;;) {
        bool fresh = false;
        uint32_t frow = 0, fcol = 0;
        if constexpr (CAMQ) {
            // ---- top up the queue with camera batches, then free lanes pop primary-ray hits ----
            const unsigned long long freem = __ballot(!live);
            const uint32_t nfree = (uint32_t)__popcll(freem);
            for (;;) {
                const uint32_t qcount = __builtin_amdgcn_readfirstlane(s_is[wave].qcount);
                if (qcount >= nfree || qcount + 64u > QN) break;
                if (!camera_batch()) break;
            }
            const uint32_t qhead = __builtin_amdgcn_readfirstlane(s_is[wave].qhead);
            const uint32_t qcount = __builtin_amdgcn_readfirstlane(s_is[wave].qcount);
            const uint32_t take = min(nfree, qcount);
            const uint32_t r = (uint32_t)__popcll(freem & lt_mask);
            if (!live && r < take) {
                const uint32_t e = (qhead + r) % QN;
                const uint32_t w0 = q_sid[wave][e];
                sid = w0 & 0x1FFFFFFFu;
                slot = w0 >> 29;
                pix = s_slotpix[wave][slot];
                hit_i = q_hit[wave][e];
                hit_t = q_t[wave][e];
                const auto& q = *cold_args<T>();
                const V3<T> pd = mk(q_d[wave][0][e], q_d[wave][1][e], q_d[wave][2][e]);
                const V3<T> po = mk(q.center[0], q.center[1], q.center[2]);
                if constexpr (kPark) park(po, pd);
                else { d = pd; o = po; }
                if constexpr (kParkC) park_c(mk(T(1.0), T(1.0), T(1.0)));
                else c = mk(T(1.0), T(1.0), T(1.0));
                k = 0;
                live = true;
                scat = true;
            }
            if (lane == 0) { s_is[wave].qhead = (qhead + take) % QN; s_is[wave].qcount = qcount - take; }
        } else {
            // ---- hand free lanes the next samples (opening new pixel slots as needed) ----
            uint32_t nsid = 0, nslot = 0, npix = 0;
            fresh = issue(__ballot(!live), nsid, nslot, npix, frow, fcol);
            if (fresh) { sid = nsid; slot = nslot; pix = npix; }
        }
        // ---- next rays: camera rays for fresh lanes, scattered rays for last iteration's hits ----
#ifdef RT_EXP_DUP_SCATTER   // timing experiment: the next-ray stage twice (same result)
        if (fresh || scat) {
            V3<T> o2 = o, d2 = d, c2 = c;
            asm volatile("" : "+v"(o2.x), "+v"(d2.x), "+v"(c2.x));
            next_ray<T, SC>(CAMQ ? false : fresh, fcol, frow, pix, sid, k, hit_i, hit_t, o2, d2, c2);
            asm volatile("" ::"v"(o2.x), "v"(o2.y), "v"(o2.z), "v"(d2.x), "v"(d2.y), "v"(d2.z), "v"(c2.x), "v"(c2.y), "v"(c2.z));
        }
#endif
        if constexpr (kPark) unpark(o, d);
        if constexpr (kParkC) c = unpark_c();
        if (fresh || scat) next_ray<T, SC>(CAMQ ? false : fresh, fcol, frow, pix, sid, k, hit_i, hit_t, o, d, c);
        if constexpr (kPark) park(o, d);
        if constexpr (kParkC) park_c(c);
        if (fresh) {
            k = 0;
            live = true;
            if (MODE == kModeV2) wave_scratch<T>(wave).y(slot, sid) = d.y;   // primary y, kept for quirk Q2
        } else if (scat) {
            k += 1u;
        }
        if (__ballot(live) == 0ull) break;   // drained, and every slot finished
        // ---- one sphere sweep for every live ray ----
        const uint32_t depth = cold_args<T>()->depth;
        const bool act = live && k < depth;
        hit_i = -1;
#ifdef RT_EXP_DUP_SWEEP   // timing experiment: the general sweep twice (same result)
        if (act) {
            V3<T> o2 = o;
            asm volatile("" : "+v"(o2.x));
            T t2;
            const int h2 = nearest_hit<T, ROOT2, SC, false, MEGA>(p, o2, d, t2);
            asm volatile("" ::"v"(h2), "v"(t2));
        }
#endif
        if (act) hit_i = nearest_hit<T, ROOT2, SC, false, MEGA>(p, o, d, hit_t);
        const unsigned long long bact = __ballot(act);
        if (lane == 0 && bact) { wcount[wave][0] += (uint32_t)__popcll(bact); wcount[wave][1] += 64u; }
        // ---- terminations: record e (and the colour of a sky hit) ----
        const bool skyhit = act && hit_i < 0;
        // A hit at the last bounce is not scattered: the ray stays enabled and reads black
        // whatever its colour (ray_tracing.rs:495-497), and the scatter draws nothing observable.
        const bool term = live && (!act || skyhit || k + 1 == depth);
        scat = act && hit_i >= 0 && k + 1 < depth;
        if constexpr (kPark) {
            if (MODE != kModeV2) { V3<T> po, pd; unpark(po, pd); d = pd; }   // the own-value modes read d
        }
        if constexpr (kParkC) c = unpark_c();
        terminate(term, skyhit, skyhit ? k : depth, slot, sid, c, d);
        live = live && !term;
    }
    if (lane == 0) {
        const auto& q = *cold_args<T>();
        const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + wave;
        unsigned long long* cc = &q.segs[(gw & (kSegShards - 1)) * kSegStride];
        atomicAdd(cc + 0, wcount[wave][0]);
        atomicAdd(cc + 1, wcount[wave][1]);
        atomicAdd(cc + 2, wcount[wave][2]);
        for (uint32_t i = 0; i < kNWork; ++i) atomicAdd(cc + kWorkSlot + i, g_work[wave][i]);
#ifdef RT_KSTATS
        for (int i = 0; i < 8; ++i) atomicAdd(cc + 3 + i, g_kst[wave][i]);
#endif
    }
}

}  // namespace rt

// ============================== host side ==============================
using namespace rt;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(x)                                                                     \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) return fail(RT_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

struct rt_context {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_first = nullptr, ev_last = nullptr;
    bool have_first = false;
    // scene, fp64 and fp32 images
    void* sph64 = nullptr; void* sph32 = nullptr;   // grouped sphere records
    void* fsph64 = nullptr; void* fsph32 = nullptr; // fp32 filter streams (for fp64 / fp32 rays)
    uint32_t n_fgroups = 0;
    float f_cmax64 = 0, f_r2max64 = 0, f_cmax32 = 0, f_r2max32 = 0, f_r2min64 = 0, f_r2min32 = 0;
    void* cam64 = nullptr; void* cam32 = nullptr;   // camera-origin tables (same size; rebuilt per launch)
    void* camf64 = nullptr; void* camf32 = nullptr; // camera filter tables (fp32 layout; rebuilt per launch)
    void* cen64 = nullptr; void* cen32 = nullptr;   // AoS centre tables
    void* camx64 = nullptr; void* camx32 = nullptr; // per-sphere camera-origin records (rebuilt per launch)
    void* cull64 = nullptr; void* cull32 = nullptr; // camera cone-cull records (fp32; rebuilt per launch)
    uint32_t n_cull = 0;                            // records: n_spheres rounded up to 64, + 64 padding
    void* rsph64 = nullptr; void* rsph32 = nullptr; // general sweep: slot-order exact groups
    void* xrec32 = nullptr;                          // fp32: the exact test's r² and scene indices per group
    void* rfsph64 = nullptr; void* rfsph32 = nullptr; // slot-order fp32 filter groups
    void* top64 = nullptr; void* top32 = nullptr;   // cluster bounds (fp32 top groups)
    void* sup64 = nullptr; void* sup32 = nullptr;   // super boxes (4 clusters each)
    void* meg64 = nullptr; void* meg32 = nullptr;   // mega boxes (4 supers each; big scenes only)
    void* lfs64 = nullptr; void* lfs32 = nullptr;   // cluster-local filter groups (big scenes only)
    void* lcl64 = nullptr; void* lcl32 = nullptr;   // ... and the per-cluster frame records
    void* lbx64[4] = {}; void* lbx32[4] = {};       // local box levels: cluster boxes, supers, megas, gigas
    uint32_t n_gg = 0;
    float l_r2max64 = 0, l_r2min64 = 0, l_r2max32 = 0, l_r2min32 = 0;
    uint32_t n_mg = 0;
    void* mtiers = nullptr;                         // the mega walk's order table (pack_mega_tiers)
    float mt_lo[3] = {0, 0, 0}, mt_inv = 0;
    uint32_t mt_n[3] = {1, 1, 1};
    uint32_t* ridx = nullptr;
    void* clus64 = nullptr; void* clus32 = nullptr;   // cluster bounding spheres {C, R} (double)
    void* cullc64 = nullptr; void* cullc32 = nullptr; // per-cluster camera cull records (rebuilt per launch)
    uint32_t n_cslots = 0, n_clp = 0;                 // slot-order cull records; cluster records (x64)
    uint32_t n_supc = 0;                              // super records after them (x64; 0: none)
    uint32_t n_top = 0, n_xg = 0, n_xs = 0;
    uint32_t n_groups64 = 0, n_groups32 = 0;
    void* mat64 = nullptr; void* mat32 = nullptr;     // per-sphere material records
    uint32_t n_spheres = 0, n_materials = 0;
    unsigned long long* segs = nullptr;
    uint32_t* err = nullptr;
    uint32_t* counter = nullptr;   // persistent-kernel block counter (zeroed before each launch)
    void* scratch = nullptr;       // per-wave ray state (grown on demand)
    size_t scratch_bytes = 0;
    int n_cu = 0;
    uint64_t samples = 0, pixels = 0;
    hipStream_t last_stream = nullptr;   // stream of the previous render (they share scratch and tables)
    bool have_last = false;
};

extern "C" const char* rt_last_error(void) { return g_err.c_str(); }
// "rt_mi355x <version> gfx950 <product|experiment> src=<hash of the sources it was built from>"
extern "C" const char* rt_version(void) { return "rt_mi355x 0.3 gfx950 " RT_BUILD_KIND " src=" RT_SRC_HASH; }

extern "C" double rt_metal_clamp_fuzz(double fuzz) { return fuzz < 1.0 ? fuzz : 1.0; }

// Camera::new, ray_tracing.rs:27-62 (f64, Vec3 ops without FMA; compiled -ffp-contract=off).
extern "C" int rt_camera_new(rt_camera* out, uint32_t w, uint32_t h, double focal_length, double view_angle_deg,
                             const double center[3], const double look_at[3], const double up[3],
                             double defocus_angle_deg) {
    if (!out || !center || !look_at || !up || w == 0 || h == 0) return fail(RT_ERR_INVALID, "rt_camera_new: bad argument");
    const double rads_per_deg = 3.141592653589793 / 180.0;              // f64::to_radians
    const double aspect = (double)w / (double)h;                         // :28
    const double vh = std::tan((view_angle_deg * rads_per_deg) / 2.0) * focal_length * 2.0;  // :29
    const double vw = vh * aspect;                                       // :32
    auto unit3 = [](const double a[3], double o[3]) {
        const double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        o[0] = a[0] / l; o[1] = a[1] / l; o[2] = a[2] / l;
    };
    double dirv[3] = {look_at[0] - center[0], look_at[1] - center[1], look_at[2] - center[2]};
    double dir[3]; unit3(dirv, dir);                                     // :34
    const double wv[3] = {-dir[0], -dir[1], -dir[2]};                    // :35
    const double cr[3] = {up[1] * wv[2] - up[2] * wv[1], up[2] * wv[0] - up[0] * wv[2], up[0] * wv[1] - up[1] * wv[0]};
    double u[3]; unit3(cr, u);                                           // :36
    const double v[3] = {wv[1] * u[2] - wv[2] * u[1], wv[2] * u[0] - wv[0] * u[2], wv[0] * u[1] - wv[1] * u[0]};  // :37
    const double dr = focal_length * std::tan((defocus_angle_deg / 2.0) * rads_per_deg);  // :43
    out->image_width = w; out->image_height = h;
    for (int i = 0; i < 3; ++i) {
        out->center[i] = center[i];
        out->vu[i] = u[i] * vw;                                          // :39
        out->vv[i] = (-v[i]) * vh;                                       // :40
        out->ulc[i] = ((center[i] - wv[i] * focal_length) - out->vu[i] / 2.0) - out->vv[i] / 2.0;  // :41
        out->du[i] = u[i] * dr;                                          // :44
        out->dv[i] = v[i] * dr;                                          // :45
    }
    return RT_OK;
}

extern "C" int rt_context_create(int device, rt_context** out) {
    if (!out) return fail(RT_ERR_INVALID, "rt_context_create: out is NULL");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID, "rt_context_create: no such device");
    HIPCHK(hipSetDevice(device));
    rt_context* c = new rt_context();
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&c->ev_first));
    HIPCHK(hipEventCreate(&c->ev_last));
    HIPCHK(hipMalloc((void**)&c->segs, sizeof(unsigned long long) * kSegShards * kSegStride));
    HIPCHK(hipMalloc((void**)&c->err, 16));
    HIPCHK(hipMalloc((void**)&c->counter, 16));
    HIPCHK(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
    HIPCHK(hipMemset(c->segs, 0, sizeof(unsigned long long) * kSegShards * kSegStride));
    HIPCHK(hipMemset(c->err, 0, 16));
    *out = c;
    return RT_OK;
}

static void free_scene(rt_context* c) {
    (void)hipFree(c->sph64); (void)hipFree(c->sph32); (void)hipFree(c->mat64); (void)hipFree(c->mat32);
    (void)hipFree(c->cam64); (void)hipFree(c->cam32);
    c->cam64 = c->cam32 = nullptr;
    (void)hipFree(c->camf64); (void)hipFree(c->camf32);
    c->camf64 = c->camf32 = nullptr;
    (void)hipFree(c->fsph64); (void)hipFree(c->fsph32);
    c->fsph64 = c->fsph32 = nullptr;
    (void)hipFree(c->cen64); (void)hipFree(c->cen32);
    (void)hipFree(c->camx64); (void)hipFree(c->camx32); (void)hipFree(c->cull64); (void)hipFree(c->cull32);
    c->camx64 = c->camx32 = c->cull64 = c->cull32 = nullptr;
    (void)hipFree(c->rsph64); (void)hipFree(c->rsph32); (void)hipFree(c->rfsph64); (void)hipFree(c->rfsph32);
    (void)hipFree(c->xrec32);
    c->xrec32 = nullptr;
    (void)hipFree(c->top64); (void)hipFree(c->top32); (void)hipFree(c->ridx);
    (void)hipFree(c->sup64); (void)hipFree(c->sup32);
    c->sup64 = c->sup32 = nullptr;
    (void)hipFree(c->meg64); (void)hipFree(c->meg32);
    (void)hipFree(c->lfs64); (void)hipFree(c->lfs32); (void)hipFree(c->lcl64); (void)hipFree(c->lcl32);
    c->lfs64 = c->lfs32 = c->lcl64 = c->lcl32 = nullptr;
    for (int lv = 0; lv < 4; ++lv) {
        (void)hipFree(c->lbx64[lv]); (void)hipFree(c->lbx32[lv]);
        c->lbx64[lv] = c->lbx32[lv] = nullptr;
    }
    c->meg64 = c->meg32 = nullptr;
    c->n_mg = 0;
    c->n_gg = 0;
    (void)hipFree(c->mtiers);
    c->mtiers = nullptr;
    (void)hipFree(c->clus64); (void)hipFree(c->clus32); (void)hipFree(c->cullc64); (void)hipFree(c->cullc32);
    c->clus64 = c->clus32 = c->cullc64 = c->cullc32 = nullptr;
    c->n_cslots = c->n_clp = c->n_supc = 0;
    c->rsph64 = c->rsph32 = c->rfsph64 = c->rfsph32 = c->top64 = c->top32 = nullptr;
    c->ridx = nullptr;
    c->n_top = c->n_xg = c->n_xs = 0;
    c->sph64 = c->sph32 = c->mat64 = c->mat32 = c->cen64 = c->cen32 = nullptr;
    c->n_spheres = c->n_materials = 0;
}

extern "C" int rt_context_destroy(rt_context* c) {
    if (!c) return RT_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    free_scene(c);
    (void)hipFree(c->segs); (void)hipFree(c->err); (void)hipFree(c->counter); (void)hipFree(c->scratch);
    (void)hipEventDestroy(c->ev_first); (void)hipEventDestroy(c->ev_last);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return RT_OK;
}

// Grouped, padded sphere records (layout at SphGroup) + AoS centre table, in precision T.
template <typename T>
static void pack_scene(const rt_scene* s, std::vector<T>& grp, std::vector<T>& cen, std::vector<MatT<T>>& mats,
                       uint32_t& n_groups) {
    const uint32_t G = kGroup<T>;
    const uint32_t n = s->n_spheres;
    n_groups = (n + G - 1) / G;
    const uint32_t npad = n_groups * G;
    cen.assign((size_t)4 * (n ? n : 1), T(0));
    for (uint32_t i = 0; i < n; ++i) {
        const T r = (T)s->radius[i];
        cen[4 * i + 0] = (T)s->center[3 * i + 0];
        cen[4 * i + 1] = (T)s->center[3 * i + 1];
        cen[4 * i + 2] = (T)s->center[3 * i + 2];
        cen[4 * i + 3] = r;       // signed radius (scalar-mode normal, objects.rs:242)
    }
    auto field = [&](uint32_t i, int f) -> T {   // dummies: centre 0, r^2 = -inf (never hit)
        if (i >= n) return f == 3 ? -std::numeric_limits<T>::infinity() : T(0);
        return f == 3 ? cen[4 * i + 3] * cen[4 * i + 3] : cen[4 * i + f];   // r.powi(2) in T (objects.rs:256)
    };
    grp.assign((size_t)64 / sizeof(T) * (n_groups + 1), T(0));   // + 1 dummy group: prefetch target
    for (uint32_t i = 0; i < npad + G; ++i) {
        const uint32_t g = i / G, j = i % G;
        T* out = &grp[(size_t)g * (64 / sizeof(T))];
        for (int f = 0; f < 4; ++f) {
            if (sizeof(T) == 4) out[8 * (j / 2) + 2 * f + (j % 2)] = field(i, f);   // pair-interleaved
            else out[4 * j + f] = field(i, f);                                     // AoS
        }
    }
    mats.resize(s->n_materials ? s->n_materials : 1);
    for (uint32_t i = 0; i < s->n_materials; ++i) {
        const rt_material& m = s->materials[i];
        const T ior = (T)m.ior, one = T(1.0);
        const T inv = one / ior;
        const T qf = (one - inv) / (one + inv), qb = (one - ior) / (one + ior);
        mats[i] = MatT<T>{m.kind, m.hollow, (T)m.albedo[0], (T)m.albedo[1], (T)m.albedo[2], (T)m.fuzz, ior,
                          inv, qf * qf, qb * qb};
    }
}

// Filter stream for rays in precision T (layout at SphGroup, fp32, 4 spheres per group): centres
// as the T kernel sees them, converted to fp32; r2f = the kernel's r^2 (r.powi(2) in T) rounded up
// to fp32; +inf for "always exact" spheres; -inf for dummies.  Returns the margin bounds over the
// other spheres: max |c|_1 (rounded up) and max r2f.
template <typename T>
static void pack_filter(const std::vector<T>& cen, uint32_t n, std::vector<float>& grp, uint32_t& n_fgroups,
                        float& cmax, float& r2max, float& r2min, std::vector<float>& frec) {
    n_fgroups = (n + 3) / 4;
    std::vector<double> key(n);
    for (uint32_t i = 0; i < n; ++i)
        key[i] = std::fabs((double)cen[4 * i]) + std::fabs((double)cen[4 * i + 1]) + std::fabs((double)cen[4 * i + 2]) +
                 std::fabs((double)cen[4 * i + 3]);
    double median = 0.0;
    if (n) {
        std::vector<double> k2 = key;
        std::nth_element(k2.begin(), k2.begin() + n / 2, k2.end());
        median = k2[n / 2];
    }
    auto up32 = [](double v) -> float {   // fp32 >= v
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    // The kernel scales each lane's filter basis by 1/sqrt(1 + m/r2min), which inflates every r2f
    // by the factor (1 + m/r2min) >= 1 + m/r2f.  A floor on r2f (tiny spheres filtered as if of the
    // floor radius, conservative) keeps one tiny sphere from inflating all the others.
    double cm = 0.0, rm = 0.0;
    for (uint32_t i = 0; i < n; ++i) {
        const double c1 = std::fabs((double)(float)cen[4 * i]) + std::fabs((double)(float)cen[4 * i + 1]) +
                          std::fabs((double)(float)cen[4 * i + 2]);
        const double r2 = (double)(cen[4 * i + 3] * cen[4 * i + 3]);
        if (std::isfinite(key[i]) && std::isfinite(r2) && std::isfinite(c1) && !(key[i] > kExactRatio * median)) {
            cm = std::max(cm, c1);
            rm = std::max(rm, r2);
        }
    }
    const double floor2 = std::max(rm * 0x1.0p-10, cm * cm * 0x1.0p-16);
    double rmin = std::numeric_limits<double>::infinity();
    cm = 0.0; rm = 0.0;
    grp.assign((size_t)16 * (n_fgroups + 1), 0.0f);
    frec.assign((size_t)4 * n, 0.0f);
    for (uint32_t i = 0; i < 4 * (n_fgroups + 1); ++i) {
        float f[4] = {0.0f, 0.0f, 0.0f, -std::numeric_limits<float>::infinity()};
        if (i < n) {
            const T r2 = cen[4 * i + 3] * cen[4 * i + 3];   // as pack_scene: r.powi(2) in T
            f[0] = (float)cen[4 * i]; f[1] = (float)cen[4 * i + 1]; f[2] = (float)cen[4 * i + 2];
            const double c1 = std::fabs((double)f[0]) + std::fabs((double)f[1]) + std::fabs((double)f[2]);
            const bool finite = std::isfinite(key[i]) && std::isfinite((double)r2) && std::isfinite(c1);
            if (!finite || key[i] > kExactRatio * median) {
                f[3] = std::numeric_limits<float>::infinity();
            } else {
                f[3] = up32(std::max((double)r2, floor2));
                cm = std::max(cm, c1);
                rm = std::max(rm, (double)f[3]);
                rmin = std::min(rmin, (double)f[3]);
            }
        }
        const uint32_t g = i / 4, j = i % 4;
        for (int q = 0; q < 4; ++q) grp[(size_t)16 * g + 8 * (j / 2) + 2 * q + (j % 2)] = f[q];   // pair-interleaved
        if (i < n) for (int q = 0; q < 4; ++q) frec[(size_t)4 * i + q] = f[q];
    }
    cmax = up32(cm);
    r2max = up32(rm);
    r2min = std::isfinite(rmin) ? (float)rmin : 0.0f;   // exact: rmin is an fp32 value
}

// Spatial clusters for the general sweep's two-level filter (nearest_hit).  Slot order: first the
// "always exact" spheres (pack_filter's rule: non-finite, or |c|_1 + r above 8x the median, e.g. a
// ground sphere; and up to kBigExact spheres of more than kBigRatio x the median radius) in scene
// order, padded to whole groups -- every ray tests them exactly; then the
// filterable spheres, split k-d style (median along the longest extent of the centres) into
// clusters of at most kClusterMax = 16 spheres, each cluster in 4 whole groups (dummy-padded).  The
// cluster count is padded to whole top groups of 4 with empty clusters (never taken).  The sweep
// visits spheres in slot order, not scene order: hit_update's tie rule (equal t -> the later scene
// index wins; scalar mode: the earlier) makes the nearest hit independent of the visiting order.
constexpr uint32_t kClusterMax = 16;
constexpr double kBigRatio = 3.0;   // "big": radius above 3x the median radius of the filtered spheres
constexpr size_t kBigExact = 8;     // at most this many big spheres join the always-exact ones
struct SweepLayout {
    std::vector<int32_t> slot;                   // slot -> scene index, -1 = dummy (4 slots per group)
    std::vector<std::vector<uint32_t>> members;  // per cluster (count padded to a multiple of 4)
    uint32_t n_xg = 0;                           // leading groups of always-exact spheres
    uint32_t n_xs = 0;                           // always-exact spheres (slots 0 .. n_xs-1)
    bool giga = false;                           // splits aligned to gigas (1024 spheres) as well
};
static SweepLayout build_layout(const rt_scene* s) {
    const uint32_t n = s->n_spheres;
    std::vector<double> key(n);
    for (uint32_t i = 0; i < n; ++i)
        key[i] = std::fabs(s->center[3 * i]) + std::fabs(s->center[3 * i + 1]) + std::fabs(s->center[3 * i + 2]) +
                 std::fabs(s->radius[i]);
    double median = 0.0;
    if (n) {
        std::vector<double> k2 = key;
        std::nth_element(k2.begin(), k2.begin() + n / 2, k2.end());
        median = k2[n / 2];
    }
    std::vector<uint32_t> filt, exact;
    for (uint32_t i = 0; i < n; ++i) {
        const bool fin = std::isfinite(key[i]) && std::isfinite(s->radius[i] * s->radius[i]);
        (fin && !(key[i] > kExactRatio * median) ? filt : exact).push_back(i);
    }
    // A few spheres far larger than the typical one (RTIOW's three radius-1 spheres among radius-0.2
    // ones) are tested exactly by every ray too: in a cluster, one of them made its box 5x taller, and
    // every ray passing over the small spheres near it walked the cluster.  At most kBigExact of them
    // (more stay in clusters: exact tests for every ray would cost more).  Same-box C fp32 +5.1 %,
    // fp64 +5.4 %, B +4.1 %, E +3.1 % (profiles/r03/experiments/big_exact.txt).
    {
        std::vector<double> rr;
        for (uint32_t i : filt) rr.push_back(std::fabs(s->radius[i]));
        if (!rr.empty()) {
            std::nth_element(rr.begin(), rr.begin() + rr.size() / 2, rr.end());
            const double mr = rr[rr.size() / 2];
            std::vector<uint32_t> keep, big;
            for (uint32_t i : filt) (std::fabs(s->radius[i]) > kBigRatio * mr ? big : keep).push_back(i);
            if (!big.empty() && big.size() <= kBigExact) {
                filt.swap(keep);
                exact.insert(exact.end(), big.begin(), big.end());
                std::sort(exact.begin(), exact.end());
            }
        }
    }
    SweepLayout L;
    for (uint32_t i : exact) L.slot.push_back((int32_t)i);
    L.n_xs = (uint32_t)exact.size();
    while (L.slot.size() % 4) L.slot.push_back(-1);
    L.n_xg = (uint32_t)(L.slot.size() / 4);
    // k-d split (median along the longest extent of the centres), aligned to the box hierarchy above
    // the clusters: a node of more than 256 spheres (4 supers = one mega) gives its left part a
    // multiple of 256, a node of 65..256 a multiple of 64 (one super), smaller nodes a multiple of 16,
    // and each child's clusters are padded with empty ones to a whole number of its parent's unit
    // (the next sibling then starts on a super / mega boundary).  So every super box and mega box
    // bounds one k-d subtree.  Round 2 split at multiples of 16 only:
    // at config E (10 000 spheres, a 313-cluster left half) every super and mega on the right of a
    // split took clusters of two subtrees, and their boxes spanned both.
    auto build = [&](auto&& self, size_t b, size_t e, size_t pad) -> void {   // pad: clusters per block
        const size_t N = e - b, c0 = L.members.size();
        if (N <= kClusterMax) {
            if (e > b) L.members.emplace_back(filt.begin() + b, filt.begin() + e);
            while ((L.members.size() - c0) % pad) L.members.emplace_back();
            return;
        }
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = b; k < e; ++k)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], s->center[3 * filt[k] + a]);
                hi[a] = std::max(hi[a], s->center[3 * filt[k] + a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a) if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
        const size_t unit = L.giga && N > 64 * kClusterMax ? 64 * kClusterMax : N > 16 * kClusterMax ? 16 * kClusterMax
                          : N > 4 * kClusterMax ? 4 * kClusterMax : kClusterMax;
        const size_t m = b + std::min(N - 1, (N + 2 * unit - 1) / (2 * unit) * unit);
        std::nth_element(filt.begin() + b, filt.begin() + m, filt.begin() + e, [&](uint32_t x, uint32_t y) {
            const double cx = s->center[3 * x + ax], cy = s->center[3 * y + ax];
            return cx < cy || (cx == cy && x < y);
        });
        self(self, b, m, unit / kClusterMax);
        self(self, m, e, unit / kClusterMax);
        while ((L.members.size() - c0) % pad) L.members.emplace_back();
    };
    L.giga = filt.size() > 128 * kClusterMax;   // the mega kernels' scenes (more than 8 super groups)
    build(build, 0, filt.size(), 1);
    while (L.members.size() % 4) L.members.emplace_back();
    // Members ordered by k-d halving (16 -> 8|8 -> 4|4 -> 2|2), so each filter group and each exact pair
    // holds neighbours: a lane's passes concentrate in fewer groups and pairs.  Scene-index order (round
    // 2) grouped spheres along the generator's loop.  Same-box C fp32 +0.5 %, fp64 +0.7 %, E +0.4 %.
    auto kd_order = [&](auto&& self, std::vector<uint32_t>& v, size_t b, size_t e) -> void {
        if (e - b <= 2) return;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = b; k < e; ++k)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], s->center[3 * v[k] + a]);
                hi[a] = std::max(hi[a], s->center[3 * v[k] + a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a) if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
        size_t half = 1;
        while (2 * half < e - b) half *= 2;   // power-of-two left part: groups of 4 stay whole
        const size_t m = b + half;
        std::nth_element(v.begin() + b, v.begin() + m, v.begin() + e, [&](uint32_t x, uint32_t y) {
            const double cx = s->center[3 * x + ax], cy = s->center[3 * y + ax];
            return cx < cy || (cx == cy && x < y);
        });
        self(self, v, b, m);
        self(self, v, m, e);
    };
    for (auto& c : L.members) {
        std::sort(c.begin(), c.end());
        kd_order(kd_order, c, 0, c.size());
        for (uint32_t k = 0; k < kClusterMax; ++k) L.slot.push_back(k < c.size() ? (int32_t)c[k] : -1);
    }
    return L;
}

// Slot-order streams for rays in precision T: the exact groups (SphGroup layout of pack_scene),
// the fp32 filter groups (pack_filter's records) and the top stream of cluster bounds: axis-aligned
// boxes {centre C, half-extent h} in fp32, 4 per 96-byte group (BoxGroup), enclosing every member
// with its filter radius sqrt(r2f) (so the floor applies: h >= sqrt(r2min) on every axis), h rounded
// up and widened by 2^-20 relative and 4 u |C| for the fp32 rounding of C; h = +inf if a member is
// always exact in T, -inf for an empty cluster.  |C|_1 + |h|_1 enters the margin bound cmax.
template <typename T>
static void pack_sweep(const std::vector<T>& cen, const std::vector<float>& frec, const SweepLayout& L,
                       std::vector<T>& rgrp, std::vector<float>& rfgrp, std::vector<float>& top, float& cmax,
                       float& r2max, std::vector<float>& sup, std::vector<float>& meg) {
    auto up32 = [](double v) -> float {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    const size_t ns = L.slot.size(), nfg = ns / 4;
    constexpr uint32_t G = kGroup<T>, NE = 64 / sizeof(T);
    rgrp.assign((size_t)NE * (ns / G + 1), T(0));
    rfgrp.assign((size_t)16 * (nfg + 1), 0.0f);
    for (size_t i = 0; i < ns + G; ++i) {   // exact groups, + one dummy group
        const int32_t sc = i < ns ? L.slot[i] : -1;
        const size_t g = i / G, j = i % G;
        for (int f = 0; f < 4; ++f) {
            T v = f == 3 ? -std::numeric_limits<T>::infinity() : T(0);
            if (sc >= 0) v = f == 3 ? cen[4 * sc + 3] * cen[4 * sc + 3] : cen[4 * sc + f];   // r.powi(2) in T
            if (sizeof(T) == 4) rgrp[g * NE + 8 * (j / 2) + 2 * f + (j % 2)] = v;
            else rgrp[g * NE + 4 * j + f] = v;
        }
    }
    for (size_t i = 0; i < ns + 4; ++i) {   // filter groups, + one dummy group (prefetch target)
        const int32_t sc = i < ns ? L.slot[i] : -1;
        for (int f = 0; f < 4; ++f) {
            const float fv = sc >= 0 ? frec[(size_t)4 * sc + f] : (f == 3 ? -INFINITY : 0.0f);
            rfgrp[(size_t)16 * (i / 4) + 8 * ((i % 4) / 2) + 2 * f + (i % 2)] = fv;
        }
    }
    const size_t nc = L.members.size();
    top.assign((size_t)kBoxFloats / 4 * (nc + 4), 0.0f);   // + one empty top group (prefetch target)
    double cm = cmax;
    for (size_t k = 0; k < nc + 4; ++k) {
        float b[6] = {0.0f, 0.0f, 0.0f, -INFINITY, -INFINITY, -INFINITY};   // empty: never passes
        if (k < nc && !L.members[k].empty()) {
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            bool inf = false;
            for (uint32_t i : L.members[k]) {
                const double r = std::sqrt((double)frec[4 * i + 3]);   // the filter's (floored) radius
                if (!(frec[4 * i + 3] < INFINITY)) inf = true;
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::min(lo[a], (double)frec[4 * i + a] - r);
                    hi[a] = std::max(hi[a], (double)frec[4 * i + a] + r);
                }
            }
            double c1 = 0.0;
            for (int a = 0; a < 3; ++a) {
                b[a] = (float)(0.5 * (lo[a] + hi[a]));
                const double h = std::max(hi[a] - (double)b[a], (double)b[a] - lo[a]);
                b[3 + a] = inf ? INFINITY : up32(h * (1.0 + 0x1.0p-20) + 0x1.0p-22 * std::fabs((double)b[a]));
                c1 += std::fabs((double)b[a]) + (double)b[3 + a];
            }
            if (!inf) cm = std::max(cm, c1);
        }
        // pair-interleaved: pair q of a group at 12 q, {cx0,cx1, cy0,cy1, cz0,cz1, hx0,hx1, hy0,hy1, hz0,hz1}
        const size_t tg = k / 4, j = k % 4;
        for (int f = 0; f < 6; ++f) top[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)] = b[f];
    }
    // Super boxes: the union of the 4 cluster boxes of each top group, same rounding; 4 per group,
    // padded with empty boxes plus one empty group (prefetch target).  Mega boxes likewise over the
    // 4 supers of each super group, when there are more than 8 super groups (one sweep chunk).
    auto unite = [&](const std::vector<float>& lower, size_t nup, std::vector<float>& upper) {
        const size_t ng = (nup + 3) / 4;
        upper.assign((size_t)kBoxFloats * (ng + 1), 0.0f);
        for (size_t k = 0; k < 4 * (ng + 1); ++k) {
            float b[6] = {0.0f, 0.0f, 0.0f, -INFINITY, -INFINITY, -INFINITY};
            if (k < nup) {
                double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                bool inf = false, any = false;
                for (size_t j = 0; j < 4; ++j) {
                    const float* t = &lower[kBoxFloats * k + 12 * (j / 2) + (j % 2)];
                    if (!(t[6] > -INFINITY)) continue;   // empty box
                    any = true;
                    for (int a = 0; a < 3; ++a) {
                        if (!(t[6 + 2 * a] < INFINITY)) inf = true;
                        lo[a] = std::min(lo[a], (double)t[2 * a] - (double)t[6 + 2 * a]);
                        hi[a] = std::max(hi[a], (double)t[2 * a] + (double)t[6 + 2 * a]);
                    }
                }
                if (any) {
                    double c1 = 0.0;
                    for (int a = 0; a < 3; ++a) {
                        b[a] = inf ? 0.0f : (float)(0.5 * (lo[a] + hi[a]));
                        const double h = std::max(hi[a] - (double)b[a], (double)b[a] - lo[a]);
                        b[3 + a] = inf ? INFINITY : up32(h * (1.0 + 0x1.0p-20) + 0x1.0p-22 * std::fabs((double)b[a]));
                        c1 += std::fabs((double)b[a]) + (double)b[3 + a];
                    }
                    if (!inf) cm = std::max(cm, c1);
                }
            }
            const size_t tg = k / 4, j = k % 4;
            for (int f = 0; f < 6; ++f) upper[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)] = b[f];
        }
    };
    const size_t nsup = nc / 4, nsg = (nsup + 3) / 4;
    unite(top, nsup, sup);
    if (nsg > 8) unite(sup, nsg, meg);
    else meg.clear();
    cmax = up32(cm);
    (void)r2max;
}

// Cluster-local filter records for the MEGA kernels (nearest_hit).  Far from the origin the scene-wide
// margin of the sphere filter, 48 u ((max|c|_1 + |o|_1)^2 + max r2f), grows with the coordinates'
// magnitudes (config E: ~0.06 against r^2 = 0.04), though the rounding it covers grows with the
// distances involved.  In a frame centred on the cluster (C_k: its box centre, an fp32 value) the
// filter sees c' = RN_f(c - C_k) and o' = o - C_k, and the same margin formula with |c'|_1 <= Rc_k and
// |o'|_1 in place of the scene-wide magnitudes bounds the same errors (tests/filter_margin_fuzz.c,
// local mode).  r2f is floored per cluster at 2^-10 of its largest (a tiny sphere cannot inflate the
// others by more than that ratio).  Slot order and group layout as the scene-wide filter stream;
// always-exact slots get dummies (they are never filtered).
template <typename T>
static void pack_local(const std::vector<T>& cen, const SweepLayout& L, const std::vector<float>& top,
                       std::vector<float>& lfgrp, std::vector<float>& lrec, std::vector<float>& r2l) {
    auto up32 = [](double v) -> float {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    const size_t ns = L.slot.size(), nc = L.members.size();
    lfgrp.assign((size_t)16 * (ns / 4 + 1), 0.0f);
    for (size_t i = 0; i < ns + 4; ++i) lfgrp[(size_t)16 * (i / 4) + 8 * ((i % 4) / 2) + 6 + (i % 2)] = -INFINITY;
    lrec.assign((size_t)8 * (nc ? nc : 1), 0.0f);
    for (size_t k = 0; k < nc; ++k) {
        const auto& m = L.members[k];
        if (m.empty()) continue;
        float Ck[3];
        for (int f = 0; f < 3; ++f) Ck[f] = top[kBoxFloats * (k / 4) + 12 * ((k % 4) / 2) + 2 * f + (k % 2)];
        double r2max = 0.0, rc = 0.0;
        for (uint32_t i : m) r2max = std::max(r2max, (double)(cen[4 * i + 3] * cen[4 * i + 3]));   // r.powi(2) in T
        const double floor2 = r2max * 0x1.0p-10;
        double r2min = INFINITY, r2fmax = 0.0;
        for (uint32_t j = 0; j < m.size(); ++j) {
            const uint32_t i = m[j];
            const size_t slot = (size_t)4 * L.n_xg + kClusterMax * k + j;   // members in cluster-slot order
            float f[4];
            for (int a = 0; a < 3; ++a) f[a] = (float)((double)cen[4 * i + a] - (double)Ck[a]);   // RN_f(c - C_k)
            const T r2 = cen[4 * i + 3] * cen[4 * i + 3];
            f[3] = up32(std::max((double)r2, floor2));
            if (r2l.size() <= i) r2l.resize((size_t)i + 1, -INFINITY);
            r2l[i] = f[3];
            rc = std::max(rc, std::fabs((double)f[0]) + std::fabs((double)f[1]) + std::fabs((double)f[2]));
            r2min = std::min(r2min, (double)f[3]);
            r2fmax = std::max(r2fmax, (double)f[3]);
            for (int q = 0; q < 4; ++q) lfgrp[(size_t)16 * (slot / 4) + 8 * ((slot % 4) / 2) + 2 * q + (slot % 2)] = f[q];
        }
        float* r = &lrec[8 * k];
        r[0] = Ck[0]; r[1] = Ck[1]; r[2] = Ck[2];
        r[3] = up32(rc);
        r[4] = up32(r2fmax);
        r[5] = up32(1.0 / r2min);
    }
}

// The MEGA kernels' box levels in group-local frames.  World boxes as pack_sweep builds them, but
// around the spheres' locally floored radii (pack_local's r2f), so a far-from-origin scene keeps its
// boxes tight: clusters, their union per super, the supers' union per mega.  Every box group is then
// stored around its own frame S (the fp32 centre of its boxes' union): 24 floats of boxes with
// C' = RN_f(C - S) and H widened by 2^-22 |C'|, then {S, Rg = max |C'|_1 + |H'|_1} (LBoxGroup); the
// lane tests it with o' = o - S and the margin from |o'|_1 + Rg (nearest_hit; tests/box_cull_fuzz.c,
// local mode).  One empty group past the end of each level (prefetch target).
constexpr uint32_t kLBoxFloats = 32;
template <typename T>
static void pack_local_boxes(const std::vector<T>& cen, const SweepLayout& L, const std::vector<float>& r2l,
                             std::vector<float>& lclb, std::vector<float>& lsup, std::vector<float>& lmeg,
                             std::vector<float>& lgig, float& r2max, float& r2min, std::vector<float>* wmeg = nullptr) {
    auto up32 = [](double v) -> float {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
        return f;
    };
    const size_t nc = L.members.size();
    // world boxes, BoxGroup layout (4 per 24 floats), like pack_sweep's, around sqrt(local r2f)
    auto put = [](std::vector<float>& v, size_t k, const float b[6]) {
        const size_t tg = k / 4, j = k % 4;
        for (int f = 0; f < 6; ++f) v[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)] = b[f];
    };
    auto get = [](const std::vector<float>& v, size_t k, float b[6]) {
        const size_t tg = k / 4, j = k % 4;
        for (int f = 0; f < 6; ++f) b[f] = v[kBoxFloats * tg + 12 * (j / 2) + 2 * f + (j % 2)];
    };
    auto box_of = [&](double lo[3], double hi[3], bool inf, float b[6]) {
        for (int a = 0; a < 3; ++a) {
            b[a] = inf ? 0.0f : (float)(0.5 * (lo[a] + hi[a]));
            const double h = std::max(hi[a] - (double)b[a], (double)b[a] - lo[a]);
            b[3 + a] = inf ? INFINITY : up32(h * (1.0 + 0x1.0p-20) + 0x1.0p-22 * std::fabs((double)b[a]));
        }
    };
    const float kEmpty[6] = {0.0f, 0.0f, 0.0f, -INFINITY, -INFINITY, -INFINITY};
    std::vector<float> wcl((size_t)kBoxFloats * ((nc + 3) / 4 + 1));
    for (size_t k = 0; k < 4 * (wcl.size() / kBoxFloats); ++k) put(wcl, k, kEmpty);
    double rmax = 0.0, rmin = INFINITY;
    for (size_t k = 0; k < nc; ++k) {
        if (L.members[k].empty()) continue;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        bool inf = false;
        for (uint32_t i : L.members[k]) {
            if (!(r2l[i] < INFINITY)) inf = true;
            rmax = std::max(rmax, (double)r2l[i]);
            rmin = std::min(rmin, (double)r2l[i]);
            const double r = std::sqrt((double)r2l[i]);
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], (double)(float)cen[4 * i + a] - r);
                hi[a] = std::max(hi[a], (double)(float)cen[4 * i + a] + r);
            }
        }
        float b[6];
        box_of(lo, hi, inf, b);
        put(wcl, k, b);
    }
    r2max = up32(rmax);
    r2min = std::isfinite(rmin) ? (float)rmin : 0.0f;
    auto unite = [&](const std::vector<float>& lower, size_t nup, std::vector<float>& upper) {
        upper.assign((size_t)kBoxFloats * ((nup + 3) / 4 + 1), 0.0f);
        for (size_t k = 0; k < 4 * (upper.size() / kBoxFloats); ++k) put(upper, k, kEmpty);
        for (size_t k = 0; k < nup; ++k) {
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            bool inf = false, any = false;
            for (size_t j = 0; j < 4; ++j) {
                float t[6];
                get(lower, 4 * k + j, t);
                if (!(t[3] > -INFINITY)) continue;
                any = true;
                for (int a = 0; a < 3; ++a) {
                    if (!(t[3 + a] < INFINITY)) inf = true;
                    lo[a] = std::min(lo[a], (double)t[a] - (double)t[3 + a]);
                    hi[a] = std::max(hi[a], (double)t[a] + (double)t[3 + a]);
                }
            }
            if (!any) continue;
            float b[6];
            box_of(lo, hi, inf, b);
            put(upper, k, b);
        }
    };
    const size_t nsup = nc / 4, nsg = (nsup + 3) / 4;
    std::vector<float> wsu, wme;
    unite(wcl, nsup, wsu);
    unite(wsu, nsg, wme);
    if (wmeg) *wmeg = wme;
    // group-local frames: group g of `world` (4 boxes) -> LBoxGroup g
    auto localise = [&](const std::vector<float>& world, size_t ng, std::vector<float>& out) {
        out.assign((size_t)kLBoxFloats * (ng + 1), 0.0f);
        for (size_t g = 0; g < ng + 1; ++g) {
            float* o = &out[kLBoxFloats * g];
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            bool any = false, inf = false;
            float bx[4][6];
            for (size_t j = 0; j < 4; ++j) {
                if (g < ng) get(world, 4 * g + j, bx[j]);
                else for (int f = 0; f < 6; ++f) bx[j][f] = kEmpty[f];
                if (!(bx[j][3] > -INFINITY)) continue;
                any = true;
                for (int a = 0; a < 3; ++a) {
                    if (!(bx[j][3 + a] < INFINITY)) { inf = true; continue; }
                    lo[a] = std::min(lo[a], (double)bx[j][a] - (double)bx[j][3 + a]);
                    hi[a] = std::max(hi[a], (double)bx[j][a] + (double)bx[j][3 + a]);
                }
            }
            float Sg[3] = {0.0f, 0.0f, 0.0f};
            if (any && !inf)
                for (int a = 0; a < 3; ++a) Sg[a] = (float)(0.5 * (lo[a] + hi[a]));
            double rg = 0.0;
            for (size_t j = 0; j < 4; ++j) {
                float b[6];
                for (int f = 0; f < 6; ++f) b[f] = bx[j][f];
                if (b[3] > -INFINITY) {
                    for (int a = 0; a < 3; ++a) {
                        const float cl = (float)((double)b[a] - (double)Sg[a]);   // RN_f(C - S)
                        b[3 + a] = b[3 + a] < INFINITY ? up32((double)b[3 + a] + 0x1.0p-22 * std::fabs((double)cl)) : INFINITY;
                        b[a] = b[3 + a] < INFINITY ? cl : 0.0f;
                    }
                    rg = std::max(rg, std::fabs((double)b[0]) + std::fabs((double)b[1]) + std::fabs((double)b[2]) +
                                          (double)b[3] + (double)b[4] + (double)b[5]);
                }
                for (int f = 0; f < 6; ++f) o[12 * (j / 2) + 2 * f + (j % 2)] = b[f];
            }
            o[24] = Sg[0]; o[25] = Sg[1]; o[26] = Sg[2];
            o[27] = std::isfinite(rg) ? up32(rg) : INFINITY;
        }
    };
    localise(wcl, (nc + 3) / 4, lclb);
    localise(wsu, nsg, lsup);
    localise(wme, (nsg + 3) / 4, lmeg);
    // gigas: the union of each mega group's 4 megas (build_layout aligns them to k-d subtrees in scenes
    // of more than 2048 filtered spheres)
    const size_t nmg = (nsg + 3) / 4;
    std::vector<float> wgi;
    unite(wme, nmg, wgi);
    localise(wgi, (nmg + 3) / 4, lgig);
}

// The mega walk's order table (nearest_hit, MEGA): a grid of cubic cells (<= 4096, <= 64 per axis)
// over the union of the mega boxes (world frame, BoxGroup layout); per cell four u64 masks over the
// megas (<= 64): those whose box touches the cell, those within a quarter and within a half of the
// median mega size, and 0 (nested, so the walk's tiers partition the passing megas; the kernel's
// default uses the first two).  A heuristic:
// the order changes which boxes get culled early, never the hits.
struct MegaTiers { std::vector<uint64_t> t; float lo[3] = {0, 0, 0}, inv = 0; uint32_t n[3] = {1, 1, 1}; };
static MegaTiers pack_mega_tiers(const std::vector<float>& wme, size_t nm) {
    MegaTiers M;
    M.t.assign(4, 0ull);
    if (nm == 0 || nm > 64) return M;
    std::vector<std::array<double, 6>> bx;
    std::vector<size_t> id;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    std::vector<double> size;
    for (size_t k = 0; k < nm; ++k) {
        std::array<double, 6> b;
        for (int f = 0; f < 6; ++f) b[f] = wme[kBoxFloats * (k / 4) + 12 * ((k % 4) / 2) + 2 * f + (k % 2)];
        if (!(b[3] > -INFINITY) || !std::isfinite(b[3] + b[4] + b[5] + b[0] + b[1] + b[2])) continue;
        bx.push_back(b);
        id.push_back(k);
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b[a] - b[3 + a]);
            hi[a] = std::max(hi[a], b[a] + b[3 + a]);
        }
        size.push_back(2.0 * std::max(b[3], std::max(b[4], b[5])));
    }
    if (bx.empty()) return M;
    std::nth_element(size.begin(), size.begin() + size.size() / 2, size.end());
    const double L = size[size.size() / 2];
    double ext = 0.0;
    for (int a = 0; a < 3; ++a) ext = std::max(ext, hi[a] - lo[a]);
    double cs = ext > 0.0 ? ext / 64.0 : 1.0;
    for (;;) {
        uint64_t prod = 1;
        for (int a = 0; a < 3; ++a) {
            M.n[a] = (uint32_t)std::min(64.0, std::max(1.0, std::ceil((hi[a] - lo[a]) / cs)));
            prod *= M.n[a];
        }
        if (prod <= 4096) break;
        cs *= 1.25;
    }
    for (int a = 0; a < 3; ++a) M.lo[a] = (float)lo[a];
    M.inv = (float)(1.0 / cs);
    M.t.assign((size_t)4 * M.n[0] * M.n[1] * M.n[2], 0ull);
    for (uint32_t z = 0; z < M.n[2]; ++z)
        for (uint32_t y = 0; y < M.n[1]; ++y)
            for (uint32_t x = 0; x < M.n[0]; ++x) {
                const double cc[3] = {lo[0] + (x + 0.5) * cs, lo[1] + (y + 0.5) * cs, lo[2] + (z + 0.5) * cs};
                uint64_t* t = &M.t[(size_t)4 * (x + M.n[0] * (y + M.n[1] * z))];
                for (size_t j = 0; j < bx.size(); ++j) {
                    double d2 = 0.0;
                    for (int a = 0; a < 3; ++a) {
                        const double g = std::max(0.0, std::fabs(cc[a] - bx[j][a]) - (0.5 * cs + bx[j][3 + a]));
                        d2 += g * g;
                    }
                    const double d = std::sqrt(d2);
                    const uint64_t bit = 1ull << id[j];
                    if (d <= 0.0) t[0] |= bit;
                    if (d <= 0.25 * L) t[1] |= bit;
                    if (d <= 0.5 * L) t[2] |= bit;
                }
            }
    return M;
}

extern "C" int rt_context_set_scene(rt_context* c, const rt_scene* s) {
    if (!c || !s) return fail(RT_ERR_INVALID, "rt_context_set_scene: NULL argument");
    if (s->n_spheres && (!s->center || !s->radius || !s->material || !s->materials))
        return fail(RT_ERR_INVALID, "rt_context_set_scene: NULL array");
    for (uint32_t i = 0; i < s->n_spheres; ++i)
        if (s->material[i] >= s->n_materials)
            return fail(RT_ERR_INVALID, "rt_context_set_scene: material index out of range (objects.rs:296 would panic)");
    for (uint32_t i = 0; i < s->n_materials; ++i)
        if (s->materials[i].kind > RT_DIELECTRIC)
            return fail(RT_ERR_INVALID, "rt_context_set_scene: unknown material kind (materials.rs:31 would panic)");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    free_scene(c);
    std::vector<double> g64, c64; std::vector<MatT<double>> m64;
    std::vector<float> g32, c32; std::vector<MatT<float>> m32;
    pack_scene(s, g64, c64, m64, c->n_groups64);
    pack_scene(s, g32, c32, m32, c->n_groups32);
    std::vector<uint32_t> sm(s->n_spheres ? s->n_spheres : 1, 0);
    for (uint32_t i = 0; i < s->n_spheres; ++i) sm[i] = s->material[i];
    auto up = [&](void** dst, const void* src, size_t bytes) -> int {
        HIPCHK(hipMalloc(dst, bytes));
        HIPCHK(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
        return RT_OK;
    };
    int rc;
    if ((rc = up(&c->sph64, g64.data(), g64.size() * sizeof(double))) != RT_OK) return rc;
    if ((rc = up(&c->sph32, g32.data(), g32.size() * sizeof(float))) != RT_OK) return rc;
    {
        std::vector<float> f64g, f32g, fr64, fr32;
        uint32_t nf = 0;
        pack_filter(c64, s->n_spheres, f64g, nf, c->f_cmax64, c->f_r2max64, c->f_r2min64, fr64);
        pack_filter(c32, s->n_spheres, f32g, c->n_fgroups, c->f_cmax32, c->f_r2max32, c->f_r2min32, fr32);
        if ((rc = up(&c->fsph64, f64g.data(), f64g.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->fsph32, f32g.data(), f32g.size() * sizeof(float))) != RT_OK) return rc;
        const SweepLayout L = build_layout(s);
        std::vector<double> rg64; std::vector<float> rg32, rf64, rf32, t64, t32, s64, s32, m64, m32;
        pack_sweep(c64, fr64, L, rg64, rf64, t64, c->f_cmax64, c->f_r2max64, s64, m64);
        pack_sweep(c32, fr32, L, rg32, rf32, t32, c->f_cmax32, c->f_r2max32, s32, m32);
        if ((rc = up(&c->sup64, s64.data(), s64.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->sup32, s32.data(), s32.size() * sizeof(float))) != RT_OK) return rc;
        c->n_mg = m32.empty() ? 0u : (uint32_t)(m32.size() / kBoxFloats - 1);   // groups, without the empty one
        if (c->n_mg) {
            if ((rc = up(&c->meg64, m64.data(), m64.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->meg32, m32.data(), m32.size() * sizeof(float))) != RT_OK) return rc;
            std::vector<float> lf64, lf32, lr64, lr32, q64, q32;
            pack_local(c64, L, t64, lf64, lr64, q64);
            pack_local(c32, L, t32, lf32, lr32, q32);
            std::vector<float> b64[4], b32[4];
            pack_local_boxes(c64, L, q64, b64[0], b64[1], b64[2], b64[3], c->l_r2max64, c->l_r2min64);
            std::vector<float> wme;
            pack_local_boxes(c32, L, q32, b32[0], b32[1], b32[2], b32[3], c->l_r2max32, c->l_r2min32, &wme);
            c->n_gg = L.giga && c->n_mg <= 16u ? (c->n_mg + 3u) / 4u : 0u;
            {
                const MegaTiers M = pack_mega_tiers(wme, (L.members.size() / 4 + 3) / 4);
                if ((rc = up(&c->mtiers, M.t.data(), M.t.size() * sizeof(uint64_t))) != RT_OK) return rc;
                for (int a = 0; a < 3; ++a) { c->mt_lo[a] = M.lo[a]; c->mt_n[a] = M.n[a]; }
                c->mt_inv = M.inv;
            }
            for (int lv = 0; lv < 4; ++lv) {
                if ((rc = up(&c->lbx64[lv], b64[lv].data(), b64[lv].size() * sizeof(float))) != RT_OK) return rc;
                if ((rc = up(&c->lbx32[lv], b32[lv].data(), b32[lv].size() * sizeof(float))) != RT_OK) return rc;
            }
            if ((rc = up(&c->lfs64, lf64.data(), lf64.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lfs32, lf32.data(), lf32.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lcl64, lr64.data(), lr64.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lcl32, lr32.data(), lr32.size() * sizeof(float))) != RT_OK) return rc;
        }
        c->n_top = (uint32_t)(L.members.size() / 4);
        c->n_xg = L.n_xg;
        c->n_xs = L.n_xs;
        // slot -> scene index (0xFFFFFFFF: dummy), padded past the last cluster by one block of 64
        // (the camera sweep's empty quarters read the slots of cluster index n_clusters)
        const uint32_t ncl = (uint32_t)L.members.size();
        c->n_cslots = 4u * L.n_xg + 16u * ncl + 64u;
        c->n_clp = (ncl + 63u) / 64u * 64u;
        std::vector<uint32_t> ridx(c->n_cslots, 0xFFFFFFFFu);
        for (size_t i = 0; i < L.slot.size(); ++i) if (L.slot[i] >= 0) ridx[i] = (uint32_t)L.slot[i];
        // cluster bounding spheres for the camera cull, per precision: centre = the members' AABB
        // centre, R >= max |c_i - C| + |r_i| over the members' T-precision centres and radii.  Scenes
        // with more than 128 clusters (config E) also get super records, the bounding spheres of the
        // 4 clusters of each super (camera_sweep tests them first), stored after the cluster records.
        const uint32_t nsup = ncl / 4u;
        c->n_supc = ncl > 128u ? (nsup + 63u) / 64u * 64u : 0u;
        auto bounds = [&](auto const& cen, std::vector<double>& out) {
            out.assign((size_t)4 * ((c->n_clp + c->n_supc) ? c->n_clp + c->n_supc : 1), 0.0);
            for (size_t k = 0; k < out.size() / 4; ++k) out[4 * k + 3] = -INFINITY;
            auto sphere = [&](size_t at, uint32_t k0, uint32_t nk) {   // the members of clusters k0 .. k0+nk-1
                double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                bool any = false;
                for (uint32_t k = k0; k < k0 + nk; ++k)
                    for (uint32_t i : L.members[k]) {
                        any = true;
                        for (int a = 0; a < 3; ++a) {
                            const double r = std::fabs((double)cen[4 * i + 3]);
                            lo[a] = std::min(lo[a], (double)cen[4 * i + a] - r);
                            hi[a] = std::max(hi[a], (double)cen[4 * i + a] + r);
                        }
                    }
                if (!any) return;
                double C[3], R = 0.0;
                for (int a = 0; a < 3; ++a) C[a] = 0.5 * (lo[a] + hi[a]);
                for (uint32_t k = k0; k < k0 + nk; ++k)
                    for (uint32_t i : L.members[k]) {
                        const double dx = (double)cen[4 * i] - C[0], dy = (double)cen[4 * i + 1] - C[1],
                                     dz = (double)cen[4 * i + 2] - C[2];
                        R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + std::fabs((double)cen[4 * i + 3]));
                    }
                out[4 * at] = C[0]; out[4 * at + 1] = C[1]; out[4 * at + 2] = C[2];
                out[4 * at + 3] = std::isfinite(R) ? R * (1.0 + 0x1.0p-40) : INFINITY;
            };
            for (uint32_t k = 0; k < ncl; ++k) sphere(k, k, 1);
            if (c->n_supc)
                for (uint32_t k = 0; k < nsup; ++k) sphere(c->n_clp + k, 4 * k, 4);
        };
        std::vector<double> cl64, cl32;
        bounds(c64, cl64);
        bounds(c32, cl32);
        if ((rc = up(&c->clus64, cl64.data(), cl64.size() * sizeof(double))) != RT_OK) return rc;
        if ((rc = up(&c->clus32, cl32.data(), cl32.size() * sizeof(double))) != RT_OK) return rc;
        HIPCHK(hipMalloc(&c->cullc64, cl64.size() / 4 * 4 * sizeof(float)));
        HIPCHK(hipMalloc(&c->cullc32, cl32.size() / 4 * 4 * sizeof(float)));
        if ((rc = up(&c->rsph64, rg64.data(), rg64.size() * sizeof(double))) != RT_OK) return rc;
        if ((rc = up(&c->rsph32, rg32.data(), rg32.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->rfsph64, rf64.data(), rf64.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->rfsph32, rf32.data(), rf32.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->top64, t64.data(), t64.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->top32, t32.data(), t32.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up((void**)&c->ridx, ridx.data(), ridx.size() * sizeof(uint32_t))) != RT_OK) return rc;
        {   // fp32 exact-test records: a walked group's centres are its filter group's (the same fp32
            // values), so a taken group loads only these 32 bytes (nearest_hit, exact4f)
            const size_t ng = rg32.size() / 16;
            std::vector<uint32_t> xr((size_t)8 * ng, 0xFFFFFFFFu);
            for (size_t g = 0; g < ng; ++g) {
                for (int q = 0; q < 2; ++q)
                    for (int h = 0; h < 2; ++h) memcpy(&xr[8 * g + 2 * q + h], &rg32[16 * g + 8 * q + 6 + h], 4);
                for (int j = 0; j < 4; ++j) if (4 * g + j < ridx.size()) xr[8 * g + 4 + j] = ridx[4 * g + j];
            }
            if ((rc = up((void**)&c->xrec32, xr.data(), xr.size() * sizeof(uint32_t))) != RT_OK) return rc;
        }
        HIPCHK(hipMalloc(&c->camf64, f64g.size() * sizeof(float)));
        HIPCHK(hipMalloc(&c->camf32, f32g.size() * sizeof(float)));
    }
    HIPCHK(hipMalloc(&c->cam64, g64.size() * sizeof(double)));
    HIPCHK(hipMalloc(&c->cam32, g32.size() * sizeof(float)));
    c->n_cull = (s->n_spheres + 63u) / 64u * 64u + 64u;
    HIPCHK(hipMalloc(&c->camx64, (size_t)4 * c->n_cslots * sizeof(double)));
    HIPCHK(hipMalloc(&c->camx32, (size_t)4 * c->n_cslots * sizeof(float)));
    HIPCHK(hipMalloc(&c->cull64, (size_t)4 * c->n_cslots * sizeof(float)));
    HIPCHK(hipMalloc(&c->cull32, (size_t)4 * c->n_cslots * sizeof(float)));
    if ((rc = up(&c->cen64, c64.data(), c64.size() * sizeof(double))) != RT_OK) return rc;
    if ((rc = up(&c->cen32, c32.data(), c32.size() * sizeof(float))) != RT_OK) return rc;
    {
        // per-sphere records: next_ray gathers a hit sphere's material in one dependent load
        std::vector<MatT<double>> s64(sm.size());
        std::vector<MatT<float>> s32(sm.size());
        for (size_t i = 0; i < sm.size(); ++i)
            if (sm[i] < m64.size()) { s64[i] = m64[sm[i]]; s32[i] = m32[sm[i]]; }
        if ((rc = up(&c->mat64, s64.data(), s64.size() * sizeof(MatT<double>))) != RT_OK) return rc;
        if ((rc = up(&c->mat32, s32.data(), s32.size() * sizeof(MatT<float>))) != RT_OK) return rc;
    }
    c->n_spheres = s->n_spheres;
    c->n_materials = s->n_materials;
    return RT_OK;
}

static bool check_range(const rt_camera* cam, const rt_tile_range* r) {
    if (r->row_count == 0 || r->col_count == 0 || r->row_step == 0) return false;
    if (r->col_begin + (uint64_t)r->col_count > cam->image_width) return false;
    const uint64_t last_row = r->row_begin + (uint64_t)(r->row_count - 1) * r->row_step;
    return last_row < cam->image_height;
}

static int ensure_scratch(rt_context* c, size_t bytes, hipStream_t st);

// The kernel instantiation for (flags, waves-per-SIMD target, camera batches, mega level).  W < 0:
// the defaults (RT_WAVES unset).  The mega level (scenes with more than 8 super groups) has its own
// live-path kernels (fp32 at 5 or 6 waves, default 6; fp64 at 4); at other W such scenes are swept
// from the super boxes (the same result, more box tests).
template <typename T, bool CAMQ>
static void (*pick_kernel(uint32_t flags, int W, bool mega, bool big))(KParams<T>) {
    const bool r2 = (flags & RT_FLAG_ROOT2) != 0u;
    constexpr bool F32 = sizeof(T) == 4;
    constexpr int WM = kWavesModes<T>;
    if (flags & RT_FLAG_MODE_SCALAR) return trace_paths<T, WM, false, kModeScalar, CAMQ>;
    if (flags & RT_FLAG_MODE_VECTORIZED3)
        return r2 ? trace_paths<T, WM, true, kModeV3, CAMQ> : trace_paths<T, WM, false, kModeV3, CAMQ>;
    if (flags & RT_FLAG_MODE_VECTORIZED)
        return r2 ? trace_paths<T, WM, true, kModeV1, CAMQ> : trace_paths<T, WM, false, kModeV1, CAMQ>;
    if (r2) return trace_paths<T, WM, true, kModeV2, CAMQ>;
    if (mega) {
        const int Wm = W < 0 ? (F32 ? (big ? kWavesMegaF32 : 5) : kWavesF64) : W;
        if constexpr (F32) {
            if (Wm == 5) return trace_paths<T, 5, false, kModeV2, CAMQ, true>;
            if (Wm == 6) return trace_paths<T, 6, false, kModeV2, CAMQ, true>;
        } else {
            if (Wm == 4) return trace_paths<T, 4, false, kModeV2, CAMQ, true>;
        }
    }
    if (W < 0) W = F32 ? (big ? kWavesF32 : 5) : kWavesF64;
    if constexpr (F32) {
        if (W >= 7) return trace_paths<T, 7, false, kModeV2, CAMQ>;
    }
    return W >= 6 ? trace_paths<T, 6, false, kModeV2, CAMQ> : W >= 5 ? trace_paths<T, 5, false, kModeV2, CAMQ>
                                                           : trace_paths<T, 4, false, kModeV2, CAMQ>;
}

template <typename T>
static int launch_t(rt_context* c, const rt_camera* cam, uint32_t depth, uint32_t spp, uint64_t seed, uint32_t flags,
                    const rt_tile_range& rg, void* d_rgb, void* d_lin, hipStream_t st) {
    KParams<T> p;
    memset(&p, 0, sizeof(p));
    const bool f64 = sizeof(T) == 8;
    p.sph = (const T*)(f64 ? c->sph64 : c->sph32);
    p.cen = (const T*)(f64 ? c->cen64 : c->cen32);
    p.n_groups = f64 ? c->n_groups64 : c->n_groups32;
    p.fsph = (const float*)(f64 ? c->fsph64 : c->fsph32);
    p.n_fgroups = c->n_fgroups;
    p.rsph = (const T*)(f64 ? c->rsph64 : c->rsph32);
    p.rfsph = (const float*)(f64 ? c->rfsph64 : c->rfsph32);
    p.xrec = f64 ? nullptr : (const uint32_t*)c->xrec32;
    p.ftop = (const float*)(f64 ? c->top64 : c->top32);
    p.fsup = (const float*)(f64 ? c->sup64 : c->sup32);
    p.fmeg = (const float*)(f64 ? c->meg64 : c->meg32);
    p.n_mg = c->n_mg;
    p.lfsph = (const float*)(f64 ? c->lfs64 : c->lfs32);
    p.lclu = (const float*)(f64 ? c->lcl64 : c->lcl32);
    p.lclb = (const float*)(f64 ? c->lbx64[0] : c->lbx32[0]);
    p.lsup = (const float*)(f64 ? c->lbx64[1] : c->lbx32[1]);
    p.lmeg = (const float*)(f64 ? c->lbx64[2] : c->lbx32[2]);
    p.lgig = (const float*)(f64 ? c->lbx64[3] : c->lbx32[3]);
    p.n_gg = c->n_gg;
    p.mtiers = (const uint64_t*)c->mtiers;
    for (int a = 0; a < 3; ++a) { p.mt_lo[a] = c->mt_lo[a]; p.mt_n[a] = c->mt_n[a]; }
    p.mt_inv = c->mt_inv;
    {
        auto up32 = [](double v) -> float {
            float f = (float)v;
            if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
            return f;
        };
        const double r2m = (double)(f64 ? c->l_r2min64 : c->l_r2min32);
        p.l_r2max = f64 ? c->l_r2max64 : c->l_r2max32;
        p.l_hir2 = up32((double)kFilterMargin * 0.5 / r2m);
        p.l_isr = up32(8.0 * 0x1.0p-24 / std::sqrt(r2m));
    }
    p.ridx = c->ridx;
    p.n_top = c->n_top;
    p.n_xg = c->n_xg;
    p.n_xs = c->n_xs;
    p.f_cmax = f64 ? c->f_cmax64 : c->f_cmax32;
    p.f_r2max = f64 ? c->f_r2max64 : c->f_r2max32;
    p.f_r2min = f64 ? c->f_r2min64 : c->f_r2min32;
    {
        auto up32 = [](double v) -> float {
            float f = (float)v;
            if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
            return f;
        };
        const double r2m = (double)p.f_r2min;   // 0 (no filtered sphere) gives +inf: every basis is zero
        p.f_ir2 = up32(1.0 / r2m);
        p.f_hir2 = up32(0.5 / r2m);
        p.f_isr = up32(8.0 * 0x1.0p-24 / std::sqrt(r2m));
    }
    bool filter_off = false;
    {   // diagnostics: every general-sweep and camera-sweep group through the exact test
        const char* e = getenv("RT_FILTER_OFF");
        filter_off = e && atoi(e) != 0;
        if (filter_off) p.f_cmax = std::numeric_limits<float>::infinity();
    }
    p.mats = (const MatT<T>*)(f64 ? c->mat64 : c->mat32);
    p.n_spheres = c->n_spheres;
    p.W = cam->image_width; p.H = cam->image_height;
    p.rW = p.W < (1u << 20) ? 1.0 / (double)p.W : 0.0;   // div_dim
    p.rH = p.H < (1u << 20) ? 1.0 / (double)p.H : 0.0;
    for (int i = 0; i < 3; ++i) {
        p.center[i] = (T)cam->center[i]; p.ulc[i] = (T)cam->ulc[i]; p.vu[i] = (T)cam->vu[i];
        p.vv[i] = (T)cam->vv[i]; p.du[i] = (T)cam->du[i]; p.dv[i] = (T)cam->dv[i];
    }
    p.spp = spp;
    p.C = (spp + 3) / 4;
    p.P = 4 * p.C;
    p.depth = depth;
    p.flags = flags;
    {
        bool pinhole = true;
        for (int i = 0; i < 3; ++i) {
            if (p.du[i] != T(0) || p.dv[i] != T(0)) pinhole = false;
            if (p.center[i] == T(0) && std::signbit(p.center[i])) pinhole = false;
        }
        if (pinhole) p.flags |= kFlagPinholeInternal;
    }
    p.s_sel = (p.C - 1) % 2;   // ray_tracing.rs:486
    p.k0 = (uint32_t)seed; p.k1 = (uint32_t)(seed >> 32);
    p.row_begin = rg.row_begin; p.row_step = rg.row_step; p.col_begin = rg.col_begin; p.col_count = rg.col_count;
    p.rgb = (uint8_t*)d_rgb;
    p.lin = (double*)d_lin;
    p.segs = c->segs;
    p.err = c->err;
    p.counter = c->counter;
    p.n_items = rg.row_count * rg.col_count;

    // Persistent grid: as many 4-wave workgroups as stay resident, never more waves than pixels.
    // Minimum waves per SIMD the register allocation targets.  RT_WAVES (4..7; read at every
    // launch, so one process can compare them) overrides it for the live-path kernels (pinhole and
    // defocus cameras); the ROOT2 and semantics-mode kernels always run at kWavesModes.
    const char* waves_env = getenv("RT_WAVES");
    const int W = waves_env && atoi(waves_env) > 0 ? atoi(waves_env) : -1;
    // Camera batches + camera-origin table when every primary ray starts at the centre.
    const bool camq = (p.flags & kFlagPinholeInternal) && depth >= 1u;
    const bool big = (uint64_t)p.n_items * spp >= kW6SamplesPerWave * 24u * (uint64_t)c->n_cu;
    void (*kern)(KParams<T>) = camq ? pick_kernel<T, true>(flags, W, p.n_mg > 0, big)
                                    : pick_kernel<T, false>(flags, W, p.n_mg > 0, big);
    if (camq) {
        p.camsph = (const T*)(f64 ? c->cam64 : c->cam32);
        p.camf = (const float*)(f64 ? c->camf64 : c->camf32);
        p.camx = (const T*)(f64 ? c->camx64 : c->camx32);
        p.cull = (const float*)(f64 ? c->cull64 : c->cull32);
        const uint32_t n_slots = (p.n_groups + 1) * kGroup<T>, n_fslots = (p.n_fgroups + 1) * 4;
        p.cullc = (const float*)(f64 ? c->cullc64 : c->cullc32);
        p.n_clp = c->n_clp;
        p.n_supc = c->n_supc;
        const uint32_t n_thr = std::max(std::max(std::max(n_slots, n_fslots), c->n_cull),
                                        std::max(c->n_cslots, c->n_clp + c->n_supc));
        auto build = (flags & RT_FLAG_MODE_SCALAR) ? build_cam_table<T, true> : build_cam_table<T, false>;
        hipLaunchKernelGGL(build, dim3((n_thr + 255) / 256), dim3(256), 0, st, p.sph, (T*)p.camsph, n_slots,
                           (float*)p.camf, n_fslots, p.center[0], p.center[1], p.center[2], (uint32_t)filter_off,
                           (T*)p.camx, (float*)p.cull, c->n_cull, c->n_spheres, c->ridx, c->n_cslots,
                           (const double*)(f64 ? c->clus64 : c->clus32), (float*)p.cullc, c->n_clp + c->n_supc);
        HIPCHK(hipGetLastError());
    }
    int per_cu = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 256, 0));
    if (per_cu < 1) per_cu = 1;
    uint64_t nblocks = (uint64_t)c->n_cu * (uint64_t)per_cu;
    const uint64_t need = ((uint64_t)p.n_items + 3) / 4;
    if (nblocks > need) nblocks = need;
    {   // G: the largest power of two <= min(kMaxBlock, kBlockSamples / spp, pixels per wave / kBlockShare),
        // raised to kClaimSpp / spp (claim rate, below) where the share bound would go under it
        const uint64_t per_wave = (uint64_t)p.n_items / (4u * nblocks);
        const uint64_t g = std::max<uint64_t>({1u, std::min<uint64_t>({(uint64_t)kMaxBlock, kBlockSamples / spp,
                                                                       per_wave / kBlockShare}),
                                               std::min<uint64_t>((uint64_t)kMaxBlock, (kClaimSpp + spp - 1) / spp)});
        uint32_t G = 1;
        while (2u * G <= g) G *= 2u;
        p.blk_g = G;
    }
    p.swide = paths_wide(p.P, depth);
    p.vbytes = paths_vbytes(p.P, p.swide, (flags & RT_FLAG_MODE_VECTORIZED3) != 0u);
    p.sbytes = paths_sbytes(p.P, sizeof(T), p.swide);
    p.scratch_stride = (size_t)p.vbytes + (size_t)kSlots * p.sbytes;
    // Keep the scratch within a fixed budget: fewer resident waves for very large spp.
    const uint64_t kScratchBudget = 24ull << 30;
    const uint64_t max_blocks = kScratchBudget / (4 * p.scratch_stride);
    if (nblocks > max_blocks) nblocks = max_blocks > 0 ? max_blocks : 1;
    const int rc = ensure_scratch(c, p.scratch_stride * nblocks * 4, st);
    if (rc != RT_OK) return rc;
    p.scratch = (char*)c->scratch;
    HIPCHK(hipMemsetAsync(c->counter, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(kern, dim3((uint32_t)nblocks), dim3(256), 0, st, p);
    HIPCHK(hipGetLastError());
    return RT_OK;
}

static int ensure_scratch(rt_context* c, size_t bytes, hipStream_t st) {
    if (bytes <= c->scratch_bytes) return RT_OK;
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipDeviceSynchronize());
    if (c->scratch) HIPCHK(hipFree(c->scratch));
    c->scratch = nullptr;
    c->scratch_bytes = 0;
    HIPCHK(hipMalloc(&c->scratch, bytes));
    c->scratch_bytes = bytes;
    return RT_OK;
}

extern "C" int rt_render_async(rt_context* c, const rt_camera* cam, uint32_t max_bounces, uint32_t spp, uint64_t seed,
                               uint32_t flags, const rt_tile_range* range, void* d_rgb8, void* d_linear, void* stream) {
    if (!c || !cam) return fail(RT_ERR_INVALID, "rt_render_async: NULL argument");
    if (spp == 0) return fail(RT_ERR_INVALID, "rt_render_async: spp == 0 (the reference panics: 0/0 in to_u8_array)");
    if (flags & ~RT_FLAG_ALL) return fail(RT_ERR_INVALID, "rt_render_async: unknown flag bits");
    {
        const uint32_t modes = flags & (RT_FLAG_MODE_VECTORIZED | RT_FLAG_MODE_SCALAR | RT_FLAG_MODE_VECTORIZED3);
        if (modes & (modes - 1u))
            return fail(RT_ERR_INVALID, "rt_render_async: the RT_FLAG_MODE_* flags are exclusive");
    }
    if (spp > (1u << 20)) return fail(RT_ERR_UNSUPPORTED, "rt_render_async: spp > 2^20");
    if (cam->image_width == 0 || cam->image_height == 0) return fail(RT_ERR_INVALID, "rt_render_async: empty image");
    if ((uint64_t)cam->image_width * cam->image_height > 0xFFFFFFFFull) return fail(RT_ERR_UNSUPPORTED, "image too large");
    rt_tile_range rg = range ? *range : rt_tile_range{0, 1, cam->image_height, 0, cam->image_width};
    if (!check_range(cam, &rg)) return fail(RT_ERR_INVALID, "rt_render_async: tile range outside the image");
    if ((uint64_t)rg.row_count * rg.col_count > 0x7FFFFFFFull) return fail(RT_ERR_UNSUPPORTED, "too many pixels in one call");
    const bool f32 = (flags & RT_FLAG_F32) != 0;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream
    // Renders on one context share its work counter, scratch and camera table: a render on a new
    // stream first waits for the previous stream, so cross-stream use serialises instead of racing.
    if (c->have_last && c->last_stream != st) HIPCHK(hipStreamSynchronize(c->last_stream));
    c->last_stream = st;
    c->have_last = true;
    if (!c->have_first) {
        HIPCHK(hipEventRecord(c->ev_first, st));
        c->have_first = true;
    }
    const int rc = f32 ? launch_t<float>(c, cam, max_bounces, spp, seed, flags, rg, d_rgb8, d_linear, st)
                       : launch_t<double>(c, cam, max_bounces, spp, seed, flags, rg, d_rgb8, d_linear, st);
    if (rc != RT_OK) return rc;
    HIPCHK(hipEventRecord(c->ev_last, st));
    c->pixels += (uint64_t)rg.row_count * rg.col_count;
    c->samples += (uint64_t)rg.row_count * rg.col_count * spp;
    return RT_OK;
}

extern "C" int rt_context_collect(rt_context* c, void* stream, rt_stats* out) {
    if (!c) return fail(RT_ERR_INVALID, "rt_context_collect: NULL context");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream
    HIPCHK(hipStreamSynchronize(st));
    std::vector<unsigned long long> segs(kSegShards * kSegStride);
    uint32_t err = 0;
    HIPCHK(hipMemcpy(segs.data(), c->segs, segs.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&err, c->err, sizeof(uint32_t), hipMemcpyDeviceToHost));
    float ms = 0.f;
    if (c->have_first) HIPCHK(hipEventElapsedTime(&ms, c->ev_first, c->ev_last));
    HIPCHK(hipMemset(c->segs, 0, segs.size() * sizeof(unsigned long long)));
    HIPCHK(hipMemset(c->err, 0, 16));
    uint64_t total = 0, slots = 0, iters = 0, kst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, work[kNWork] = {};
    for (int i = 0; i < kSegShards; ++i)
        for (int j = 0; j < 8; ++j) kst[j] += segs[(size_t)i * kSegStride + 3 + j];
    if (kst[0] | kst[1] | kst[2] | kst[3])   // instrumented build (make kstats) only
        fprintf(stderr, "rt_kstats: general taken_groups %llu sweeps %llu clusters %llu top_groups %llu  camera "
                "candidates %llu sweeps %llu  finish_pixel %llu  filter_lanes_passing %llu\n",
                (unsigned long long)kst[0], (unsigned long long)kst[1], (unsigned long long)kst[4],
                (unsigned long long)kst[5], (unsigned long long)kst[2], (unsigned long long)kst[3],
                (unsigned long long)kst[6], (unsigned long long)kst[7]);
    for (int i = 0; i < kSegShards; ++i) {
        total += segs[(size_t)i * kSegStride];
        slots += segs[(size_t)i * kSegStride + 1];
        iters += segs[(size_t)i * kSegStride + 2];
        for (uint32_t j = 0; j < kNWork; ++j) work[j] += segs[(size_t)i * kSegStride + kWorkSlot + j];
    }
    if (out) {
        memset(out, 0, sizeof(*out));
        out->kernel_ms = ms;
        out->pixels = c->pixels;
        out->samples = c->samples;
        out->ray_segments = total;
        out->lane_slots = slots;
        out->bounce_iters = iters;
        out->pixels_per_second = ms > 0.f ? (double)c->pixels / ((double)ms * 1e-3) : 0.0;
        out->box_groups = work[kWBox];
        out->filter_groups = work[kWFilt];
        out->exact_tests = work[kWExact];
        out->cone_tests = work[kWCone];
        out->camera_exact_tests = work[kWCExact];
    }
    c->have_first = false;
    c->pixels = c->samples = 0;
    if (err) return fail(RT_ERR_RANGE, "a pixel channel exceeded 2.0 (Color::to_u8_array would panic, color.rs:55-57)");
    return RT_OK;
}

extern "C" int rt_device_alloc(rt_context* c, size_t bytes, void** out) {
    if (!c || !out) return fail(RT_ERR_INVALID, "rt_device_alloc: NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMalloc(out, bytes ? bytes : 1));
    return RT_OK;
}
extern "C" int rt_device_free(rt_context* c, void* ptr) {
    if (!c) return fail(RT_ERR_INVALID, "rt_device_free: NULL context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipFree(ptr));
    return RT_OK;
}
extern "C" int rt_memcpy_d2h(rt_context* c, void* dst, const void* src, size_t bytes) {
    if (!c || !dst || !src) return fail(RT_ERR_INVALID, "rt_memcpy_d2h: NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}

extern "C" int rt_render(const rt_scene* scene, const rt_camera* cam, uint32_t max_bounces, uint32_t spp, uint64_t seed,
                         uint32_t flags, const rt_tile_range* range, uint8_t* rgb8, double* linear, rt_stats* stats) {
    if (!scene || !cam) return fail(RT_ERR_INVALID, "rt_render: NULL argument");
    const auto t0 = std::chrono::steady_clock::now();
    rt_context* c = nullptr;
    int rc = rt_context_create(0, &c);
    if (rc != RT_OK) return rc;
    struct Guard { rt_context* c; void* a = nullptr; void* b = nullptr;
        ~Guard() { if (a) rt_device_free(c, a); if (b) rt_device_free(c, b); rt_context_destroy(c); } } g{c};
    rc = rt_context_set_scene(c, scene);
    if (rc != RT_OK) return rc;
    const rt_tile_range rg = range ? *range : rt_tile_range{0, 1, cam->image_height, 0, cam->image_width};
    const size_t npx = (size_t)rg.row_count * rg.col_count;
    if (rgb8 && (rc = rt_device_alloc(c, npx * 3, &g.a)) != RT_OK) return rc;
    if (linear && (rc = rt_device_alloc(c, npx * 3 * sizeof(double), &g.b)) != RT_OK) return rc;
    rc = rt_render_async(c, cam, max_bounces, spp, seed, flags, &rg, g.a, g.b, nullptr);
    if (rc != RT_OK) return rc;
    rt_stats st;
    const int crc = rt_context_collect(c, nullptr, &st);
    if (crc != RT_OK && crc != RT_ERR_RANGE) return crc;
    if (rgb8 && (rc = rt_memcpy_d2h(c, rgb8, g.a, npx * 3)) != RT_OK) return rc;
    if (linear && (rc = rt_memcpy_d2h(c, linear, g.b, npx * 3 * sizeof(double))) != RT_OK) return rc;
    st.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    st.pixels_per_second = st.seconds > 0 ? (double)st.pixels / st.seconds : 0.0;
    if (stats) *stats = st;
    if (crc == RT_ERR_RANGE) return fail(RT_ERR_RANGE, "a pixel channel exceeded 2.0 (Color::to_u8_array would panic, color.rs:55-57)");
    return RT_OK;
}
