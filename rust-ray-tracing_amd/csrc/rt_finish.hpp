// rt_finish.hpp — per-wave record scratch and finish_pixel: the replay of trace_vectorized2's
// positions from the termination bounces, quirk Q3's final read (ray_tracing.rs:486-504) and the
// reduction in the reference's order, /spp and Color::to_u8_array (renderer.rs:161, color.rs:54-64).
#pragma once
#include "rt_common.hpp"

namespace rt {

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
constexpr uint32_t kSlots = 8;   // pixels a wave may have in flight (lane s holds slot s's metadata)
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

// The final reduction in the reference's order (ray_tracing.rs:499-502, color.rs:226-232): per lane l of
// PackedColor<4>, chunks j = 0..C-1 from +0.0, over the values vals(q, r, g, b) forms for positions
// q < P.  All 64 lanes form the values of 64 positions at a time into LDS (stage, transposed); lanes
// ch * 4 + l then add theirs in order, the 12 running sums kept in LDS (hist) between batches: a short
// live range keeps this loop from raising the kernel's register peak.  Returns lane ch * 4 + l's sum.
template <typename T, typename F>
__device__ __forceinline__ T reduce_positions(uint32_t P, uint32_t* hist, T (*stage)[64], F&& vals) {
    const uint32_t lane = threadIdx.x & 63u;
    T* accl = (T*)hist;
    if (lane < 12u) accl[lane] = T(0.0);
    for (uint32_t qb = 0; qb < P; qb += 64u) {
        const uint32_t qq = qb + lane;
        T vr = T(0.0), vg = T(0.0), vb = T(0.0);
        if (qq < P) vals(qq, vr, vg, vb);
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return lane < 12u ? accl[lane] : T(0.0);
}


// The live path's final reduction (ray_tracing.rs:488-504) over whole batches of 64 positions with a u16
// position map (LDS or the wave's scratch): the same values and the same order of adds as
// reduce_positions with finish_pixel's generic value lambda (the partial last batch, spp % 64, goes through
// that lambda), specialised: no bounds test in whole batches, a three-op map decode, a branch-free record
// load for positions without an entry (clamped to a valid record, value 0), the 12 running sums in a VGPR,
// and two batches per iteration: the y, map and record loads of both are issued together and the batches
// staged and summed one after the other, so a 512-position pixel waits for 4 load round trips, not 8
// (round 5, same-box C fp32 +0.4 %, fp64 +0.6 %, E +0.6 %; prefetching the next pair's map entries as well
// lost, profiles/r05/reduce_pair_ab.txt).
template <typename T, typename G>
__device__ __forceinline__ T reduce_live16(const PScratch<T>& sc, uint32_t s, uint32_t spp, uint32_t P, const uint16_t* lmap,
                                           bool lm, uint32_t* hist, T (*stage)[64], G&& generic) {
    const uint32_t lane = threadIdx.x & 63u;
    T* accl = (T*)hist;
    T racc = T(0.0);
    if (lane < 12u) accl[lane] = T(0.0);
    const uint32_t nfull = spp & ~63u;
    const uint16_t* gmap = (const uint16_t*)sc.base;
    const uint32_t si = 16u * (lane & 3u) + (lane >> 2);
    auto mapat = [&](uint32_t qi) -> uint32_t { return lm ? (uint32_t)lmap[qi] : (uint32_t)gmap[qi]; };
    // values of one batch (positions qb + lane) from its y, map entry and record
    auto vals16 = [&](T y, uint32_t m16, const C3<T>& cm, T& vr, T& vg, T& vb) {
        const bool has = m16 != 0xFFFFu, wh = m16 >= 0x8000u;
        const V3<T> sk = sky(y);
        vr = has ? (wh ? sk.x : cm.x * sk.x) : T(0.0);   // (white x sky) == sky, bit for bit
        vg = has ? (wh ? sk.y : cm.y * sk.y) : T(0.0);
        vb = has ? (wh ? sk.z : cm.z * sk.z) : T(0.0);
    };
    auto rec = [&](uint32_t m16) -> C3<T> { return sc.c(s, min(m16 & 0x7FFFu, spp - 1u)); };   // clamped when none
    // the 12 lanes' running sums over one staged batch, in position order
    auto sum16 = [&](T vr, T vg, T vb) {
        stage[0][si] = vr; stage[1][si] = vg; stage[2][si] = vb;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane < 12u) {
            const T* sv = &stage[lane >> 2][16u * (lane & 3u)];
            T a = racc;
#pragma unroll
            for (uint32_t u0 = 0; u0 < 16u; u0 += 4u) {
                T v[4];
#pragma unroll
                for (uint32_t u = 0; u < 4u; ++u) v[u] = sv[u0 + u];
#pragma unroll
                for (uint32_t u = 0; u < 4u; ++u) a = a + v[u];
            }
            racc = a;
        }
        __builtin_amdgcn_wave_barrier();
    };
    uint32_t qb = 0;
    for (; qb + 128u <= nfull; qb += 128u) {   // two batches per round trip
        const uint32_t qq = qb + lane;
        const uint32_t m0 = mapat(qq), m1 = mapat(qq + 64u);
        const T y0 = sc.y(s, qq), y1 = sc.y(s, qq + 64u);
        const C3<T> c0 = rec(m0), c1 = rec(m1);
        T r0, g0, b0, r1, g1, b1;
        vals16(y0, m0, c0, r0, g0, b0);
        vals16(y1, m1, c1, r1, g1, b1);
        sum16(r0, g0, b0);
        sum16(r1, g1, b1);
    }
    if (qb < nfull) {   // a leftover single batch
        const uint32_t qq = qb + lane, m0 = mapat(qq);
        T r0, g0, b0;
        vals16(sc.y(s, qq), m0, rec(m0), r0, g0, b0);
        sum16(r0, g0, b0);
    }
    if (lane < 12u) accl[lane] = racc;
    // the partial last batch (and positions past spp): the generic path, continuing the same sums
    for (uint32_t qb = nfull; qb < P; qb += 64u) {
        const uint32_t qq = qb + lane;
        T vr = T(0.0), vg = T(0.0), vb = T(0.0);
        if (qq < P) generic(qq, vr, vg, vb);
        stage[0][si] = vr; stage[1][si] = vg; stage[2][si] = vb;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane < 12u) {
            const uint32_t nu = min(16u, (P - qb) / 4u);
            const T* sv = &stage[lane >> 2][16u * (lane & 3u)];
            T a = accl[lane];
            for (uint32_t u = 0; u < nu; ++u) a = a + sv[u];
            accl[lane] = a;
        }
        __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return lane < 12u ? accl[lane] : T(0.0);
}

// The pixel's value: PackedColor::sum of the 4 lanes' sums (or the scalar mode's average), / spp
// (renderer.rs:161), Color::to_u8_array's assert and bytes (color.rs:54-64).
template <typename T, int MODE>
__device__ __forceinline__ void write_pixel(T acc, uint32_t item) {
    const auto& q = *cold_args<T>();
    const uint32_t lane = threadIdx.x & 63u;
    const T s1 = __shfl(acc, (int)((lane + 1) & 63u)), s2 = __shfl(acc, (int)((lane + 2) & 63u)),
            s3 = __shfl(acc, (int)((lane + 3) & 63u));
    const bool writer = MODE == kModeScalar ? lane < 3u : (lane < 12u && (lane & 3u) == 0u);
    if (writer) {
        const uint32_t ch = MODE == kModeScalar ? lane : lane >> 2;
        const T tot = MODE == kModeScalar ? acc : (((T(0.0) + acc) + s1) + s2) + s3;
        const T v = tot / (T)q.spp;                                 // renderer.rs:161
        if (!(v <= T(2.0))) atomicOr(q.err, 1u);                    // color.rs:55-57 assert
        if (q.rgb) q.rgb[(size_t)item * 3 + ch] = q8(v);
        if (q.lin) q.lin[(size_t)item * 3 + ch] = (double)v;
    }
}

// A sky pixel finished without tracing (trace_paths, camera batches: a pixel whose camera candidate
// list is empty, so none of its primary rays can hit a sphere and every sample escapes at bounce 0;
// depth > 1).  As finish_pixel's sky path (the replay is the identity, position q < spp holds
// sky(y_q)), with y_q the primary direction's y that Camera::get_ray (ray_tracing.rs:77-89) gives
// sample q, computed here exactly as the camera batches compute it; positions past spp hold sky(0).
template <typename T>
__device__ __forceinline__ void finish_sky_direct(uint32_t item, uint32_t col, uint32_t row, uint32_t pix,
                                                  uint32_t* hist, T (*stage)[64]) {
    const auto& q = *cold_args<T>();
    const uint32_t spp = q.spp;
    const V3<T> s0 = sky(T(0.0));
    const T acc = reduce_positions<T>(q.P, hist, stage, [&](uint32_t qq, T& vr, T& vg, T& vb) {
        if (qq >= spp) { vr = s0.x; vg = s0.y; vb = s0.z; return; }
        const auto& qc = *cold_args<T>();
        const U4 r = rng<T>(qq, pix, 0u, 0u, qc.k0, qc.k1);
        const T s1 = div_dim((T)col + u01a(r, T(0)), qc.W, qc.rW);
        const T s2 = div_dim((T)row + u01b(r, T(0)), qc.H, qc.rH);
        const V3<T> vu = mk(qc.vu[0], qc.vu[1], qc.vu[2]), vv = mk(qc.vv[0], qc.vv[1], qc.vv[2]);
        const V3<T> pc = add(mk(qc.ulc[0], qc.ulc[1], qc.ulc[2]), add(mul(vu, s1), mul(vv, s2)));
        const V3<T> sk = sky(unit(sub(pc, mk(qc.center[0], qc.center[1], qc.center[2]))).y);
        vr = sk.x; vg = sk.y; vb = sk.z;
    });
    write_pixel<T, kModeV2>(acc, item);
}

// Replay pixel slot s's positions from its records, apply the retire rule, reduce, write the
// pixel (whole wave; returns the number of bounce iterations the reference runs for the pixel).
// all_e0: every sample of the slot terminated at bounce 0 (trace_paths tracks it per slot).
// The position map in LDS (live-path kernels without the mega level, P <= kLMapCap positions: config C's
// 512 spp): the replay's scattered u16 writes, the map's initialisation and the reduction's reads stay
// on the CU instead of going to HBM as partial lines.  Larger P uses the global map in PScratch.
template <typename T, int MODE, bool BALLOT01 = true>
__device__ __forceinline__ uint32_t finish_pixel(const PScratch<T>& sc, uint32_t s, uint32_t item, uint32_t* hist,
                                                 T (*stage)[64], uint16_t* lmap, bool all_e0 = false) {
    const auto& q = *cold_args<T>();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t spp = q.spp, P = q.P, C = q.C, depth = q.depth;
    constexpr uint32_t kNone = PScratch<T>::kNone;
    const bool lm = kLMapCap > 0u && lmap != nullptr && P <= kLMapCap;   // wave-uniform
    auto set_map = [&](uint32_t qq, uint32_t smp) {
        if (lm) lmap[qq] = PScratch<T>::to16(smp);
        else sc.set_map(qq, smp);
    };
    // Bounce iterations the reference runs: K = min(depth, max e + 1).  The same pass builds the
    // histogram of the termination bounces below 64 (a sample terminated iff e < depth, and then
    // e < K); it is only used when K <= 64.
    // (An incremental histogram kept by terminate as samples end, skipping this pass, measured -1.7 %
    // at config C fp32 and -1.0 % fp64: its per-termination LDS atomics cost more than the pass.)
    // all_e0 (trace_paths: no sample of the slot terminated at a bounce e > 0): K = 1 without the pass.
    uint32_t K = 0;
    const bool known1 = MODE == kModeV2 && all_e0 && depth > 1u;
    const bool hist_on = MODE == kModeV2 && depth > 0u && !known1;
    if (hist_on) {
        hist[lane] = 0u;
        __builtin_amdgcn_wave_barrier();
    }
    if (known1) K = 1u;
    else if (depth > 0) {
        // BALLOT01: the two commonest bounces (e = 0, the sky at bounce 0: 43 % of config C's samples; e = 1)
        // are counted with ballots into wave-uniform sums, LDS atomics only for e >= 2 (64 lanes adding to one
        // LDS word serialise): C fp32 +0.4 %, fp64 +0.1 %; the mega kernels (config E, fewer bounce-0 skies)
        // lost 0.3 % and keep the atomics (profiles/r05/hist01_ab.txt)
        uint32_t me = 0, h0 = 0, h1 = 0;   // #{e == 0}, #{e == 1} (wave-uniform)
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
                const bool hk = hist_on && b + 64u * u + lane < spp && ev[u] < depth && ev[u] < 64u;
                if constexpr (BALLOT01) {
                    h0 += (uint32_t)__popcll(__ballot(hk && ev[u] == 0u));
                    h1 += (uint32_t)__popcll(__ballot(hk && ev[u] == 1u));
                    if (hk && ev[u] >= 2u) atomicAdd(&hist[ev[u]], 1u);
                } else if (hk) {
                    atomicAdd(&hist[ev[u]], 1u);
                }
            }
        }
        K = min(depth, __builtin_amdgcn_readfirstlane(wave_max(me)) + 1u);
        if (BALLOT01 && hist_on) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0u) hist[0] = h0;
            if (lane == 1u) hist[1] = h1;
        }
    }
    // Sky pixels: K = 1 with depth > 1 means every sample hit the sky at bounce 0 (e = 0 < depth), so
    // the replay is the identity (bounce 0 retires every position: lo = 0, and pold = pnew = i) and
    // position q < spp holds white x sky(y_q) = sky(y_q).  No map, no replay, no colour reads (config C:
    // the top third of the frame).
    const bool sky_only = MODE == kModeV2 && depth > 1u && K == 1u;
    // Map init: no position holds a terminated sample's value yet (survivors and never-written
    // positions read 0; positions [spp, P), the missing lanes of a partial last chunk, get their
    // fixed value in the final reduction).  Two u16 entries per u32 store.
    if (MODE == kModeV2 && !sky_only) {
        if (lm) {
            for (uint32_t qi = 2u * lane; qi < P; qi += 128u) *(uint32_t*)(lmap + qi) = 0xFFFFFFFFu;
        } else if (sc.wide & 2u) {
            for (uint32_t qi = lane; qi < P; qi += 64u) sc.set_map(qi, kNone);
        } else {
            for (uint32_t qi = 2u * lane; qi < P; qi += 128u) *(uint32_t*)(sc.base + 2u * qi) = 0xFFFFFFFFu;
        }
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
    bool replayed = sky_only;
    if (MODE == kModeV2 && K > 0u && K <= 64u && !sky_only) {
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
                // this lane's index k (lane k's count of e == k).  The masks are kept as 32-bit halves, B and Bk
                // all-ones or zero per lane (v_bfe_i32), each update one v_bitop3 / v_and_or per half (truth
                // table index S0 << 2 | S1 << 1 | S2): 11 VALU per plane, where the 64-bit form took ~22 (the
                // compiler built the lane masks with cndmasks).  Every plane is applied, without a branch (a
                // skipped plane cost loop-carried copies): a plane no lane sets leaves eq and gt unchanged in the
                // lanes that use them and clears eqk in the lanes k with that bit.  Round 5, same-box with the
                // reduction below: C fp32 +1.9 %, fp64 +2.4 %, E +1.3 % (profiles/r05/finish_ab.txt).
                uint32_t eql = (uint32_t)inm, eqh = (uint32_t)(inm >> 32), gtl = 0u, gth = 0u;
                uint32_t eqkl = eql, eqkh = eqh;
                for (uint32_t bb = nb; bb-- > 0u;) {
                    const uint32_t B = (uint32_t)__builtin_amdgcn_sbfe((int)ec, bb, 1u);     // this lane's bit
                    const unsigned long long P = __ballot(B != 0u) & inm;
                    const uint32_t Pl = (uint32_t)P, Ph = (uint32_t)(P >> 32);
                    const uint32_t Bk = (uint32_t)__builtin_amdgcn_sbfe((int)lane, bb, 1u);  // bit of k = lane
                    // gt |= eq & P & ~B (equal so far, 1 where this lane has 0: greater)
                    gtl = ((eql & ~B) & Pl) | gtl;
                    gth = ((eqh & ~B) & Ph) | gth;
                    // eq &= ~(P ^ B) (still equal), eqk &= ~(P ^ Bk): table 0x90
                    eql = __builtin_amdgcn_bitop3_b32(eql, Pl, B, 0x90);
                    eqh = __builtin_amdgcn_bitop3_b32(eqh, Ph, B, 0x90);
                    eqkl = __builtin_amdgcn_bitop3_b32(eqkl, Pl, Bk, 0x90);
                    eqkh = __builtin_amdgcn_bitop3_b32(eqkh, Ph, Bk, 0x90);
                }
                const unsigned long long eq = ((unsigned long long)eqh << 32) | eql;
                const unsigned long long gt = ((unsigned long long)gth << 32) | gtl;
                const unsigned long long eqk = ((unsigned long long)eqkh << 32) | eqkl;
                const uint32_t ek = ret ? e : 0u;
                // the earlier chunks' counts at this lane's bounce
                const uint32_t cg = (uint32_t)__shfl((int)cge, (int)ek), cq = (uint32_t)__shfl((int)ceq, (int)ek);
                const uint32_t nn = (uint32_t)__shfl((int)nn_l, (int)ek);
                // lane k < K: #{e == k} in this chunk (lanes k >= 2^nb or > K are never read)
                const uint32_t h = (uint32_t)__popcll(eqk);
                // lane k <= K: #{in && e >= k} = #{in} - #{e < k}
                cge += (uint32_t)__popcll(inm) - (wave_scan_dpp(h) - h);
                ceq += h;
                if (ret) {
                    // Sample i, terminated at bounce e, sat at pold = #{s' < i : e_s' >= e} during bounce e
                    // and moves to pnew = n_{e+1} + #{s' < i : e_s' == e}
                    const uint32_t pold = cg + lanes_below(gt | eq);
                    const uint32_t pnew = nn + cq + lanes_below(eq);
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
    }
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
                const uint32_t rd = cd + lanes_below(bd), rf = ce + lanes_below(be);
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
                const uint32_t rd = cd + lanes_below(bd), re = ne - 1u - (ce + lanes_below(be));
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
                    const uint32_t pold = cge + lanes_below(bge);
                    const uint32_t pnew = n_next + ceq + lanes_below(beq);
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
        auto vals = [&](uint32_t qq, T& vr, T& vg, T& vb) {
            if (MODE == kModeV3) {
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
            } else if (qq >= spp) {
                if (MODE == kModeV2) {
                    if (depth > 0u) { vr = s0.x; vg = s0.y; vb = s0.z; }
                    else if (white0) { vr = T(1.0); vg = T(1.0); vb = T(1.0); }
                }
            } else if (MODE == kModeV2 && sky_only) {
                const V3<T> sk = sky(sc.y(s, qq));
                vr = sk.x; vg = sk.y; vb = sk.z;
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
        };
        if (MODE == kModeV2 && !sky_only && !(sc.wide & 2u)) acc = reduce_live16<T>(sc, s, spp, P, lmap, lm, hist, stage, vals);
        else acc = reduce_positions<T>(P, hist, stage, vals);
    }
    write_pixel<T, MODE>(acc, item);
    return K;
}

}  // namespace rt
