// rt_trace.hpp — the persistent path-regeneration kernel trace_paths: work distribution (guided
// blocks through a workgroup pool), camera batches and their LDS queue, the per-iteration
// next-ray / sweep / terminate loop (TileRenderTask::render_vectorized2, renderer.rs:141-176).
#pragma once
#include "rt_sweep.hpp"
#include "rt_camera.hpp"
#include "rt_finish.hpp"

namespace rt {

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
// The blocks past the first gridDim.x (one per workgroup, taken without an atomic) are dealt round-robin
// to kStreams claim streams, stream s holding blocks gridDim.x + s + kStreams c (c = 0, 1, ...) behind its
// own counter, kCtrStride words apart (256 B: separate lines and memory channels).  A workgroup claims
// from stream blockIdx.x % kStreams (the XCD the hardware dispatches it to), and from the others once its
// own runs dry, so the counters of a launch are not one word every CU hammers: the sky rows' cheap
// pixels otherwise claimed faster than one word serves (~88 claims/us).
constexpr uint32_t kStreams = 8;
constexpr uint32_t kCtrStride = 64;

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
    __shared__ unsigned long long wcount[4][4];   // segments, lane slots, bounce iterations, direct sky samples
    // 8-byte aligned: finish_pixel keeps its 12 running sums (T, fp64 too) in this array
    __shared__ __attribute__((aligned(16))) uint32_t s_hist[4][64];
    __shared__ __attribute__((aligned(16))) T s_stage[4][3][64];   // finish_pixel: 64 positions' values per wave
    __shared__ IssueState s_is[4];
    __shared__ unsigned long long s_pool;   // the workgroup's pool of claimed items: next << 32 | end
    __shared__ uint32_t s_dry;              // claim streams this workgroup found exhausted (bit s)
    __shared__ uint32_t q_sid[QW][QN];   // sid | slot << 29 (the pixel: s_slotpix[slot])
    __shared__ uint32_t s_slotpix[4][kSlots];   // the pixel of each open slot
    // ... and its work item (read at finish_pixel, not held in a VGPR)
    __shared__ uint32_t s_item[4][kSlots];
    __shared__ int q_hit[QW][QN];
    __shared__ T q_t[QW][QN], q_d[QW][3][QN];
    // camera candidate list of each open pixel slot (pixel_list): [0] = count (0xFFFF: none, sweep per batch)
    __shared__ alignas(16) uint16_t s_clist[QW][CAMQ ? kSlots : 1][kCList];   // 16 B lists: one LDS read (fp64)
    // fp32 at 6 waves per SIMD (80 VGPRs): each lane's ray origin and direction are parked in LDS
    // across the sphere sweeps and the camera batches and re-read right before the scatter, instead
    // of being held in VGPRs (the allocator otherwise spills them to scratch memory around the sweep).
    constexpr bool kPark = (sizeof(T) == 4 && W >= 6) || kF64Park;
    // the mega-level kernels park the path colour as well (their four-level sweep holds more state), and
    // so does fp32 at W6 since issue() finishes sky pixels (it pushed the colour into scratch spills
    // around the scatter; parked: C +0.9 % same-box, LDS 26.8 of 27.3 KB per workgroup)
    constexpr bool kParkC = kPark && (MEGA || (sizeof(T) == 4 && W == 6));
    __shared__ T s_park[kPark ? 4 : 1][kParkC ? 9 : 6][64];
    // finish_pixel's position map (P <= kLMapCap) in LDS: the fp64 live-path kernels without the mega level
    // (fp64 C +1.1 % same-box).  fp32 lost 7 % with it (the extra finish_pixel code pushed 5 more spills
    // into the hot loop at 80 VGPRs); the mega kernels' LDS is full at 6 waves per SIMD.
    constexpr bool kLMap = MODE == kModeV2 && !MEGA && kLMapCap > 0u && sizeof(T) == 8 && !kF64Park;
    __shared__ __attribute__((aligned(16))) uint16_t s_lmap[kLMap ? 4 : 1][kLMap ? kLMapCap : 2];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (lane == 0) { wcount[wave][0] = 0; wcount[wave][1] = 0; wcount[wave][2] = 0; wcount[wave][3] = 0; }
    if (lane < kNWork) g_work[wave][lane] = 0ull;
#ifdef RT_KSTATS
    if (lane < 8) g_kst[wave][lane] = 0;
#endif
    if (lane == 0) s_is[wave] = IssueState{0u, 0u, cold_args<T>()->spp, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    // The workgroup's first block is block blockIdx.x, taken without an atomic (the counter's claims
    // start at gridDim.x): the launch's opening burst of one global atomic per workgroup is gone.
    {
        const auto& q = *cold_args<T>();
        uint32_t b0 = 0, b1 = 0;
        const bool got = guided_block(q.n_items, max(1u, kTMul * gridDim.x), q.blk_g, blockIdx.x, b0, b1);
        if (threadIdx.x == 0) {
            s_pool = got ? ((unsigned long long)b0 << 32) | b1 : 0ull;   // {next, end}; {0, 0}: empty
            s_dry = 0u;
        }
    }
    __syncthreads();
    V3<T> o = mk(T(0), T(0), T(0)), d = o, c = o;
    // the lane's sample and pixel slot in one VGPR, sid | slot << 29 (as in the camera queue: spp <= 2^20,
    // kSlots <= 8); the slot's pixel is read from s_slotpix where the scatter needs it
    uint32_t ss = 0, k = 0;
    // The mega kernels keep ss in LDS, in this lane's word of the finish stage (s_stage, free outside
    // finish_pixel; terminate saves and restores it around the call): at 80 VGPRs the allocator
    // otherwise spills ss to scratch at every queue pop (config E's last hot-loop spill store).
    constexpr bool kParkSS = MEGA;
    uint32_t* const ssp = (uint32_t*)&s_stage[wave][0][0] + lane;
    auto ss_get = [&]() -> uint32_t {
        if constexpr (kParkSS) { asm volatile("" ::: "memory"); return *ssp; }
        else return ss;
    };
    auto ss_set = [&](uint32_t v) {
        if constexpr (kParkSS) *ssp = v;
        else ss = v;
    };
    if constexpr (kParkSS) *ssp = 0u;
    // lane s < kSlots: slot s's samples not yet terminated, | kSlotNZ once one of them terminated at a
    // bounce e > 0 (so finish_pixel knows a sky pixel without reading its records).  In a VGPR, not LDS:
    // the LDS round trip sat on terminate's path every iteration (config E -4.6 %, C +-0 against this)
    constexpr uint32_t kSlotNZ = 0x80000000u;
    uint32_t slot_left = 0;
    auto sid_of = [](uint32_t v) -> uint32_t { return v & 0x1FFFFFFFu; };
    auto slot_of = [](uint32_t v) -> uint32_t { return v >> 29; };
    bool live = false;
    bool scat = false;                 // hit at bounce k last iteration, still below depth: scatter now
    int hit_i = -1;
    T hit_t = T(0);
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
    // Camera batches on the live path: pixels whose camera candidate list is empty finish at claim time
    constexpr bool kDirectSky = CAMQ && MODE == kModeV2;
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
        uint32_t opened = 0, listed = 0;
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
                        uint32_t b0 = 0, b1 = 0;
                        bool claimed = false;
                        for (uint32_t r = 0; it == 0xFFFFFFFFu && r < kStreams && !claimed; ++r) {
                            const uint32_t s = (blockIdx.x + r) % kStreams;
                            if ((__hip_atomic_load(&s_dry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >> s) & 1u) continue;
                            const uint32_t j = gridDim.x + s + kStreams * atomicAdd(q.counter + kCtrStride * s, 1u);
                            claimed = guided_block(q.n_items, max(1u, kTMul * gridDim.x), q.blk_g, j, b0, b1);
                            if (!claimed) atomicOr(&s_dry, 1u << s);   // blocks of a stream only grow in j
                        }
                        if (claimed) {
                            it = b0;
                            if (b1 > b0 + 1u && atomicCAS(&s_pool, pv, ((unsigned long long)(b0 + 1u) << 32) | b1) != pv) {
                                nb = b0 + 1u;   // the pool was refilled meanwhile: keep the rest
                                ne = b1;
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
                if constexpr (kDirectSky) {
                    if (cold_args<T>()->depth > 1u) {
                        // the pixel's camera candidate list now, not at its slot's first batch: an empty
                        // one means no primary ray of the pixel can hit a sphere, so every sample escapes
                        // at bounce 0 and the pixel is finished here without tracing (finish_sky_direct);
                        // its slot stays free
                        const uint32_t nl = pixel_list<T, MEGA>(cur_col, cur_row, s_clist[wave][s]);
                        if (nl == 0u) {
                            const uint32_t ss_keep = kParkSS ? *ssp : 0u;   // the stage is overwritten
                            finish_sky_direct<T>(item, cur_col, cur_row, cur_pix, s_hist[wave], s_stage[wave]);
                            if constexpr (kParkSS) {
                                __builtin_amdgcn_wave_barrier();
                                *ssp = ss_keep;
                            }
                            // its spp primary segments and one bounce iteration, as traced; no lane held them
                            if (lane == 0) { wcount[wave][0] += spp; wcount[wave][3] += spp; wcount[wave][2] += 1u; }
                            continue;
                        }
                        listed |= 1u << s;
                    }
                }
                if (lane == 0) { s_slotpix[wave][s] = cur_pix; s_item[wave][s] = item; }
                if (lane == s) slot_left = spp;
                busy |= 1u << s;
                opened |= 1u << s;
                cur = s;
                cur_next = 0;
            }
            const bool isw = (want >> lane) & 1ull;
            const uint32_t take = min((uint32_t)__popcll(want), spp - cur_next);
            const uint32_t r = lanes_below(want);
            const bool mine = isw && r < take;
            if (mine) { got = true; i_sid = cur_next + r; i_slot = cur; i_pix = cur_pix; i_row = cur_row; i_col = cur_col; }
            want &= ~__ballot(mine);
            cur_next += take;
        }
        if (lane == 0) {
            s_is[wave].busy = busy; s_is[wave].cur = cur; s_is[wave].cur_next = cur_next; s_is[wave].cur_pix = cur_pix;
            s_is[wave].cur_row = cur_row; s_is[wave].cur_col = cur_col; s_is[wave].drained = drained ? 1u : 0u;
            s_is[wave].blk_next = blk_next; s_is[wave].blk_end = blk_end;
            if (CAMQ) s_is[wave].need |= opened & ~listed;
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
        const unsigned long long nzl = MODE == kModeV2 ? __ballot(term && e != 0u) : 0ull;
        bool synced = false;
        while (tm != 0ull) {
            const uint32_t s = __builtin_amdgcn_readlane(t_slot, __builtin_ctzll(tm));
            const unsigned long long m = __ballot(term && t_slot == s);
            tm &= ~m;
            if (lane == s) slot_left = (slot_left - (uint32_t)__popcll(m)) | ((m & nzl) != 0ull ? kSlotNZ : 0u);
            const uint32_t left = __builtin_amdgcn_readlane(slot_left, s);
            // pixel complete: once per spp samples -- marked unlikely, so the register allocator
            // places any spill code here rather than in the sphere sweeps
            if (__builtin_expect((left & ~kSlotNZ) == 0u, 0)) {
                const uint32_t ss_keep = kParkSS ? *ssp : 0u;   // finish_pixel overwrites the stage
                if (!synced) { wave_mem_sync(); synced = true; }
                KSTAT(6);
                const uint32_t K = finish_pixel<T, MODE, !MEGA>(
                    wave_scratch<T>(wave), s, __builtin_amdgcn_readfirstlane(s_item[wave][s]), s_hist[wave], s_stage[wave],
                    kLMap ? s_lmap[wave] : nullptr, (left & kSlotNZ) == 0u);
                if constexpr (kParkSS) {
                    __builtin_amdgcn_wave_barrier();
                    *ssp = ss_keep;
                }
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
        if (v) {   // Camera::get_ray (ray_tracing.rs:77-89) with origin == centre
            const U4 r = [&] {
                const auto& q0 = *cold_args<T>();
                return rng<T>(bsid, bpix, 0u, 0u, q0.k0, q0.k1);
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
                    (void)pixel_list<T, MEGA>(pxi - row * iw, row, s_clist[wave][sl]);
                }
            }
            bool listed = true;
            for (uint32_t m = smask; m != 0u; m &= m - 1u)
                if (__builtin_amdgcn_readfirstlane(s_clist[wave][__builtin_ctz(m)][0]) == 0xFFFFu) listed = false;
            if (listed) bi = camera_listed<T, ROOT2, SC>(v, bd, bt, s_clist[wave], smask);
            else bi = camera_sweep<T, ROOT2, SC, MEGA>(v, bd, bt);   // whole wave: lanes are spheres in the cull
        }
        if (lane == 0) { wcount[wave][0] += (uint32_t)__popcll(vm); wcount[wave][1] += 64u; }
        const uint32_t depth = cold_args<T>()->depth;
        const bool skyhit = v && bi < 0;
        const bool term = v && (skyhit || depth == 1u);
        const bool push = v && !term;
        const unsigned long long pm = __ballot(push);
        const uint32_t qhead = __builtin_amdgcn_readfirstlane(s_is[wave].qhead);
        const uint32_t qcount = __builtin_amdgcn_readfirstlane(s_is[wave].qcount);
        if (push) {
            const uint32_t e = (qhead + qcount + lanes_below(pm)) % QN;
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
        uint32_t frow = 0, fcol = 0, npix = 0;
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
            const uint32_t r = lanes_below(freem);
            if (!live && r < take) {
                const uint32_t e = (qhead + r) % QN;
                ss_set(q_sid[wave][e]);
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
            uint32_t nsid = 0, nslot = 0;
            fresh = issue(__ballot(!live), nsid, nslot, npix, frow, fcol);
            if (fresh) ss_set(nsid | (nslot << 29));
        }
        // ---- next rays: camera rays for fresh lanes, scattered rays for last iteration's hits ----
        if constexpr (kPark) unpark(o, d);
        if constexpr (kParkC) c = unpark_c();
        if (fresh || scat) {
            const uint32_t ssv = ss_get();
            const uint32_t pix = (!CAMQ && fresh) ? npix : s_slotpix[wave][slot_of(ssv)];
            next_ray<T, SC>(CAMQ ? false : fresh, fcol, frow, pix, sid_of(ssv), k, hit_i, hit_t, o, d, c);
        }
        if constexpr (kPark) park(o, d);
        if constexpr (kParkC) park_c(c);
        if (fresh) {
            k = 0;
            live = true;
            if (MODE == kModeV2) {   // primary y (quirk Q2)
                const uint32_t ssv = ss_get();
                wave_scratch<T>(wave).y(slot_of(ssv), sid_of(ssv)) = d.y;
            }
        } else if (scat) {
            k += 1u;
        }
        if (__ballot(live) == 0ull) break;   // drained, and every slot finished
        // ---- one sphere sweep for every live ray ----
        const uint32_t depth = cold_args<T>()->depth;
        const bool act = live && k < depth;
        hit_i = -1;
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
        {
            const uint32_t ssv = ss_get();
            terminate(term, skyhit, skyhit ? k : depth, slot_of(ssv), sid_of(ssv), c, d);
        }
        live = live && !term;
    }
    if (lane == 0) {
        const auto& q = *cold_args<T>();
        const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + wave;
        unsigned long long* cc = &q.segs[(gw & (kSegShards - 1)) * kSegStride];
        atomicAdd(cc + 0, wcount[wave][0]);
        atomicAdd(cc + 1, wcount[wave][1]);
        atomicAdd(cc + 2, wcount[wave][2]);
        if (wcount[wave][3]) atomicAdd(cc + kDirectSkySlot, wcount[wave][3]);
        for (uint32_t i = 0; i < kNWork; ++i) atomicAdd(cc + kWorkSlot + i, g_work[wave][i]);
#ifdef RT_KSTATS
        for (int i = 0; i < 8; ++i) atomicAdd(cc + 3 + i, g_kst[wave][i]);
#endif
    }
}

}  // namespace rt
