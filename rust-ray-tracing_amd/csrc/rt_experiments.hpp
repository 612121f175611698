// rt_experiments.hpp — build kinds and the A/B knobs: the only product source that names an RT_EXP_
// macro.
//
// The product library (make) defines RT_PRODUCT and refuses every experiment macro below; the A/B
// builds (make exp / kstats) define RT_EXPERIMENT, and rt_version() says so, which
// rt_mi355x.load_library refuses unless RT_ALLOW_EXPERIMENT=1.  Timing experiments that add code (a
// stage run twice, DESIGN.md §5 "where the time goes") are not in the product sources at all: they are
// patches under tools/exp/, applied by `make exp` to a copy of csrc/.  tests/test_abi.py checks that
// this fence lists every RT_EXP_ macro the sources and those patches test.  Every experiment keeps the
// results bit-identical (timing or ordering changes only).
#pragma once

#if defined(RT_PRODUCT) && defined(RT_EXPERIMENT)
#error "RT_PRODUCT and RT_EXPERIMENT are exclusive"
#endif
#if defined(RT_PRODUCT) && (defined(RT_EXP_BLOCK_SAMPLES) || defined(RT_EXP_TMUL) || defined(RT_EXP_LMAP_CAP) ||      \
                            defined(RT_EXP_DUP_FINISH) || defined(RT_EXP_DUP_CAMRAY) || defined(RT_EXP_DUP_CAM) ||     \
                            defined(RT_EXP_DUP_SCATTER) || defined(RT_EXP_DUP_SWEEP) || defined(RT_EXP_DUP_CLBOX) ||   \
                            defined(RT_EXP_DUP_FILTER) || defined(RT_EXP_DUP_SUPBOX) || defined(RT_EXP_DUP_MEGABOX) || \
                            defined(RT_EXP_DUP_PLIST) || defined(RT_EXP_DUP_REPLAY) || defined(RT_EXP_DUP_REDUCE) ||   \
                            defined(RT_EXP_TIMELINE) || \
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

// Work distribution (rt_trace.hpp, guided_block): the samples a block may hold and the T multiplier.
#ifdef RT_EXP_BLOCK_SAMPLES
constexpr uint32_t kBlockSamples = RT_EXP_BLOCK_SAMPLES;
#else
// 32768 (round 6; was 8192): config E (2048 spp, 1350 pixels per wave) takes G = 16 instead of 4, E fp32 +0.4 %,
// fp64 +0.5 % same-box (profiles/r06/block_samples_ab.txt).  It changes G only where kBlockSamples / spp was the
// binding bound; C (whole frame 8, row shards 2), D (4) and B keep theirs: the share bound decides for them
constexpr uint32_t kBlockSamples = 32768;
#endif
#ifdef RT_EXP_TMUL
constexpr uint32_t kTMul = RT_EXP_TMUL;
#else
constexpr uint32_t kTMul = 8;
#endif
// finish_pixel's position map in LDS up to this many positions (fp64 live-path kernels, rt_finish.hpp).
#ifdef RT_EXP_LMAP_CAP
constexpr uint32_t kLMapCap = RT_EXP_LMAP_CAP;
#else
constexpr uint32_t kLMapCap = 512;
#endif

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

}  // namespace rt
