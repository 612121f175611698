# A/B patch: finish_pixel's histogram pass counts the two commonest termination bounces (e = 0: the sky at
# bounce 0, 43 % of config C's samples; e = 1) with ballots into wave-uniform sums, and LDS atomics only for
# e >= 2: 64 lanes adding to the same LDS word serialise.
import sys
d = sys.argv[1]
p = f"{d}/rt_finish.hpp"; s = open(p).read()
old = """        uint32_t me = 0;
        for (uint32_t b = 0; b < spp; b += 512u) {"""
new = """        uint32_t me = 0, h0 = 0, h1 = 0;   // #{e == 0}, #{e == 1} (wave-uniform)
        for (uint32_t b = 0; b < spp; b += 512u) {"""
assert old in s; s = s.replace(old, new)
old = """                if (hist_on && b + 64u * u + lane < spp && ev[u] < depth && ev[u] < 64u) atomicAdd(&hist[ev[u]], 1u);"""
new = """                const bool hk = hist_on && b + 64u * u + lane < spp && ev[u] < depth && ev[u] < 64u;
                h0 += (uint32_t)__popcll(__ballot(hk && ev[u] == 0u));
                h1 += (uint32_t)__popcll(__ballot(hk && ev[u] == 1u));
                if (hk && ev[u] >= 2u) atomicAdd(&hist[ev[u]], 1u);"""
assert old in s; s = s.replace(old, new)
old = """        K = min(depth, __builtin_amdgcn_readfirstlane(wave_max(me)) + 1u);"""
new = """        K = min(depth, __builtin_amdgcn_readfirstlane(wave_max(me)) + 1u);
        if (hist_on) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0u) hist[0] = h0;
            if (lane == 1u) hist[1] = h1;
        }"""
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
