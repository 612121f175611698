"""A/B patch (round 6): finish_pixel keeps the first pass's termination bounces in registers for the replay when the
pixel has at most 512 samples (config C's 512 spp: one pass block), instead of loading all of them again from the
wave's scratch (8 byte loads per lane and their wait)."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_finish.hpp", """        uint32_t me = 0, h0 = 0, h1 = 0;   // #{e == 0}, #{e == 1} (wave-uniform)
        for (uint32_t b = 0; b < spp; b += 512u) {
            uint32_t ev[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t i = b + 64u * u + lane;
                ev[u] = i < spp ? sc.e(s, i) : 0u;
            }""", """        uint32_t me = 0, h0 = 0, h1 = 0;   // #{e == 0}, #{e == 1} (wave-uniform)
        for (uint32_t b = 0; b < spp; b += 512u) {
            uint32_t ev[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t i = b + 64u * u + lane;
                ev[u] = i < spp ? sc.e(s, i) : 0u;
                ev1[u] = ev[u];
            }""")
sub("rt_finish.hpp", """    uint32_t K = 0;
    const bool known1 = MODE == kModeV2 && all_e0 && depth > 1u;""", """    uint32_t K = 0;
    uint32_t ev1[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};   // pass 1's bounces (the last block), for the replay
    const bool known1 = MODE == kModeV2 && all_e0 && depth > 1u;""")
sub("rt_finish.hpp", """            uint32_t ev[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t i = b + 64u * u + lane;
                ev[u] = i < spp ? sc.e(s, i) : 0xFFFFFFFFu;
            }""", """            uint32_t ev[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t i = b + 64u * u + lane;
                ev[u] = i < spp ? (spp <= 512u ? ev1[u] : sc.e(s, i)) : 0xFFFFFFFFu;
            }""")
