"""A/B patch (round 6): launches with at least 2^17 samples per wave (config C's whole frame: 337 pixels x 512 spp per
wave; D's shard: 169 x 1024) take the largest claim block (16, within kBlockSamples) instead of the share bound's 8
or 4.  Smaller launches (row shards of C: 86 400 samples per wave at N = 2) keep the share bound, where G = 16 lost
(profiles/r06/block_samples_ab.txt)."""
import sys
d = sys.argv[1]
p = f"{d}/rt_kernel.hip"
s = open(p).read()
old = """        uint32_t G = 1;
        while (2u * G <= g) G *= 2u;
"""
new = """        uint32_t G = 1;
        while (2u * G <= g) G *= 2u;
        if (per_wave * spp >= (1ull << 17)) G = (uint32_t)std::min<uint64_t>((uint64_t)kMaxBlock, kBlockSamples / spp);
"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
