"""A/B patch (round 6): the largest claim block raised from 16 to 32 pixels (kMaxBlock), so RT_BLOCK_G=32 can be
measured; the host's default choice of G is unchanged."""
import sys
d = sys.argv[1]
p = f"{d}/rt_trace.hpp"
s = open(p).read()
old = "constexpr uint32_t kMaxBlock = 16;"
assert old in s
s = s.replace(old, "constexpr uint32_t kMaxBlock = 32;")
open(p, "w").write(s)
