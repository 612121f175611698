# A/B patch: finish_pixel's whole-batch reduction (reduce_live16) loads a colour record only for map
# entries that have one (not for kWhite bounce-0 sky hits, 43 % of config C's samples, nor for positions
# without an entry): an exec-masked load instead of a clamped load for every lane.
import sys
d = sys.argv[1]
p = f"{d}/rt_finish.hpp"; s = open(p).read()
old = """        const uint32_t smp = min(m16 & 0x7FFFu, spp - 1u);   // a clamped (unused) record without an entry
        const C3<T> cm = sc.c(s, smp);"""
new = """        C3<T> cm = {T(0.0), T(0.0), T(0.0)};
        if (m16 < 0x8000u) cm = sc.c(s, m16);   // exec-masked: only positions holding a record"""
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
