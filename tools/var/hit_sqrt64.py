# A/B patch: hit_update's sqrt(disc) in fp64 through sqrt_len (the library's sequence without the
# range scaling and the class fix-up, taken when every candidate lane's disc is in [2^-100, 2^100];
# otherwise the library sqrt).  fp32 is unchanged (sqrt_len(float) is sqrtf).
import sys
d = sys.argv[1]
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
old = """    const T sd = sqrt(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270"""
new = """    const T sd = sqrt_len(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270"""
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
