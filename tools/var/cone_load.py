# A/B patch: the cone test's record read as one 16-byte load.  `wc.w > -inf && (...)` made the compiler load
# w first, wait for it and branch, then load x, y, z: two dependent global round trips per member test.
import sys
d = sys.argv[1]
p = f"{d}/rt_camera.hpp"; s = open(p).read()
old = "        return wc.w > -INFINITY && (all || !(f > wc.w));   // NaN f passes"
new = "        return (wc.w > -INFINITY) & (all | !(f > wc.w));   // NaN f passes; bitwise: one load, no branch"
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
