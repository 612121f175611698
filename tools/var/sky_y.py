# A/B patch: finish_sky_direct forms only the y component of the primary direction (unit(v).y = v.y / |v|, the
# same correctly rounded quotient the full unit() gives, so the same bits) instead of all three.
import sys
d = sys.argv[1]
p = f"{d}/rt_finish.hpp"; s = open(p).read()
old = "        const V3<T> sk = sky(unit(sub(pc, mk(qc.center[0], qc.center[1], qc.center[2]))).y);"
new = """        const V3<T> dv = sub(pc, mk(qc.center[0], qc.center[1], qc.center[2]));
        const V3<T> sk = sky(dv.y / sqrt_len(len2(dv)));   // unit(dv).y: the same correctly rounded quotient"""
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
