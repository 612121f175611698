"""A/B patch (round 6): fp32 sqrt_len (unit(): camera rays, the scatter's normal length, the hit test's sqrt(disc))
through sqrt_nd -- v_sqrt_f32 and the compiler's own +-1 ulp residual correction, without its scaling of
arguments below 2^-96 and its special-value select -- when no lane has a tiny positive argument (a wave ballot;
otherwise the library sqrtf).  The same correctly rounded value (sqrt_nd's contract, rt_device.hpp).  The library
sequence is ~16 VALU ops, most of them single-issue (compares, selects, constant operands)."""
import sys
d = sys.argv[1]
p = f"{d}/rt_device.hpp"
s = open(p).read()
old = "__device__ __forceinline__ float sqrt_len(float x) { return sqrtf(x); }"
new = """__device__ __forceinline__ float sqrt_len(float x) {
    if (__builtin_expect(__ballot(x > 0.0f && x < 0x1.0p-96f) == 0ull, 1)) return sqrt_nd(x);
    return sqrtf(x);
}"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
