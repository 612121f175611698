"""A/B patch (round 6): fp64 camera coordinates x / W (Camera::get_ray, ray_tracing.rs:78-79) from the host's
r = RN(1/W) and two residual corrections instead of the compiler's division (div_scale x2, rcp, four FMAs, a
multiply, div_fmas, div_fixup): q1 = fma(fma(-x r, W, x), r, x r) is within an ulp of x / W, and Markstein's theorem
(a correctly rounded reciprocal, a faithful quotient) makes q2 = fma(fma(-q1, W, x), r, q1) the correctly rounded
quotient.  tools/div_dim_check.c checks 2.2e8 camera coordinates (BASELINE widths, edge and random W <
2^20, quotients next to midpoints) against x / W."""
import sys
d = sys.argv[1]
p = f"{d}/rt_common.hpp"
s = open(p).read()
old = """template <typename T> __device__ __forceinline__ T div_dim(T x, uint32_t W, double r) {
    if constexpr (sizeof(T) == 4) {
        if (r != 0.0) return (float)((double)x * r);
    }
    return x / (T)W;
}"""
new = """template <typename T> __device__ __forceinline__ T div_dim(T x, uint32_t W, double r) {
    if (r != 0.0) {
        if constexpr (sizeof(T) == 4) {
            return (float)((double)x * r);
        } else {
            // fp64: q1 = x r + r (x - W x r) is within an ulp of x / W, and with r correctly rounded one more
            // residual step rounds correctly (Markstein); 5 ops against the division's 10
            // (tools/div_dim_check.c: 2.2e8 camera coordinates, equal to x / W)
            const double w = (double)W, q0 = x * r;
            const double q1 = fma(fma(-q0, w, x), r, q0);
            return fma(fma(-q1, w, x), r, q1);
        }
    }
    return x / (T)W;
}"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
