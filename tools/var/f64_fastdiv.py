# A/B patch: fp64 unit vectors (unit(), next_ray's normal) through the compiler's own f64 division and sqrt
# sequences without their range scaling and special-value fixups when every lane is in range: one shared
# refined reciprocal for the three components (rcp + 4 FMAs, then 3 ops per component, as div_scale /
# div_fmas / div_fixup compute them when nothing is scaled or special), and the sqrt's rsq refinement
# without the ldexp scaling and the zero / inf select.  Bit-identical by construction; the fp32 forms
# are rt_device.hpp's dvs<float> and sqrt_nd(float).
import sys
d = sys.argv[1]
p = f"{d}/rt_device.hpp"; s = open(p).read()
old = "__device__ __forceinline__ double sqrt_nd(double x) { return sqrt(x); }"
new = '''__device__ __forceinline__ double sqrt_nd(double x) { return sqrt(x); }
// fp64 a / s, s > 0, for three components: the compiler's f64 division (div_scale x2, rcp, two Newton steps,
// the residual FMA, div_fmas, div_fixup) where div_scale scales nothing and div_fixup has nothing to fix
// (every lane: 2^-20 <= s <= 2^20 and every |a_i| >= 2^-100): the same operations, the reciprocal shared.
template <> __device__ __forceinline__ V3<double> dvs(V3<double> a, double s) {
    const double mn = fmin(fmin(fabs(a.x), fabs(a.y)), fabs(a.z));
    const bool ok = s >= 0x1.0p-20 && s <= 0x1.0p20 && mn >= 0x1.0p-100;
    if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
        double r = __builtin_amdgcn_rcp(s);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
        r = __builtin_fma(r, __builtin_fma(-s, r, 1.0), r);
        auto q = [&](double x) {
            const double m = x * r;
            return __builtin_fma(__builtin_fma(-s, m, x), r, m);
        };
        return mk(q(a.x), q(a.y), q(a.z));
    }
    return mk(a.x / s, a.y / s, a.z / s);
}
// sqrt(x), x = |v|^2 of a direction: the compiler's f64 sqrt (rsq, then Goldschmidt/Newton refinement) without
// its ldexp scaling for x < 2^-767 and its select for zero / inf, when every lane has 2^-100 <= x <= 2^100.
__device__ __forceinline__ double sqrt_len(double x) {
    if (__builtin_expect(__ballot(!(x >= 0x1.0p-100 && x <= 0x1.0p100)) == 0ull, 1)) {
        const double g0 = __builtin_amdgcn_rsq(x);
        double sq = x * g0, h = g0 * 0.5;
        const double r = __builtin_fma(-h, sq, 0.5);
        sq = __builtin_fma(sq, r, sq);
        const double d0 = __builtin_fma(-sq, sq, x);
        h = __builtin_fma(h, r, h);
        sq = __builtin_fma(d0, h, sq);
        const double d1 = __builtin_fma(-sq, sq, x);
        return __builtin_fma(d1, h, sq);
    }
    return sqrt(x);
}
__device__ __forceinline__ float sqrt_len(float x) { return sqrtf(x); }'''
assert old in s; s = s.replace(old, new)
old = "template <typename T> __device__ __forceinline__ V3<T> unit(V3<T> a) { return dvs(a, sqrt(len2(a))); }"
new = "template <typename T> __device__ __forceinline__ V3<T> unit(V3<T> a) { return dvs(a, sqrt_len(len2(a))); }"
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
p = f"{d}/rt_camera.hpp"; s = open(p).read()
old = "    const T len = (SCALAR && !cam) ? rad : sqrt(l2);"
new = "    const T len = (SCALAR && !cam) ? rad : sqrt_len(l2);"
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
