# A/B patch: cheaper correctly rounded fp32 sqrt where the argument is provably zero, >= 2^-96, +inf or NaN
# (unit_vec, the dielectric's sin, refract), and v / len for a vector and its length through one shared
# reciprocal when every lane's operands are in range (else the full division).  argv[2]: "sqrt" = only the
# sqrt part.
import sys
d = sys.argv[1]; mode = sys.argv[2] if len(sys.argv) > 2 else "all"
p = f"{d}/rt_device.hpp"; s = open(p).read()
old = "template <typename T> __device__ __forceinline__ V3<T> dvs(V3<T> a, T s) { return mk(a.x / s, a.y / s, a.z / s); }"
new = '''template <typename T> __device__ __forceinline__ V3<T> dvs(V3<T> a, T s) { return mk(a.x / s, a.y / s, a.z / s); }
__DVS_F32__
// sqrt, correctly rounded, of an argument known to be +-0, >= 2^-96, +inf, negative or NaN (never a tiny
// positive one): v_sqrt_f32 (within 1 ulp) and the compiler's own correction by the residuals of the two
// neighbours, without its scaling for arguments below 2^-96 and its special-value select (both no-ops
// here: 0, +inf and NaN come through the correction unchanged).  fp64: the library sqrt.
__device__ __forceinline__ float sqrt_nd(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __int_as_float(__float_as_int(s) - 1), sup = __int_as_float(__float_as_int(s) + 1);
    float r = __builtin_fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
    r = __builtin_fmaf(-sup, s, x) > 0.0f ? sup : r;
    return r;
}
__device__ __forceinline__ double sqrt_nd(double x) { return sqrt(x); }'''
dvs32 = '''// a / |a| for fp32 (unit(), next_ray's normal): the compiler's correctly rounded division is
// div_scale x2, rcp, 6 FMAs, div_fmas, div_fixup per component; when v_div_scale would scale nothing and
// div_fixup has no special case to fix (every lane: 2^-20 <= len <= 2^20 and every |component| >= 2^-100,
// which bounds |a_i / len| by ~1 since |a_i| <= len), the same sequence without them gives the same bits,
// with the denominator's refined reciprocal shared by the three components.  Otherwise the full division.
template <> __device__ __forceinline__ V3<float> dvs(V3<float> a, float s) {
    const float mn = fminf(fminf(fabsf(a.x), fabsf(a.y)), fabsf(a.z));
    const bool ok = s >= 0x1.0p-20f && s <= 0x1.0p20f && mn >= 0x1.0p-100f;
    if (__builtin_expect(__ballot(!ok) == 0ull, 1)) {
        const float r0 = __builtin_amdgcn_rcpf(s);
        const float r1 = __builtin_fmaf(__builtin_fmaf(-s, r0, 1.0f), r0, r0);
        auto q = [&](float x) {
            const float m = x * r1;
            const float f3 = __builtin_fmaf(__builtin_fmaf(-s, m, x), r1, m);
            return __builtin_fmaf(__builtin_fmaf(-s, f3, x), r1, f3);
        };
        return mk(q(a.x), q(a.y), q(a.z));
    }
    return mk(a.x / s, a.y / s, a.z / s);
}'''
new = new.replace("__DVS_F32__", dvs32 if mode == "all" else "")
assert old in s; s = s.replace(old, new)
s = s.replace("    V3<T> rpar = mul(n, -(sqrt(fabs(T(1.0) - len2(rperp)))));", "    V3<T> rpar = mul(n, -(sqrt_nd(fabs(T(1.0) - len2(rperp)))));   // |1 - x| is 0 or >= 2^-24")
s = s.replace("    const T r = sqrt(T(1.0) - z * z);", "    const T r = sqrt_nd(T(1.0) - z * z);   // z = 1 - 2 u1: 1 - z^2 is 0 or >= 2^-24")
# sqrt_nd is declared after refract/unit_vec users? move check
assert s.index("float sqrt_nd") < s.index("V3<T> rpar")
open(p, "w").write(s)
p = f"{d}/rt_camera.hpp"; s = open(p).read()
old = "        const T st = sqrt(T(1.0) - ct * ct);"
new = "        const T st = sqrt_nd(T(1.0) - ct * ct);   // ct <= 1: 0, >= 2^-24 or negative"
assert old in s; s = s.replace(old, new)
if mode == "all":
    old = "    const V3<T> u = mk(vec.x / len, vec.y / len, vec.z / len);"
    new = "    const V3<T> u = dvs(vec, len);"
    assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
