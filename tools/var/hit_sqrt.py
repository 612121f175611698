# A/B patch: hit_update's sqrt(disc) through sqrt_nd when no candidate lane has a tiny positive
# discriminant (< 2^-96; else the library sqrt), and 1 / |d|^2 through the shared-reciprocal division
# sequence when every lane's a is in [2^-20, 2^20].
import sys
d = sys.argv[1]
p = f"{d}/rt_device.hpp"; s = open(p).read()
old = "__device__ __forceinline__ double sqrt_nd(double x) { return sqrt(x); }"
new = old + '''
// sqrt of a candidate's discriminant (>= +0, maybe +inf): sqrt_nd unless some lane's is tiny and positive
__device__ __forceinline__ float sqrt_cand(float x) {
    if (__builtin_expect(__ballot(x < 0x1.0p-96f && x != 0.0f) == 0ull, 1)) return sqrt_nd(x);
    return sqrtf(x);
}
__device__ __forceinline__ double sqrt_cand(double x) { return sqrt(x); }
// 1 / a, correctly rounded: the compiler's division sequence without div_scale / div_fmas / div_fixup
// (no-ops when every lane's a is in [2^-20, 2^20]); otherwise the division
__device__ __forceinline__ float recip(float a) {
    if (__builtin_expect(__ballot(!(a >= 0x1.0p-20f && a <= 0x1.0p20f)) == 0ull, 1)) {
        const float r0 = __builtin_amdgcn_rcpf(a);
        const float r1 = __builtin_fmaf(__builtin_fmaf(-a, r0, 1.0f), r0, r0);
        const float f3 = __builtin_fmaf(__builtin_fmaf(-a, r1, 1.0f), r1, r1);
        return __builtin_fmaf(__builtin_fmaf(-a, f3, 1.0f), r1, f3);
    }
    return 1.0f / a;
}
__device__ __forceinline__ double recip(double a) { return 1.0 / a; }'''
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
old = '''    const T sd = sqrt(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270'''
new = '''    const T sd = sqrt_cand(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270'''
assert old in s; s = s.replace(old, new)
old = "    const T inv_a = SCALAR ? T(0) : T(1.0) / a;      // objects.rs:254 (loop-invariant)"
new = "    const T inv_a = SCALAR ? T(0) : recip(a);        // objects.rs:254 (loop-invariant)"
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
p = f"{d}/rt_camera.hpp"; s = open(p).read()
old = "    const T inv_a = SCALAR ? T(0) : T(1.0) / a;      // objects.rs:254"
assert s.count(old) == 2
s = s.replace(old, "    const T inv_a = SCALAR ? T(0) : recip(a);        // objects.rs:254"); open(p, "w").write(s)
