# A/B patch: the fp64 general sweep's exact test of a taken group requests the group's two 64-byte exact halves
# (4 spheres x {cx, cy, cz, r^2} in double) together, then waits once, instead of the loads the compiler sinks
# into each passing sphere's branch (one dependent scalar round trip per passing sphere, the fp64 sweep's
# waits).  The scene indices are requested first, so their load is in flight too.
import sys
d = sys.argv[1]
p = f"{d}/rt_common.hpp"; s = open(p).read()
old = "typedef float f2 __attribute__((ext_vector_type(2)));"
new = old + '''
// Two consecutive 64-byte groups into SGPRs with one wait (s_load_dwordx16 x2, then lgkmcnt(0)): both
// requests are in flight together.  The asm waits for its own loads, so the compiler's counters stay exact.
typedef int v16i __attribute__((ext_vector_type(16)));
template <typename T>
__device__ __forceinline__ void load_group_pair(const __attribute__((address_space(4))) T* f, uint32_t g, SphGroup<T>& c0,
                                                SphGroup<T>& c1) {
    v16i a, b;
    const __attribute__((address_space(4))) char* p = (const __attribute__((address_space(4))) char*)f + 64u * g;
    asm volatile("s_load_dwordx16 %0, %2, 0x0\\n\\ts_load_dwordx16 %1, %2, 0x40\\n\\ts_waitcnt lgkmcnt(0)"
                 : "=s"(a), "=s"(b) : "s"(p) : "memory");
    __builtin_memcpy(&c0, &a, 64);
    __builtin_memcpy(&c1, &b, 64);
}'''
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
old = '''            } else {
                const SphGroup<T> c0 = load_group(fe, 2 * g), c1 = load_group(fe, 2 * g + 1);
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (!((pairs >> j) & 1u)) continue;'''
new = '''            } else {
                const Q4 si = sidx(g);
                SphGroup<T> c0, c1;
                load_group_pair(fe, 2 * g, c0, c1);
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (!((pairs >> j) & 1u)) continue;'''
assert old in s; s = s.replace(old, new)
old = '''                const Q4 si = sidx(g);
                const uint32_t sv[4] = {si.x, si.y, si.z, si.w};'''
new = '''                const uint32_t sv[4] = {si.x, si.y, si.z, si.w};'''
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
