# A/B patch: fp32 general sweep (scene-frame filter groups, not MEGA): a walked cluster's exact-test records
# (xrec: the group's r^2 and scene indices, one s_load_dwordx8) are requested with the next filter group's
# prefetch, before the filter of this group runs, instead of after its ballot.  A taken group then finds
# them landed; an untaken group wastes one K$ hit.  +8 SGPRs in the walk.
import sys
d = sys.argv[1]
p = f"{d}/rt_common.hpp"; s = open(p).read()
old = "template <typename T, typename F>\n__device__ __forceinline__ void sphere_loop(cptr<T> f, uint32_t ng, F&& group) {"
new = '''// sphere_loop over exactly 4 filter groups (a walked cluster) with each group's 32-byte exact record
// requested together with the next group's prefetch (before this group's filter runs).
struct XRec { uint32_t v[8]; };
__device__ __forceinline__ XRec load_xrec(cptr<uint32_t> x, uint32_t g) {
    XRec r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[j] = x[8u * g + (uint32_t)j];
    return r;
}
template <typename F>
__device__ __forceinline__ void sphere_loop4x(cptr<float> f, cptr<uint32_t> x, F&& group) {
    SphGroup<float> A = load_group(f, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t g = 0; g < 4u; g += 2) {
        XRec X = load_xrec(x, g);
        const SphGroup<float> B = load_group(f, g + 1);
        __builtin_amdgcn_sched_barrier(0);
        group(A, X, g);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        X = load_xrec(x, g + 1);
        if (g + 2 < 4u) A = load_group(f, g + 2);
        __builtin_amdgcn_sched_barrier(0);
        group(B, X, g + 1);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
    }
}

''' + old
assert old in s; s = s.replace(old, new); open(p, "w").write(s)

p = f"{d}/rt_sweep.hpp"; s = open(p).read()
# exact4f taking its record from the caller
old = '''        auto exact4f = [&](const SphGroup<float>& cur, uint32_t g, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                const auto& qx = *cold_args<T>();
                cptr<uint32_t> xr = (cptr<uint32_t>)__builtin_assume_aligned(qx.xrec, 32);
                uint32_t rec[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) rec[j] = xr[8u * g + (uint32_t)j];'''
new = '''        auto exact4f = [&](const SphGroup<float>& cur, const XRec& xrc, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                const uint32_t* rec = xrc.v;'''
assert old in s; s = s.replace(old, new)
old = '''                sphere_loop(fg + 16u * g0, 4u, [&](const SphGroup<float>& cur, uint32_t g) {
                    uint32_t s0, s1;'''
new = '''                auto grp = [&](const SphGroup<float>& cur, const XRec& xrc, uint32_t g) {
                    uint32_t s0, s1;'''
assert old in s; s = s.replace(old, new)
old = '''                        if constexpr (sizeof(T) == 4 && !MEGA && !CAMT) exact4f(cur, g0 + g, pairs);
                        else
                            exact4(g0 + g, pairs);
                    }
                });'''
new = '''                        if constexpr (sizeof(T) == 4 && !MEGA && !CAMT) exact4f(cur, xrc, pairs);
                        else
                            exact4(g0 + g, pairs);
                    }
                };
                if constexpr (sizeof(T) == 4 && !MEGA && !CAMT) {
                    const auto& qx = *cold_args<T>();
                    cptr<uint32_t> xr = (cptr<uint32_t>)__builtin_assume_aligned(qx.xrec, 32);
                    sphere_loop4x(fg + 16u * g0, xr + 8u * g0, grp);
                } else {
                    const XRec none{};
                    sphere_loop(fg + 16u * g0, 4u, [&](const SphGroup<float>& cur, uint32_t g) { grp(cur, none, g); });
                }'''
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
