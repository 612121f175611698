# A/B patch: prefetch a walked cluster's exact-test data into the scalar cache together with its first filter
# group (one dummy SGPR, waited by the filter pipeline's first s_waitcnt).  python3 pf_exact.py <dir>
import sys
d = sys.argv[1]
p = f"{d}/rt_common.hpp"; s = open(p).read()
old = "template <typename T, typename F>\n__device__ __forceinline__ void sphere_loop(cptr<T> f, uint32_t ng, F&& group) {"
new = '''// sphere_loop with a scalar-cache prefetch issued next to its first group's load: pf() issues s_load_dwords
// into one dummy SGPR (never read), kept live until the first wait has drained them.
template <typename T, typename F, typename PF>
__device__ __forceinline__ void sphere_loop_pf(cptr<T> f, uint32_t ng, F&& group, PF&& pf) {
    const uint32_t dummy = pf();
    SphGroup<T> A = load_group(f, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::"s"(dummy));
    uint32_t g = 0;
    for (; g + 1 < ng; g += 2) {
        const SphGroup<T> B = load_group(f, g + 1);
        __builtin_amdgcn_sched_barrier(0);
        group(A, g);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        A = load_group(f, g + 2);
        __builtin_amdgcn_sched_barrier(0);
        group(B, g + 1);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (g < ng) group(A, g);
}
''' + old
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
old = "                sphere_loop(fg + 16u * g0, 4u, [&](const SphGroup<float>& cur, uint32_t g) {"
new = "                sphere_loop_pf(fg + 16u * g0, 4u, [&](const SphGroup<float>& cur, uint32_t g) {"
assert old in s; s = s.replace(old, new)
old = '''                        if constexpr (sizeof(T) == 4 && !MEGA && !CAMT) exact4f(cur, g0 + g, pairs);
                        else
                            exact4(g0 + g, pairs);
                    }
                });'''
new = '''                        if constexpr (sizeof(T) == 4 && !MEGA && !CAMT) exact4f(cur, g0 + g, pairs);
                        else
                            exact4(g0 + g, pairs);
                    }
                }, [&]() -> uint32_t {
                    const auto& qp = *cold_args<T>();
                    uint32_t dm;
                    if constexpr (sizeof(T) == 4 && !MEGA) {   // xrec: 32 B per group
                        const char* xp = (const char*)qp.xrec + 32u * g0;
                        asm volatile("s_load_dword %0, %1, 0x0\\n\\ts_load_dword %0, %1, 0x40\\n\\ts_load_dword %0, %1, 0x7c"
                                     : "=&s"(dm) : "s"(xp));
                    } else if constexpr (sizeof(T) == 8) {     // 128 B exact data per group, 16 B indices
                        const char* xp = (const char*)qp.rsph + 128u * g0;
                        const char* ip = (const char*)qp.ridx + 16u * g0;
                        asm volatile("s_load_dword %0, %1, 0x0\\n\\ts_load_dword %0, %1, 0x40\\n\\ts_load_dword %0, %1, 0x80\\n\\t"
                                     "s_load_dword %0, %1, 0xc0\\n\\ts_load_dword %0, %1, 0x100\\n\\ts_load_dword %0, %1, 0x140\\n\\t"
                                     "s_load_dword %0, %1, 0x180\\n\\ts_load_dword %0, %1, 0x1c0\\n\\t"
                                     "s_load_dword %0, %2, 0x0\\n\\ts_load_dword %0, %2, 0x3c"
                                     : "=&s"(dm) : "s"(xp), "s"(ip));
                    } else {                                   // MEGA fp32: 64 B exact group, 16 B indices
                        const char* xp = (const char*)qp.rsph + 64u * g0;
                        const char* ip = (const char*)qp.ridx + 16u * g0;
                        asm volatile("s_load_dword %0, %1, 0x0\\n\\ts_load_dword %0, %1, 0x40\\n\\ts_load_dword %0, %1, 0x80\\n\\t"
                                     "s_load_dword %0, %1, 0xc0\\n\\ts_load_dword %0, %2, 0x0\\n\\ts_load_dword %0, %2, 0x3c"
                                     : "=&s"(dm) : "s"(xp), "s"(ip));
                    }
                    return dm;
                });'''
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
