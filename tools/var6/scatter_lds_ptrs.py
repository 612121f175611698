"""A/B patch (round 6): the scatter's two table pointers (sphere centres, material records) copied into LDS once per
workgroup and read from there in next_ray, instead of from the kernel arguments: after a sphere sweep has streamed
its groups through the scalar cache, the kernel-argument line is likely gone and its reload is an L2 round trip in
front of the dependent record gather."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_camera.hpp", """template <typename T, bool SCALAR>
__device__ __forceinline__ void next_ray(bool cam, uint32_t colx, uint32_t rowy, uint32_t pix, uint32_t sid,
                                         uint32_t k, int hit_i, T hit_t, V3<T>& o, V3<T>& d, V3<T>& c) {""",
    """template <typename T, bool SCALAR>
__device__ __forceinline__ void next_ray(bool cam, uint32_t colx, uint32_t rowy, uint32_t pix, uint32_t sid,
                                         uint32_t k, int hit_i, T hit_t, V3<T>& o, V3<T>& d, V3<T>& c,
                                         const T* tcen, const MatT<T>* tmats) {""")
sub("rt_camera.hpp", """    const auto& qg = *cold_args<T>();
    const T* sgp = qg.cen + 4 * hg;""", """    const T* sgp = tcen + 4 * hg;""")
sub("rt_camera.hpp", """    const MatT<T> m = qg.mats[hg];""", """    const MatT<T> m = tmats[hg];""")
sub("rt_trace.hpp", """    __shared__ unsigned long long s_pool;   // the workgroup's pool of claimed items: next << 32 | end""",
    """    __shared__ unsigned long long s_pool;   // the workgroup's pool of claimed items: next << 32 | end
    __shared__ const void* s_tabs[2];       // the scatter's tables (centres, materials): LDS, not kernel arguments""")
sub("rt_trace.hpp", """            s_pool = got ? ((unsigned long long)b0 << 32) | b1 : 0ull;   // {next, end}; {0, 0}: empty
            s_dry = 0u;""", """            s_pool = got ? ((unsigned long long)b0 << 32) | b1 : 0ull;   // {next, end}; {0, 0}: empty
            s_dry = 0u;
            s_tabs[0] = q.cen;
            s_tabs[1] = q.mats;""")
sub("rt_trace.hpp", """            next_ray<T, SC>(CAMQ ? false : fresh, fcol, frow, pix, sid_of(ssv), k, hit_i, hit_t, o, d, c);""",
    """            next_ray<T, SC>(CAMQ ? false : fresh, fcol, frow, pix, sid_of(ssv), k, hit_i, hit_t, o, d, c,
                            (const T*)s_tabs[0], (const MatT<T>*)s_tabs[1]);""")
