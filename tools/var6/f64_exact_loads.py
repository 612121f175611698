"""A/B patch (round 6): fp64 exact test (nearest_hit's exact4) loads both 64-byte groups of spheres 4g..4g+3 and (in a
walked cluster) their inline scene indices in one scalar round trip: three s_loads and one wait in one asm statement.
The compiler had sunk each sphere's part of the loads into its pair-mask branch, so a taken group waited for up to
four scalar round trips one after the other."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_sweep.hpp", """            } else {
                const SphGroup<T> c0 = load_group(fe, 2 * g), c1 = load_group(fe, 2 * g + 1);
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (!((pairs >> j) & 1u)) continue;""", """            } else {
                typedef double d8 __attribute__((ext_vector_type(8)));
                typedef uint32_t u4v __attribute__((ext_vector_type(4)));
                d8 ga, gb;
                Q4 si;
                const auto* gp = fe + 16u * g;   // the two groups of spheres 4g..4g+3
                if (ip != nullptr) {
                    u4v iv;
                    asm volatile("s_load_dwordx16 %0, %3, 0x0\\n\\ts_load_dwordx16 %1, %3, 0x40\\n\\t"
                                 "s_load_dwordx4 %2, %4, 0x0\\n\\ts_waitcnt lgkmcnt(0)"
                                 : "=s"(ga), "=s"(gb), "=s"(iv) : "s"(gp), "s"(ip));
                    si = Q4{iv.x, iv.y, iv.z, iv.w};
                } else {
                    asm volatile("s_load_dwordx16 %0, %2, 0x0\\n\\ts_load_dwordx16 %1, %2, 0x40\\n\\ts_waitcnt lgkmcnt(0)"
                                 : "=s"(ga), "=s"(gb) : "s"(gp));
                    si = sidx(g, nullptr);
                }
                SphGroup<T> c0, c1;
#pragma unroll
                for (int e = 0; e < 8; ++e) { c0.v[e] = ga[e]; c1.v[e] = gb[e]; }
                T hb[4], disc[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (!((pairs >> j) & 1u)) continue;""")
sub("rt_sweep.hpp", """                const Q4 si = sidx(g, ip);
                const uint32_t sv[4] = {si.x, si.y, si.z, si.w};""", """                const uint32_t sv[4] = {si.x, si.y, si.z, si.w};""")
