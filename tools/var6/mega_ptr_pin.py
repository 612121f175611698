"""A/B patch (round 6): the mega kernels' sweep pins the cluster-box and local-filter stream pointers in SGPRs once
per sweep, instead of reloading them from the kernel arguments at every walked super / cluster (a dependent scalar
round trip before each box group and each cluster block)."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_sweep.hpp", """        const uint32_t nsg = (ntop + 3u) / 4u;   // super groups (ntop supers, one per cluster top group)""",
    """        const uint32_t nsg = (ntop + 3u) / 4u;   // super groups (ntop supers, one per cluster top group)
        cptr<float> p_lclb = (cptr<float>)qa.lclb, p_lfs = (cptr<float>)qa.lfsph;
        if constexpr (MEGA) asm volatile("" : "+s"(p_lclb), "+s"(p_lfs));   // pinned for the sweep""")
sub("rt_sweep.hpp", """                mask = lmask(load_lbox((cptr<float>)__builtin_assume_aligned(qa.lclb, 64), sup));""",
    """                mask = lmask(load_lbox(p_lclb, sup));""")
sub("rt_sweep.hpp", """                    fg = (cptr<float>)__builtin_assume_aligned(ql.lfsph, 64) + 16u * nxg + 96u * kc;""",
    """                    fg = p_lfs + 16u * nxg + 96u * kc;""")
