"""A/B patch (round 6): in each cluster block the records of groups 2 and 3 come first (slot g ^ 2).  The walk's group
pipeline requests "group 4" -- the records' first line -- while it tests group 2; groups 0 and 1 were tested before
that request either way, so the line it prefetches now holds the records the last two groups need."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_sweep.hpp", """                        if constexpr (kInl) exact4f(cur, fgb + 64u + 8u * g, pairs);
                        else
                            exact4(g0 + g, pairs, fgb + 68u + 8u * g);""", """                        if constexpr (kInl) exact4f(cur, fgb + 64u + 8u * (g ^ 2u), pairs);
                        else
                            exact4(g0 + g, pairs, fgb + 68u + 8u * (g ^ 2u));""")
sub("rt_kernel.hip", """                    memcpy(b + 64 + 8 * q, rec, 32);""", """                    memcpy(b + 64 + 8 * (q ^ 2), rec, 32);   // groups 2, 3 first: the line the walk prefetches""")
