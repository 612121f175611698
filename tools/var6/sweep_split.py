"""A/B probe (round 6): how much of a general sweep's work comes from mixing
unrelated rays in one wave?  The live lanes are split into classes and each class sweeps on its own
(nearest_hit called once per non-empty class, lanes of other classes masked off), so a sweep's box and
filter groups are the union over one class's rays only.  Same hits, same image; more sweeps.
argv[2]: "bounce" (k == 1 | k >= 2), "bounce3" (k == 1 | k == 2 | k >= 3), "octant" (sign bits of d).
Measured with the kstats build (VARIANT_FLAGS=-DRT_KSTATS): clusters / filter groups per segment."""
import sys
d, mode = sys.argv[1], sys.argv[2]
p = f"{d}/rt_trace.hpp"
s = open(p).read()
old = """        hit_i = -1;
        if (act) hit_i = nearest_hit<T, ROOT2, SC, false, MEGA>(p, o, d, hit_t);"""
assert old in s
cls = {"bounce": "(k == 1u ? 0u : 1u)", "bounce3": "(k == 1u ? 0u : (k == 2u ? 1u : 2u))",
       "octant": "((d.x < T(0) ? 1u : 0u) | (d.y < T(0) ? 2u : 0u) | (d.z < T(0) ? 4u : 0u))"}[mode]
new = f"""        hit_i = -1;
        {{
            const uint32_t mycls = {cls};
            unsigned long long rem = __ballot(act);
            while (rem != 0ull) {{
                const uint32_t cc = __builtin_amdgcn_readlane(mycls, (int)__builtin_ctzll(rem));
                const bool mine = act && mycls == cc;
                rem &= ~__ballot(mine);
                if (mine) hit_i = nearest_hit<T, ROOT2, SC, false, MEGA>(p, o, d, hit_t);
            }}
        }}"""
s = s.replace(old, new)
open(p, "w").write(s)
