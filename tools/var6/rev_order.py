"""A/B patch (round 6): claim the work items in reverse order (item' = n_items - 1 - item), so a launch ends on
the top rows -- for the RTIOW camera the sky, whose pixels finish at claim time (finish_sky_direct) -- instead of
the ground and sphere rows.  Cheap items at the end act as filler: waves that finish early take more of them, so
the launch's drain shrinks.  Pixels are independent and keyed by their own index: the same image."""
import sys
d = sys.argv[1]
p = f"{d}/rt_trace.hpp"
s = open(p).read()
old = "                const uint32_t s = __builtin_ctz(avail);\n                const uint32_t ri = item / q.col_count, ci = item % q.col_count;"
new = "                const uint32_t s = __builtin_ctz(avail);\n                item = q.n_items - 1u - item;\n                const uint32_t ri = item / q.col_count, ci = item % q.col_count;"
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
