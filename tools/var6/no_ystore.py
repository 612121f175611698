"""Timing-only probe (round 6; results differ from the oracle in the pixel values, not in the paths): the camera
batches do not store the primary rays' y.  Tests whether the fp64 scatter's waits (80 % of its added cycles,
profiles/r06/stage_issue_C_f64.txt) come from vmcnt ordering: the scatter's hit-record loads are issued after
the camera batches' stores, and gfx950 has one in-order vector-memory counter for loads and stores."""
import sys
d = sys.argv[1]
p = f"{d}/rt_trace.hpp"
s = open(p).read()
old = "            if (MODE == kModeV2) wave_scratch<T>(wave).y(bslot, bsid) = bd.y;   // primary y (quirk Q2)\n"
assert old in s
s = s.replace(old, "")
open(p, "w").write(s)
