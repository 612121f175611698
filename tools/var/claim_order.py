# A/B patch: claim order and sky pixels per issue() call.  argv[2] = "<order>,<cap>": order "bup" renders
# the range bottom row first (the sky rows at the top of config C's frame come last, as cheap filler while
# the in-flight paths drain), "tdn" keeps top-down; cap > 0 stops issue() after finishing that many sky
# pixels at claim time when the wave has other work (live lanes or queued rays), so its stragglers keep
# running instead of waiting behind a run of sky pixels.
import sys
d = sys.argv[1]; order, cap = sys.argv[2].split(",")
p = f"{d}/rt_trace.hpp"; s = open(p).read()
if order == "bup":
    old = "                const uint32_t ri = item / q.col_count, ci = item % q.col_count;"
    new = ("                const uint32_t ri0 = item / q.col_count, ci = item % q.col_count;\n"
           "                const uint32_t ri = (q.n_items / q.col_count - 1u) - ri0;   // bottom row first")
    assert old in s; s = s.replace(old, new)
if int(cap) > 0:
    old = "        uint32_t opened = 0, listed = 0;\n        while (want != 0ull && !drained) {"
    new = ("        uint32_t opened = 0, listed = 0, nsky = 0;\n"
           "        const bool has_work = __ballot(live) != 0ull || __builtin_amdgcn_readfirstlane(s_is[wave].qcount) != 0u;\n"
           "        while (want != 0ull && !drained) {")
    assert old in s; s = s.replace(old, new)
    old = "            if (cur_next == spp) {\n                const uint32_t avail = ~busy & ((1u << kSlots) - 1u);\n                if (avail == 0u) break;   // every slot waits for straggler rays"
    new = ("            if (cur_next == spp) {\n                const uint32_t avail = ~busy & ((1u << kSlots) - 1u);\n                if (avail == 0u) break;   // every slot waits for straggler rays\n"
           f"                if (has_work && nsky >= {cap}u) break;   // back to the live rays")
    assert old in s; s = s.replace(old, new)
    old = "                            if (lane == 0) { wcount[wave][0] += spp; wcount[wave][3] += spp; wcount[wave][2] += 1u; }\n                            continue;"
    new = "                            if (lane == 0) { wcount[wave][0] += spp; wcount[wave][3] += spp; wcount[wave][2] += 1u; }\n                            ++nsky;\n                            continue;"
    assert old in s; s = s.replace(old, new)
    # `live` must be declared before issue(): it is (bool live = false;) -- check
    assert s.index("bool live = false;") < s.index("auto issue = [&]")
open(p, "w").write(s)
