# A/B patch: PackedHitRecords::update (objects.rs:140-155) as selects instead of control flow.  The
# compiler lowered `valid && (root < best || (root == best && i > best_i))` to nested exec-mask
# branches (two s_and_saveexec, ~15 SALU per candidate sphere); with bitwise ands/ors of the compares
# the update is two v_cndmask under one combined mask.  Same compares, same result.
import sys
d = sys.argv[1]
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
old = """    if (valid && (root < best_t || (root == best_t && (int)i > best))) { best_t = root; best = (int)i; }   // ties: later wins (:141)"""
new = """    // ties: later wins (:141); bitwise, so the update is two selects, not nested exec-mask branches
    const bool take = valid & ((root < best_t) | ((root == best_t) & ((int)i > best)));
    best_t = take ? root : best_t;
    best = take ? (int)i : best;"""
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
