"""A/B patch (round 6): the box test's max(tn, 0) with a VGPR holding +0 instead of the inline constant.  A VALU op
with an SGPR or constant operand never co-issues (1 VALU quad-cycle); an all-VGPR max may take half of one
(profiles/r06/issue_counters.txt).  Same passes bit for bit (v_max_f32 with +0, either operand form)."""
import sys
d = sys.argv[1]
p = f"{d}/rt_sweep.hpp"
s = open(p).read()
old = '''    auto pass = [bt](float nx, float ny, float nz, float fx, float fy, float fz, auto bitc) -> uint32_t {'''
new = '''    float vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));   // +0 in a VGPR (one per box pair)
    auto pass = [bt, vz](float nx, float ny, float nz, float fx, float fy, float fz, auto bitc) -> uint32_t {'''
assert old in s
s = s.replace(old, new)
old = '''            "v_max_f32 %[tn], 0, %[tn]\\n\\t"'''
new = '''            "v_max_f32 %[tn], %[vz], %[tn]\\n\\t"'''
assert old in s, old
s = s.replace(old, new)
old = '''              [bit] "n"(bit)'''
new = '''              [bit] "n"(bit), [vz] "v"(vz)'''
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
