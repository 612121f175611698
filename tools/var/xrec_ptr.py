# A/B patch: fp32 general sweep: the exact records' base pointer (xrec) read once per sweep with the other
# sweep constants, instead of from the laundered kernel arguments at every taken group (a dependent scalar
# load before the record's own).  +2 SGPRs held through the sweep.
import sys
d = sys.argv[1]
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
old = """        auto exact4f = [&](const SphGroup<float>& cur, uint32_t g, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                const auto& qx = *cold_args<T>();
                cptr<uint32_t> xr = (cptr<uint32_t>)__builtin_assume_aligned(qx.xrec, 32);"""
new = """        cptr<uint32_t> xr = (cptr<uint32_t>)__builtin_assume_aligned(qa.xrec, 32);
        auto exact4f = [&](const SphGroup<float>& cur, uint32_t g, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {"""
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
