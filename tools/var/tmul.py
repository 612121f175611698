# A/B patch: the guided schedule's single-pixel tail length T = kTMul x workgroups (argv[2] = kTMul; product 8).
import sys
d = sys.argv[1]; n = int(sys.argv[2])
p = f"{d}/rt_experiments.hpp"; s = open(p).read()
old = "constexpr uint32_t kTMul = 8;"
assert old in s; s = s.replace(old, f"constexpr uint32_t kTMul = {n};"); open(p, "w").write(s)
