# A/B patch: the passing clusters of one super box walked as one stream of filter groups (kernels without the
# mega level).  sphere_loop per cluster loaded each cluster's first group with nothing to hide it behind and
# prefetched the group after its last one (the next cluster in memory, usually not walked); the stream
# prefetches the next walked cluster's first group while the current cluster's last group is tested.
import sys
d = sys.argv[1]
p = f"{d}/rt_sweep.hpp"; s = open(p).read()
a = s.index("            while (mask != 0u) {\n                const uint32_t kc = 4u * sup + (uint32_t)__builtin_ctz(mask);   // cluster")
b = s.index("        // The top level is the super boxes, or (MEGA")
old = s[a:b]
# the per-group body, with the group's absolute index ga and the filter constants as parameters
body_start = old.index("                    uint32_t s0, s1;")
body_end = old.index("                });\n            }\n        };")
body = old[body_start:body_end].replace("g0 + g", "ga")
body = "\n".join(l[4:] if l.startswith("    ") else l for l in body.split("\n"))
fgroup = ("            // one filter group (absolute index ga) against the filter constants L0..L3\n"
          "            auto fgroup = [&](const SphGroup<float>& cur, uint32_t ga, f2 L0, f2 L1, f2 L2, f2 L3) {\n"
          + body + "            };\n")
stream = """            if constexpr (!MEGA) {
                // The passing clusters' groups as one stream, two groups per step: the next walked
                // cluster's first group is requested while this cluster's last group is tested.
                if (mask == 0u) return;
                auto next_cluster = [&]() -> uint32_t {
                    const uint32_t kc = 4u * sup + (uint32_t)__builtin_ctz(mask);   // cluster
                    mask &= mask - 1u;
                    KSTAT(4);
                    n_filt += 4u;
                    return nxg + 4u * kc;
                };
                uint32_t gc = next_cluster();
                SphGroup<float> A = load_group(ff, gc);
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_sched_barrier(0);
                bool first = true;   // gc is a cluster's first group (else its third)
                for (;;) {
                    const SphGroup<float> B = load_group(ff, gc + 1u);
                    __builtin_amdgcn_sched_barrier(0);
                    fgroup(A, gc, K0, K1, K2, K3);
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // B has landed
                    __builtin_amdgcn_sched_barrier(0);
                    const bool last = !first && mask == 0u;
                    const uint32_t gn = first ? gc + 2u : (last ? gc : next_cluster());
                    if (!last) A = load_group(ff, gn);
                    __builtin_amdgcn_sched_barrier(0);
                    fgroup(B, gc + 1u, K0, K1, K2, K3);
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // A has landed
                    __builtin_amdgcn_sched_barrier(0);
                    if (last) break;
                    gc = gn;
                    first = !first;
                }
                return;
            }
"""
new_loop = old[:body_start] + "                    fgroup(cur, g0 + g, L0, L1, L2, L3);\n" + old[body_end:]
s = s[:a] + fgroup + stream + new_loop + s[b:]
open(p, "w").write(s)
