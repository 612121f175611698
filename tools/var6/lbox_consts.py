"""A/B patch (round 6): the mega kernels' local-frame margin constants (l_r2max, l_hir2, l_isr) in every local box
group's unused words v[28..30], so lmask reads them with the group instead of from the kernel arguments at every box
group (a scalar load in front of each group's frame arithmetic)."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_common.hpp", """    for (uint32_t e = 0; e < 28; ++e) r.v[e] = f[g * 32u + e];""",
    """    for (uint32_t e = 0; e < 31; ++e) r.v[e] = f[g * 32u + e];   // + the margin constants at 28..30""")
sub("rt_sweep.hpp", """            const float kp = __builtin_fmaf(__builtin_fmaf(pmg, pmg, ql.l_r2max), ql.l_hir2,
                                            __builtin_fmaf(pmg, ql.l_isr, 1.0f));""",
    """            const float kp = __builtin_fmaf(__builtin_fmaf(pmg, pmg, g.v[28]), g.v[29],
                                            __builtin_fmaf(pmg, g.v[30], 1.0f));   // l_r2max, l_hir2, l_isr""")
sub("rt_kernel.hip", """            pack_local_boxes(c32, L, q32, b32[0], b32[1], b32[2], b32[3], c->l_r2max32, c->l_r2min32, &wme);""",
    """            pack_local_boxes(c32, L, q32, b32[0], b32[1], b32[2], b32[3], c->l_r2max32, c->l_r2min32, &wme);
            {   // the margin constants in every local box group's words 28..30 (lmask), as launch_t computes them
                auto up32c = [](double v) -> float {
                    float f = (float)v;
                    if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
                    return f;
                };
                auto fill = [&](std::vector<float>* b, float r2max, float r2min) {
                    const float k[3] = {r2max, up32c((double)kFilterMargin * 0.5 / (double)r2min),
                                        up32c(8.0 * 0x1.0p-24 / std::sqrt((double)r2min))};
                    for (int lv = 0; lv < 4; ++lv)
                        for (size_t g = 0; g + 1 <= b[lv].size() / 32; ++g)
                            for (int j = 0; j < 3; ++j) b[lv][32 * g + 28 + j] = k[j];
                };
                fill(b64, c->l_r2max64, c->l_r2min64);
                fill(b32, c->l_r2max32, c->l_r2min32);
            }""")
