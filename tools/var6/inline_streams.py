"""A/B patch (round 6, after xrec_inline): the same inline layout for the fp64 filter stream and the mega kernels'
local streams.  Each cluster's 4 filter groups are followed by 4 records {r^2 of the pairs (fp32 scene-frame stream
only), 4 scene indices} and, in the mega streams, the cluster's frame record (8 floats, was a separate table).  A
taken group's scene indices and a walked cluster's frame are then loads from the stream pointer the walk already
holds, instead of a kernel-argument load followed by the dependent record load (fp64 exact4's sidx, the mega
kernels' ridx and lclu)."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


# ---- device ----
sub("rt_sweep.hpp", """        auto sidx = [&](uint32_t g) -> Q4 {   // scene indices of slot group g (one s_load_dwordx4)
            const auto& qi = *cold_args<T>();
            cptr<uint32_t> ri = (cptr<uint32_t>)__builtin_assume_aligned(qi.ridx, 16);
            return Q4{ri[4 * g], ri[4 * g + 1], ri[4 * g + 2], ri[4 * g + 3]};
        };""", """        // scene indices of slot group g: from the inline record ip (a walked cluster's group) or the slot table
        auto sidx = [&](uint32_t g, cptr<float> ip) -> Q4 {
            if (ip != nullptr) {
                cptr<uint32_t> r = (cptr<uint32_t>)ip;
                return Q4{r[0], r[1], r[2], r[3]};
            }
            const auto& qi = *cold_args<T>();
            cptr<uint32_t> ri = (cptr<uint32_t>)__builtin_assume_aligned(qi.ridx, 16);
            return Q4{ri[4 * g], ri[4 * g + 1], ri[4 * g + 2], ri[4 * g + 3]};
        };""")
sub("rt_sweep.hpp", """        auto exact4 = [&](uint32_t g, uint32_t pairs = sizeof(T) == 4 ? 3u : 15u) {""",
    """        auto exact4 = [&](uint32_t g, uint32_t pairs = sizeof(T) == 4 ? 3u : 15u, cptr<float> ip = nullptr) {""")
sub("rt_sweep.hpp", """                const Q4 si = sidx(g);""", """                const Q4 si = sidx(g, ip);""", count=2)
sub("rt_sweep.hpp", """                    const auto& ql = *cold_args<T>();
                    cptr<float> lr = (cptr<float>)__builtin_assume_aligned(ql.lclu, 32);
                    const f2 Ckxy = {lr[8u * kc], lr[8u * kc + 1u]};
                    const float Ckz = lr[8u * kc + 2u];
                    const float Rc = lr[8u * kc + 3u], r2x = lr[8u * kc + 4u], ir2 = lr[8u * kc + 5u];""",
    """                    const auto& ql = *cold_args<T>();
                    // the cluster's block in the local stream: 4 groups, then 4 records whose unused r^2 words
                    // hold the frame {C_k, Rc} (record 0) and {r2max, 1/r2min} (record 1)
                    fg = (cptr<float>)__builtin_assume_aligned(ql.lfsph, 64) + 16u * nxg + 96u * kc;
                    const f2 Ckxy = {fg[64], fg[65]};
                    const float Ckz = fg[66];
                    const float Rc = fg[67], r2x = fg[72], ir2 = fg[73];""")
sub("rt_sweep.hpp", """                    L3 = f2{-oe1l, -oe2l};
                    fg = (cptr<float>)__builtin_assume_aligned(ql.lfsph, 64);
                }""", """                    L3 = f2{-oe1l, -oe2l};
                }""")
sub("rt_sweep.hpp", """                // fp32 scene-frame kernels: cluster kc's block in the filter stream is its 4 groups, then their
                // 4 exact records (pack_sweep_inline)
                constexpr bool kInl = sizeof(T) == 4 && !MEGA && !CAMT;
                const cptr<float> fgb = kInl ? ff + 16u * nxg + 96u * kc : fg + 16u * g0;""",
    """                // cluster kc's block in the filter stream: its 4 groups, then their 4 records (r^2 for the fp32
                // scene-frame stream, the scene indices), then (mega streams) the frame record (inline_stream)
                constexpr bool kInl = sizeof(T) == 4 && !MEGA && !CAMT;
                const cptr<float> fgb = MEGA ? fg : ff + 16u * nxg + 96u * kc;""")
sub("rt_sweep.hpp", """                        if constexpr (kInl) exact4f(cur, fgb + 64u + 8u * g, pairs);
                        else
                            exact4(g0 + g, pairs);""", """                        if constexpr (kInl) exact4f(cur, fgb + 64u + 8u * g, pairs);
                        else
                            exact4(g0 + g, pairs, fgb + 68u + 8u * g);""")
# ---- host ----
s = open(f"{d}/rt_kernel.hip").read()
i = s.index("        {   // fp32: each cluster's 4 filter groups followed by their 4 exact records")
j = s.index("            if ((rc = up(&c->rfsph32, rx.data(), rx.size() * sizeof(float))) != RT_OK) return rc;\n        }\n", i)
j += len("            if ((rc = up(&c->rfsph32, rx.data(), rx.size() * sizeof(float))) != RT_OK) return rc;\n        }\n")
new = """        // General-sweep filter streams, inline layout (nearest_hit): the always-exact groups, then per cluster its 4
        // filter groups, 4 records of 8 words {r^2 of pair 0 (2), r^2 of pair 1 (2), 4 scene indices} (r^2: the
        // fp32 scene-frame stream, whose exact test takes the centres from the filter group; in the mega kernels'
        // local streams the r^2 words of records 0 and 1 hold the cluster's frame record); then a dummy group (the
        // loop's prefetch).  96 floats per cluster keep every group on its own 64-byte line.  A
        // taken group's record and a walked cluster's frame are loads from the pointer the walk already holds.
        auto inline_stream = [&](const std::vector<float>& src, bool r2, const std::vector<float>* frame) {
            const size_t blk = 96, ngf = src.size() / 16 - 1, nxg = c->n_xg, nk = (ngf - nxg) / 4;
            std::vector<float> rx((size_t)16 * nxg + blk * nk + 32, 0.0f);
            for (size_t g = 0; g < 16 * nxg; ++g) rx[g] = src[g];
            for (size_t k = 0; k < nk; ++k) {
                float* b = &rx[16 * nxg + blk * k];
                for (size_t j = 0; j < 64; ++j) b[j] = src[16 * (nxg + 4 * k) + j];
                for (size_t q = 0; q < 4; ++q) {
                    const size_t g = nxg + 4 * k + q;
                    uint32_t rec[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
                    if (r2) for (int h = 0; h < 4; ++h) memcpy(&rec[h], &rg32[16 * g + 8 * (h / 2) + 6 + (h % 2)], 4);
                    for (int j = 0; j < 4; ++j) rec[4 + j] = 4 * g + j < ridx.size() ? ridx[4 * g + j] : 0xFFFFFFFFu;
                    memcpy(b + 64 + 8 * q, rec, 32);
                }
                if (frame) for (size_t j = 0; j < 4; ++j) { b[64 + j] = (*frame)[8 * k + j]; b[72 + j] = (*frame)[8 * k + 4 + j]; }
            }
            for (size_t j = 0; j < 16; ++j) rx[16 * nxg + blk * nk + j] = src[16 * ngf + j];   // the dummy group
            return rx;
        };
        {
            const std::vector<float> rx32 = inline_stream(rf32, true, nullptr), rx64 = inline_stream(rf64, false, nullptr);
            if ((rc = up(&c->rfsph32, rx32.data(), rx32.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->rfsph64, rx64.data(), rx64.size() * sizeof(float))) != RT_OK) return rc;
        }
        if (c->n_mg) {
            const std::vector<float> lx32 = inline_stream(lf32, false, &lr32), lx64 = inline_stream(lf64, false, &lr64);
            if ((rc = up(&c->lfs32, lx32.data(), lx32.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lfs64, lx64.data(), lx64.size() * sizeof(float))) != RT_OK) return rc;
        }
"""
s = s[:i] + new + s[j:]
open(f"{d}/rt_kernel.hip", "w").write(s)
sub("rt_kernel.hip", """        if ((rc = up(&c->rfsph64, rf64.data(), rf64.size() * sizeof(float))) != RT_OK) return rc;\n""", "")
sub("rt_kernel.hip", """            std::vector<float> lf64, lf32, lr64, lr32, q64, q32;""", """            std::vector<float> q64, q32;""")
sub("rt_kernel.hip", """        std::vector<double> rg64; std::vector<float> rg32, rf64, rf32, t64, t32, s64, s32, m64, m32;""",
    """        std::vector<double> rg64; std::vector<float> rg32, rf64, rf32, t64, t32, s64, s32, m64, m32;
        std::vector<float> lf64, lf32, lr64, lr32;   // the mega kernels' local streams (uploaded inline below)""")
sub("rt_kernel.hip", """            if ((rc = up(&c->lfs64, lf64.data(), lf64.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lfs32, lf32.data(), lf32.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lcl64, lr64.data(), lr64.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lcl32, lr32.data(), lr32.size() * sizeof(float))) != RT_OK) return rc;
""", "")
