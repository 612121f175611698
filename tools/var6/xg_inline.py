"""A/B patch (round 6): the always-exact groups' records inline too.  After the always-exact filter groups, their
records (r^2 of the pairs, 4 scene indices; padded to whole 64-byte lines) precede the cluster blocks, and the fp32
scene-frame kernels test an always-exact group like a walked one (exact4f: centres from the filter group, r^2 and
indices from the record) -- the sweep's first step, which sets the best hit the box tests cull with, then reads one
stream through one pointer instead of the exact group and the index table behind two kernel-argument loads."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_sweep.hpp", """        for (uint32_t g = 0; g < nxg; ++g) {
            const uint32_t pr = sizeof(T) == 4 ? (4u * g + 2u >= qa.n_xs ? 1u : 3u) : 15u;
            n_exact += pr == 1u ? 2u : 4u;
            exact4(g, pr);
        }""", """        // cluster blocks start after the always-exact groups and their records (whole 64-byte lines)
        const uint32_t cbase = 16u * nxg + 16u * ((nxg + 1u) / 2u);
        for (uint32_t g = 0; g < nxg; ++g) {
            const uint32_t pr = sizeof(T) == 4 ? (4u * g + 2u >= qa.n_xs ? 1u : 3u) : 15u;
            n_exact += pr == 1u ? 2u : 4u;
            if constexpr (sizeof(T) == 4 && !MEGA) exact4f(load_group(ff, g), ff + 16u * nxg + 8u * g, pr);
            else exact4(g, pr);
        }""")
sub("rt_sweep.hpp", """                    fg = (cptr<float>)__builtin_assume_aligned(ql.lfsph, 64) + 16u * nxg + 96u * kc;""",
    """                    fg = (cptr<float>)__builtin_assume_aligned(ql.lfsph, 64) + cbase + 96u * kc;""")
sub("rt_sweep.hpp", """                const cptr<float> fgb = MEGA ? fg : ff + 16u * nxg + 96u * kc;""",
    """                const cptr<float> fgb = MEGA ? fg : ff + cbase + 96u * kc;""")
# host: records of the always-exact groups after them, padded to whole lines
sub("rt_kernel.hip", """            const size_t blk = 96, ngf = src.size() / 16 - 1, nxg = c->n_xg, nk = (ngf - nxg) / 4;
            std::vector<float> rx((size_t)16 * nxg + blk * nk + 32, 0.0f);
            for (size_t g = 0; g < 16 * nxg; ++g) rx[g] = src[g];""",
    """            const size_t blk = 96, ngf = src.size() / 16 - 1, nxg = c->n_xg, nk = (ngf - nxg) / 4;
            const size_t cb = 16 * nxg + 16 * ((nxg + 1) / 2);   // the cluster blocks' start (device: cbase)
            std::vector<float> rx(cb + blk * nk + 32, 0.0f);
            for (size_t g = 0; g < 16 * nxg; ++g) rx[g] = src[g];
            for (size_t g = 0; g < nxg; ++g) {   // the always-exact groups' records
                uint32_t rec[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
                if (r2) for (int h = 0; h < 4; ++h) memcpy(&rec[h], &rg32[16 * g + 8 * (h / 2) + 6 + (h % 2)], 4);
                for (int j = 0; j < 4; ++j) rec[4 + j] = 4 * g + j < ridx.size() ? ridx[4 * g + j] : 0xFFFFFFFFu;
                memcpy(&rx[16 * nxg + 8 * g], rec, 32);
            }""")
sub("rt_kernel.hip", """                float* b = &rx[16 * nxg + blk * k];""", """                float* b = &rx[cb + blk * k];""")
sub("rt_kernel.hip", """            for (size_t j = 0; j < 16; ++j) rx[16 * nxg + blk * nk + j] = src[16 * ngf + j];   // the dummy group""",
    """            for (size_t j = 0; j < 16; ++j) rx[cb + blk * nk + j] = src[16 * ngf + j];   // the dummy group""")
