"""A/B patch (round 6): the fp32 general sweep's exact records inside the filter stream.  Each cluster's block is its
4 filter groups (256 B) followed by their 4 exact records (r^2 of the two pairs and the 4 scene indices, 128 B), so a
taken group's record address is the cluster's filter pointer + 256 + 32 g: one scalar load from SGPRs the loop
already holds, where the separate table (xrec) needed the kernel-argument load of its base first (two dependent
scalar round trips per taken group).  fp64 and the mega kernels keep their streams."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_sweep.hpp", """        auto exact4f = [&](const SphGroup<float>& cur, uint32_t g, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                const auto& qx = *cold_args<T>();
                cptr<uint32_t> xr = (cptr<uint32_t>)__builtin_assume_aligned(qx.xrec, 32);
                uint32_t rec[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) rec[j] = xr[8u * g + (uint32_t)j];""",
    """        auto exact4f = [&](const SphGroup<float>& cur, cptr<float> recp, uint32_t pairs) {
            KSTAT(0);
            if constexpr (sizeof(T) == 4) {
                cptr<uint32_t> xr = (cptr<uint32_t>)recp;
                uint32_t rec[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) rec[j] = xr[(uint32_t)j];""")
sub("rt_sweep.hpp", """                sphere_loop(fg + 16u * g0, 4u, [&](const SphGroup<float>& cur, uint32_t g) {""",
    """                // fp32 scene-frame kernels: cluster kc's block in the filter stream is its 4 groups, then their
                // 4 exact records (pack_sweep_inline)
                constexpr bool kInl = sizeof(T) == 4 && !MEGA && !CAMT;
                const cptr<float> fgb = kInl ? ff + 16u * nxg + 96u * kc : fg + 16u * g0;
                sphere_loop(fgb, 4u, [&](const SphGroup<float>& cur, uint32_t g) {""")
sub("rt_sweep.hpp", """                        if constexpr (sizeof(T) == 4 && !MEGA && !CAMT) exact4f(cur, g0 + g, pairs);""",
    """                        if constexpr (kInl) exact4f(cur, fgb + 64u + 8u * g, pairs);""")
sub("rt_kernel.hip", """        if ((rc = up(&c->rfsph32, rf32.data(), rf32.size() * sizeof(float))) != RT_OK) return rc;""",
    """        {   // fp32: each cluster's 4 filter groups followed by their 4 exact records (nearest_hit, exact4f): the
            // always-exact groups first, then 96 floats per cluster, then a dummy group (the loop's prefetch)
            const size_t ngf = rf32.size() / 16 - 1, nxg = c->n_xg, ncl = (ngf - nxg) / 4;
            std::vector<float> rx((size_t)16 * nxg + (size_t)96 * ncl + 32, 0.0f);
            for (size_t g = 0; g < 16 * nxg; ++g) rx[g] = rf32[g];
            for (size_t k = 0; k < ncl; ++k) {
                float* b = &rx[16 * nxg + 96 * k];
                for (size_t j = 0; j < 64; ++j) b[j] = rf32[16 * (nxg + 4 * k) + j];
                for (size_t q = 0; q < 4; ++q) {
                    const size_t g = nxg + 4 * k + q;
                    uint32_t rec[8];
                    for (int h = 0; h < 4; ++h) memcpy(&rec[h], &rg32[16 * g + 8 * (h / 2) + 6 + (h % 2)], 4);
                    for (int j = 0; j < 4; ++j) rec[4 + j] = 4 * g + j < ridx.size() ? ridx[4 * g + j] : 0xFFFFFFFFu;
                    memcpy(b + 64 + 8 * q, rec, 32);
                }
            }
            for (size_t j = 0; j < 16; ++j) rx[16 * nxg + 96 * ncl + j] = rf32[16 * ngf + j];   // the dummy group
            if ((rc = up(&c->rfsph32, rx.data(), rx.size() * sizeof(float))) != RT_OK) return rc;
        }""")
