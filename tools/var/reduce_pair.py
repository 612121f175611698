# A/B patch: reduce_live16 takes two batches of 64 positions per iteration -- the y, map and colour-record
# loads of both issued together, then the two batches staged and summed one after the other in the same
# order -- so a pixel of 512 positions waits for 4 load round trips instead of 8 (REDUCE waits 60 % of its
# added cycles, profiles/r05/stage_issue_C_f32.txt).  A leftover single batch runs the one-batch body.
import sys
d = sys.argv[1]; pf = len(sys.argv) > 2 and sys.argv[2] == "pf"   # pf: the next pair's map entries loaded one iteration ahead
p = f"{d}/rt_finish.hpp"; s = open(p).read()
i0 = s.index("    uint32_t m16n = nfull ? (lm ? (uint32_t)lmap[lane] : (uint32_t)gmap[lane]) : 0xFFFFu;\n    for (uint32_t qb = 0; qb < nfull; qb += 64u) {")
i1 = s.index("    if (lane < 12u) accl[lane] = racc;\n    // the partial last batch")
new = r'''    auto mapat = [&](uint32_t qi) -> uint32_t { return lm ? (uint32_t)lmap[qi] : (uint32_t)gmap[qi]; };
    // values of one batch (positions qb + lane) from its y, map entry and record
    auto vals16 = [&](T y, uint32_t m16, const C3<T>& cm, T& vr, T& vg, T& vb) {
        const bool has = m16 != 0xFFFFu, wh = m16 >= 0x8000u;
        const V3<T> sk = sky(y);
        vr = has ? (wh ? sk.x : cm.x * sk.x) : T(0.0);   // (white x sky) == sky, bit for bit
        vg = has ? (wh ? sk.y : cm.y * sk.y) : T(0.0);
        vb = has ? (wh ? sk.z : cm.z * sk.z) : T(0.0);
    };
    auto rec = [&](uint32_t m16) -> C3<T> { return sc.c(s, min(m16 & 0x7FFFu, spp - 1u)); };   // clamped when none
    // the 12 lanes' running sums over one staged batch, in position order
    auto sum16 = [&](T vr, T vg, T vb) {
        stage[0][si] = vr; stage[1][si] = vg; stage[2][si] = vb;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane < 12u) {
            const T* sv = &stage[lane >> 2][16u * (lane & 3u)];
            T a = racc;
#pragma unroll
            for (uint32_t u0 = 0; u0 < 16u; u0 += 4u) {
                T v[4];
#pragma unroll
                for (uint32_t u = 0; u < 4u; ++u) v[u] = sv[u0 + u];
#pragma unroll
                for (uint32_t u = 0; u < 4u; ++u) a = a + v[u];
            }
            racc = a;
        }
        __builtin_amdgcn_wave_barrier();
    };
    uint32_t qb = 0;
__PFINIT__
    for (; qb + 128u <= nfull; qb += 128u) {   // two batches per round trip
        const uint32_t qq = qb + lane;
__PFLOAD__
        const T y0 = sc.y(s, qq), y1 = sc.y(s, qq + 64u);
        const C3<T> c0 = rec(m0), c1 = rec(m1);
        T r0, g0, b0, r1, g1, b1;
        vals16(y0, m0, c0, r0, g0, b0);
        vals16(y1, m1, c1, r1, g1, b1);
        sum16(r0, g0, b0);
        sum16(r1, g1, b1);
    }
    if (qb < nfull) {   // a leftover single batch
        const uint32_t qq = qb + lane, m0 = mapat(qq);
        T r0, g0, b0;
        vals16(sc.y(s, qq), m0, rec(m0), r0, g0, b0);
        sum16(r0, g0, b0);
    }
'''
if pf:
    new = new.replace("__PFINIT__", "    uint32_t n0 = nfull >= 128u ? mapat(lane) : 0xFFFFu, n1 = nfull >= 128u ? mapat(lane + 64u) : 0xFFFFu;")
    new = new.replace("__PFLOAD__", "        const uint32_t m0 = n0, m1 = n1;\n        if (qb + 256u <= nfull) { n0 = mapat(qq + 128u); n1 = mapat(qq + 192u); }")
else:
    new = new.replace("__PFINIT__\n", "")
    new = new.replace("__PFLOAD__", "        const uint32_t m0 = mapat(qq), m1 = mapat(qq + 64u);")
s = s[:i0] + new + s[i1:]
open(p, "w").write(s)
