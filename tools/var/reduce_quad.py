# A/B patch: reduce_live16 with four batches per iteration (the loads of 256 positions issued together) instead
# of two.
import sys
d = sys.argv[1]
p = f"{d}/rt_finish.hpp"; s = open(p).read()
old = '''    for (; qb + 128u <= nfull; qb += 128u) {   // two batches per round trip
        const uint32_t qq = qb + lane;
        const uint32_t m0 = mapat(qq), m1 = mapat(qq + 64u);
        const T y0 = sc.y(s, qq), y1 = sc.y(s, qq + 64u);
        const C3<T> c0 = rec(m0), c1 = rec(m1);
        T r0, g0, b0, r1, g1, b1;
        vals16(y0, m0, c0, r0, g0, b0);
        vals16(y1, m1, c1, r1, g1, b1);
        sum16(r0, g0, b0);
        sum16(r1, g1, b1);
    }'''
new = '''    for (; qb + 256u <= nfull; qb += 256u) {   // four batches per round trip
        const uint32_t qq = qb + lane;
        uint32_t m[4];
        T y[4];
        C3<T> c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = mapat(qq + 64u * k);
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = sc.y(s, qq + 64u * k);
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = rec(m[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            T r0, g0, b0;
            vals16(y[k], m[k], c[k], r0, g0, b0);
            sum16(r0, g0, b0);
        }
    }
    for (; qb + 128u <= nfull; qb += 128u) {   // two batches per round trip
        const uint32_t qq = qb + lane;
        const uint32_t m0 = mapat(qq), m1 = mapat(qq + 64u);
        const T y0 = sc.y(s, qq), y1 = sc.y(s, qq + 64u);
        const C3<T> c0 = rec(m0), c1 = rec(m1);
        T r0, g0, b0, r1, g1, b1;
        vals16(y0, m0, c0, r0, g0, b0);
        vals16(y1, m1, c1, r1, g1, b1);
        sum16(r0, g0, b0);
        sum16(r1, g1, b1);
    }'''
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
