# A/B patch: finish_pixel's final reduction on the live path (not sky-only, u16 map in LDS or global) through a
# specialised loop: whole batches need no bounds test, the map decode is three ops, a position without an
# entry loads a clamped record (branch-free), the y load does not wait for the map.
# argv[2] (optional): "reg" keeps the 12 running sums in a VGPR instead of LDS; "pf" also prefetches the next
# batch's map entry.
import sys
d = sys.argv[1]; mode = sys.argv[2] if len(sys.argv) > 2 else ""
p = f"{d}/rt_finish.hpp"; s = open(p).read()
helper = r'''
// The live path's final reduction (ray_tracing.rs:488-504) over whole batches of 64 positions with a u16
// position map (LDS or the wave's scratch): the same values and the same order of adds as
// reduce_positions with finish_pixel's generic value lambda; the partial last batch (spp % 64) goes
// through the generic lambda.
template <typename T, typename G>
__device__ __forceinline__ T reduce_live16(const PScratch<T>& sc, uint32_t s, uint32_t spp, uint32_t P, const uint16_t* lmap,
                                           bool lm, uint32_t* hist, T (*stage)[64], G&& generic) {
    const uint32_t lane = threadIdx.x & 63u;
    T* accl = (T*)hist;
    __REGACC_DECL__
    if (lane < 12u) accl[lane] = T(0.0);
    const uint32_t nfull = spp & ~63u;
    const uint16_t* gmap = (const uint16_t*)sc.base;
    const uint32_t si = 16u * (lane & 3u) + (lane >> 2);
    __PF_INIT__
    for (uint32_t qb = 0; qb < nfull; qb += 64u) {
        const uint32_t qq = qb + lane;
        const T y = sc.y(s, qq);
        __PF_LOAD__
        const bool has = m16 != 0xFFFFu, wh = m16 >= 0x8000u;
        const uint32_t smp = min(m16 & 0x7FFFu, spp - 1u);   // a clamped (unused) record without an entry
        const C3<T> cm = sc.c(s, smp);
        const V3<T> sk = sky(y);
        const T vr = has ? (wh ? sk.x : cm.x * sk.x) : T(0.0);   // (white x sky) == sky, bit for bit
        const T vg = has ? (wh ? sk.y : cm.y * sk.y) : T(0.0);
        const T vb = has ? (wh ? sk.z : cm.z * sk.z) : T(0.0);
        stage[0][si] = vr; stage[1][si] = vg; stage[2][si] = vb;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane < 12u) {
            const T* sv = &stage[lane >> 2][16u * (lane & 3u)];
            T a = __ACC_LOAD__;
#pragma unroll
            for (uint32_t u0 = 0; u0 < 16u; u0 += 4u) {
                T v[4];
#pragma unroll
                for (uint32_t u = 0; u < 4u; ++u) v[u] = sv[u0 + u];
#pragma unroll
                for (uint32_t u = 0; u < 4u; ++u) a = a + v[u];
            }
            __ACC_STORE__
        }
        __builtin_amdgcn_wave_barrier();
    }
    __REGACC_FLUSH__
    // the partial last batch (and positions past spp): the generic path, continuing the same sums
    for (uint32_t qb = nfull; qb < P; qb += 64u) {
        const uint32_t qq = qb + lane;
        T vr = T(0.0), vg = T(0.0), vb = T(0.0);
        if (qq < P) generic(qq, vr, vg, vb);
        stage[0][si] = vr; stage[1][si] = vg; stage[2][si] = vb;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane < 12u) {
            const uint32_t nu = min(16u, (P - qb) / 4u);
            const T* sv = &stage[lane >> 2][16u * (lane & 3u)];
            T a = accl[lane];
            for (uint32_t u = 0; u < nu; ++u) a = a + sv[u];
            accl[lane] = a;
        }
        __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return lane < 12u ? accl[lane] : T(0.0);
}
'''
if mode == "reg" or mode == "regpf":
    helper = helper.replace("__REGACC_DECL__", "T racc = T(0.0);").replace("__ACC_LOAD__", "racc").replace("__ACC_STORE__", "racc = a;") \
                   .replace("__REGACC_FLUSH__", "if (lane < 12u) accl[lane] = racc;")
else:
    helper = helper.replace("__REGACC_DECL__", "").replace("__ACC_LOAD__", "accl[lane]").replace("__ACC_STORE__", "accl[lane] = a;") \
                   .replace("__REGACC_FLUSH__", "")
if mode == "regpf2":   # two-stage pipeline: batch b+1's record and y loads issued before batch b's sum
    helper = helper.replace("__REGACC_DECL__", "T racc = T(0.0);").replace("__ACC_LOAD__", "racc").replace("__ACC_STORE__", "racc = a;") \
                   .replace("__REGACC_FLUSH__", "if (lane < 12u) accl[lane] = racc;")
    old_body = """        const uint32_t qq = qb + lane;
        const T y = sc.y(s, qq);
        __PF_LOAD__
        const bool has = m16 != 0xFFFFu, wh = m16 >= 0x8000u;
        const uint32_t smp = min(m16 & 0x7FFFu, spp - 1u);   // a clamped (unused) record without an entry
        const C3<T> cm = sc.c(s, smp);
"""
    new_body = """        const uint32_t qq = qb + lane;
        const T y = yn;
        const uint32_t m16 = m16n;
        const C3<T> cm = cn;
        if (qb + 64u < nfull) {   // batch b+1: its record and y (its map entry arrived during batch b-1), b+2's map entry
            const uint32_t m1 = m16nn;
            yn = sc.y(s, qq + 64u);
            cn = sc.c(s, min(m1 & 0x7FFFu, spp - 1u));
            m16n = m1;
            if (qb + 128u < nfull) m16nn = lm ? (uint32_t)lmap[qq + 128u] : (uint32_t)gmap[qq + 128u];
        }
        const bool has = m16 != 0xFFFFu, wh = m16 >= 0x8000u;
"""
    assert old_body in helper; helper = helper.replace(old_body, new_body)
    helper = helper.replace("__PF_INIT__", """uint32_t m16n = 0xFFFFu, m16nn = 0xFFFFu;
    T yn = T(0.0);
    C3<T> cn = {T(0.0), T(0.0), T(0.0)};
    if (nfull) {
        m16n = lm ? (uint32_t)lmap[lane] : (uint32_t)gmap[lane];
        if (64u < nfull) m16nn = lm ? (uint32_t)lmap[64u + lane] : (uint32_t)gmap[64u + lane];
        yn = sc.y(s, lane);
        cn = sc.c(s, min(m16n & 0x7FFFu, spp - 1u));
    }""")
elif mode in ("pf", "regpf"):
    helper = helper.replace("__PF_INIT__", "uint32_t m16n = nfull ? (lm ? (uint32_t)lmap[lane] : (uint32_t)gmap[lane]) : 0xFFFFu;") \
                   .replace("__PF_LOAD__", "const uint32_t m16 = m16n;\n        if (qb + 64u < nfull) m16n = lm ? (uint32_t)lmap[qq + 64u] : (uint32_t)gmap[qq + 64u];")
else:
    helper = helper.replace("__PF_INIT__", "").replace("__PF_LOAD__", "const uint32_t m16 = lm ? (uint32_t)lmap[qq] : (uint32_t)gmap[qq];")
anchor = "// The pixel's value: PackedColor::sum of the 4 lanes' sums"
assert anchor in s; s = s.replace(anchor, helper + "\n" + anchor)
old = '''        acc = reduce_positions<T>(P, hist, stage, [&](uint32_t qq, T& vr, T& vg, T& vb) {'''
new = '''        auto vals = [&](uint32_t qq, T& vr, T& vg, T& vb) {'''
assert old in s; s = s.replace(old, new)
old = '''            } else {
                const C3<T> cm = sc.c(s, qq);
                vr = cm.x; vg = cm.y; vb = cm.z;
            }
        });
    }'''
new = '''            } else {
                const C3<T> cm = sc.c(s, qq);
                vr = cm.x; vg = cm.y; vb = cm.z;
            }
        };
        if (MODE == kModeV2 && !sky_only && !(sc.wide & 2u)) acc = reduce_live16<T>(sc, s, spp, P, lmap, lm, hist, stage, vals);
        else acc = reduce_positions<T>(P, hist, stage, vals);
    }'''
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
