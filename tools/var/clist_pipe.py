# A/B patch: camera_listed reads a slot's whole candidate list with one 16-byte LDS read (the entries
# unpacked from SGPRs) and requests the next listed sphere's camera-origin record and scene index while
# the current one is tested: per listed sphere an LDS read, then the scalar loads it addresses, then the
# test, each waited on in turn before.
import sys
d = sys.argv[1]
p = f"{d}/rt_camera.hpp"; s = open(p).read()
old = """    uint32_t n_cx = 0;
    for (; smask != 0u; smask &= smask - 1u) {
        const uint16_t* l = lists[__builtin_ctz(smask)];
        const uint32_t n = __builtin_amdgcn_readfirstlane(l[0]);
        for (uint32_t j = 0; j < n; ++j) {
            ++n_cx;
            camera_exact<T, root2, SCALAR>(q, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, best_t, best);
        }
    }"""
new = """    uint32_t n_cx = 0;
    cptr<T> cxt = (cptr<T>)__builtin_assume_aligned(q.camx, 16);
    cptr<uint32_t> ri = (cptr<uint32_t>)q.ridx;
    struct CX { uint32_t i; T ox, oy, oz, c; };
    auto fetch = [&](uint32_t sl) -> CX { return CX{ri[sl], cxt[4 * sl], cxt[4 * sl + 1], cxt[4 * sl + 2], cxt[4 * sl + 3]}; };
    constexpr bool kBothRoots = root2 || SCALAR;
    for (; smask != 0u; smask &= smask - 1u) {
        const uint4 w = *(const uint4*)lists[__builtin_ctz(smask)];   // the whole list: n, then up to 7 slots
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(w.x), w1 = __builtin_amdgcn_readfirstlane(w.y),
                       w2 = __builtin_amdgcn_readfirstlane(w.z), w3 = __builtin_amdgcn_readfirstlane(w.w);
        const uint32_t n = w0 & 0xFFFFu;
        auto entry = [&](uint32_t j) -> uint32_t {   // list[j], 1 <= j < kCList
            const uint32_t ww = j < 2u ? w0 : (j < 4u ? w1 : (j < 6u ? w2 : w3));
            return (ww >> (16u * (j & 1u))) & 0xFFFFu;
        };
        if (n == 0u) continue;
        CX cur = fetch(entry(1u));
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        for (uint32_t j = 0; j < n; ++j) {
            ++n_cx;
            // the next listed sphere's record (this one's again past the end: never unused entries)
            const CX nxt = fetch(j + 1u < n ? entry(j + 2u) : entry(j + 1u));
            __builtin_amdgcn_sched_barrier(0);
            KSTAT(2);
            if (v) {
                T hb, disc;
                if constexpr (SCALAR) {   // objects.rs:217-222
                    hb = (cur.ox * d.x + cur.oy * d.y) + cur.oz * d.z;
                    disc = hb * hb - a * cur.c;
                } else {                  // objects.rs:255, 257
                    hb = fma(cur.oz, d.z, fma(cur.oy, d.y, cur.ox * d.x));
                    disc = fma(hb, hb, (-a) * cur.c);
                }
                if (kBothRoots ? disc >= T(0.0) : (disc >= T(0.0) && hb <= T(0.0)))
                    hit_update<T, root2, SCALAR>(hb, disc, cur.i, a, inv_a, best_t, best);
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_sched_barrier(0);
            cur = nxt;
        }
    }"""
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
p = f"{d}/rt_trace.hpp"; s = open(p).read()
old = "    __shared__ uint16_t s_clist[QW][CAMQ ? kSlots : 1][kCList];"
assert old in s; s = s.replace(old, "    __shared__ alignas(16) uint16_t s_clist[QW][CAMQ ? kSlots : 1][kCList];")
open(p, "w").write(s)
