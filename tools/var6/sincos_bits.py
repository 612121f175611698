"""A/B patch (round 6): sincos2pi's quadrant switch without branches.  With q = floor(4u) and the octant swap sw, the
result is sin = (sw ^ odd(q) ? c : s) with its sign flipped when q & 2, cos = (sw ^ odd(q) ? s : c) flipped when
(q + 1) & 2: two selects and two sign-bit xors (the same bits as the switch's negations), where the compiler built
the switch as nested exec-mask branches, every one of them run by a wave with lanes in all four quadrants."""
import sys
d = sys.argv[1]
p = f"{d}/rt_device.hpp"
s = open(p).read()
old = """    T s = fma(x * x2, ps, x);
    T c = fma(x2, pc, T(1.0));
    if (sw) { const T tmp = s; s = c; c = tmp; }
    switch (q & 3) {
        case 0: so = s; co = c; break;
        case 1: so = c; co = -s; break;
        case 2: so = -s; co = -c; break;
        default: so = -c; co = s; break;
    }
}"""
new = """    const T s = fma(x * x2, ps, x);
    const T c = fma(x2, pc, T(1.0));
    // quadrant q (0..3) of the un-swapped (s, c): sin = q odd ? c : s, negated for q & 2; cos = q odd ? s : c,
    // negated for (q + 1) & 2 -- the octant swap sw toggles the choice.  Branch-free: two selects, two sign xors.
    const uint32_t qs = (uint32_t)q << 30;                  // bit 31: q & 2, bit 30: q & 1
    const bool swp = sw != ((qs & 0x40000000u) != 0u);
    const T sm = swp ? c : s, cm = swp ? s : c;
    if constexpr (sizeof(T) == 4) {
        so = __uint_as_float(__float_as_uint(sm) ^ (qs & 0x80000000u));
        co = __uint_as_float(__float_as_uint(cm) ^ ((qs + 0x40000000u) & 0x80000000u));
    } else {
        so = __longlong_as_double(__double_as_longlong(sm) ^ ((long long)(qs & 0x80000000u) << 32));
        co = __longlong_as_double(__double_as_longlong(cm) ^ ((long long)((qs + 0x40000000u) & 0x80000000u) << 32));
    }
}"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
