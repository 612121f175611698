"""A/B patch (round 6): fp64 unit_vec's r = sqrt(1 - z^2) through sqrt_len (the library's fp64 sqrt sequence without
its range scaling and class fix-up when every lane's argument is in [2^-100, 2^100]; 1 - z^2 is 0 or >= ~2^-53, and a
wave with a 0 takes the library sqrt).  The same bits.  fp32 keeps sqrt_nd."""
import sys
d = sys.argv[1]
p = f"{d}/rt_device.hpp"
s = open(p).read()
old = "    const T r = sqrt_nd(T(1.0) - z * z);   // z = 1 - 2 u1: 1 - z^2 is 0 or >= 2^-24"
new = """    // z = 1 - 2 u1: 1 - z^2 is 0 or >= 2^-24 (fp32) / ~2^-53 (fp64); fp64 through sqrt_len's in-range fast form
    T r;
    if constexpr (sizeof(T) == 8) r = sqrt_len(T(1.0) - z * z);
    else r = sqrt_nd(T(1.0) - z * z);"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
