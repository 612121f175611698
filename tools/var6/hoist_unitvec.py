"""A/B patch (round 6): the scatter's random unit vector computed before the hit normal, outside the material branch,
so its sincos polynomial chains and the normal's sqrt / reciprocal chain are one basic block the scheduler can
interleave (the fp64 scatter waits ~80 % of its cycles at 4 waves per SIMD).  Waves whose hits are all dielectric
compute it for nothing."""
import sys
d = sys.argv[1]


def sub(path, old, new):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == 1, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_camera.hpp", """    } else {
        base = mk(o.x + d.x * hit_t, o.y + d.y * hit_t, o.z + d.z * hit_t);   // at_t""",
    """    } else {
        rvh = unit_vec(ua, ub);   // random_unit_vector (materials.rs), independent of the normal below
        base = mk(o.x + d.x * hit_t, o.y + d.y * hit_t, o.z + d.z * hit_t);   // at_t""")
sub("rt_camera.hpp", """    V3<T> vec, base;
    T l2, rad = T(1.0);""", """    V3<T> vec, base, rvh = mk(T(0), T(0), T(0));
    T l2, rad = T(1.0);""")
sub("rt_camera.hpp", """        const V3<T> rv = unit_vec(ua, ub);""", """        const V3<T> rv = rvh;""")
