"""A/B patch (round 6, after mat_compact): the hit sphere's centre joins its material record, so the scatter
gathers one record per hit (fp64: 64 bytes, one aligned half line; fp32: 48) instead of a material record and a
separate centre.  The centre stream (cen) stays for the scalar mode's radius."""
import sys
d = sys.argv[1]


def sub(path, old, new):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == 1, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_common.hpp", """    T p[4];
};""", """    T p[4];
    T c[3];   // the sphere's centre (the record is per sphere): one gather per hit
};""")
sub("rt_kernel.hip", """        for (size_t i = 0; i < sm.size(); ++i)
            if (sm[i] < m64.size()) { s64[i] = m64[sm[i]]; s32[i] = m32[sm[i]]; }""",
    """        for (size_t i = 0; i < sm.size(); ++i) {
            if (sm[i] < m64.size()) { s64[i] = m64[sm[i]]; s32[i] = m32[sm[i]]; }
            for (int f = 0; f < 3; ++f) { s64[i].c[f] = c64[4 * i + f]; s32[i].c[f] = c32[4 * i + f]; }
        }""")
sub("rt_camera.hpp", """    const T* sgp = qg.cen + 4 * hg;
    const V3<T> hcen = mk(sgp[0], sgp[1], sgp[2]);
    const T hrad = sgp[3];
    const MatT<T> m = qg.mats[hg];                       // = materials[material[hit_i]] (objects.rs:296)""",
    """    const MatT<T> m = qg.mats[hg];                       // = materials[material[hit_i]] (objects.rs:296) + centre
    const V3<T> hcen = mk(m.c[0], m.c[1], m.c[2]);
    const T hrad = SCALAR ? qg.cen[4 * hg + 3] : T(0);""")
