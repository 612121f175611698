"""A/B patch (round 6): the per-sphere material record the scatter gathers, compacted to the fields its kind uses:
{kind, hollow, p[4]} with p = {albedo r, g, b, fuzz} (Lambertian, metal) or {ior, 1/ior, r0_front, r0_back}
(dielectric).  fp64 72 -> 40 bytes, fp32 40 -> 24: fewer vector loads and registers per scatter."""
import sys
d = sys.argv[1]


def sub(path, old, new):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == 1, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_common.hpp", """template <typename T> struct MatT {
    uint32_t kind, hollow;
    T ar, ag, ab, fuzz, ior;
    // Dielectric constants precomputed on the host in T with the reference's operations (IEEE,
    // no contraction, so the bits equal the per-ray device computation): 1/ior (materials.rs:131)
    // and Schlick's r0 = ((1-ratio)/(1+ratio))^2 (materials.rs:122) for ratio = 1/ior and ior.
    T inv_ior, r0_front, r0_back;
};""", """template <typename T> struct MatT {
    uint32_t kind, hollow;
    // Lambertian / metal: {albedo r, g, b, fuzz}; dielectric: {ior, 1/ior, r0_front, r0_back} -- the constants
    // precomputed on the host in T with the reference's operations (IEEE, no contraction, so the bits equal the
    // per-ray device computation): 1/ior (materials.rs:131) and Schlick's r0 = ((1-ratio)/(1+ratio))^2
    // (materials.rs:122) for ratio = 1/ior and ior.  Only the fields of the record's kind: fp64 40 bytes, fp32 24.
    T p[4];
};""")
sub("rt_layout.hpp", """        mats[i] = MatT<T>{m.kind, m.hollow, (T)m.albedo[0], (T)m.albedo[1], (T)m.albedo[2], (T)m.fuzz, ior,
                          inv, qf * qf, qb * qb};""", """        if (m.kind == RT_DIELECTRIC) mats[i] = MatT<T>{m.kind, m.hollow, {ior, inv, qf * qf, qb * qb}};
        else mats[i] = MatT<T>{m.kind, m.hollow, {(T)m.albedo[0], (T)m.albedo[1], (T)m.albedo[2], (T)m.fuzz}};""")
sub("rt_camera.hpp", """            nd = add(reflect(d, nrm), mul(rv, m.fuzz));""", """            nd = add(reflect(d, nrm), mul(rv, m.p[3]));   // fuzz""")
sub("rt_camera.hpp", """        c = mk(c.x * m.ar, c.y * m.ag, c.z * m.ab);""", """        c = mk(c.x * m.p[0], c.y * m.p[1], c.z * m.p[2]);   // albedo""")
sub("rt_camera.hpp", """        const T ratio = front ? m.inv_ior : m.ior;""", """        const T ratio = front ? m.p[1] : m.p[0];   // 1/ior : ior""")
sub("rt_camera.hpp", """            const T r0 = front ? m.r0_front : m.r0_back;""", """            const T r0 = front ? m.p[2] : m.p[3];   // r0_front : r0_back""")
