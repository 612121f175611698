# A/B patch: next_ray's scatter issues its two per-lane gathers -- the hit sphere's centre (q.cen) and its
# material record (q.mats) -- before the Philox block, from the un-laundered kernel arguments, so their
# latencies overlap each other and the RNG; the product loads the centre after the RNG (its pointer comes
# from the kernarg view laundered on the draw) and the material kind after that, then the rest by kind:
# three dependent round trips (SCATTER waits 51 % of its added cycles, profiles/r05/stage_issue_C_f32.txt).
import sys
d = sys.argv[1]
p = f"{d}/rt_camera.hpp"; s = open(p).read()
old = """    const U4 r = [&] {
        const auto& q0 = *cold_args<T>();
        return rng<T>(sid, pix, cam ? 0u : k, cam ? 0u : 2u, q0.k0, q0.k1);
    }();
    const auto& q = *cold_args_after<T>(r.a ^ r.b);"""
new = """    // the hit sphere's centre and material, requested before the draw (scatter lanes; a camera lane reads
    // record 0, unused)
    const int hg = cam ? 0 : hit_i;
    const auto& qg = *cold_args<T>();
    const T* sgp = qg.cen + 4 * hg;
    const V3<T> hcen = mk(sgp[0], sgp[1], sgp[2]);
    const T hrad = sgp[3];
    const MatT<T> m = qg.mats[hg];                       // = materials[material[hit_i]] (objects.rs:296)
    const U4 r = [&] {
        const auto& q0 = *cold_args<T>();
        return rng<T>(sid, pix, cam ? 0u : k, cam ? 0u : 2u, q0.k0, q0.k1);
    }();
    const auto& q = *cold_args_after<T>(r.a ^ r.b);"""
assert old in s; s = s.replace(old, new)
old = """        const T* sg = q.cen + 4 * hit_i;
        vec = sub(base, mk(sg[0], sg[1], sg[2]));        // normal = at_t(t) - center (objects.rs:279-280)
        if constexpr (SCALAR) rad = sg[3];"""
new = """        vec = sub(base, hcen);                           // normal = at_t(t) - center (objects.rs:279-280)
        if constexpr (SCALAR) rad = hrad;"""
assert old in s; s = s.replace(old, new)
old = "    const MatT<T> m = q.mats[hit_i];                     // = materials[material[hit_i]] (objects.rs:296)\n    V3<T> nd;"
new = "    V3<T> nd;"
assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
