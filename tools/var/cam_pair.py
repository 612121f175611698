# A/B patch: camera_listed tests a pixel's listed spheres two at a time with both spheres' records (scene
# index, camera-origin record) requested together, instead of one load round trip per listed sphere
# (CAM waits 56 % of its added cycles, profiles/r05/stage_issue_C_f32.txt).
import sys
d = sys.argv[1]
p = f"{d}/rt_camera.hpp"; s = open(p).read()
old = '''        for (uint32_t j = 0; j < n; ++j) {
            ++n_cx;
            camera_exact<T, root2, SCALAR>(q, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, best_t, best);
        }'''
new = '''        for (uint32_t j = 0; j < n; j += 2u) {
            const bool two = j + 1u < n;
            const uint32_t s0 = __builtin_amdgcn_readfirstlane(l[1u + j]);
            const uint32_t s1 = two ? __builtin_amdgcn_readfirstlane(l[2u + j]) : s0;
            cptr<T> cxt = (cptr<T>)__builtin_assume_aligned(q.camx, 16);
            cptr<uint32_t> ri = (cptr<uint32_t>)q.ridx;
            const uint32_t i0 = ri[s0], i1 = ri[s1];
            const T x0 = cxt[4 * s0], y0 = cxt[4 * s0 + 1], z0 = cxt[4 * s0 + 2], c0 = cxt[4 * s0 + 3];
            const T x1 = cxt[4 * s1], y1 = cxt[4 * s1 + 1], z1 = cxt[4 * s1 + 2], c1 = cxt[4 * s1 + 3];
            n_cx += two ? 2u : 1u;
            camera_exact_rec<T, root2, SCALAR>(i0, x0, y0, z0, c0, v, d, a, inv_a, best_t, best);
            if (two) camera_exact_rec<T, root2, SCALAR>(i1, x1, y1, z1, c1, v, d, a, inv_a, best_t, best);
        }'''
assert old in s; s = s.replace(old, new)
# camera_exact split: the record-taking body
old = "template <typename T, bool root2, bool SCALAR, typename KP>\n__device__ __forceinline__ void camera_exact("
if old not in s:
    i = s.index("__device__ __forceinline__ void camera_exact(")
    j = s.rfind("template", 0, i)
    hdr = s[j:i]
else:
    j = s.index(old); hdr = None
k = s.index("__device__ __forceinline__ void camera_exact(")
tmpl_start = s.rfind("template", 0, k)
body = '''template <typename T, bool root2, bool SCALAR>
__device__ __forceinline__ void camera_exact_rec(uint32_t i, T ocx, T ocy, T ocz, T c, bool v, const V3<T>& d, T a, T inv_a,
                                                 T& best_t, int& best) {
    KSTAT(2);
    constexpr bool kBothRoots = root2 || SCALAR;
    if (v) {
        T hb, disc;
        if constexpr (SCALAR) {   // objects.rs:217-222
            hb = (ocx * d.x + ocy * d.y) + ocz * d.z;
            disc = hb * hb - a * c;
        } else {                  // objects.rs:255, 257
            hb = fma(ocz, d.z, fma(ocy, d.y, ocx * d.x));
            disc = fma(hb, hb, (-a) * c);
        }
        if (kBothRoots ? disc >= T(0.0) : (disc >= T(0.0) && hb <= T(0.0)))
            hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, best_t, best);
    }
}
'''
s = s[:tmpl_start] + body + s[tmpl_start:]
open(p, "w").write(s)
