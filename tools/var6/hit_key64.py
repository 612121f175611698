"""A/B patch (round 6): fp32 best-hit state as one 64-bit key, (bits(t) - bits(0.001f)) << 32 | ~index (32-bit
wrap-around in the high half).  Non-negative floats order as their bits, so PackedHitRecords::update's rule (a
smaller t, or the same t and a later sphere, objects.rs:140-155) is one unsigned 64-bit compare; with the offset a
root below 0.001 (or negative, -0, NaN) wraps or lands above every valid key, and +inf meets the initial key
(+inf, ~(-1) = 0) with ~index >= 1: the compare is the whole of valid && better.  Replaces 5 compares, 4 SALU mask
ops, a move and two selects per candidate with a subtract, a move, one compare and two selects."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:60], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_sweep.hpp", """template <typename T, bool root2, bool SCALAR>
__device__ __forceinline__ void hit_update(T hb, T disc, uint32_t i, T a, T inv_a, T& best_t, int& best) {
    if constexpr (SCALAR) {""", """// The best hit so far (PackedHitRecords' t and sphere, objects.rs:121-155).  fp32: one 64-bit key bits(t) << 32 |
// ~index.  Non-negative floats order as their bits, so "a smaller t, or the same t and a later sphere" (:141) is
// one unsigned 64-bit compare; the key starts at +inf and ~(-1) = 0.
template <typename T> struct HitBest {
    T t = T(INFINITY);
    int i = -1;
    __device__ __forceinline__ T bt() const { return t; }
    __device__ __forceinline__ int bi() const { return i; }
    __device__ __forceinline__ void set(T r, uint32_t j) { t = r; i = (int)j; }
};
constexpr uint32_t kT001 = 0x3A83126Fu;   // bits of 0.001f (RN), the smallest valid root
__device__ __forceinline__ uint64_t hit_key(float r, uint32_t j) {
    return ((uint64_t)(__float_as_uint(r) - kT001) << 32) | (uint64_t)~j;
}
template <> struct HitBest<float> {
    uint64_t k = (uint64_t)(0x7F800000u - kT001) << 32;
    __device__ __forceinline__ float bt() const { return __uint_as_float((uint32_t)(k >> 32) + kT001); }
    __device__ __forceinline__ int bi() const { return (int)~(uint32_t)k; }
    __device__ __forceinline__ void set(float r, uint32_t j) { k = hit_key(r, j); }
};
template <typename T, bool root2, bool SCALAR>
__device__ __forceinline__ void hit_update(T hb, T disc, uint32_t i, T a, T inv_a, HitBest<T>& bh) {
    if constexpr (SCALAR) {""")
sub("rt_sweep.hpp", """        if (root < best_t || (root == best_t && (int)i < best)) { best_t = root; best = (int)i; }   // first wins""",
    """        if (root < bh.bt() || (root == bh.bt() && (int)i < bh.bi())) bh.set(root, i);   // first wins""")
sub("rt_sweep.hpp", """    const T sd = sqrt_len(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270
""", """    const T sd = sqrt_len(disc);
    const T r1 = (-hb - sd) * inv_a;                       // :270
    if constexpr (sizeof(T) == 4 && !root2) {
        // valid (:272) && better (:141) in one compare (HitBest<float>)
        const uint64_t key = hit_key(r1, i);
        bh.k = key < bh.k ? key : bh.k;
        return;
    }
""")
sub("rt_sweep.hpp", """    const bool take = valid & ((root < best_t) | ((root == best_t) & ((int)i > best)));
    best_t = take ? root : best_t;
    best = take ? (int)i : best;""", """    if constexpr (sizeof(T) == 4) {
        const uint64_t key = hit_key(root, i);
        const bool take = valid & (key < bh.k);
        bh.k = take ? key : bh.k;
    } else {
        const bool take = valid & ((root < bh.t) | ((root == bh.t) & ((int)i > bh.i)));
        bh.t = take ? root : bh.t;
        bh.i = take ? (int)i : bh.i;
    }""")
sub("rt_sweep.hpp", """    T best_t = T(INFINITY);          // PackedHitRecords::default, objects.rs:128
    int best = -1;""", """    HitBest<T> bh;                   // PackedHitRecords::default, objects.rs:128""")
sub("rt_sweep.hpp", """hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, best_t, best); };""",
    """hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, bh); };""")
sub("rt_sweep.hpp", """            if constexpr (sizeof(T) == 4) return best_t;
            else return (float)best_t * (1.0f + 0x1.0p-22f);""", """            if constexpr (sizeof(T) == 4) return bh.bt();
            else return (float)bh.bt() * (1.0f + 0x1.0p-22f);""")
sub("rt_sweep.hpp", """    t_out = best_t;
    return best;
}

}  // namespace rt""", """    t_out = bh.bt();
    return bh.bi();
}

}  // namespace rt""")
sub("rt_camera.hpp", """__device__ __forceinline__ void camera_exact(const KP& q, uint32_t sl, bool v, const V3<T>& d, T a, T inv_a, T& best_t,
                                             int& best) {""", """__device__ __forceinline__ void camera_exact(const KP& q, uint32_t sl, bool v, const V3<T>& d, T a, T inv_a,
                                             HitBest<T>& bh) {""")
sub("rt_camera.hpp", """            hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, best_t, best);""",
    """            hit_update<T, root2, SCALAR>(hb, disc, i, a, inv_a, bh);""")
sub("rt_camera.hpp", """    T best_t = T(INFINITY);
    int best = -1;""", """    HitBest<T> bh;""", count=2)
sub("rt_camera.hpp", """camera_exact<T, root2, SCALAR>(q, sl, v, d, a, inv_a, best_t, best);""",
    """camera_exact<T, root2, SCALAR>(q, sl, v, d, a, inv_a, bh);""")
sub("rt_camera.hpp", """    t_out = best_t;
    return best;""", """    t_out = bh.bt();
    return bh.bi();""", count=2)
sub("rt_camera.hpp", """hit_update<T, root2, SCALAR>(hb, disc, cur.i, a, inv_a, best_t, best);""",
    """hit_update<T, root2, SCALAR>(hb, disc, cur.i, a, inv_a, bh);""")
sub("rt_camera.hpp", """camera_exact<T, root2, SCALAR>(q, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, best_t, best);""",
    """camera_exact<T, root2, SCALAR>(q, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, bh);""")
