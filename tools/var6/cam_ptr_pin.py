"""A/B patch (round 6): the camera batches' exact tests read the camera-origin table and the slot -> scene index table
through two pointers loaded once per batch and pinned in SGPRs, instead of reloading both pointers from the kernel
arguments at every listed sphere (two dependent scalar round trips per listed sphere)."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_camera.hpp", """template <typename T, bool root2, bool SCALAR, typename KP>
__device__ __forceinline__ void camera_exact(const KP& q, uint32_t sl, bool v, const V3<T>& d, T a, T inv_a,
                                             HitBest<T>& bh) {
    KSTAT(2);
    constexpr bool kBothRoots = root2 || SCALAR;
    cptr<T> cxt = (cptr<T>)__builtin_assume_aligned(q.camx, 16);
    cptr<uint32_t> ri = (cptr<uint32_t>)q.ridx;""", """// cxt, ri: the camera-origin table and the slot -> scene index table, loaded once by the caller (CamPtrs).
template <typename T> struct CamPtrs {
    cptr<T> cxt;
    cptr<uint32_t> ri;
};
template <typename T, typename KP> __device__ __forceinline__ CamPtrs<T> cam_ptrs(const KP& q) {
    CamPtrs<T> c{(cptr<T>)__builtin_assume_aligned(q.camx, 16), (cptr<uint32_t>)q.ridx};
    asm volatile("" : "+s"(c.cxt), "+s"(c.ri));   // pinned in SGPRs: not reloaded from the kernel arguments
    return c;
}
template <typename T, bool root2, bool SCALAR>
__device__ __forceinline__ void camera_exact(const CamPtrs<T>& cp, uint32_t sl, bool v, const V3<T>& d, T a, T inv_a,
                                             HitBest<T>& bh) {
    KSTAT(2);
    constexpr bool kBothRoots = root2 || SCALAR;
    cptr<T> cxt = cp.cxt;
    cptr<uint32_t> ri = cp.ri;""")
sub("rt_camera.hpp", """    uint32_t n_cx = 0;   // executed-work counts (work_add below)
    const uint32_t n_cone = cone_walk<MEGA>(q, ax, ay, az, S, Cc, all, xw0, kw0, [&](uint32_t sl) {
        ++n_cx;
        camera_exact<T, root2, SCALAR>(q, sl, v, d, a, inv_a, bh);""", """    uint32_t n_cx = 0;   // executed-work counts (work_add below)
    const CamPtrs<T> cp = cam_ptrs<T>(q);
    const uint32_t n_cone = cone_walk<MEGA>(q, ax, ay, az, S, Cc, all, xw0, kw0, [&](uint32_t sl) {
        ++n_cx;
        camera_exact<T, root2, SCALAR>(cp, sl, v, d, a, inv_a, bh);""")
sub("rt_camera.hpp", """    } else {
        for (; smask != 0u; smask &= smask - 1u) {
            const uint16_t* l = lists[__builtin_ctz(smask)];
            const uint32_t n = __builtin_amdgcn_readfirstlane(l[0]);
            for (uint32_t j = 0; j < n; ++j) {
                ++n_cx;
                camera_exact<T, root2, SCALAR>(q, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, bh);""",
    """    } else {
        const CamPtrs<T> cp = cam_ptrs<T>(q);
        for (; smask != 0u; smask &= smask - 1u) {
            const uint16_t* l = lists[__builtin_ctz(smask)];
            const uint32_t n = __builtin_amdgcn_readfirstlane(l[0]);
            for (uint32_t j = 0; j < n; ++j) {
                ++n_cx;
                camera_exact<T, root2, SCALAR>(cp, __builtin_amdgcn_readfirstlane(l[1u + j]), v, d, a, inv_a, bh);""")
