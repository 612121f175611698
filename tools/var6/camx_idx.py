"""A/B patch (round 6): the fp32 camera-origin record carries its slot's scene index: {ocx, ocy, ocz, c, index, pad}
(32 bytes, one s_load_dwordx8), so a camera batch's exact test reads one record per listed sphere instead of the
record and a separate slot -> index table (two cache lines, two pointers from the kernel arguments).  fp64 keeps its
16-byte... 32-byte records and the table."""
import sys
d = sys.argv[1]


def sub(path, old, new, count=1):
    p = f"{d}/{path}"
    s = open(p).read()
    assert s.count(old) == count, (path, old[:70], s.count(old))
    open(p, "w").write(s.replace(old, new))


sub("rt_camera.hpp", """    cptr<T> cxt = (cptr<T>)__builtin_assume_aligned(q.camx, 16);
    cptr<uint32_t> ri = (cptr<uint32_t>)q.ridx;
    const uint32_t i = ri[sl];
    const T ocx = cxt[4 * sl], ocy = cxt[4 * sl + 1], ocz = cxt[4 * sl + 2], c = cxt[4 * sl + 3];""",
    """    // fp32: {ocx, ocy, ocz, c, scene index, pad} per slot (one 32-byte record); fp64: {ocx, ocy, ocz, c} and
    // the slot -> index table
    constexpr uint32_t CS = sizeof(T) == 4 ? 8u : 4u;
    cptr<T> cxt = (cptr<T>)__builtin_assume_aligned(q.camx, 16);
    uint32_t i;
    if constexpr (sizeof(T) == 4) i = __float_as_uint(cxt[CS * sl + 4]);
    else i = ((cptr<uint32_t>)q.ridx)[sl];
    const T ocx = cxt[CS * sl], ocy = cxt[CS * sl + 1], ocz = cxt[CS * sl + 2], c = cxt[CS * sl + 3];""")
sub("rt_camera.hpp", """        camx[4 * i] = ex; camx[4 * i + 1] = ey; camx[4 * i + 2] = ez; camx[4 * i + 3] = ec;""",
    """        constexpr uint32_t CS = sizeof(T) == 4 ? 8u : 4u;   // fp32 records carry the scene index (camera_exact)
        camx[CS * i] = ex; camx[CS * i + 1] = ey; camx[CS * i + 2] = ez; camx[CS * i + 3] = ec;
        if constexpr (sizeof(T) == 4) {
            ((uint32_t*)camx)[CS * i + 4] = sj;
            camx[CS * i + 5] = T(0); camx[CS * i + 6] = T(0); camx[CS * i + 7] = T(0);
        }""")
sub("rt_kernel.hip", """    HIPCHK(hipMalloc(&c->camx32, (size_t)4 * c->n_cslots * sizeof(float)));""",
    """    HIPCHK(hipMalloc(&c->camx32, (size_t)8 * c->n_cslots * sizeof(float)));   // + the scene index (camera_exact)""")
