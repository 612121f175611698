# Timing-only A/B patch (results differ from the oracle): fp32 draws from Philox2x32-10 (one 32x32->64
# multiply per round instead of two) keyed (pixel, sample | stream code << 20) with key seed_lo ^ seed_hi.
import sys
d = sys.argv[1]
p = f"{d}/rt_device.hpp"; s = open(p).read()
old = "// Uniform [0,1): f64 from 53 bits of (a,b) / (c,d); f32 from 24 bits of a / b."
new = '''// Philox2x32-10 (Random123): counter (pixel, sample | code << 20), key seed_lo ^ seed_hi; code 0 camera,
// 1 + i disk try i, 257 + k scatter at bounce k.  fp32 draws (24 bits of each output word).
__device__ __forceinline__ U4 philox2(uint32_t c0, uint32_t c1, uint32_t k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p = (uint64_t)0xD256D193u * c0;
        c0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p >> 32), c1, k, 0x96);
        c1 = (uint32_t)p;
        k += 0x9E3779B9u;
    }
    return U4{c0, c1, 0u, 0u};
}
template <typename T> __device__ __forceinline__ U4 draw(uint32_t sid, uint32_t pix, uint32_t kk, uint32_t stream, uint32_t k0, uint32_t k1) {
    if constexpr (sizeof(T) == 4) {
        const uint32_t code = stream == 0u ? 0u : stream == 1u ? 1u + kk : 257u + kk;
        return philox2(pix, sid | (code << 20), k0 ^ k1);
    } else {
        return philox(sid, pix, kk, stream, k0, k1);
    }
}
''' + old
assert old in s; s = s.replace(old, new); open(p, "w").write(s)
for f, olds in (("rt_camera.hpp", ["return philox(sid, pix, cam ? 0u : k, cam ? 0u : 2u, q0.k0, q0.k1);", "const U4 qq = philox(sid, pix, i, 1u, k0, k1);"]),
                ("rt_finish.hpp", ["const U4 r = philox(qq, pix, 0u, 0u, qc.k0, qc.k1);"]),
                ("rt_trace.hpp", ["return philox(bsid, bpix, 0u, 0u, q0.k0, q0.k1);"])):
    p = f"{d}/{f}"; s = open(p).read()
    for o in olds:
        assert o in s, o
        s = s.replace(o, o.replace("philox(", "draw<T>("))
    open(p, "w").write(s)
