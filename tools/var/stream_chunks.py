# A/B patch: claim streams in runs of M consecutive blocks (argv[2] = M) instead of block by block, so the
# pixels an XCD's workgroups claim one after another stay adjacent in the frame at small block sizes (the
# 8-way shards run G = 2: stream s's consecutive blocks were 8 blocks apart); argv[3] = "perm" also deals the
# workgroups' first blocks (block blockIdx.x, no atomic) so that an XCD's workgroups start on adjacent blocks.
import sys
d = sys.argv[1]; M = int(sys.argv[2]); perm = len(sys.argv) > 3 and sys.argv[3] == "perm"
p = f"{d}/rt_trace.hpp"; s = open(p).read()
old = "                            const uint32_t j = gridDim.x + s + kStreams * atomicAdd(q.counter + kCtrStride * s, 1u);"
new = f"""                            const uint32_t cc = atomicAdd(q.counter + kCtrStride * s, 1u);
                            const uint32_t j = gridDim.x + ((cc / {M}u) * kStreams + s) * {M}u + cc % {M}u;"""
assert old in s; s = s.replace(old, new)
if perm:
    old = "        const bool got = guided_block(q.n_items, max(1u, kTMul * gridDim.x), q.blk_g, blockIdx.x, b0, b1);"
    new = """        const uint32_t b0i = gridDim.x % kStreams == 0u ? (blockIdx.x % kStreams) * (gridDim.x / kStreams) + blockIdx.x / kStreams
                                                        : blockIdx.x;
        const bool got = guided_block(q.n_items, max(1u, kTMul * gridDim.x), q.blk_g, b0i, b0, b1);"""
    assert old in s; s = s.replace(old, new)
open(p, "w").write(s)
