#!/usr/bin/env python3
"""Claim-block size of N-way row shards, same process (round 6): the whole frame at the default block size,
then each rank's shard under every RT_BLOCK_G in the list (the diagnostic override of the largest claim
block, read at each launch; "d" = the default), REPS rounds interleaved, so every setting sees the same
box.  Prints per setting the median over rounds of the slowest shard against 1/N of the whole frame.

    python tools/shard_g_ab.py [config] [N] [reps] [G,...]
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 7
GS = (sys.argv[4] if len(sys.argv) > 4 else "d,1,2").split(",")
r = rt.GpuRenderer(precision=os.environ.get("PREC", "f32"), lib=rt.load_library())
W, H, n, spp, depth = rt.scenes.CONFIGS[cfg]
flat = rt.scenes.config_scene(cfg).flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)


def kms(g, tr=None):
    if g == "d":
        os.environ.pop("RT_BLOCK_G", None)
    else:
        os.environ["RT_BLOCK_G"] = g
    return r.render_flat(depth, spp, flat, cam, tile_range=tr)[2].kernel_ms


kms("d", abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
whole = statistics.median(kms("d") for _ in range(5))
print(f"{cfg} N={N} whole frame {whole:.3f} ms (ideal shard {whole / N:.3f})", flush=True)
slow = {g: [] for g in GS}
summ = {g: [] for g in GS}
for i in range(REPS):
    for g in GS:
        t = [kms(g, parallel.shard_range(W, H, N, k)) for k in range(N)]
        slow[g].append(max(t))
        summ[g].append(sum(t))
for g in GS:
    m = statistics.median(slow[g])
    print(f"  G={g:>2}: slowest shard median {m:.3f} ms = {whole / N / m:.3f} of ideal (min {whole / N / max(slow[g]):.3f}, "
          f"max {whole / N / min(slow[g]):.3f}); shards summed {statistics.median(summ[g]) / whole:.3f} of the whole", flush=True)
