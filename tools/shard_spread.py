#!/usr/bin/env python3
"""Spread of the N-way row shards' kernel times on one GPU: config C (or another
config) rendered as each rank's shard of an N-way split, REPS times round-robin over the ranks, so every
rank's shard is timed REPS times on the same box.  Prints per rank the median and max of its launches, then
per repetition the slowest shard (the N-GPU frame time) against 1/N of the whole frame's median: median,
min and max of that ratio.  Informational.

    python tools/shard_spread.py [config] [N,...] [reps]
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
NS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8").split(",")]
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 7
prec = os.environ.get("PREC", "f32")
lib = rt.load_library()
r = rt.GpuRenderer(precision=prec, lib=lib)
W, H, n, spp, depth = rt.scenes.CONFIGS[cfg]
flat = rt.scenes.config_scene(cfg).flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
for k in ("RT_WAVES", "RT_BLOCK_G"):
    os.environ.pop(k, None)
wh = [r.render_flat(depth, spp, flat, cam)[2].kernel_ms for _ in range(REPS)]
whole = statistics.median(wh)
print(f"{prec} {cfg} whole frame: median {whole:.3f} ms, min {min(wh):.3f}, max {max(wh):.3f} over {REPS}", flush=True)
for N in NS:
    t = [[0.0] * N for _ in range(REPS)]
    kid = set()
    for i in range(REPS):
        for k in range(N):
            st = r.render_flat(depth, spp, flat, cam, tile_range=parallel.shard_range(W, H, N, k))[2]
            t[i][k] = st.kernel_ms
            kid.add(abi.kernel_name(st.kernel_id))
    ideal = whole / N
    print(f" N={N} (ideal {ideal:.3f} ms, kernel {', '.join(sorted(kid))}):", flush=True)
    for k in range(N):
        v = [t[i][k] for i in range(REPS)]
        print(f"   rank {k}: median {statistics.median(v):.3f}  min {min(v):.3f}  max {max(v):.3f}  "
              f"max/min {max(v) / min(v):.3f}", flush=True)
    slow = [max(t[i]) for i in range(REPS)]
    eff = [ideal / s for s in slow]
    print(f"   slowest shard per repetition: {[round(s, 3) for s in slow]}", flush=True)
    print(f"   of ideal: median {statistics.median(eff):.3f}  min {min(eff):.3f}  max {max(eff):.3f}; "
          f"slowest max/min {max(slow) / min(slow):.3f}; shards summed (median rep) "
          f"{statistics.median([sum(t[i]) for i in range(REPS)]) / whole:.3f} of the whole frame", flush=True)
