#!/usr/bin/env python3
"""Launch-to-launch jitter of one launch shape on one GPU: config C's whole frame and
rank 0's shard of an N-way row split, each REPS times back to back; prints every kernel time (HIP events
around the launch) and the distribution.  Separates a spike that every launch shape shows (the box) from
one that only small launches show (the drain).

    python tools/launch_jitter.py [N] [reps]
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 40
prec = os.environ.get("PREC", "f32")
r = rt.GpuRenderer(precision=prec, lib=rt.load_library())
W, H, n, spp, depth = rt.scenes.CONFIGS["C"]
flat = rt.scenes.config_scene("C").flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
for label, tr in (("whole", None), (f"shard 0/{N}", parallel.shard_range(W, H, N, 0)),
                  (f"shard {N - 1}/{N}", parallel.shard_range(W, H, N, N - 1))):
    t = [r.render_flat(depth, spp, flat, cam, tile_range=tr)[2].kernel_ms for _ in range(REPS)]
    med = statistics.median(t)
    print(f"{prec} {label}: median {med:.3f} ms  min {min(t):.3f}  max {max(t):.3f}  "
          f"p90 {sorted(t)[int(0.9 * len(t))]:.3f}  launches over 1.05x median: {sum(v > 1.05 * med for v in t)}/{len(t)}",
          flush=True)
    print("   " + " ".join(f"{v:.3f}" for v in t), flush=True)
