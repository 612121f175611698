#!/usr/bin/env python3
"""The fixed cost of one launch: config C's rows every 8th row (an 8-way rank's shard shape),
the first R of them for R = 1 .. 135, kernel time by HIP events (median of REPS); a least-squares line
time = a + b * rows over the larger launches gives the per-launch intercept a against the per-row cost b.

    python tools/launch_fixed_cost.py [reps]
"""
import os
import statistics
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
prec = os.environ.get("PREC", "f32")
r = rt.GpuRenderer(precision=prec, lib=rt.load_library())
W, H, n, spp, depth = rt.scenes.CONFIGS["C"]
flat = rt.scenes.config_scene("C").flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 8, 1, 0, W))   # warm-up
xs, ys = [], []
for rows in (1, 2, 4, 8, 16, 32, 48, 64, 96, 135):
    t = statistics.median(r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 8, rows, 0, W))[2].kernel_ms
                          for _ in range(REPS))
    print(f"{prec} rows {rows:4d} (every 8th, {rows * W} px): {t:.3f} ms", flush=True)
    xs.append(rows); ys.append(t)
sel = [i for i, x in enumerate(xs) if x >= 16]
b, a = np.polyfit([xs[i] for i in sel], [ys[i] for i in sel], 1)
print(f"fit over >= 16 rows: {a:.3f} ms per launch + {b * 1e3:.2f} us per row ({b * 135:.3f} ms for the 135-row shard)")
