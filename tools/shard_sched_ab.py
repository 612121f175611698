#!/usr/bin/env python3
"""One variant of the work distribution (the library RT_MI355X_LIB names, RT_BLOCK_G / RT_WAVES from the
environment): config C's whole frame and its N-way row shards, round-robin over the ranks, REPS times;
prints one JSON line (medians, the slowest shard per repetition against 1/N of the whole frame).  Run
several variants alternately on one box (tools/shard_sched_ab.sh) so clock differences cancel.

    python tools/shard_sched_ab.py NAME [N] [reps]
"""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

name = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 5
prec = os.environ.get("PREC", "f32")
r = rt.GpuRenderer(precision=prec, lib=rt.load_library())
W, H, n, spp, depth = rt.scenes.CONFIGS["C"]
flat = rt.scenes.config_scene("C").flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
wh = [r.render_flat(depth, spp, flat, cam)[2].kernel_ms for _ in range(REPS)]
whole = statistics.median(wh)
t = [[r.render_flat(depth, spp, flat, cam, tile_range=parallel.shard_range(W, H, N, k))[2].kernel_ms for k in range(N)]
     for _ in range(REPS)]
slow = [max(x) for x in t]
print(json.dumps({"name": name, "prec": prec, "N": N, "whole_ms": round(whole, 3),
                  "shard_median_ms": round(statistics.median([v for x in t for v in x]), 3),
                  "slowest": [round(v, 3) for v in slow],
                  "of_ideal_median": round(statistics.median([whole / N / v for v in slow]), 4),
                  "of_whole_frame_med": round(whole / N / statistics.median(slow), 4),
                  "slowest_max_min": round(max(slow) / min(slow), 4),
                  "summed_over_whole": round(statistics.median([sum(x) for x in t]) / whole, 4)}), flush=True)
