#!/usr/bin/env python3
"""Work and time of the N-way row shards of a config against the whole frame, on one GPU (round 6): the
in-kernel work counters (rt_stats: box / filter groups, exact tests, camera exact tests, cone tests, ray
segments) summed over the N shard launches, each over the whole frame's, and the same for the kernel time.
Work ratio ~1 with time ratio > 1: the shards lose to ramp, drain or occupancy; work ratio > 1: to coherence.

    python tools/shard_work.py [config] [N,...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
NS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,8").split(",")]
r = rt.GpuRenderer(precision=os.environ.get("PREC", "f32"), lib=rt.load_library())
W, H, n, spp, depth = rt.scenes.CONFIGS[cfg]
flat = rt.scenes.config_scene(cfg).flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
K = ("kernel_ms", "ray_segments", "lane_slots", "box_groups", "filter_groups", "exact_tests", "camera_exact_tests", "cone_tests")


def run(tr=None):
    st = r.render_flat(depth, spp, flat, cam, tile_range=tr)[2]
    return {k: float(getattr(st, k)) for k in K}


run(abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
whole = [run() for _ in range(3)]
wm = {k: sorted(w[k] for w in whole)[1] for k in K}
print(f"{cfg} whole frame:", {k: round(v, 3) if k == "kernel_ms" else int(v) for k, v in wm.items()}, flush=True)
for N in NS:
    tot = {k: 0.0 for k in K}
    mx = 0.0
    for rank in range(N):
        s = run(parallel.shard_range(W, H, N, rank))
        mx = max(mx, s["kernel_ms"])
        for k in K:
            tot[k] += s[k]
    print(f" N={N}: summed / whole:", {k: round(tot[k] / wm[k], 4) if wm[k] else None for k in K},
          f"slowest {mx:.3f} ms (ideal {wm['kernel_ms'] / N:.3f})", flush=True)
