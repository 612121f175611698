#!/usr/bin/env python3
"""Occupancy A/B on one GPU, same process: every fp32 launch shape the multi-GPU bench produces (config C
whole and as each rank's shard of a 2/4/8/16-way split, B's 4- and 8-way shards, one 8-way shard of D, 8- and 32-way shards of E),
rendered at RT_WAVES=5 and 6 alternately (RT_WAVES is read per launch).  For an N-way split the slowest
shard sets the frame time, so each line reports max over the ranks' kernel times.  Informational:
the evidence for kWavesF32 / kWavesMegaF32."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

WAVES = sys.argv[1].split(",") if len(sys.argv) > 1 else ["5", "6"]
REPS = 2
lib = rt.load_library()
r = rt.GpuRenderer(precision="f32", lib=lib)
cases = [("C", 1, None), ("C", 2, None), ("C", 4, None), ("C", 8, None), ("C", 16, None), ("B", 4, None),
         ("B", 8, None), ("D", 8, [0]), ("E", 8, [0]), ("E", 32, [0, 16])]
for cfg, N, ranks in cases:
    W, H, n, spp, depth = rt.scenes.CONFIGS[cfg]
    flat = rt.scenes.config_scene(cfg).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
    ranks = ranks if ranks is not None else list(range(N))
    res = {w: [] for w in WAVES}
    for _ in range(REPS):
        for w in WAVES:
            os.environ["RT_WAVES"] = w
            ms = [r.render_flat(depth, spp, flat, cam, tile_range=parallel.shard_range(W, H, N, k))[2].kernel_ms
                  for k in ranks]
            res[w].append(max(ms))
    os.environ.pop("RT_WAVES", None)
    line = " | ".join(f"W{w}: {min(v):8.2f} ms" for w, v in res.items())
    base = min(res[WAVES[0]])
    gains = " ".join(f"W{w}/W{WAVES[0]} {base / min(v):.3f}" for w, v in res.items() if w != WAVES[0])
    print(f"{cfg} {N:2d}-way (ranks {ranks if len(ranks) < N else 'all'}): {line}   {gains}", flush=True)
