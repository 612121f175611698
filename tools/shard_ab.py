#!/usr/bin/env python3
"""Strong-scaling A/B on one GPU, same process: config C's N-way row shards (every rank's shard; the
slowest sets the N-GPU frame time) at each (waves per SIMD, largest block G) combination, against the
whole frame at the defaults.  RT_WAVES and RT_BLOCK_G are read per launch.  Informational: the evidence
for the host's per-launch W and G choice.

    python tools/shard_ab.py [N] [waves,...] [G,...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
WAVES = sys.argv[2].split(",") if len(sys.argv) > 2 else ["5", "6"]
GS = sys.argv[3].split(",") if len(sys.argv) > 3 else ["2", "4", "8", "16"]
REPS = 2
prec = os.environ.get("PREC", "f32")
lib = rt.load_library()
r = rt.GpuRenderer(precision=prec, lib=lib)
W, H, n, spp, depth = rt.scenes.CONFIGS["C"]
flat = rt.scenes.config_scene("C").flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
for k in ("RT_WAVES", "RT_BLOCK_G"):
    os.environ.pop(k, None)
whole = min(r.render_flat(depth, spp, flat, cam)[2].kernel_ms for _ in range(REPS))
print(f"{prec} C whole frame (defaults): {whole:.3f} ms; ideal 1/{N}: {whole / N:.3f} ms", flush=True)
res = {}
for _ in range(REPS):
    for w in WAVES:
        for g in GS + ["auto"]:
            os.environ["RT_WAVES"] = w
            if g == "auto":
                os.environ.pop("RT_BLOCK_G", None)
            else:
                os.environ["RT_BLOCK_G"] = g
            ms = [r.render_flat(depth, spp, flat, cam, tile_range=parallel.shard_range(W, H, N, k))[2].kernel_ms
                  for k in range(N)]
            res.setdefault((w, g), []).append(max(ms))
for (w, g), v in sorted(res.items()):
    m = min(v)
    print(f"  W{w} G={g:>4}: slowest shard {m:.3f} ms  ({whole / N / m:.3f} of ideal)  runs {[round(x, 3) for x in v]}",
          flush=True)
