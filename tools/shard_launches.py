#!/usr/bin/env python3
"""One warm-up, one whole frame of config C, then its N row-interleaved shards, each launch synchronised:
the program tools/shard_pmc.sh runs under rocprofv3 --pmc, so per-dispatch counters of the whole frame
and of the shards (which sum to the same samples) can be compared.   python tools/shard_launches.py [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
r = rt.GpuRenderer(precision=os.environ.get("PREC", "f32"), lib=rt.load_library())
W, H, n, spp, depth = rt.scenes.CONFIGS["C"]
flat = rt.scenes.config_scene("C").flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 64, 1, 0, W))   # warm-up
ms = [r.render_flat(depth, spp, flat, cam)[2].kernel_ms]
ms += [r.render_flat(depth, spp, flat, cam, tile_range=parallel.shard_range(W, H, N, k))[2].kernel_ms for k in range(N)]
print("kernel_ms whole", round(ms[0], 3), "shards", [round(x, 3) for x in ms[1:]], "sum", round(sum(ms[1:]), 3))
