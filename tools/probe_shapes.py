#!/usr/bin/env python3
"""Kernel time across image sizes, sphere counts and spp (fp32, one GPU; informational).

This probe found the per-pixel atomic bottleneck: 1280x720 took 10.6 ms at 32, 64, 128 and 256 spp
alike (work distribution).  Prints one JSON line per shape."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt
from rt_mi355x import abi, parallel
lib = rt.load_library()
r = rt.GpuRenderer(precision="f32", lib=lib)
for (W, H, nsph, spp) in [(1280, 720, 100, 128), (1280, 720, 100, 512), (1280, 720, 500, 128), (1920, 1080, 100, 512),
                          (1920, 1080, 500, 128), (1920, 1080, 500, 512), (640, 360, 100, 128), (1280, 720, 100, 32), (1280, 720, 100, 64), (1280, 720, 100, 256)]:
    flat = rt.scenes.random_spheres(nsph).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    r.render_flat(50, spp, flat, cam, tile_range=abi.RtTileRange(0, 8, 1, 0, W))
    best = 1e9
    for _ in range(2):
        _, _, st, _ = r.render_flat(50, spp, flat, cam, tile_range=parallel.shard_range(W, H, 1, 0))
        best = min(best, st.kernel_ms)
    print(json.dumps({"W": W, "H": H, "nsph": nsph, "spp": spp, "ms": round(best, 3),
                      "Msps": round(W * H * spp / best / 1e3, 1), "segs": round(st.ray_segments / (W * H * spp), 3)}), flush=True)
