#!/usr/bin/env python3
"""Time every BASELINE config on ONE GPU (informational; bench.py is the judged line).

D and E are full 3840x2160 frames meant for 8 GPUs; here a row-strided subset (every 8th row, i.e.
exactly one rank's shard of the 8-GPU partition) is timed and reported per GPU.
Prints one JSON line per (config, precision)."""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402


def run(config, precision, stride):
    lib = rt.load_library()
    W, H, n_sph, spp, depth = rt.scenes.CONFIGS[config]
    flat = rt.scenes.config_scene(config).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    r = rt.GpuRenderer(precision=precision, lib=lib)
    tile = parallel.shard_range(W, H, stride, 0)
    r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, stride, 1, 0, W))  # warm-up (1 row)
    t0 = time.perf_counter()
    rgb, _, st, rc = r.render_flat(depth, spp, flat, cam, tile_range=tile)
    wall = time.perf_counter() - t0
    r.close()
    samples = tile.row_count * W * spp
    return {"config": config, "precision": precision, "rows": f"every {stride} row(s)", "pixels": tile.row_count * W,
            "spp": spp, "spheres": n_sph, "kernel_ms": round(st.kernel_ms, 2),
            "msamples_per_s_per_gpu": round(samples / (st.kernel_ms / 1e3) / 1e6, 1),
            "brute_force_equiv_tflops": round(17 * n_sph * st.ray_segments / (st.kernel_ms / 1e3) / 1e12, 2),
            "roofline_frac": round(sum(f / (pk * 1e12) for f, pk in zip(abi.executed_flop(st, precision), (157.3, 78.6)))
                                   / (st.kernel_ms / 1e3), 4),
            "segments_per_sample": round(st.ray_segments / samples, 4),
            "lane_utilisation": round(rt.abi.lane_utilisation(st), 4), "wall_s": round(wall, 2)}


if __name__ == "__main__":
    for cfg, stride in (("B", 1), ("C", 1), ("D", 8), ("E", 8)):
        for prec in ("f32", "f64"):
            print(json.dumps(run(cfg, prec, stride)), flush=True)
