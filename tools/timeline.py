#!/usr/bin/env python3
"""Per-wave timeline of one launch (experiment build with RT_EXP_TIMELINE, tools/exp/timeline.patch):
when each wave started, when it found the work exhausted ("drained": no pixel left to open), when it
ended.  Splits a launch into ramp-up, steady state and the drain tail, for the launch shapes of the
multi-GPU bench (config C whole and as 2/4/8-way row shards, a quarter of B).

    make -C rust-ray-tracing_amd exp EXP=-DRT_EXP_TIMELINE
    RT_ALLOW_EXPERIMENT=1 RT_MI355X_LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_exp.so python tools/timeline.py
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

lib = rt.load_library(os.environ.get("RT_MI355X_LIB") or None)
lib.rt_exp_timeline.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int)]
prec = sys.argv[1] if len(sys.argv) > 1 else "f32"
shapes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["C1", "C2", "C4", "C8", "B4"]
r = rt.GpuRenderer(precision=prec, lib=lib)
NW = 16384


def launch(cfg, n, rank=0):
    W, H, nsph, spp, depth = rt.scenes.CONFIGS[cfg]
    flat = rt.scenes.config_scene(cfg).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    tr = parallel.shard_range(W, H, n, rank)
    r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 8, 1, 0, W))   # warm-up (1 row)
    buf = np.zeros((NW, 8), dtype=np.uint64)
    khz = ctypes.c_int()
    abi.check(lib, lib.rt_exp_timeline(r.ctx, buf.ctypes.data, NW, ctypes.byref(khz)))   # clear
    _, _, st, _ = r.render_flat(depth, spp, flat, cam, tile_range=tr)
    abi.check(lib, lib.rt_exp_timeline(r.ctx, buf.ctypes.data, NW, ctypes.byref(khz)))
    return buf, khz.value, st, tr.row_count * W * spp


for s in shapes:
    cfg, n = s[0], int(s[1:])
    buf, khz, st, samples = launch(cfg, n)
    w = buf[buf[:, 2] != 0]
    us = 1e3 / khz   # microseconds per tick
    t0 = w[:, 0].min()
    start = (w[:, 0] - t0) * us
    end = (w[:, 2] - t0) * us
    dr = np.where(w[:, 1] != 0, (w[:, 1].astype(np.int64) - t0) * us, end)
    tail = end - dr
    span = end.max()
    print(f"{prec} {cfg} 1/{n}: kernel {st.kernel_ms:.3f} ms, waves {len(w)}, samples/wave {samples / len(w):.0f}, "
          f"span {span / 1e3:.3f} ms | start p50 {np.median(start):.1f} max {start.max():.1f} us | "
          f"drained p10 {np.percentile(dr, 10) / 1e3:.3f} p50 {np.median(dr) / 1e3:.3f} p90 {np.percentile(dr, 90) / 1e3:.3f} "
          f"ms | end p10 {np.percentile(end, 10) / 1e3:.3f} p50 {np.median(end) / 1e3:.3f} max {span / 1e3:.3f} ms | "
          f"tail (end - drained) p50 {np.median(tail):.1f} p90 {np.percentile(tail, 90):.1f} max {tail.max():.1f} us | "
          f"iters p50 {np.median(w[:, 3]):.0f} | wave-time after drain {1 - dr.mean() / span:.3f}",
          flush=True)
    # time per iteration by phase (median over waves): iterations 0-8, 8-32, 32-128, 128-drained
    cp = [(w[:, 4 + j].astype(np.int64) - t0) * us for j in range(3)]
    its = w[:, 3].astype(np.float64)
    ph = [("0-8", start, cp[0], 8), ("8-32", cp[0], cp[1], 24), ("32-128", cp[1], cp[2], 96)]
    out = []
    for name, a, b, n_it in ph:
        ok = w[:, 4 + [p_[0] for p_ in ph].index(name)] != 0
        if ok.any():
            out.append(f"{name} {np.median((b - a)[ok]) / n_it:.2f}")
    ok = (w[:, 6] != 0) & (w[:, 1] != 0)
    if ok.any():
        out.append(f"128-drained {np.median(((dr - cp[2]) / np.maximum(its - 129, 1))[ok]):.2f}")
    print("    us per iteration by phase (p50 over waves): " + ", ".join(out), flush=True)
