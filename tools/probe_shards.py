#!/usr/bin/env python3
"""Strong-scaling rehearsal on one GPU: config C rendered as each rank's row shard of an N-way split
(N = 1, 2, 4, 8), kernel time per shard.  The slowest shard sets the N-GPU frame time; `sum` is the
shards' total (ideal: the whole frame's time).  Informational; DESIGN.md §4, work distribution."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

lib = rt.load_library()
for prec in ("f32", "f64"):
    r = rt.GpuRenderer(precision=prec, lib=lib)
    W, H, n, spp, depth = rt.scenes.CONFIGS["C"]
    flat = rt.scenes.config_scene("C").flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 8, 1, 0, W))   # warm-up (1 row)
    out = []
    t1 = None
    for N in (1, 2, 4, 8):
        ms = []
        for rank in range(N):
            _, _, st, _ = r.render_flat(depth, spp, flat, cam, tile_range=parallel.shard_range(W, H, N, rank))
            ms.append(st.kernel_ms)
        t1 = t1 or ms[0]
        out.append(f"N={N}: max {max(ms):.2f} ms (ideal {t1 / N:.2f}), mean/max {sum(ms) / N / max(ms):.3f}, "
                   f"sum {sum(ms):.1f}")
    print(prec, " | ".join(out), flush=True)
