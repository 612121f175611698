#!/usr/bin/env python3
"""Back-to-back shard launches on one GPU, as bench.py issues its steps (HIP events around each launch on the
render stream, no host synchronisation in between): config C's N-way row shards, each rank's shard REPS
times in a row, then all ranks round-robin REPS times.  Separates the launch-to-launch spread of one shard
from the host gaps of tools/shard_spread.py.  Informational.

    python tools/shard_b2b.py [config] [N] [reps]
"""
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 7
prec = os.environ.get("PREC", "f32")
flags = abi.RT_FLAG_F32 if prec == "f32" else 0
lib = rt.load_library()
torch.cuda.init()
stream = torch.cuda.current_stream()
sptr = ctypes.c_void_p(stream.cuda_stream)
ctx = ctypes.c_void_p()
abi.check(lib, lib.rt_context_create(0, ctypes.byref(ctx)))
W, H, n, spp, depth = rt.scenes.CONFIGS[cfg]
flat = rt.scenes.config_scene(cfg).flatten()
abi.check(lib, lib.rt_context_set_scene(ctx, ctypes.byref(flat.abi)))
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
out = torch.empty((H * W * 3,), dtype=torch.uint8, device="cuda")


def launch(tile):
    abi.check(lib, lib.rt_render_async(ctx, ctypes.byref(cam), depth, spp, 0x5EED0001, flags, ctypes.byref(tile),
                                       ctypes.c_void_p(out.data_ptr()), None, sptr), allow=(abi.RT_ERR_RANGE,))


def timed(tiles):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in tiles]
    for t, (a, b) in zip(tiles, evs):
        a.record(stream)
        launch(t)
        b.record(stream)
    torch.cuda.synchronize()
    abi.check(lib, lib.rt_context_collect(ctx, sptr, ctypes.byref(abi.RtStats())), allow=(abi.RT_ERR_RANGE,))
    return [a.elapsed_time(b) for a, b in evs]


whole_tile = abi.RtTileRange(0, 1, H, 0, W)
timed([abi.RtTileRange(0, 64, 1, 0, W)] * 3)   # warm-up
wh = timed([whole_tile] * REPS)
whole = statistics.median(wh)
print(f"{prec} {cfg} whole frame back to back: median {whole:.3f} ms, min {min(wh):.3f}, max {max(wh):.3f}", flush=True)
ideal = whole / N
tiles = [parallel.shard_range(W, H, N, k) for k in range(N)]
print(f" N={N}, ideal {ideal:.3f} ms; each rank {REPS} launches in a row:", flush=True)
per = []
for k in range(N):
    v = timed([tiles[k]] * REPS)
    per.append(v)
    print(f"   rank {k}: median {statistics.median(v):.3f}  min {min(v):.3f}  max {max(v):.3f}  max/min {max(v) / min(v):.3f}  "
          f"{[round(x, 3) for x in v]}", flush=True)
slow = [max(per[k][i] for k in range(N)) for i in range(REPS)]
print(f"   slowest rank per launch index: median {statistics.median(slow):.3f} ({ideal / statistics.median(slow):.3f} of ideal), "
      f"max {max(slow):.3f} ({ideal / max(slow):.3f})", flush=True)
rr = timed(tiles * REPS)
rounds = [rr[i * N:(i + 1) * N] for i in range(REPS)]
slow = [max(r) for r in rounds]
print(f" round-robin over the ranks, {REPS} rounds: slowest shard per round median {statistics.median(slow):.3f} "
      f"({ideal / statistics.median(slow):.3f} of ideal), min {min(slow):.3f}, max {max(slow):.3f}; "
      f"shards summed median {statistics.median([sum(r) for r in rounds]) / whole:.3f} of the whole frame", flush=True)
