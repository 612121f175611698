#!/usr/bin/env python3
"""Where an N-way shard of config C loses against 1/N of the whole frame, on one GPU, same process:
for the row-interleaved shards bench.py uses (parallel.shard_range) and for contiguous row bands,
print the slowest, mean and summed kernel time of the N launches.  sum/whole > 1 is throughput lost
per launch (ramp, tail, locality); max/mean > 1 is imbalance between shards.  Informational.

    python tools/shard_layout.py [N] [reps]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
prec = os.environ.get("PREC", "f32")
r = rt.GpuRenderer(precision=prec, lib=rt.load_library())
W, H, n, spp, depth = rt.scenes.CONFIGS["C"]
flat = rt.scenes.config_scene("C").flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
r.render_flat(depth, spp, flat, cam, tile_range=abi.RtTileRange(0, 64, 1, 0, W))   # warm-up


def kms(tr=None):
    return r.render_flat(depth, spp, flat, cam, tile_range=tr)[2].kernel_ms


def band(k):
    b = (H + N - 1) // N
    lo = k * b
    return abi.RtTileRange(lo, 1, max(0, min(H, lo + b) - lo), 0, W)


layouts = {"interleaved": lambda k: parallel.shard_range(W, H, N, k), "bands": band}
whole = []
res = {name: [] for name in layouts}
for _ in range(REPS):
    whole.append(kms())
    for name, f in layouts.items():
        res[name].append([kms(f(k)) for k in range(N)])
wm = min(whole)
print(f"{prec} C whole frame: {wm:.3f} ms (runs {[round(x, 3) for x in whole]}); 1/{N} = {wm / N:.3f} ms", flush=True)
for name, runs in res.items():
    best = min(runs, key=max)
    mx, mean, tot = max(best), sum(best) / N, sum(best)
    print(f"  {name:12s} slowest {mx:.3f} ms ({wm / N / mx:.3f} of ideal)  mean {mean:.3f}  sum/whole {tot / wm:.3f}"
          f"  max/mean {mx / mean:.3f}  shards {[round(x, 3) for x in best]}", flush=True)

# The same N interleaved shards queued back to back (one collect: kernel_ms spans all N launches, no
# host gap between them), and the whole frame at each largest block G: separates per-launch cost and
# clock ramp after an idle gap from the claim rate of small blocks.
import ctypes  # noqa: E402

lib = r.lib
buf = ctypes.c_void_p()   # one whole-frame output buffer; each launch writes its compact shard at its start


def queued(ranges):
    for tr in ranges:
        rt.abi.check(lib, lib.rt_render_async(r.ctx, ctypes.byref(cam), depth, spp, r.seed, r.flags, ctypes.byref(tr),
                                              buf, None, None))
    st = rt.abi.RtStats()
    lib.rt_context_collect(r.ctx, None, ctypes.byref(st))
    last[0] = st
    return st.kernel_ms


last = [None]
WORK = ("ray_segments", "lane_slots", "bounce_iters", "box_groups", "filter_groups", "exact_tests", "cone_tests",
        "camera_exact_tests")


def per_sample(st):
    return {k: round(getattr(st, k) / st.samples, 4) for k in WORK}


full = abi.RtTileRange(0, 1, H, 0, W)
rt.abi.check(lib, lib.rt_device_alloc(r.ctx, W * H * 3, ctypes.byref(buf)))
q8 = min(queued([parallel.shard_range(W, H, N, k) for k in range(N)]) for _ in range(REPS))
w8 = per_sample(last[0])
q1 = min(queued([full]) for _ in range(REPS))
w1 = per_sample(last[0])
print(f"  work per sample, whole frame: {w1}\n  work per sample, {N} shards:   {w8}", flush=True)
qq = min(queued([full, full]) for _ in range(REPS)) - q1
print(f"  queued: {N} interleaved shards back to back {q8:.3f} ms ({q8 / wm:.3f} of the whole frame); whole frame "
      f"alone {q1:.3f}, a second whole frame queued behind it {qq:.3f}", flush=True)
for g in ("1", "2", "4", "8", "16"):
    os.environ["RT_BLOCK_G"] = g
    print(f"  whole frame at G={g:>2}: {min(queued([full]) for _ in range(REPS)):.3f} ms", flush=True)
os.environ.pop("RT_BLOCK_G", None)
