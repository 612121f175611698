#!/usr/bin/env python3
"""Frame overlap probe (round 6): REPS back-to-back launches of a config's whole frame or one N-way row shard,
(a) all on one context and stream, each waiting for the one before (the bench's loop), and (b) alternating
between two contexts on two HIP streams, so launch k+1's workgroups start on the CUs that launch k's drain
frees.  Wall time per launch, same process, interleaved rounds.  Informational.

    python tools/overlap_probe.py [config] [N,...] [reps] [rounds]
"""
import ctypes
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
import torch  # noqa: E402
import rt_mi355x as rt  # noqa: E402
from rt_mi355x import abi, parallel  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
NS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 20
ROUNDS = int(sys.argv[4]) if len(sys.argv) > 4 else 3
flags = abi.RT_FLAG_F32 if os.environ.get("PREC", "f32") == "f32" else 0
lib = rt.load_library()
W, H, n, spp, depth = rt.scenes.CONFIGS[cfg]
flat = rt.scenes.config_scene(cfg).flatten()
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
torch.cuda.set_device(0)
ctxs = []
for _ in range(2):
    c = ctypes.c_void_p()
    abi.check(lib, lib.rt_context_create(0, ctypes.byref(c)))
    abi.check(lib, lib.rt_context_set_scene(c, ctypes.byref(flat.abi)))
    ctxs.append(c)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
bufs = [torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]


def run(N, two):
    tr = parallel.shard_range(W, H, N, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(REPS):
        i = k % 2 if two else 0
        s = streams[i]
        abi.check(lib, lib.rt_render_async(ctxs[i], ctypes.byref(cam), depth, spp, 0x5EED, flags, ctypes.byref(tr),
                                           ctypes.c_void_p(bufs[k % 2].data_ptr()), None, ctypes.c_void_p(s.cuda_stream)))
        if two:   # launch k+1 may start only after launch k-1 (same context) is done: its stream is that context's
            pass
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / REPS * 1e3


for N in NS:
    run(N, False)
    run(N, True)
    a, b = [], []
    for _ in range(ROUNDS):
        a.append(run(N, False))
        b.append(run(N, True))
    ma, mb = statistics.median(a), statistics.median(b)
    print(f"{cfg} N={N} (shard 0): one stream {ma:.3f} ms/launch, two contexts/streams {mb:.3f} ms/launch "
          f"({ma / mb:.4f}x)", flush=True)
    st = abi.RtStats()
    for c in ctxs:
        abi.check(lib, lib.rt_context_collect(c, None, ctypes.byref(st)), allow=(abi.RT_ERR_RANGE,))
for c in ctxs:
    lib.rt_context_destroy(c)
