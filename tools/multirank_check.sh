#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: (1) torchrun world 1 over nccl (RCCL init with the
# library loaded), (2) 2 ranks sharing the GPU over gloo, (3) plain `bench.py --gpus 2` (it launches
# its own 2 ranks, as the driver runs it) over gloo; compare the assembled images bit-for-bit with a
# plain single-process run; (4) the dynamic schedule (--schedule dynamic: ranks pull chunks from the
# store's queue, RCCL/gloo reduce) at world 1 over nccl and world 2 over gloo; (5) round 4: plain
# `bench.py --gpus 8` on config C, the SCALE run's workload (8 self-launched ranks sharing the one GPU over
# gloo), static and dynamic, against a single-process frame of C.
# Usage: bash tools/multirank_check.sh <outdir>
set -eu
OUT=${1:-gpurun_out/multirank}
mkdir -p "$OUT"
ARGS="--config B --steps 2 --warmup 1 --cpu-seconds 0 --other-precision 0"
RT_BENCH_SAVE=$OUT/single.npy timeout -k 10 200 python3 bench.py $ARGS > "$OUT/single.log" 2>&1
RT_BENCH_SAVE=$OUT/nccl1.npy timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 $ARGS > "$OUT/nccl1.log" 2>&1
RT_BENCH_BACKEND=gloo RT_BENCH_SAVE=$OUT/gloo2.npy timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 $ARGS > "$OUT/gloo2.log" 2>&1
RT_BENCH_BACKEND=gloo RT_BENCH_SAVE=$OUT/self2.npy timeout -k 10 300 python3 bench.py --gpus 2 $ARGS > "$OUT/self2.log" 2>&1
RT_BENCH_SAVE=$OUT/dyn1.npy timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --schedule dynamic $ARGS > "$OUT/dyn1.log" 2>&1
RT_BENCH_BACKEND=gloo RT_BENCH_SAVE=$OUT/dyn2.npy timeout -k 10 300 python3 bench.py --gpus 2 --schedule dynamic \
    $ARGS > "$OUT/dyn2.log" 2>&1
ARGC="--config C --steps 2 --warmup 1 --cpu-seconds 0 --other-precision 0"
RT_BENCH_SAVE=$OUT/singleC.npy timeout -k 10 200 python3 bench.py $ARGC > "$OUT/singleC.log" 2>&1
RT_BENCH_BACKEND=gloo RT_BENCH_SAVE=$OUT/self8.npy timeout -k 10 400 python3 bench.py --gpus 8 $ARGC > "$OUT/self8.log" 2>&1
RT_BENCH_BACKEND=gloo RT_BENCH_SAVE=$OUT/dyn8.npy timeout -k 10 400 python3 bench.py --gpus 8 --schedule dynamic \
    $ARGC > "$OUT/dyn8.log" 2>&1
# round 6: the double-buffered gather (parallel.PipelinedGather) in the real bench, 8 gloo ranks, host-staged
RT_BENCH_BACKEND=gloo RT_BENCH_SAVE=$OUT/pipe8.npy timeout -k 10 400 python3 bench.py --gpus 8 --overlap-gloo \
    --config C --steps 3 --warmup 1 --cpu-seconds 0 --other-precision 0 > "$OUT/pipe8.log" 2>&1
python3 - "$OUT" <<'PY'
import json, sys, numpy as np
o = sys.argv[1]
names = ("single", "nccl1", "gloo2", "self2", "dyn1", "dyn2", "singleC", "self8", "dyn8", "pipe8")
a, b, c, d, e, f, g, h, i, j = (np.load(f"{o}/{n}.npy") for n in names)
print("nccl world-1 identical:", np.array_equal(a, b), " gloo world-2 identical:", np.array_equal(a, c),
      " self-launched world-2 identical:", np.array_equal(a, d), " dynamic world-1 (nccl) identical:",
      np.array_equal(a, e), " dynamic world-2 (gloo) identical:", np.array_equal(a, f), a.shape)
print("config C: self-launched world-8 identical:", np.array_equal(g, h), " dynamic world-8 identical:",
      np.array_equal(g, i), " pipelined gather world-8 identical:", np.array_equal(g, j), g.shape)
for n in names:   # the decomposition rank 0 prints (bench.py "dist")
    line = json.loads([l for l in open(f"{o}/{n}.log") if l.startswith("{")][-1])
    dd = line["dist"]
    print(n, "value", line["value"], "n_gpus", line["n_gpus"], "backend", dd["backend"], "world_size_initialised",
          dd["world_size_initialised"], "rccl", dd["rccl_version"], "imbalance", dd.get("imbalance"))
    for r in dd["per_rank"]:
        print("   rank", r["rank"], "render_ms", r["render_ms"], "gather_ms", r["gather_ms"], "assemble_ms",
              r["assemble_ms"], "wall_s", r["wall_s"], "px_per_s", r["px_per_s"], "pixels", r.get("pixels"),
              "chunks", r.get("chunks"))
assert all(np.array_equal(a, x) for x in (b, c, d, e, f)) and all(np.array_equal(g, x) for x in (h, i, j))
PY
