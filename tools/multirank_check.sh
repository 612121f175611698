#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: (1) torchrun world 1 over nccl (RCCL init with the
# library loaded), (2) 2 ranks sharing the GPU over gloo, (3) plain `bench.py --gpus 2` (it launches
# its own 2 ranks, as the driver runs it) over gloo; compare the assembled images bit-for-bit with a
# plain single-process run.  Usage: bash tools/multirank_check.sh <outdir>
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
python3 - "$OUT" <<'PY'
import json, sys, numpy as np
o = sys.argv[1]
a, b, c, d = (np.load(f"{o}/{n}.npy") for n in ("single", "nccl1", "gloo2", "self2"))
print("nccl world-1 identical:", np.array_equal(a, b), " gloo world-2 identical:", np.array_equal(a, c),
      " self-launched world-2 identical:", np.array_equal(a, d), a.shape)
for n in ("single", "nccl1", "gloo2", "self2"):   # the decomposition rank 0 prints (bench.py "dist")
    line = json.loads([l for l in open(f"{o}/{n}.log") if l.startswith("{")][-1])
    dd = line["dist"]
    print(n, "value", line["value"], "n_gpus", line["n_gpus"], "backend", dd["backend"], "world_size_initialised",
          dd["world_size_initialised"], "rccl", dd["rccl_version"], "imbalance", dd.get("imbalance"))
    for r in dd["per_rank"]:
        print("   rank", r["rank"], "render_ms", r["render_ms"], "gather_ms", r["gather_ms"], "assemble_ms",
              r["assemble_ms"], "wall_s", r["wall_s"], "px_per_s", r["px_per_s"])
assert np.array_equal(a, b) and np.array_equal(a, c) and np.array_equal(a, d)
PY
