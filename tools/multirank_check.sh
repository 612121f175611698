#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: (1) torchrun world 1 over nccl (RCCL init with the
# library loaded), (2) 2 ranks sharing the GPU over gloo; compare the assembled images bit-for-bit
# with a plain single-process run.  Usage: bash tools/multirank_check.sh <outdir>
set -eu
OUT=${1:-gpurun_out/multirank}
mkdir -p "$OUT"
ARGS="--config B --steps 1 --warmup 0 --cpu-seconds 0"
RT_BENCH_SAVE=$OUT/single.npy timeout -k 10 200 python3 bench.py $ARGS > "$OUT/single.log" 2>&1
RT_BENCH_SAVE=$OUT/nccl1.npy timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 $ARGS > "$OUT/nccl1.log" 2>&1
RT_BENCH_BACKEND=gloo RT_BENCH_SAVE=$OUT/gloo2.npy timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 $ARGS > "$OUT/gloo2.log" 2>&1
python3 - "$OUT" <<'PY'
import sys, numpy as np
o = sys.argv[1]
a, b, c = (np.load(f"{o}/{n}.npy") for n in ("single", "nccl1", "gloo2"))
print("nccl world-1 identical:", np.array_equal(a, b), " gloo world-2 identical:", np.array_equal(a, c), a.shape)
assert np.array_equal(a, b) and np.array_equal(a, c)
PY
