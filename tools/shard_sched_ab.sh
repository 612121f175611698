#!/bin/bash
# alternate the work-distribution variants of tools/shard_sched_ab.py on one box: NAME[@G] (lib NAME, RT_BLOCK_G=G); bash tools/shard_sched_ab.sh ROUNDS VARIANT...
set -e
R=$1; shift
mkdir -p gpurun_out/sab
for i in $(seq 1 $R); do
  for V in "$@"; do
    N=${V%@*}; G=""; [ "$V" != "$N" ] && G=${V#*@}
    LIB=""; [ "$N" != base ] && LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_$N.so
    RT_BLOCK_G=$G RT_ALLOW_EXPERIMENT=1 RT_MI355X_LIB=$LIB timeout -k 10 120 python tools/shard_sched_ab.py $V 8 5 >> gpurun_out/sab/all.jsonl
  done
done
python3 - "$@" <<'PY'
import json, sys, statistics
rows = [json.loads(l) for l in open("gpurun_out/sab/all.jsonl")]
for v in sys.argv[1:]:
    x = [r for r in rows if r["name"] == v]
    print(f"{v:10s} whole {statistics.median([r['whole_ms'] for r in x]):.3f}  of_ideal {[r['of_ideal_median'] for r in x]}  "
          f"max/min {[r['slowest_max_min'] for r in x]}  summed {[r['summed_over_whole'] for r in x]}")
PY
