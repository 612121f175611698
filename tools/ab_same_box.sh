#!/bin/bash
# Same-box A/B of the product library against lib/librt_mi355x_exp.so (make exp EXP=...):
# alternating bench runs, so box-to-box clock differences cancel.  Usage: bash tools/ab_same_box.sh [prec] [rounds]
set -e
PREC=${1:-f32}; R=${2:-3}
for i in $(seq 1 $R); do
  for L in base exp; do
    LIB=""; [ $L = exp ] && LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_exp.so
    RT_ALLOW_EXPERIMENT=1 RT_MI355X_LIB=$LIB timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 3 --precision $PREC > gpurun_out/abx_${PREC}_${L}_$i.log 2>&1
  done
done
python3 - "$PREC" "$R" <<'PY'
import json, sys
prec, R = sys.argv[1], int(sys.argv[2])
for L in ("base", "exp"):
    v = [json.loads([l for l in open(f"gpurun_out/abx_{prec}_{L}_{i}.log") if l.startswith("{")][-1])["value"] for i in range(1, R + 1)]
    print(L, prec, [round(x) for x in v], "mean", round(sum(v) / len(v), 1))
PY
