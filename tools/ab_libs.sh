#!/bin/bash
# Same-box A/B of several builds, alternating bench runs so box-to-box clock differences cancel.
#   bash tools/ab_libs.sh <prec> <rounds> <config> <variant>...
# A variant is NAME or NAME@W: NAME "base" = lib/librt_mi355x.so, otherwise lib/librt_mi355x_NAME.so;
# @W sets RT_WAVES=W.  Prints one line per variant: the bench values and their mean.
set -e
PREC=$1; R=$2; CFG=$3; shift 3
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for V in "$@"; do
    N=${V%@*}; W=""; [ "$V" != "$N" ] && W=${V#*@}
    LIB=""; [ "$N" != base ] && LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_$N.so
    RT_WAVES=$W RT_ALLOW_EXPERIMENT=1 RT_MI355X_LIB=$LIB timeout -k 10 120 python bench.py --config $CFG --cpu-seconds 0 --steps 3 \
        --other-precision 0 --precision $PREC > gpurun_out/ab/${PREC}_${CFG}_${V}_$i.log 2>&1
  done
done
python3 - "$PREC" "$R" "$CFG" "$@" <<'PY'
import json, sys
prec, R, cfg, vs = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4:]
for v in vs:
    x = [json.loads([l for l in open(f"gpurun_out/ab/{prec}_{cfg}_{v}_{i}.log") if l.startswith("{")][-1])["value"]
         for i in range(1, R + 1)]
    print(f"{cfg} {prec} {v:12s}", [round(t) for t in x], "mean", round(sum(x) / len(x), 1))
PY
