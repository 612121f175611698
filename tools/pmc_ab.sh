#!/bin/bash
# Instruction counts of the trace kernel for several library builds (one counter pass each):
#   bash tools/pmc_ab.sh <prec> <config> <variant>...   (variant as in tools/ab_libs.sh: base or NAME)
# Prints, per variant, the per-launch SQ_INSTS_VALU / SALU / LDS / SMEM / VMEM of trace_paths.
set -u
PREC=$1; CFG=$2; shift 2
OUT=gpurun_out/pmc_ab; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for V in "$@"; do
  LIB=""; [ "$V" != base ] && LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_$V.so
  RT_ALLOW_EXPERIMENT=1 RT_MI355X_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
      -d $OUT/${PREC}_${CFG}_$V -o run --output-format csv -- python3 bench.py --config $CFG --precision $PREC --steps 1 --warmup 0 \
      --cpu-seconds 0 --other-precision 0 > $OUT/${PREC}_${CFG}_$V.log 2>&1 || { echo "$V failed"; exit 1; }
done
python3 - $OUT $PREC $CFG "$@" <<'PY'
import csv, glob, sys
out, prec, cfg, vs = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
for v in vs:
    d, n = {}, {}
    for f in glob.glob(f"{out}/{prec}_{cfg}_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace_paths" in r["Kernel_Name"]:
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                n[r["Counter_Name"]] = n.get(r["Counter_Name"], 0) + 1
    # counters summed over the launches of the run (one warm-up row launch + the timed one): per launch = the max
    print(cfg, prec, f"{v:10s}", {k: f"{d[k] / 1e9:.3f}G" for k in sorted(d)})
PY
