#!/bin/bash
# Where the trace kernel's wave cycles go, per config: one SQ pass (wave-parked on s_waitcnt, issue
# stalls, active) and one scalar-cache pass, each a one-launch bench run under rocprofv3 --pmc.
#   bash tools/stall_pass.sh <out> <prec> <config>...
set -u
OUT=$1; PREC=$2; shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQ="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
SQC="SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM"
for CFG in "$@"; do
  for P in sq sqc; do
    [ $P = sq ] && CTR=$SQ || CTR=$SQC
    timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$OUT/${CFG}_$P" -o run --output-format csv -- \
        python3 bench.py --config $CFG --precision $PREC --steps 1 --warmup 0 --cpu-seconds 0 --other-precision 0 \
        > "$OUT/${CFG}_$P.log" 2>&1 || echo "$CFG $P failed rc=$?"
  done
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, sys
out, cfgs = sys.argv[1], sys.argv[2:]
for c in cfgs:
    d = {}
    for p in ("sq", "sqc"):
        for f in glob.glob(f"{out}/{c}_{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "trace_paths" in r["Kernel_Name"]:
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    print(c, {k: f"{v:.4g}" for k, v in sorted(d.items())})
    print(c, "parked %.3f  issue-stall %.3f  active %.3f" % (d.get("SQ_WAIT_ANY", 0) / wc,
          d.get("SQ_WAIT_INST_ANY", 0) / wc, d.get("SQ_ACTIVE_INST_ANY", 0) / wc))
PY
