#!/bin/bash
# Where the trace kernel's memory waits come from: per instruction class, the
# instructions issued and their in-flight level summed over cycles (SQ_INST_LEVEL_* / SQ_INSTS_* =
# average latency, Little's law), plus the LDS issue waits; one PMC pass per config, counters only.
#   bash tools/stall_split.sh <out> <prec> <config>...
set -u
OUT=$1; PREC=$2; shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/list_avail.txt" 2>&1 || true
# rocprofv3's derived latency metrics (accumulate(SQ_INST_LEVEL_X, HIGH_RES) / SQ_INSTS_X, in cycles),
# one pass each, then the instruction counts and wait cycles
for CFG in "$@"; do
  for M in SmemLatency VmemLatency LdsLatency "SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES"; do
    N=$(echo $M | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $M -d "$OUT/${CFG}_$N" -o run --output-format csv -- \
        python3 bench.py --config $CFG --precision $PREC --steps 1 --warmup 0 --cpu-seconds 0 --other-precision 0 \
        > "$OUT/${CFG}_$N.log" 2>&1 || echo "$CFG $N failed rc=$?"
  done
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, sys
out, cfgs = sys.argv[1], sys.argv[2:]
for c in cfgs:
    d = {}
    for f in glob.glob(f"{out}/{c}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace_paths" in r["Kernel_Name"]:
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(c, {k: f"{v:.4g}" for k, v in sorted(d.items())})
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    for k in ("Smem", "Vmem", "Lds"):
        lat, n = d.get(f"{k}Latency"), d.get(f"SQ_INSTS_{k.upper()}")
        if lat and n:
            # Little's law: instructions x latency = wave-cycles with that class in flight
            print(f"  {k}: {n:.4g} insts x {lat:.0f} cycles = {n * lat / wc:.3f} of wave-cycles in flight")
    if "SQ_WAIT_ANY" in d:
        print(f"  waiting (s_waitcnt) {d['SQ_WAIT_ANY'] / wc:.3f} of wave-cycles; LDS issue waits {4 * d.get('SQ_WAIT_INST_LDS', 0) / wc:.3f}")
PY
