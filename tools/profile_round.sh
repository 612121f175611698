#!/bin/bash
# One GPU call that produces the judged artefacts for a round:
#   <out>/bench.json            default bench line (N=1)
#   <out>/ktrace/*stats.csv     rocprofv3 --kernel-trace --stats of the same bench command
#   <out>/pmc_*                 FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU passes (separate, counters only)
#   profiles/traffic.json       HBM bytes per launch (FETCH doubled per MI355X_MICROARCH.md §HBM)
# Usage (GPU box): bash tools/profile_round.sh gpurun_out/round [precision]
set -u
OUT=${1:-gpurun_out/round}
PREC=${2:-f32}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS=5
for C in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex trace_ -d "$OUT/pmc_$C" -o run --output-format csv -- \
      python3 bench.py --precision "$PREC" --steps 1 --warmup 0 --cpu-seconds 0 > "$OUT/pmc_$C.log" 2>&1 || exit $?
done
python3 - "$OUT" "$PREC" <<'EOF'
import csv, glob, json, os, sys
out, prec = sys.argv[1], sys.argv[2]
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU"):
    rows = [r for f in glob.glob(f"{out}/pmc_{c}/**/*counter_collection.csv", recursive=True)
            for r in csv.DictReader(open(f)) if "trace_" in r["Kernel_Name"]]
    vals[c] = sum(float(r["Counter_Value"]) for r in rows) / max(1, len({r["Dispatch_Id"] for r in rows}))
fetch_b, write_b = vals["FETCH_SIZE"] * 1024, vals["WRITE_SIZE"] * 1024
rec = {"hbm_bytes_per_launch": 2 * fetch_b + write_b, "fetch_bytes_raw": fetch_b, "write_bytes": write_b,
       "valu_insts_per_launch": vals["SQ_INSTS_VALU"],
       "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half of wide streaming reads); "
               "per launch of config C on one GPU"}
path = "profiles/traffic.json"
db = json.load(open(path)) if os.path.exists(path) else {}
db[f"C:{prec}:1"] = rec
json.dump(db, open(path, "w"), indent=1)
json.dump(rec, open(f"{out}/traffic.json", "w"), indent=1)
print(json.dumps(rec))
EOF
# bench line and kernel trace after the traffic passes, so bench.json reads this round's traffic
timeout -k 10 300 python3 bench.py --precision "$PREC" --steps $STEPS > "$OUT/bench.log" 2>&1 || exit $?
grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace" -o run --output-format csv -- \
    python3 bench.py --precision "$PREC" --steps $STEPS --cpu-seconds 0 > "$OUT/ktrace.log" 2>&1 || exit $?
