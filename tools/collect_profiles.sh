#!/bin/bash
# Copy the judged artefacts of a tools/profile_round.sh call (gpurun_out/<tag>_{f32,f64}) into
# profiles/<round>/{f32,f64} and profiles/traffic.json.  Usage: bash tools/collect_profiles.sh <tag> [round]
set -eu
TAG=$1; ROUND=${2:-r01}
for P in f32 f64; do
  SRC=gpurun_out/${TAG}_$P
  [ -d "$SRC" ] || continue
  DST=profiles/$ROUND/$P
  mkdir -p "$DST"
  cp "$SRC/bench.json" "$DST/bench.json"
  cp "$SRC/ktrace/run_kernel_stats.csv" "$DST/kernel_stats.csv"
  cp "$SRC/traffic.json" "$DST/traffic.json"
  python3 - "$SRC/traffic.json" "$P" <<'PY'
import json, os, sys
rec = json.load(open(sys.argv[1]))
path = "profiles/traffic.json"
db = json.load(open(path)) if os.path.exists(path) else {}
db[f"C:{sys.argv[2]}:1"] = rec
json.dump(db, open(path, "w"), indent=1)
PY
done
