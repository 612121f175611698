#!/bin/bash
# Copy the judged artefacts of tools/profile_round.sh calls (gpurun_out/<tag>_{f32,f64}) into
# profiles/<round>/{f32,f64}/ and merge their pmc.json records into profiles/pmc.json, stamped with the
# commit they were measured at (run this from the commit the GPU call was made from, tree clean).
# Usage: bash tools/collect_profiles.sh <tag> <round>
set -eu
TAG=$1; ROUND=$2
if [ -n "$(git status --porcelain -- rust-ray-tracing_amd/csrc include)" ]; then
  echo "kernel sources differ from HEAD: commit first, then profile" >&2; exit 1
fi
HEAD=$(git rev-parse --short=12 HEAD)
for P in f32 f64; do
  SRC=gpurun_out/${TAG}_$P
  [ -d "$SRC" ] || continue
  DST=profiles/$ROUND/$P
  mkdir -p "$DST"
  cp "$SRC/bench.json" "$DST/bench.json"
  cp "$SRC/ktrace/run_kernel_stats.csv" "$DST/kernel_stats.csv"
  cp "$SRC/pmc.json" "$DST/pmc.json"
  cp "$SRC/pmc_summary.txt" "$DST/pmc_summary.txt"
  for pass in pmc_fetch pmc_write pmc_sq ubench_sq; do
    [ -f "$SRC/$pass/run_counter_collection.csv" ] && cp "$SRC/$pass/run_counter_collection.csv" "$DST/${pass}_counter_collection.csv"
  done
  python3 - "$SRC/pmc.json" "$HEAD" <<'PY'
import json, os, sys
rec = json.load(open(sys.argv[1]))
path = "profiles/pmc.json"
db = json.load(open(path)) if os.path.exists(path) else {}
for k, v in rec.items():
    v["commit"] = sys.argv[2]
    db[k] = v
json.dump(db, open(path, "w"), indent=1)
PY
done
