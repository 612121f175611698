#!/bin/bash
# Collect the round-6 profile calls (gpurun_out/r06f_{f32,f64,E}: tools/profile_round.sh) into profiles/r06/{f32,f64,E_f32}/
# and merge their PMC records into profiles/pmc.json, each keeping the commit it was measured at (RT_COMMIT).
set -eu
for T in f32:f32 f64:f64 E:E_f32; do
  S=gpurun_out/r06f_${T%%:*}; D=profiles/r06/${T#*:}
  [ -d "$S" ] || continue
  mkdir -p "$D"
  cp "$S/bench.json" "$S/pmc.json" "$S/pmc_summary.txt" "$D/"
  cp "$S/ktrace/run_kernel_stats.csv" "$D/kernel_stats.csv"
  for p in pmc_fetch pmc_write pmc_sq pmc_issue ubench_sq ubench_issue; do
    [ -f "$S/$p/run_counter_collection.csv" ] && cp "$S/$p/run_counter_collection.csv" "$D/${p}_counter_collection.csv"
  done
done
python3 - <<'PY'
import json, os
db = json.load(open("profiles/pmc.json"))
for name in ("f32", "f64", "E_f32"):
    p = f"profiles/r06/{name}/pmc.json"
    if not os.path.exists(p):
        continue
    for k, v in json.load(open(p)).items():
        db[k] = v
    b = json.load(open(f"profiles/r06/{name}/bench.json")); r = b["roofline"]
    print(name, b["value"], b["ms_per_step"], "frac", round(r["frac"], 4), "issue_frac", round(r["issue_frac"], 3),
          "vs ubench", round(r["issue_frac_vs_ubench"], 3), "pmc_flop_frac", round(r["pmc_flop_frac"], 3),
          "traffic GB", round(r["traffic"] / 1e9, 1), "stale", r["pmc_source"]["stale"],
          "other leg", {k: b[k]["value"] for k in ("f32", "f64") if k in b})
json.dump(db, open("profiles/pmc.json", "w"), indent=1)
PY
