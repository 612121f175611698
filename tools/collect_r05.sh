#!/bin/bash
# Collect tools/_run_final.sh's outputs (gpurun_out/r05f_{f32,f64,E}) into profiles/r05/ and merge the PMC records
# into profiles/pmc.json (run from the commit the GPU call was made from, kernel sources clean).
set -eu
bash tools/collect_profiles.sh r05f r05
S=gpurun_out/r05f_E; D=profiles/r05/E_f32
mkdir -p $D
cp $S/bench.json $S/pmc.json $S/pmc_summary.txt $D/
cp $S/ktrace/run_kernel_stats.csv $D/kernel_stats.csv
for p in pmc_fetch pmc_write pmc_sq ubench_sq; do cp $S/$p/run_counter_collection.csv $D/${p}_counter_collection.csv; done
grep '^{' $S/benchE_f64.log | tail -1 > profiles/r05/benchE_f64.json
python3 - <<'PY'
import json, subprocess
head = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
db = json.load(open("profiles/pmc.json"))
for k, v in json.load(open("profiles/r05/E_f32/pmc.json")).items():
    v["commit"] = head; db[k] = v
json.dump(db, open("profiles/pmc.json", "w"), indent=1)
for name in ("f32", "f64", "E_f32"):
    b = json.load(open(f"profiles/r05/{name}/bench.json")); r = b["roofline"]
    m = json.load(open(f"profiles/r05/{name}/pmc.json")); k = list(m.values())[0]
    S = 3840 * 2160 * 2048 if name == "E_f32" else 1920 * 1080 * 512
    print(name, b["value"], b["ms_per_step"], "frac", round(r["frac"], 4), "traffic GB", round(r["traffic"] / 1e9, 1),
          "valu_busy", round(r["valu_busy"], 3), "stale", r["pmc_source"]["stale"], "written B/sample", round(k["write_bytes"] / S, 2),
          "VALU/sample", round(k["sq"]["SQ_INSTS_VALU"] / S, 2), "f64 leg", b.get("f64", {}).get("value"),
          "brute TF/s", round(r["brute_force_equiv"]["tflops"], 1), "cpu", (b.get("cpu_baseline") or {}).get("value"))
b = json.load(open("profiles/r05/benchE_f64.json")); print("E f64", b["value"], b["ms_per_step"], round(b["roofline"]["frac"], 4))
PY
