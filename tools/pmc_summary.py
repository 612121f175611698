#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: totals per counter for the trace kernel + derived ratios."""
import csv
import glob
import json
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
tot, dispatches = {}, set()
for f in sorted(glob.glob(f"{d}/pass*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "trace_" not in r["Kernel_Name"]:
            continue
        dispatches.add((f, r["Dispatch_Id"]))
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.4e}")
g = tot.get
out = {}
if g("SQ_WAVE_CYCLES"):
    w = tot["SQ_WAVE_CYCLES"]
    out["wait_any_frac"] = g("SQ_WAIT_ANY", 0) / w
    out["wait_inst_any_frac"] = g("SQ_WAIT_INST_ANY", 0) / w
    out["active_any_frac"] = g("SQ_ACTIVE_INST_ANY", 0) / w
if g("SQ_INSTS_VALU"):
    out["salu_per_valu"] = g("SQ_INSTS_SALU", 0) / tot["SQ_INSTS_VALU"]
    out["lane_util_valu"] = g("SQ_THREAD_CYCLES_VALU", 0) / (64 * g("SQ_ACTIVE_INST_VALU", 1)) if g("SQ_ACTIVE_INST_VALU") else None
if g("FETCH_SIZE") is not None:
    out["fetch_kb"] = g("FETCH_SIZE")
    out["write_kb"] = g("WRITE_SIZE", 0)
print(json.dumps(out, indent=1))
