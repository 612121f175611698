#!/usr/bin/env python3
"""VALU issue on counters (round 6): per instruction kind of the microbenchmarks (tools/ubench_mix.hip,
tools/ubench_bank2.hip) and for the timed kernel, SIMD-cycles per wave-instruction next to what
SQ_ACTIVE_INST_VALU (VALU quad-cycles: 1 per instruction, 2 per fp32 transcendental, 4 per fp64 one) and
SQ_ACTIVE_INST_VALU2 (quad-cycles in which two VALU instructions issued together) count per instruction.
The VALU pipe's occupancy is then 4 (ACTIVE - VALU2) / the dispatch's SIMD-cycles (GRBM_GUI_ACTIVE / 8 x 1024).
    python3 tools/issue_counters.py <dir with issue_ub/, issue_C_f32/, issue_C_f64/ rocprofv3 --pmc outputs>"""
import collections
import csv
import glob
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r6"


def load(d, pat):
    per, names = collections.defaultdict(dict), {}
    for f in glob.glob(f"{D}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                i = int(r["Dispatch_Id"])
                per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                names[i] = r["Kernel_Name"]
    return per, names


def row(x):
    v, cyc = x["SQ_INSTS_VALU"], x["GRBM_GUI_ACTIVE"] / 8 * 1024
    return (cyc / v, x["SQ_ACTIVE_INST_VALU"] / v, x["SQ_ACTIVE_INST_VALU2"] / v,
            4 * (x["SQ_ACTIVE_INST_VALU"] - x["SQ_ACTIVE_INST_VALU2"]) / cyc)


print(f"{'kind':24s} {'SIMD-cyc/inst':>13s} {'ACTIVE/inst':>11s} {'VALU2/inst':>10s} {'VALU occupancy':>14s}")
per, names = load("issue_ub", "chains")
last = {}
for i in sorted(per):
    last[names[i].split("chains<")[-1].split(">")[0]] = per[i]   # the last dispatch of each kind (clocks up)
for n, x in last.items():
    a, b, c, o = row(x)
    print(f"{n:24s} {a:13.2f} {b:11.2f} {c:10.3f} {o:14.3f}")
for pat, d in (("trace_paths", "issue_C_f32"), ("trace_paths", "issue_C_f64")):
    per, _ = load(d, pat)
    if per:
        x = per[max(per, key=lambda i: per[i]["GRBM_GUI_ACTIVE"])]   # the timed frame, not the one-row warm-up
        a, b, c, o = row(x)
        print(f"{'kernel ' + d[8:]:24s} {a:13.2f} {b:11.2f} {c:10.3f} {o:14.3f}   dual-issued share "
              f"{2 * x['SQ_ACTIVE_INST_VALU2'] / x['SQ_INSTS_VALU']:.3f}, VALU lane use "
              f"{x['SQ_THREAD_CYCLES_VALU'] / 64 / x['SQ_INSTS_VALU']:.3f}")
