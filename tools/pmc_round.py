#!/usr/bin/env python3
"""Turn tools/profile_round.sh's PMC passes into one pmc.json record per launch of the trace kernel.

  python3 tools/pmc_round.py <out> <key: CONFIG:PREC:WORLD>

* HBM traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; FETCH_SIZE doubled per MI355X_MICROARCH.md
  §HBM: gfx950 reports half the bytes of wide reads).  Infinity-Cache hits count too (same section).
* VALU busy = SQ_ACTIVE_INST_VALU per SIMD per cycle of the dispatch, where cycles = GRBM_GUI_ACTIVE / 8
  (the 8 XCDs summed, MI355X_MICROARCH.md §DVFS), and calibrated by the same ratio measured on
  ubench_valu's FMA chains (8 waves per SIMD, nothing but independent VALU): busy = ratio(kernel) /
  ratio(ubench).  The raw ratio is reported too.
* FLOP counters: SQ_INSTS_VALU_FLOPS_FP32/FP64 x the lane scale found on the ubench (its FMA count is
  known exactly), so the executed-FLOP count of the in-kernel counters can be checked against them.
"""
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
from rt_mi355x import abi  # noqa: E402  (source_hash: no GPU needed)

out, key = sys.argv[1], sys.argv[2]
N_SIMD = 1024


def load(name, match):
    rows = [r for f in glob.glob(f"{out}/{name}/**/*counter_collection.csv", recursive=True)
            for r in csv.DictReader(open(f)) if match(r["Kernel_Name"])]
    per = {}
    for r in rows:
        d = per.setdefault(r["Dispatch_Id"], {"_t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9,
                                              "_k": r["Kernel_Name"]})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(per.values())


def one(name):
    d = load(name, lambda k: "trace_paths" in k)
    assert len(d) == 1, (name, len(d))
    return d[0]


fetch, write, sq = one("pmc_fetch"), one("pmc_write"), one("pmc_sq")


def busy_ratio(d):
    return d["SQ_ACTIVE_INST_VALU"] / (N_SIMD * d["GRBM_GUI_ACTIVE"] / 8.0)


# The GPU box has no .git: the caller passes the commit in RT_COMMIT (expanded where the tree was sent
# from); the source hash is what bench.py checks (the library's rt_version() carries the same hash).
commit = os.environ.get("RT_COMMIT") or subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                                        text=True, cwd=REPO).stdout.strip() or None
rec = {
    "commit": commit,
    "src_hash": abi.source_hash(),
    "kernel": sq["_k"],
    "launch_ms": sq["_t"] * 1e3,
    "fetch_bytes_raw": fetch["FETCH_SIZE"] * 1024,
    "write_bytes": write["WRITE_SIZE"] * 1024,
    "hbm_bytes_per_launch": 2 * fetch["FETCH_SIZE"] * 1024 + write["WRITE_SIZE"] * 1024,
    "sq": {k: v for k, v in sq.items() if not k.startswith("_")},
    "effective_clock_ghz": sq["GRBM_GUI_ACTIVE"] / 8.0 / sq["_t"] / 1e9,
    "valu_active_per_simd_cycle_raw": busy_ratio(sq),
}
ub = load("ubench_sq", lambda k: "chains" in k)
if ub:
    # tools/ubench_valu: 2048 blocks x 4 waves x 4096 iterations x 16 independent FMAs per lane; 8 waves
    # per SIMD, nothing but VALU: its instructions per SIMD-cycle is the issue ceiling of that instruction.
    winst = 2048 * 4 * 4096 * 16
    cal = {}
    for d in ub:
        kind = "f64" if "double" in d["_k"] else ("pk_f32" if "vector" in d["_k"] else "f32")
        c = cal.setdefault(kind, {"insts_per_simd_cycle": [], "cu_busy": [], "flops_fp32_per_inst": [],
                                  "clock_ghz": []})
        c["insts_per_simd_cycle"].append(busy_ratio(d))
        c["cu_busy"].append(d["SQ_BUSY_CU_CYCLES"] / 256 / (d["GRBM_GUI_ACTIVE"] / 8.0))
        c["flops_fp32_per_inst"].append(d["SQ_INSTS_VALU_FLOPS_FP32"] / winst)
        c["clock_ghz"].append(d["GRBM_GUI_ACTIVE"] / 8.0 / d["_t"] / 1e9)
    cal = {k: {m: sum(v) / len(v) for m, v in c.items()} for k, c in cal.items()}
    rec["ubench_calibration"] = cal
    # SQ_INSTS_VALU_FLOPS_FP32 counts FLOP per lane per wave instruction (ubench: 2 per v_fma_f32, 4 per
    # v_pk_fma_f32), so x 64 is the FLOP the wave executed.
    rec["pmc_flop_fp32"] = sq["SQ_INSTS_VALU_FLOPS_FP32"] * 64
    rec["pmc_flop_fp64"] = sq["SQ_INSTS_VALU_FLOPS_FP64"] * 64
    cu = sq["SQ_BUSY_CU_CYCLES"] / 256 / (sq["GRBM_GUI_ACTIVE"] / 8.0)
    rec["cu_busy"] = cu
    rec["cycles_per_valu_inst"] = 1.0 / rec["valu_active_per_simd_cycle_raw"]
    # VALU busy against the issue ceilings the ubench measures for v_fma_f32 (~2 cycles per wave64
    # instruction) and v_pk_fma_f32 (~4): both per CU-busy cycle.
    for k in ("f32", "pk_f32"):
        if k in cal:
            rec[f"valu_busy_vs_{k}"] = (rec["valu_active_per_simd_cycle_raw"] / cu) / (
                cal[k]["insts_per_simd_cycle"] / cal[k]["cu_busy"])
    rec["valu_busy"] = rec.get("valu_busy_vs_f32")
# Issue occupancy on a counter (round 6).  SQ_ACTIVE_INST_VALU counts VALU quad-cycles (1 per instruction, 2 per
# fp32 transcendental, 4 per fp64 one) and SQ_ACTIVE_INST_VALU2 the quad-cycles in which two VALU instructions
# issued together (fp32/int32 ops whose operands are all VGPRs: ~2 per quad-cycle; an SGPR or constant operand,
# a packed, 64-bit, compare, select, cvt or 3-input op takes a quad-cycle alone: tools/ubench_bank2.hip).  So the
# VALU pipe is busy 4 (ACTIVE - VALU2) SIMD-cycles; issue_frac is that over the dispatch's SIMD-cycles (1.0 = a
# VALU quad-cycle in every 4 cycles of every SIMD), issue_frac_vs_ubench the same against ubench_valu's
# independent FMA chains (8 waves per SIMD, nothing but VALU), the best rate measured on the chip.
try:
    iss = one("pmc_issue")
except (AssertionError, KeyError):
    iss = None
if iss:
    def quads(d):
        return (d["SQ_ACTIVE_INST_VALU"] - d["SQ_ACTIVE_INST_VALU2"]) / (N_SIMD * d["GRBM_GUI_ACTIVE"] / 8.0)
    rec["issue"] = {k: v for k, v in iss.items() if not k.startswith("_")}
    rec["issue_frac"] = 4.0 * quads(iss)
    rec["valu_dual_issue_share"] = 2.0 * iss["SQ_ACTIVE_INST_VALU2"] / iss["SQ_INSTS_VALU"]
    rec["valu_lane_util"] = iss["SQ_THREAD_CYCLES_VALU"] / 64.0 / iss["SQ_INSTS_VALU"]
    ubi = load("ubench_issue", lambda k: "chains" in k)
    if ubi:
        best = max(4.0 * quads(d) for d in ubi)
        rec["issue_frac_ubench_best"] = best
        rec["issue_frac_vs_ubench"] = rec["issue_frac"] / best
# The PMC FLOP counters at the vector peaks (157.3 TF fp32, 78.6 TF fp64), over the PMC pass's own launch time:
# every fp32/fp64 FLOP the kernel executes, where roofline.frac counts only the culls' and exact tests' FLOP.
if "pmc_flop_fp32" in rec:
    rec["pmc_flop_frac"] = (rec["pmc_flop_fp32"] / 157.3e12 + rec["pmc_flop_fp64"] / 78.6e12) / sq["_t"]
json.dump({key: rec}, open(f"{out}/pmc.json", "w"), indent=1)
print(json.dumps(rec, indent=1))
