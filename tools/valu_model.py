#!/usr/bin/env python3
"""Issue-cost model of the timed kernel's VALU work ("What bounds it").

Counts: the SQ_INSTS_VALU_* classes of the timed dispatch (tools/mix_pass.sh, profiles/r05/valu_mix/<prec>_mix*.csv).
Costs: SIMD-cycles per wave-instruction from tools/ubench_mix.hip and tools/ubench_bank.hip on the same chip
(profiles/r05/valu_mix/ubench_*.txt).  The ubench run under the same counters shows how each kind is counted:
v_pk_fma_f32 counts once in FMA_F32 (not twice), v_sqrt/rsq_f32 in TRANS_F32, v_mad_u64_u32 in INT64, v_add_u32 in
INT32, v_cvt in CVT; logic ops, selects, compares and moves fall in no class ("other").
The model's VALU-busy fraction = sum(count x cost) / the dispatch's SIMD-cycles (GRBM_GUI_ACTIVE / 8 XCDs x 1024
SIMDs), bracketed by the unknowns: the packed share of FMA_F32 and the cost of an "other" instruction.
    python3 tools/valu_model.py [dir]"""
import collections
import csv
import glob
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "profiles", "r05", "valu_mix")


def counters(prec):
    tot = {}
    for f in sorted(glob.glob(os.path.join(D, f"{prec}_mix*.csv"))):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if "trace_paths" in r["Kernel_Name"]:
                d = per[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        k = max(per, key=lambda i: sum(per[i].values()))   # the timed frame, not the one-row warm-up
        tot.update(per[k])
    return tot


# SIMD-cycles per wave-instruction (ubench_mix / ubench_bank, warm clocks, 2.4 GHz)
COST = {"FMA_F32_scalar": 2.5, "FMA_F32_packed": 4.6, "FMA_F64": 4.3, "ADD_F64": 4.3, "MUL_F64": 4.3,
        "MUL_F32": 2.5, "ADD_F32": 2.5, "TRANS_F32": 8.9, "TRANS_F64": 16.3, "INT32": 2.9, "INT64": 4.5, "CVT": 4.7}
# "other": moves and logic cost 2.5-2.7, compares (e32 or e64) and selects on a lane mask 4.1-4.7; the C kernel's
# static code has about as many compares and selects as moves and logic ops, so "other" averages ~3.4: the model
# brackets it with 3.0 and 3.7 (and prints the extremes 2.5 / 4.4 for reference)

for prec, packed in (("f32", (0.5, 0.9)), ("f64", (0.5, 0.9))):
    c = counters(prec)
    simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024
    v = c["SQ_INSTS_VALU"]
    cls = {k[14:]: x for k, x in c.items() if k.startswith("SQ_INSTS_VALU_")}
    other = v - sum(cls.values())
    print(f"{prec}: {v:.3e} VALU wave-instructions, {simd_cycles:.3e} SIMD-cycles; classes (share): "
          + ", ".join(f"{k} {x / v:.3f}" for k, x in sorted(cls.items()) if x) + f", other {other / v:.3f}")
    lo = hi = None
    for pk in packed:
        for oc in (2.5, 3.0, 3.7, 4.4):
            cyc = sum(x * COST[k] for k, x in cls.items() if k != "FMA_F32")
            cyc += cls.get("FMA_F32", 0.0) * (pk * COST["FMA_F32_packed"] + (1 - pk) * COST["FMA_F32_scalar"])
            cyc += other * oc
            b = cyc / simd_cycles
            if oc in (3.0, 3.7):
                lo = b if lo is None else min(lo, b)
                hi = b if hi is None else max(hi, b)
            print(f"   packed share of FMA_F32 {pk:.1f}, other {oc} cycles: VALU pipe busy {b:.2f}")
    print(f"   {prec}: VALU pipe busy {lo:.2f}-{hi:.2f} of the dispatch's SIMD-cycles; the fma_f32-rate measure "
          f"(valu_busy) reads {v * 2.3 / simd_cycles:.2f}")
