#!/bin/bash
# Per-stage VALU issue rates at one config: one SQ counter pass (rocprofv3 --pmc, counters only) of the
# product library and of each stage-duplication build (tools/build_dups.sh).  A stage's share of the
# kernel is dGRBM_GUI_ACTIVE / GRBM_GUI_ACTIVE(base); its issue rate is the VALU instructions it adds per
# SIMD per cycle it adds, dSQ_INSTS_VALU / (dGRBM_GUI_ACTIVE / 8 x 1024 SIMDs), beside the whole
# kernel's rate; SQ_ACTIVE_INST_VALU gives the same per busy-cycle measure.
#   bash tools/stage_issue.sh <out> <prec> <config> <STAGE>...
set -u
OUT=$1; PREC=$2; CFG=$3; shift 3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CTR="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for V in base "$@"; do
  LIB=""; [ "$V" != base ] && LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_dup$V.so
  RT_ALLOW_EXPERIMENT=1 RT_MI355X_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$OUT/$V" -o run \
      --output-format csv -- python3 bench.py --config $CFG --precision $PREC --steps 1 --warmup 0 --cpu-seconds 0 \
      --other-precision 0 > "$OUT/$V.log" 2>&1 || { echo "$V failed"; exit 1; }
done
python3 - "$OUT" base "$@" <<'PY'
import csv, glob, sys
out, vs = sys.argv[1], sys.argv[2:]
def load(v):
    per = {}
    for f in glob.glob(f"{out}/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace_paths" in r["Kernel_Name"]:
                d = per.setdefault(int(r["Dispatch_Id"]), {})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per[max(per, key=lambda k: per[k].get("GRBM_GUI_ACTIVE", 0))]   # the timed frame (not the warm-up row)
B = load("base")
cyc = lambda d: d["GRBM_GUI_ACTIVE"] / 8 * 1024   # SIMD-cycles of the dispatch
print(f"base: {B['GRBM_GUI_ACTIVE'] / 8 / 1e6:.2f} M cycles, VALU/SIMD-cycle {B['SQ_INSTS_VALU'] / cyc(B):.3f}, "
      f"ACTIVE_VALU/SIMD-cycle {B['SQ_ACTIVE_INST_VALU'] / cyc(B):.3f}, SALU {B['SQ_INSTS_SALU'] / cyc(B):.3f}, "
      f"LDS {B['SQ_INSTS_LDS'] / cyc(B):.4f}, SMEM {B['SQ_INSTS_SMEM'] / cyc(B):.4f}, "
      f"waiting {B['SQ_WAIT_ANY'] / B['SQ_WAVE_CYCLES']:.3f}, issue-stalled {B['SQ_WAIT_INST_ANY'] / B['SQ_WAVE_CYCLES']:.3f}")
for v in vs[1:]:
    D = load(v)
    dc = D["GRBM_GUI_ACTIVE"] - B["GRBM_GUI_ACTIVE"]
    dd = {k: D[k] - B[k] for k in B}
    sc = dc / 8 * 1024
    print(f"{v:8s} share {dc / B['GRBM_GUI_ACTIVE']:.3f}  VALU {dd['SQ_INSTS_VALU'] / B['SQ_INSTS_VALU']:.3f} of base's  "
          f"VALU/SIMD-cycle {dd['SQ_INSTS_VALU'] / sc:.3f}  ACTIVE_VALU/SIMD-cycle {dd['SQ_ACTIVE_INST_VALU'] / sc:.3f}  "
          f"SALU {dd['SQ_INSTS_SALU'] / sc:.3f}  LDS {dd['SQ_INSTS_LDS'] / sc:.4f}  SMEM {dd['SQ_INSTS_SMEM'] / sc:.4f}  "
          f"waiting {dd['SQ_WAIT_ANY'] / max(dd['SQ_WAVE_CYCLES'], 1):.3f}")
PY
