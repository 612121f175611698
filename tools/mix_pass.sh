#!/bin/bash
# VALU instruction mix of the timed kernel (two rocprofv3 --pmc passes, counters only), for splitting the
# issue-stalled wave-cycles into multi-cycle VALU work and the rest.
#   bash tools/mix_pass.sh <out> <prec> <config>
set -u
OUT=$1; PREC=$2; CFG=$3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--config $CFG --precision $PREC --steps 1 --warmup 0 --cpu-seconds 0 --other-precision 0"
A="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT"
C="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY"
if [ ! -x tools/bin/ubench_mix ]; then
  mkdir -p tools/bin && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_mix tools/ubench_mix.hip || exit 1
fi
for pass in "mixA $A" "mixB $B" "mixC $C"; do
  set -- $pass; name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc $* -d "$OUT/$name" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1 || { echo "$name failed"; exit 1; }
done
for pass in "mixA $A" "mixB $B"; do
  set -- $pass; name=u$1; shift
  timeout -s KILL 60 rocprofv3 --pmc $* -d "$OUT/$name" -o run --output-format csv -- ./tools/bin/ubench_mix > "$OUT/$name.log" 2>&1 || { echo "$name failed"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
def load(name, pat):
    per = collections.defaultdict(dict)
    for f in glob.glob(f"{out}/{name}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                d = per[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per
tot = {}
for n in ("mixA", "mixB", "mixC"):
    per = load(n, "trace_paths")
    k = max(per, key=lambda i: per[i].get("SQ_INSTS_VALU", per[i].get("SQ_INSTS_VALU_FMA_F32", per[i].get("SQ_WAVE_CYCLES", 0))))
    tot.update(per[k])
for k in sorted(tot): print(f"{k:28s} {tot[k]:.4e}")
v = tot["SQ_INSTS_VALU"]
print("fractions of VALU instructions:", {k[14:]: round(tot[k] / v, 3) for k in tot if k.startswith("SQ_INSTS_VALU_")})
print("SQ_THREAD_CYCLES_VALU / SQ_INSTS_VALU:", round(tot["SQ_THREAD_CYCLES_VALU"] / v, 2))
print(open(f"{out}/umixA.log").read())
names = {}
for n in ("umixA", "umixB"):
    for f in glob.glob(f"{out}/{n}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"].split("chains<")[-1].split(">")[0]
    per = load(n, "chains")
    for i, d in sorted(per.items()):
        v = d.get("SQ_INSTS_VALU") or d.get("SQ_INSTS_VALU_FMA_F32", 0) + 1e-9
        print(n, i, names.get(i, "?"), {k[14:] or k: round(x / (2048 * 4 * 1024 * 16 + 1e-9), 3) for k, x in d.items() if x})
PY
