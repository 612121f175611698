#!/bin/bash
# Per-dispatch PMC of config C's whole frame against its N row shards (tools/shard_launches.py), one
# rocprofv3 --pmc pass per counter group: where the shards' extra time per sample goes.
#   bash tools/shard_pmc.sh <out> [N]
set -u
OUT=$1; N=${2:-8}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
declare -A P
P[sq]="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P[mem]="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES"
P[sqc]="SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM"
P[tcc]="TCC_HIT_sum TCC_MISS_sum"
P[fetch]="FETCH_SIZE"
P[write]="WRITE_SIZE"
for k in sq mem sqc tcc fetch write; do
  timeout -s KILL 120 rocprofv3 --pmc ${P[$k]} -d "$OUT/$k" -o run --output-format csv -- \
      python3 tools/shard_launches.py $N > "$OUT/$k.log" 2>&1 || { echo "$k failed rc=$?"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
rows = collections.defaultdict(dict)   # pass -> dispatch -> counter -> value
for p in ("sq", "mem", "sqc", "tcc", "fetch", "write"):
    for f in glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "trace_paths" in r["Kernel_Name"]:
                d = rows[p].setdefault(int(r["Dispatch_Id"]), {})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
tot = {"whole": {}, "shards": {}}
for p, ds in rows.items():
    ids = sorted(ds)[1:]   # drop the warm-up
    for i, di in enumerate(ids):
        t = tot["whole" if i == 0 else "shards"]
        for c, v in ds[di].items():
            t[c] = t.get(c, 0.0) + v
for c in sorted(tot["whole"]):
    a, b = tot["whole"][c], tot["shards"].get(c, 0.0)
    print(f"{c:24s} whole {a:12.4g}  shards {b:12.4g}  ratio {b / a if a else float('nan'):.3f}")
PY
