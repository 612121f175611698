#!/bin/bash
# HBM traffic of the trace kernel per build: FETCH_SIZE and WRITE_SIZE passes (one counter group each)
# of a one-launch bench run, for several libraries (traffic experiments: which record writes cost what).
#   bash tools/traffic_exp.sh <out> <config> <prec> <variant>...
# variant NAME: "base" = lib/librt_mi355x.so, else lib/librt_mi355x_NAME.so.  Prints GB per launch.
set -u
OUT=$1; CFG=$2; PREC=$3; shift 3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for V in "$@"; do
  LIB=""; [ "$V" != base ] && LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_$V.so
  for C in FETCH_SIZE WRITE_SIZE; do
    RT_ALLOW_EXPERIMENT=1 RT_MI355X_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/${V}_$C" -o run --output-format csv -- \
        python3 bench.py --config $CFG --precision $PREC --steps 1 --warmup 0 --cpu-seconds 0 --other-precision 0 \
        > "$OUT/${V}_$C.log" 2>&1 || { echo "$V $C failed"; exit 1; }
  done
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, sys
out, vs = sys.argv[1], sys.argv[2:]
for v in vs:
    r = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [x for f in glob.glob(f"{out}/{v}_{c}/**/*counter_collection.csv", recursive=True)
                for x in csv.DictReader(open(f)) if "trace_paths" in x["Kernel_Name"]]
        r[c] = sum(float(x["Counter_Value"]) for x in rows) * 1024 / 1e9
    print(f"{v:12s} fetch(x2) {2 * r['FETCH_SIZE']:7.2f} GB  write {r['WRITE_SIZE']:7.2f} GB  "
          f"total {2 * r['FETCH_SIZE'] + r['WRITE_SIZE']:7.2f} GB")
PY
