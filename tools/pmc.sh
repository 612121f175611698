#!/bin/bash
# Collect rocprofv3 PMC counters for the bench's trace kernel, one counter group per pass
# (never combined with tracing domains, per the GPU pool's rules).  Usage on the GPU box:
#   bash tools/pmc.sh <outdir> [bench args...]
# Writes <outdir>/pass<N>/*counter_collection.csv and <outdir>/list.txt.
set -u
OUT=${1:-gpurun_out/pmc}
shift || true
ARGS=${*:-"--cpu-seconds 0 --warmup 0 --steps 1"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SALU SQ_INSTS_VSKIPPED SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex trace_ -d "$OUT/pass$i" -o run \
      --output-format csv -- python3 bench.py $ARGS > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
