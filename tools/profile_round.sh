#!/bin/bash
# One GPU call that produces the judged profile artefacts of a round for one config/precision:
#   <out>/pmc_{fetch,write,sq,issue}/  rocprofv3 --pmc passes of bench.py (one counter group each, counters only)
#   <out>/ubench_sq/              the same SQ pass over tools/bin/ubench_valu (VALU-saturating FMA chains:
#                                 calibrates SQ_ACTIVE_INST_VALU's unit and the FLOPS counters' lane scale)
#   <out>/bench.json              the bench line (after the PMC passes, so it reads this call's pmc.json)
#   <out>/ktrace/*stats.csv       rocprofv3 --kernel-trace --stats of the same bench command
#   <out>/pmc.json                HBM bytes / VALU busy / FLOP counters per launch (tools/pmc_round.py)
# Usage (GPU box): bash tools/profile_round.sh <out> [precision] [config]
set -u
OUT=${1:-gpurun_out/round}
PREC=${2:-f32}
CFG=${3:-C}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--config $CFG --precision $PREC --steps 1 --warmup 0 --cpu-seconds 0 --other-precision 0"
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_FMA_F32 GRBM_GUI_ACTIVE"
pass() {   # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$OUT/$name" -o run --output-format csv -- "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/status.txt"
  return $rc
}
pass pmc_fetch FETCH_SIZE python3 bench.py $ARGS || exit 1
pass pmc_write WRITE_SIZE python3 bench.py $ARGS || exit 1
pass pmc_sq "$SQ" python3 bench.py $ARGS || exit 1
# VALU pipe occupancy (round 6): SQ_ACTIVE_INST_VALU counts VALU quad-cycles (1 per instruction, 2 for an
# fp32 transcendental, 4 for an fp64 one) and SQ_ACTIVE_INST_VALU2 the quad-cycles in which two VALU
# instructions issued together (VGPR-only fp32/int32 ops), so 4 (ACTIVE - VALU2) is the SIMD-cycles the VALU
# pipe is occupied (tools/ubench_mix.hip, tools/ubench_bank2.hip: profiles/r06/issue_counters.txt)
ISSUE="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
pass pmc_issue "$ISSUE" python3 bench.py $ARGS || exit 1
# the VALU issue ceiling (valu_busy's denominator): built here if this tree has no binary
if [ ! -x tools/bin/ubench_valu ]; then
  mkdir -p tools/bin && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_valu tools/ubench_valu.hip \
      || { echo "ubench_valu build failed: no valu_busy" >> "$OUT/status.txt"; exit 1; }
fi
pass ubench_sq "$SQ" ./tools/bin/ubench_valu || exit 1
pass ubench_issue "$ISSUE" ./tools/bin/ubench_valu || exit 1
python3 tools/pmc_round.py "$OUT" "$CFG:$PREC:1" > "$OUT/pmc_summary.txt" 2>&1 || exit 1
# LINE_ARGS: the bench line's steps (config E: --steps 3 --warmup 1 --cpu-seconds 0; its CPU baseline on 10 000
# spheres outlasts the GPU box's silence limit)
LINE_ARGS=${LINE_ARGS:---steps 10 --warmup 2}
timeout -k 10 300 python3 bench.py --config "$CFG" --precision "$PREC" $LINE_ARGS --pmc "$OUT/pmc.json" \
    > "$OUT/bench.log" 2>&1 || exit 1
grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace" -o run --output-format csv -- \
    python3 bench.py --config "$CFG" --precision "$PREC" $LINE_ARGS --cpu-seconds 0 --other-precision 0 \
    --pmc "$OUT/pmc.json" > "$OUT/ktrace.log" 2>&1 || exit 1
echo "profile_round done" >> "$OUT/status.txt"
