#!/bin/bash
# Build the stage-duplication experiment libraries (tools/exp/dup_stages.patch: RT_EXP_DUP_<STAGE> runs
# one stage twice, so time(dup) - time(base) is that stage's share) as lib/librt_mi355x_dup<STAGE>.so,
# four at a time.   bash tools/build_dups.sh [STAGE...]   (default: every stage the patch defines)
set -e
cd "$(dirname "$0")/../rust-ray-tracing_amd"
STAGES=${*:-$(grep -o 'RT_EXP_DUP_[A-Z]*' ../tools/exp/dup_stages.patch | sed 's/RT_EXP_DUP_//' | sort -u)}
HASH=$(cat csrc/*.hip csrc/*.hpp | sha256sum | cut -c1-12)
build() {
  local S=$1 D=build/exp_$1
  rm -rf "$D" && mkdir -p "$D" && cp csrc/*.hip csrc/*.hpp "$D/"
  for p in ../tools/exp/*.patch; do patch -s -p1 -d "$D" < "$p"; done
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -std=c++17 -Wno-unused-function \
      -mllvm -disable-vector-combine -Icsrc -DRT_EXPERIMENT -DRT_SRC_HASH=\"$HASH\" -DRT_EXP_DUP_$S \
      -shared -o lib/librt_mi355x_dup$S.so "$D/rt_kernel.hip"
  echo "built dup$S"
}
N=0
for S in $STAGES; do
  build "$S" &
  N=$((N + 1))
  if [ $((N % 4)) -eq 0 ]; then wait; fi
done
wait
