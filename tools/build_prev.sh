#!/bin/bash
# Build the kernel sources of a git revision (default HEAD) as lib/librt_mi355x_exp.so for same-box A/B
# against the working tree (tools/ab_same_box.sh).  Usage: bash tools/build_prev.sh [rev] [extra hipcc flags]
# Works for revisions before the round-4 split (one rt_kernel.hip) and after it (csrc/*.hpp too).
set -e
REV=${1:-HEAD}; shift || true
cd "$(dirname "$0")/../rust-ray-tracing_amd"
D=build/prev
rm -rf "$D" && mkdir -p "$D"
git archive "$REV" csrc | tar -x -C "$D" --strip-components=1
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -std=c++17 -Wno-unused-function \
    -mllvm -disable-vector-combine -Icsrc -DRT_EXPERIMENT "$@" -shared -o lib/librt_mi355x_exp.so "$D/rt_kernel.hip"
