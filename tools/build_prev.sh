#!/bin/bash
# Build the kernel source of a git revision (default HEAD) as lib/librt_mi355x_exp.so for same-box A/B
# against the working tree (tools/ab_same_box.sh).  Usage: bash tools/build_prev.sh [rev] [extra hipcc flags]
set -e
REV=${1:-HEAD}; shift || true
cd "$(dirname "$0")/../rust-ray-tracing_amd"
git show "$REV:rust-ray-tracing_amd/csrc/rt_kernel.hip" > csrc/_ab_prev.hip
trap 'rm -f csrc/_ab_prev.hip' EXIT
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -std=c++17 -Wno-unused-function "$@" -shared \
    -o lib/librt_mi355x_exp.so csrc/_ab_prev.hip
