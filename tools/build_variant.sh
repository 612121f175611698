#!/bin/bash
# Build an A/B variant of the kernel library from a copy of csrc/ (an experiment build: rt_version() says
# "experiment", so the loader takes it only with RT_ALLOW_EXPERIMENT=1, as tools/ab_libs.sh sets).
#   bash tools/build_variant.sh <name> [patch.py ...]
# copies rust-ray-tracing_amd/csrc to rust-ray-tracing_amd/vsrc_<name>/, runs each patch script there (python3
# <patch> <dir> [arg], written patch.py or patch.py:arg), and builds rust-ray-tracing_amd/lib/librt_mi355x_<name>.so.  vsrc_*/ and the variant
# libraries stay out of git and off the GPU push (.gitignore, .gpurunignore) except the libraries the A/B
# run names (VARIANT_FLAGS: extra compiler flags, e.g. -DRT_KSTATS); delete them (rm rust-ray-tracing_amd/lib/librt_mi355x_v*.so) after the measurement.
set -eo pipefail
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/rust-ray-tracing_amd/vsrc_$NAME
rm -rf "$D" && mkdir -p "$D" && cp "$R"/rust-ray-tracing_amd/csrc/*.hip "$R"/rust-ray-tracing_amd/csrc/*.hpp "$D"/
for P in "$@"; do python3 "${P%%:*}" "$D" $([ "$P" != "${P%%:*}" ] && echo "${P#*:}"); done
rm -f "$R"/rust-ray-tracing_amd/lib/librt_mi355x_$NAME.so   # a failed build must not leave the previous variant
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -std=c++17 -Wall -Wno-unused-function \
    -mllvm -disable-vector-combine -DRT_EXPERIMENT -DRT_SRC_HASH=\"v_$NAME\" ${VARIANT_FLAGS:-} -shared \
    -o "$R"/rust-ray-tracing_amd/lib/librt_mi355x_$NAME.so "$D"/rt_kernel.hip 2>&1 | { grep -E "error|warning: failed" || true; }
ls -la "$R"/rust-ray-tracing_amd/lib/librt_mi355x_$NAME.so
