#!/bin/bash
# Parity, then the waves-per-SIMD sweep of the default kernel (bench lines under gpurun_out/).
set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/t5.log 2>&1
for W in ${WAVES_F32:-4 5 6 8}; do
  RT_WAVES=$W timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 2 > gpurun_out/b5_f32_w$W.log 2>&1
done
for W in ${WAVES_F64:-4 5 6}; do
  RT_WAVES=$W timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 2 --precision f64 > gpurun_out/b5_f64_w$W.log 2>&1
done
