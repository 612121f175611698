#!/bin/bash
# A/B the two kernel schedules (RT_KERNEL=paths|waves) after a parity run; logs under gpurun_out/.
set -e
timeout -k 10 120 python -m pytest tests/test_gpu_parity.py -x -q -k "config_a_full" > gpurun_out/par0.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/par.log 2>&1
for K in paths waves; do for P in f32 f64; do
  RT_KERNEL=$K timeout -k 10 200 python bench.py --precision $P --steps 3 --cpu-seconds 0 > gpurun_out/ab_${K}_$P.log 2>&1
done; done
