set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/t5.log 2>&1
for W in 1 4 5 6 8; do
  RT_WAVES=$W timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 2 > gpurun_out/b5_f32_w$W.log 2>&1
  RT_WAVES=$W timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 2 --precision f64 > gpurun_out/b5_f64_w$W.log 2>&1
done
