mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cone_cull or filter_off or camera_inside or every_primary" > gpurun_out/r3/gputests.log 2>&1 || exit $?
for i in 1 2; do for W in 6 5; do RT_WAVES=$W timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 5 --precision f32 > gpurun_out/r3/b_f32_W${W}_$i.log 2>&1 || exit $?; done; done
timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 5 --precision f64 > gpurun_out/r3/b_f64.log 2>&1 || exit $?
