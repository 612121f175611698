mkdir -p gpurun_out/r10
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r10/gputests.log 2>&1 || exit $?
bash tools/ab_same_box.sh f32 3 > gpurun_out/r10/ab_f32.txt 2>&1 || exit $?
bash tools/ab_same_box.sh f64 2 > gpurun_out/r10/ab_f64.txt 2>&1 || exit $?
