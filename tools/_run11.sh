mkdir -p gpurun_out/r11
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r11/gputests.log 2>&1 || exit $?
bash tools/ab_same_box.sh f32 3 > gpurun_out/r11/ab_f32.txt 2>&1 || exit $?
bash tools/ab_same_box.sh f64 2 > gpurun_out/r11/ab_f64.txt 2>&1 || exit $?
RT_MI355X_LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_kstats.so timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 1 --warmup 0 > gpurun_out/r11/kstats_f32.log 2>&1 || exit $?
