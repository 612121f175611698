mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/gputests.log 2>&1 || exit $?
for P in f32 f64; do bash tools/ab_same_box.sh $P 2 > gpurun_out/r4/ab_$P.txt 2>&1 || exit $?; done
