mkdir -p gpurun_out/r9
for i in 1 2; do for L in base CAM SCATTER SWEEP; do
  LIB=""; [ $L != base ] && LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_dup_$L.so
  RT_MI355X_LIB=$LIB timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 3 > gpurun_out/r9/${L}_$i.log 2>&1 || exit $?
done; done
