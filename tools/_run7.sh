mkdir -p gpurun_out/r7
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RT_MI355X_LIB=$PWD/rust-ray-tracing_amd/lib/librt_mi355x_exp.so timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 -d gpurun_out/r7/pcs -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --steps 1 --warmup 0 > gpurun_out/r7/pcs.log 2>&1
echo "rc=$?" >> gpurun_out/r7/pcs.log
ls -la gpurun_out/r7/pcs >> gpurun_out/r7/pcs.log 2>&1
