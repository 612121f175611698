mkdir -p gpurun_out/r6
bash tools/ab_same_box.sh f32 2 > gpurun_out/r6/ab_skipreplay.txt 2>&1 || exit $?
bash tools/pmc.sh gpurun_out/r6/pmc > gpurun_out/r6/pmc.log 2>&1 || exit $?
