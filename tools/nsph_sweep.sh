for N in 4 20 100 250 500; do
  timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 2 --max-spheres $N > gpurun_out/nsph_$N.log 2>&1 || exit 1
done
