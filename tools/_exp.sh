mkdir -p gpurun_out/sx
for m in 0 1 2; do
  RK_SWEEP_EXP=$m timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sx/e$m -o p -- python3 bench.py --no-cpu --steps 1 --warmup 1 > gpurun_out/sx/e$m.log 2>&1
done
