mkdir -p gpurun_out/sx
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sx/t0 -o p -- python3 bench.py --no-cpu --steps 1 --warmup 1 > gpurun_out/sx/t0.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/sx/pa -o p -- python3 bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/sx/pa.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d gpurun_out/sx/pb -o p -- python3 bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/sx/pb.log 2>&1
