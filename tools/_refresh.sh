#!/bin/bash
# Profile refresh (on the GPU box, from the repo root): the driver's bench
# command (20 steps, 5 warmup, with the CPU baseline), the rocprofv3
# kernel-trace summary of the same command (no CPU leg), the PMC traffic
# passes, cfg5 on one GPU and the ratio-pair batch.  usage: tools/_refresh.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/refresh}
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || exit 2
bash tools/pmc_run.sh $O/pmc --no-cpu --steps 3 --warmup 1 || exit 3
timeout -k 10 600 python3 bench.py --gpus 1 --config cfg5 --steps 3 --warmup 1 --no-cpu > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 4
timeout -k 10 600 python3 tools/pairs_bench.py > $O/pairs.json 2> $O/pairs.err || exit 5
