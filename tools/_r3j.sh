#!/bin/bash
# Round 3 refresh on HEAD: the driver's bench command, rocprof summary, PMC traffic passes.
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || exit 2
bash tools/pmc_run.sh $O/pmc --no-cpu --steps 3 --warmup 1 || exit 3
