#!/bin/bash
# Profile refresh (on the GPU box, from the repo root): the bench line with the
# CPU baseline, the rocprofv3 kernel-trace summary of the same command (no CPU
# leg), and the PMC traffic passes.  usage: tools/_refresh.sh OUTDIR
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/refresh}
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof.log 2>&1
tools/pmc_run.sh $O/pmc --no-cpu --steps 3 --warmup 1
