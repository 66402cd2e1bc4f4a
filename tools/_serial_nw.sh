#!/bin/bash
# Record pipeline with every kernel on one stream: rocprof kernel stats per
# digit width, then the HBM traffic passes.  usage: tools/_serial_nw.sh OUTDIR
export TMPDIR=/tmp
O=${1:-gpurun_out/snw}
mkdir -p $O
export RK_ONE_STREAM=1
for B in 8 10; do
  export RK_NW_BITS=$B
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$B -o p -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/k$B.log 2>&1 || exit 1
done
export RK_NW_BITS=8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o p -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/pf.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o p -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/pw.log 2>&1 || exit 3
