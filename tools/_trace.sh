#!/bin/bash
# traced record pipeline (one stream), then the GPU parity file and a bench
export TMPDIR=/tmp
O=${1:-gpurun_out/tr}
mkdir -p $O
RK_ONE_STREAM=1 RK_NW_TRACE=$O/t8.bin timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu > $O/b8.json 2> $O/b8.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > $O/b.json 2> $O/b.err || exit 3
