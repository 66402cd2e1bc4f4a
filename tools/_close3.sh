#!/bin/bash
# round-3 close after the timer change: smoke, the GPU suite, the N>1 rehearsal
export TMPDIR=/tmp
O=gpurun_out/close3
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
bash tools/_rehearse.sh $O/reh > $O/reh.log 2>&1 || exit 3
