#!/bin/bash
# The whole GPU suite and smoke(), as the driver runs them at round end.
export TMPDIR=/tmp
O=${1:-gpurun_out/suite}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
