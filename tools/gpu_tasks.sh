#!/bin/bash
# GPU-box command tasks for gpurun (run from the repo root).  Every GPU step
# has its own time limit and a task stops at its first failure.
#
#   bash tools/gpu_tasks.sh TASK OUTDIR [ARGS...]
#
#   suite     smoke() and the whole GPU suite, as the driver runs them
#   bench     the driver's bench command (cfg3, 20 steps, CPU baseline)
#   parity    tests/test_gpu_parity.py (both pipelines against the oracle)
#   check     parity + sharded tests, the cfg5q digests, the cfg5 bench, a
#             2-rank rehearsal
#   refresh   bench + rocprofv3 --kernel-trace --stats of it + the PMC passes
#             (tools/pmc_run.sh) + cfg5 on one GPU + the ratio-pair batch
#   cfg5      tools/cfg5_check.py (1B fragments: timing, determinism,
#             properties) and the cfg5 bench line
#   ablib     record-pipeline parity, then benches of the working tree's
#             library interleaved with ablib_base/ (a build of an earlier
#             HEAD) through RK_LIB
#   abenv     the same with environment variants: ARGS = "VAR=a" "VAR=b" ...
#   abenv5    parity + cfg5q digests, then cfg5 with environment variants
#   trace     per-tile phase times of every record pass (RK_NW_TRACE)
#   shard     sharded parity tests (+ the large sharded digests with ARGS=large)
#             and the world-1 sharded bench
#   rehearse  the N > 1 bench line on one GPU: 2 and 4 ranks (ARGS) on device 0
#             over gloo host callbacks, cfg3's one 50M set strong-scaled with
#             its digest gathered; then the world-1 sharded leg
#   io        tools/io_bench.py at cfg3 (the file path against the reference)
#   fast      the sharded fast path: its tests, the sharded suite, rehearsals, world 1
#   rehearse_rccl  the same over RCCL (which refuses two ranks on one GPU:
#             value null with the error)
#   serial    per-kernel times with every kernel on one stream (RK_ONE_STREAM=1)
#   pmc5      the PMC passes at cfg5 (one timed step) -> OUTDIR/pmc5
#   shprof    rocprofv3 --kernel-trace --stats of the world-1 sharded bench
export TMPDIR=/tmp
TASK=$1
O=${2:-gpurun_out/$TASK}
shift 2
mkdir -p $O

bench() {  # bench NAME [bench args...]
  local name=$1
  shift
  timeout -k 10 600 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err
}

case $TASK in
suite)
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
  timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
  ;;
bench)
  bench bench --gpus 1 --steps 20 --warmup 5 || exit 1
  ;;
refresh)
  bench bench --gpus 1 --steps 20 --warmup 5 || exit 1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof.log 2>&1 || exit 2
  bash tools/pmc_run.sh $O/pmc --no-cpu --steps 3 --warmup 1 || exit 3
  bench bench_cfg5 --gpus 1 --config cfg5 --steps 3 --warmup 1 --no-cpu || exit 4
  timeout -k 10 600 python3 tools/pairs_bench.py > $O/pairs.json 2> $O/pairs.err || exit 5
  ;;
cfg5)
  timeout -k 10 600 python3 -u tools/cfg5_check.py --out $O/cfg5_check.json > $O/cfg5_check.log 2>&1 || exit 1
  bench bench_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 2
  ;;
longprof)  # the long-run walk's counters (RK_SWEEP_PROF build under tools/mb/prof)
  RK_LIB=tools/mb/prof/librepkiller_amd.so bench long_cfg5 --config cfg5 --no-cpu --steps 1 --warmup 0 || exit 1
  RK_LIB=tools/mb/prof/librepkiller_amd.so bench long_cfg3 --no-cpu --steps 1 --warmup 0 || exit 2
  ;;
lprof)  # parity + cfg3 bench of the working tree, then the long-run walk's counters at cfg5 with / without the list dedup
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  bench bench --no-cpu --steps 20 --warmup 5 || exit 2
  RK_LIB=tools/mb/prof/librepkiller_amd.so bench long_cfg5 --config cfg5 --no-cpu --steps 1 --warmup 0 || exit 3
  RK_LIB=tools/mb/nodedup/librepkiller_amd.so bench long_cfg5_nodedup --config cfg5 --no-cpu --steps 1 --warmup 0 || exit 4
  ;;
lcheck)  # the long-run walk: parity (long runs, cfg5q digests), the cfg5 bench, its counters (RK_SWEEP_PROF build)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  timeout -k 10 900 python3 -u -m pytest tests/test_large_configs.py -x -v -k cfg5q --timeout 600 --timeout-method thread > $O/cfg5q.log 2>&1 || exit 2
  bench bench_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 3
  RK_LIB=tools/mb/prof/librepkiller_amd.so bench long_cfg5 --config cfg5 --no-cpu --steps 1 --warmup 0 || exit 4
  ;;
lwhere)  # where k_sweep_long32's time goes at cfg5: a kernel trace of one step, and the counters of every sweep
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/ktrace -o p -- python3 bench.py --config cfg5 --no-cpu --steps 1 --warmup 1 > $O/ktrace.log 2>&1 || exit 1
  RK_LIB=tools/mb/prof/librepkiller_amd.so bench long_cfg5 --config cfg5 --no-cpu --steps 1 --warmup 0 || exit 2
  ;;
heap)  # the depth-limit heapsort: parity of the std::sort emulation, then the killers' times
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v -k "std_sort" --timeout 300 --timeout-method thread > $O/heap_tests.log 2>&1 || exit 1
  timeout -k 10 600 python3 -u tools/heap_killer_check.py --tied ${@:-10000 100000 1000000} > $O/heap_killer.log 2>&1 || exit 2
  ;;
abw5)  # k_sweep_long32 at 5 wavefronts per SIMD (tools/mb/w5) against the working tree at cfg5
  RK_LIB=tools/mb/w5/librepkiller_amd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "long or synthetic" --timeout 300 --timeout-method thread > $O/parity_w5.log 2>&1 || exit 1
  for rep in 1 2; do
    RK_LIB=tools/mb/w5/librepkiller_amd.so bench w5_cfg5_$rep --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 2
    RK_LIB=repkiller_amd/librepkiller_amd.so bench main_cfg5_$rep --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 3
  done
  ;;
sprof3)  # the window sweep's sampled phase cycles at cfg3 (RK_SWEEP_PROF build under tools/mb/prof)
  RK_LIB=tools/mb/prof/librepkiller_amd.so bench sprof3 --no-cpu --steps 1 --warmup 0 || exit 1
  ;;
heapprof)  # kernel times of the tied killer (ARGS: sizes)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hprof -o p -- python3 tools/heap_killer_check.py --tied ${@:-100000} > $O/hprof.log 2>&1 || exit 1
  ;;
abcfg5)  # parity, then cfg5 / cfg3 against the HEAD build under tools/mb/base, then the counters
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  RK_LIB=repkiller_amd/librepkiller_amd.so bench new_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 2
  RK_LIB=tools/mb/base/librepkiller_amd.so bench base_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 3
  for rep in 1 2; do
    RK_LIB=repkiller_amd/librepkiller_amd.so bench new_$rep --gpus 1 --steps 20 --warmup 5 --no-cpu || exit 4
    RK_LIB=ablib_base/librepkiller_amd.so bench base_$rep --gpus 1 --steps 20 --warmup 5 --no-cpu || exit 5
  done
  RK_LIB=tools/mb/prof/librepkiller_amd.so bench long_cfg5 --config cfg5 --no-cpu --steps 1 --warmup 0 || exit 6
  ;;
abcap)  # the long-run walk's own-list capacity at cfg5 (RK_LCAP builds under tools/mb/l*)
  for v in ${@:-l256 l512}; do
    RK_LIB=tools/mb/$v/librepkiller_amd.so bench ${v}_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 1
  done
  RK_LIB=repkiller_amd/librepkiller_amd.so bench main_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 2
  ;;
absplit)  # phase A / B boundary at cfg5 (RK_SPLIT_T builds under tools/mb/s*)
  for v in ${@:-s1024 s2048}; do
    RK_LIB=tools/mb/$v/librepkiller_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k std_sort --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || exit 1
    RK_LIB=tools/mb/$v/librepkiller_amd.so bench ${v}_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 2
  done
  ;;
parity)  # the record / generic pipelines against the oracle and the fixtures
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  ;;
check)  # parity + sharded tests + the cfg5q digests (one device, 8 ranks) + cfg5 bench + 2-rank rehearsal
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  timeout -k 10 900 python3 -u -m pytest tests/test_large_configs.py -x -v -k cfg5q --timeout 600 --timeout-method thread > $O/cfg5q.log 2>&1 || exit 2
  bench bench_cfg5 --config cfg5 --no-cpu --steps 3 --warmup 1 || exit 3
  RK_BENCH_SAME_GPU=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --comm host --steps 2 --warmup 1 --sharded-timeout 500 > $O/host2.json 2> $O/host2.err || exit 4
  ;;
ablib)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  for rep in 1 2 3; do
    RK_LIB=repkiller_amd/librepkiller_amd.so bench new_$rep --gpus 1 --steps 20 --warmup 5 --no-cpu || exit 2
    RK_LIB=ablib_base/librepkiller_amd.so bench base_$rep --gpus 1 --steps 20 --warmup 5 --no-cpu || exit 3
  done
  ;;
abenv)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  for rep in 1 2; do
    i=0
    for E in "$@"; do
      i=$((i+1))
      env $E timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/v${i}_$rep.json 2> $O/v${i}_$rep.err || exit 2
    done
  done
  ;;
abenv5)  # parity + the cfg5q digests, then cfg5 with environment variants (ARGS: "VAR=a" "VAR=b" ...) interleaved, two rounds
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  timeout -k 10 900 python3 -u -m pytest tests/test_large_configs.py -x -v -k cfg5q --timeout 600 --timeout-method thread > $O/cfg5q.log 2>&1 || exit 2
  for rep in 1 2; do
    i=0
    for E in "$@"; do
      i=$((i+1))
      env $E timeout -k 10 600 python3 bench.py --config cfg5 --no-cpu --steps 3 --warmup 1 > $O/v${i}_$rep.json 2> $O/v${i}_$rep.err || exit 3
    done
  done
  ;;
qpart)  # phase A's queue partition: std::sort parity + switches, the cfg5q digest, cfg5 with / without it
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v -k "std_sort or repeat_rich" --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  timeout -k 10 600 python3 -u -m pytest tests/test_large_configs.py -x -v -k "cfg5q_oracle_digest and not sharded" --timeout 500 --timeout-method thread > $O/cfg5q.log 2>&1 || exit 2
  for rep in 1 2; do
    for E in RK_SPLIT_Q=1 RK_SPLIT_Q=0; do
      env $E timeout -k 10 300 python3 bench.py --config cfg5 --no-cpu --steps 2 --warmup 1 > $O/${E}_$rep.json 2> $O/${E}_$rep.err || exit 3
    done
  done
  ;;
qvar)  # phase A's queue partition: parity of the working tree, then cfg5 against library variants (ARGS: dirs with a librepkiller_amd.so)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v -k "std_sort or repeat_rich" --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || exit 1
  timeout -k 10 600 python3 -u -m pytest tests/test_large_configs.py -x -v -k "cfg5q_oracle_digest and not sharded" --timeout 500 --timeout-method thread > $O/cfg5q.log 2>&1 || exit 2
  for rep in 1 2; do
    for D in repkiller_amd "$@"; do
      n=$(basename $D)
      RK_LIB=$D/librepkiller_amd.so timeout -k 10 300 python3 bench.py --config cfg5 --no-cpu --steps 2 --warmup 1 > $O/${n}_$rep.json 2> $O/${n}_$rep.err || exit 3
    done
    RK_SPLIT_Q=0 timeout -k 10 300 python3 bench.py --config cfg5 --no-cpu --steps 2 --warmup 1 > $O/listpart_$rep.json 2> $O/listpart_$rep.err || exit 4
  done
  ;;
env5)  # cfg5 with environment variants (ARGS: "VAR=a" "VAR=b" ...) interleaved, two rounds, no parity
  for rep in 1 2; do
    i=0
    for E in "$@"; do
      i=$((i+1))
      env $E timeout -k 10 600 python3 bench.py --config cfg5 --no-cpu --steps 2 --warmup 1 > $O/v${i}_$rep.json 2> $O/v${i}_$rep.err || exit 3
    done
  done
  ;;
trace)
  RK_NW_TRACE=$O/trace.bin timeout -k 10 300 python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/bt.json 2> $O/bt.err || exit 1
  python3 tools/nw_trace.py $O/trace.bin > $O/trace.txt 2>&1
  rm -f $O/trace.bin
  ;;
shard)
  timeout -k 10 600 python3 -u -m pytest tests/test_sharded.py -x -v --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 1
  if [ "$1" = large ]; then
    timeout -k 10 900 python3 -u -m pytest tests/test_large_configs.py -x -q -k sharded --timeout 600 --timeout-method thread > $O/large_tests.log 2>&1 || exit 2
  fi
  bench sharded_w1 --mode sharded --steps 20 --warmup 5 --no-cpu || exit 3
  ;;
rehearse)  # ARGS: world sizes (default 2 4); cfg3's one 50M set strong-scaled, parity gathered
  for W in ${@:-2 4}; do
    RK_BENCH_SAME_GPU=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29610 + W)) bench.py --gpus $W --comm host --steps 2 --warmup 1 --sharded-timeout 500 > $O/host$W.json 2> $O/host$W.err || exit 1
  done
  bench sharded_w1 --mode sharded --no-cpu --steps 5 --warmup 2 || exit 3
  ;;
fast)  # the sharded fast path: its tests, the whole sharded suite, the 2- and 4-rank rehearsals, world 1
  timeout -k 10 900 python3 -u -m pytest tests/test_sharded.py -x -v -k "fast" --timeout 300 --timeout-method thread > $O/fast_tests.log 2>&1 || exit 1
  timeout -k 10 1100 python3 -u -m pytest tests/test_sharded.py -x -v --timeout 300 --timeout-method thread > $O/sharded_tests.log 2>&1 || exit 2
  for W in 2 4; do
    RK_BENCH_SAME_GPU=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29610 + W)) bench.py --gpus $W --comm host --steps 2 --warmup 1 --sharded-timeout 500 > $O/host$W.json 2> $O/host$W.err || exit 3
  done
  bench sharded_w1 --mode sharded --no-cpu --steps 20 --warmup 5 || exit 4
  ;;
io)  # the whole file path at cfg3 (CSV in -> classify -> CSV out) against the reference on the same file
  T=/tmp
  if [ "$(df -Pk /dev/shm | awk 'NR==2 {print $4}')" -gt 30000000 ]; then T=/dev/shm; fi
  df -h /tmp /dev/shm > $O/df.txt 2>&1
  timeout -k 10 1100 python3 -u tools/io_bench.py --tmp $T > $O/io_bench.json 2> $O/io_bench.err || exit 1
  ;;
rehearse_rccl)  # RCCL refuses two ranks on one GPU: value null with the error
  RK_BENCH_SAME_GPU=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --config cfg2 --steps 3 --warmup 1 --sharded-timeout 60 > $O/rccl2.json 2> $O/rccl2.err
  echo "rccl2 exit $?" > $O/rccl2.rc
  ;;
serial)
  RK_ONE_STREAM=1 bench cfg3 --no-cpu || exit 1
  RK_ONE_STREAM=1 bench cfg5 --config cfg5 --no-cpu --steps 2 --warmup 1 || exit 2
  ;;
pmc5)
  bash tools/pmc_run.sh $O/pmc5 --config cfg5 --no-cpu --steps 1 --warmup 1 || exit 1
  ;;
shprof)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shprof -o p -- python3 bench.py --mode sharded --no-cpu --steps 10 --warmup 3 > $O/shprof.json 2> $O/shprof.err || exit 1
  ;;
*)
  echo "unknown task $TASK" >&2
  exit 64
  ;;
esac
