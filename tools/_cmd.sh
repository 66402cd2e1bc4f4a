export TMPDIR=/tmp; mkdir -p gpurun_out/r2v
for v in 9 10 9 10; do RK_ORDER_BITS=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r2v/b$v.$RANDOM.json 2>> gpurun_out/r2v/err || exit 1; done
