set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r1b
timeout -k 10 120 ./tools/crc_explore 4096 $((1<<20)) 3 400 > $R/gpurun_out/r1b/explore_4k.log 2>&1
PRISKV_BENCH_TRACE=1 timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r1b/bench_w3.log 2>&1
PRISKV_BENCH_TRACE=1 timeout -k 10 120 python bench.py --steps 100 --warmup 50 --no-cpu-baseline > $R/gpurun_out/r1b/bench_w50.log 2>&1
PRISKV_BENCH_TRACE=1 timeout -k 10 120 python bench.py --steps 300 --warmup 300 --no-cpu-baseline > $R/gpurun_out/r1b/bench_w300.log 2>&1
echo ALLDONE
