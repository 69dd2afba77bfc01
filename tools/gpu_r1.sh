set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r1
timeout -k 10 300 python -m pytest tests -x -q -m "gpu and not slow" > $R/gpurun_out/r1/pytest.log 2>&1
timeout -k 10 120 ./tools/crc_explore 4096 > $R/gpurun_out/r1/explore_4k.log 2>&1
timeout -k 10 120 ./tools/crc_explore 65536 > $R/gpurun_out/r1/explore_64k.log 2>&1
timeout -k 10 120 ./tools/crc_explore 1048576 > $R/gpurun_out/r1/explore_1m.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r1/ktrace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r1/bench_ktrace.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r1/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r1/bench_pmc_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r1/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r1/bench_pmc_write.log 2>&1
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/r1/counters.txt 2>&1 || true
echo ALLDONE
