set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1z
mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m "gpu" > $O/pytest.log 2>&1
timeout -k 10 200 python bench.py > $O/bench.log 2>&1
timeout -k 10 200 env PRISKV_CRC_XCD_WEIGHTS=1:1 python bench.py --no-cpu-baseline > $O/bench_equal_split.log 2>&1
timeout -k 10 200 python bench.py > $O/bench2.log 2>&1
timeout -k 10 200 python bench.py --config sweep64k --no-cpu-baseline > $O/bench_64k.log 2>&1
timeout -k 10 200 python bench.py --config sweep1m --no-cpu-baseline > $O/bench_1m.log 2>&1
timeout -k 10 400 python tools/bench_paths.py > $O/paths.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_ktrace.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_pmc_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_pmc_write.log 2>&1
echo ALLDONE
