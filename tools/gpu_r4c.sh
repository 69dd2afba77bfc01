# validation of the rebuilt tree (fresh container): all GPU tests, smoke, C executables, bench, kernel trace
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 120 ./tests/c/test_crc_gpu > $O/c_gpu.log 2>&1
timeout -k 10 120 ./tests/c/test_crc_host > $O/c_host.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_kt.json 2> $O/bench_kt.err
echo ALLDONE
