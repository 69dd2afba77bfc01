set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ze
mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m "gpu" -k "batcher or verify or ranges_host" > $O/pytest.log 2>&1
timeout -k 10 300 ./tools/batch_bench 4 4096 16 2 1 > $O/batch_bench_1.log 2>&1
timeout -k 10 300 ./tools/batch_bench 4 4096 16 2 16 > $O/batch_bench_16.log 2>&1
echo ALLDONE
