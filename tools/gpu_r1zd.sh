set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zd
mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m "gpu" > $O/pytest.log 2>&1
timeout -k 10 300 ./tools/batch_bench 4 4096 16 2 > $O/batch_bench.log 2>&1
echo ALLDONE
