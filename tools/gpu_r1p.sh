set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1p
mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m "gpu" > $O/pytest.log 2>&1
timeout -k 10 400 python tools/bench_paths.py > $O/paths.log 2>&1
timeout -k 10 200 python bench.py > $O/bench.log 2>&1
echo ALLDONE
