set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1m
mkdir -p $O
timeout -k 10 400 python -m pytest tests -x -q -m "gpu" > $O/pytest.log 2>&1
timeout -k 10 400 python tools/bench_paths.py ranges host > $O/paths.log 2>&1
echo ALLDONE
