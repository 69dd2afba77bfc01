# extents kernel in 16-wave workgroups with progress priority: gpu suite, paths sweep of the extents cases, C test
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python tools/bench_paths.py blocks ranges > $O/paths.jsonl 2> $O/paths.err
PRISKV_CRC_PRIO=0 timeout -k 10 300 python tools/bench_paths.py blocks ranges > $O/paths_noprio.jsonl 2> $O/paths_noprio.err
echo ALLDONE
