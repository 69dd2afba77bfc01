# G16 plans at one workgroup per CU: gpu suite, blocks paths with and without priority
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python tools/bench_paths.py blocks > $O/paths.jsonl 2> $O/paths.err
PRISKV_CRC_PRIO=0 timeout -k 10 300 python tools/bench_paths.py blocks > $O/paths_noprio.jsonl 2> $O/paths_noprio.err
echo ALLDONE
