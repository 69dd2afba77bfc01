# segmentation limit 8192: all GPU tests, small-call latency, paths for ranges
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python tools/small_call_latency.py > $O/small_call_latency.jsonl 2> $O/small_call_latency.err
timeout -k 10 300 python tools/bench_paths.py seglimit > $O/seglimit.jsonl 2> $O/seglimit.err
echo ALLDONE
