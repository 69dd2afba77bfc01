# pooled scratch of the *_dev paths: all GPU tests, small-call latency (pool on / off), few-values paths
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "scratch_pool or concurrent or graph" --timeout 200 --timeout-method thread > $O/pytest_pool.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python tools/small_call_latency.py > $O/small_call_latency_pool.jsonl 2> $O/scl.err
PRISKV_CRC_SCRATCH_POOL=0 timeout -k 10 200 python tools/small_call_latency.py > $O/small_call_latency_nopool.jsonl 2>> $O/scl.err
timeout -k 10 300 python tools/bench_paths.py few > $O/few.jsonl 2> $O/few.err
echo ALLDONE
