# one segment size per call: gpu suite first, then ranges paths
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "segment or ranges" --timeout 200 --timeout-method thread > $O/pytest_seg.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
timeout -k 10 300 python tools/bench_paths.py ranges > $O/paths_$i.jsonl 2> $O/paths_$i.err
done
echo ALLDONE
