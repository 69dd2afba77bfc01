# byte-balanced extents split: gpu suite (first the new test alone), then ranges paths with/without it
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k balanced_split --timeout 200 --timeout-method thread > $O/pytest_bal.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
timeout -k 10 300 python tools/bench_paths.py ranges > $O/paths_$i.jsonl 2> $O/paths_$i.err
PRISKV_CRC_BALANCE=0 timeout -k 10 300 python tools/bench_paths.py ranges > $O/paths_nobal_$i.jsonl 2> $O/paths_nobal_$i.err
done
echo ALLDONE
