# segmentation rule with host length hints: full gpu tests, few-values timing, every-path sweep
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python tools/bench_paths.py few > $O/few.jsonl 2> $O/few.err
timeout -k 10 500 python tools/bench_paths.py ranges host memfile > $O/paths.jsonl 2> $O/paths.err
echo ALLDONE
