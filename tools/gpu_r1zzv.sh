# 1024-thread plan + 64-way segment search: parity (many extents), count-rule sweep 512 vs 16384
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzv
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 500 python tools/bench_paths.py seglimit > $O/seglimit.jsonl 2> $O/seglimit.err
echo ALLDONE
