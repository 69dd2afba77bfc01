# parallel segment combine (rows path): parity incl. single 48-64 MiB blocks, few-large timing
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzl
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python tools/bench_paths.py few > $O/few.jsonl 2> $O/few.err
echo ALLDONE
