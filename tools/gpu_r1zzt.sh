# count rule 2048 adopted: full gpu suite, few-values + seglimit timing
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzt
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python tools/bench_paths.py few seglimit > $O/few.jsonl 2> $O/few.err
echo ALLDONE
