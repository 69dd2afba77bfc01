# new plan table (G64 for 8 KiB and up), small kernel nibble fold: tests, path sweep, bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zv
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 500 python tools/bench_paths.py > $O/paths.jsonl 2> $O/paths.err
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --config sweep64k > $O/bench_64k.log 2>&1
timeout -k 10 300 python bench.py --config sweep1m > $O/bench_1m.log 2>&1
echo ALLDONE
