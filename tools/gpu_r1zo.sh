# HEAD verification after container re-creation: gpu tests, smoke, bench, kernel-trace stats
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zo
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/ktrace.log 2>&1
echo ALLDONE
