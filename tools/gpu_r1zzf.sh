# concurrency test (threads x streams x segmented paths), full gpu suite, smoke, bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzf
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
echo ALLDONE
