# binding argument checks: full gpu suite
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzi
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo ALLDONE
