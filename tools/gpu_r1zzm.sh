# HIP graph capture / replay of the device paths (incl. stream-ordered scratch)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "graph" --timeout 200 --timeout-method thread > $O/pytest_graph.log 2>&1
echo ALLDONE
