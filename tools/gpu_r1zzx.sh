# C executables (PrisKV unit-test style) on the GPU box
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzx
mkdir -p $O
timeout -k 10 200 ./tests/c/test_crc_gpu > $O/test_crc_gpu.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_c_executables.py -v -m gpu --timeout 200 --timeout-method thread > $O/pytest_c.log 2>&1
echo ALLDONE
