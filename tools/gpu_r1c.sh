set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r1c
timeout -k 10 300 python -m pytest tests -x -q -m "gpu and not slow" > $R/gpurun_out/r1c/pytest.log 2>&1
timeout -k 10 150 ./tools/crc_explore 4096 $((1<<20)) 4 200 > $R/gpurun_out/r1c/explore_4k.log 2>&1
timeout -k 10 150 ./tools/crc_explore 65536 $((1<<16)) 4 200 > $R/gpurun_out/r1c/explore_64k.log 2>&1
timeout -k 10 150 ./tools/crc_explore 1048576 4096 4 200 > $R/gpurun_out/r1c/explore_1m.log 2>&1
timeout -k 10 200 python bench.py > $R/gpurun_out/r1c/bench.log 2>&1
echo ALLDONE
