set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1k
mkdir -p $O
timeout -k 10 400 python -m pytest tests -x -q -m "gpu and not slow" > $O/pytest.log 2>&1
export EXPLORE_FILTER="crc G,roof G64 CH4 NBUF2 AUX2 wg/cu2"
timeout -k 10 200 ./tools/crc_explore 4096 $((1<<20)) 10 50 > $O/explore_4k.log 2>&1
echo ALLDONE
