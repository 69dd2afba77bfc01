set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1i
mkdir -p $O
timeout -k 10 400 python -m pytest tests -x -q -m "gpu and not slow" > $O/pytest.log 2>&1
export EXPLORE_FILTER="crc G16 CH16 NBUF2 AUX2 wg/cu1,crc G32 CH8 NBUF2 AUX2 wg/cu1,crc2 G32 CH4 NBUF2 AUX2 wg/cu1,roof G64 CH4 NBUF2 AUX2 wg/cu2,crc G64 CH4 NBUF2 AUX2 wg/cu1"
timeout -k 10 200 ./tools/crc_explore 4096 $((1<<20)) 10 50 > $O/explore_4k.log 2>&1
timeout -k 10 200 ./tools/crc_explore 65536 $((1<<16)) 10 50 > $O/explore_64k.log 2>&1
timeout -k 10 200 python bench.py > $O/bench.log 2>&1
echo ALLDONE
