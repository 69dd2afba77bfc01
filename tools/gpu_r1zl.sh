set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zl
mkdir -p $O
F="crc G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw0,opt2 xw31:29,oversub,roof G32 CH8 NBUF2 AUX2 wg/cu1 xw0"
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 8 20 > $O/explore_4k.log 2>&1
F="crc G64 CH4 NBUF2 AUX2 wg/cu1 opt0 xw0,G64 CH4 NBUF2 AUX2 wg/cu1 opt0 xw31,oversub,roof G64 CH4 NBUF2 AUX2 wg/cu2 xw0"
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 65536 65536 8 20 > $O/explore_64k.log 2>&1
echo ALLDONE
