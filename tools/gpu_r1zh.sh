set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zh
mkdir -p $O
F="opt2 xw0,opt2 xw31,crc pair,roof pair,roof G32 CH8 NBUF2 AUX2 wg/cu1 xw0,roof G64 CH4 NBUF2 AUX2 wg/cu2 xw0,G64 CH4 NBUF2 AUX2 wg/cu1 opt0 xw0"
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 8 20 > $O/explore_4k.log 2>&1
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 65536 65536 8 20 > $O/explore_64k.log 2>&1
echo ALLDONE
