set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1h_$1
mkdir -p $O
export EXPLORE_FILTER="crc G16 CH16 NBUF2 AUX2 wg/cu1,crc G32 CH8 NBUF2 AUX2 wg/cu1,crc2 G32 CH4 NBUF2 AUX2 wg/cu1,crc G16 CH8 NBUF2 AUX2 wg/cu2,roof G64 CH4 NBUF2 AUX2 wg/cu2"
timeout -k 10 200 ./tools/crc_explore 4096 $((1<<20)) 12 50 > $O/explore_4k.log 2>&1
export EXPLORE_FILTER="crc G64 CH4 NBUF2 AUX2 wg/cu1,crc2 G64 CH2 NBUF2 AUX2 wg/cu1,crc G32 CH8 NBUF2 AUX2 wg/cu1,roof G64 CH4 NBUF2 AUX2 wg/cu2"
timeout -k 10 200 ./tools/crc_explore 65536 $((1<<16)) 12 50 > $O/explore_64k.log 2>&1
echo ALLDONE
