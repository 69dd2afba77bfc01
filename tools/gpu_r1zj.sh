set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zj
mkdir -p $O
F="crc G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw0,crc pair G32,roof pair G32,roof G32 CH8 NBUF2 AUX2 wg/cu1 xw0"
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 8 20 > $O/explore_4k.log 2>&1
echo ALLDONE
