# XCD weights for the G64 plans: 64 KiB and 1 MiB (bit-matrix fold), 8 KiB (nibble fold)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2c
mkdir -p $O
EXPLORE_FILTER="crc G64 CH4 NBUF2 AUX2 wg/cu1 opt0 xw" timeout -k 10 300 ./tools/crc_explore 65536 $((1<<16)) 12 10 > $O/explore_64k_xw.log 2>&1
EXPLORE_FILTER="crc G64 CH4 NBUF2 AUX2 wg/cu1 opt0 xw" timeout -k 10 300 ./tools/crc_explore $((1<<20)) 4096 12 10 > $O/explore_1m_xw.log 2>&1
EXPLORE_FILTER="nib G64 CH4 NBUF2 AUX2 wg/cu1 opt0 xw" timeout -k 10 300 ./tools/crc_explore 8192 $((1<<19)) 12 10 > $O/explore_8k_xw.log 2>&1
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw8:7,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31:29,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw7:6,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw21:19" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 16 10 > $O/explore_4k_xw.log 2>&1
echo ALLDONE
