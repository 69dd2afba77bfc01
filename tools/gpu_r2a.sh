# XCD weight sweep for the nibble-fold 4 KiB product (explorer, same process), finer ratios
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2a
mkdir -p $O
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 16 10 > $O/explore_4k_nib_xw.log 2>&1
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 16 10 > $O/explore_4k_nib_xw_b.log 2>&1
echo ALLDONE
