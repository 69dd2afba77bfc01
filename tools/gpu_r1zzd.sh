# slice-by-8 pair steps (s8) vs the nibble-fold product at 4 KiB (explorer, in-process)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzd
mkdir -p $O
EXPLORE_FILTER="G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31:29,s8 G32,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt6,roof G32 CH8 NBUF2 AUX2 wg/cu1 xw31:29,G32 CH8 NBUF2 AUX2 wg/cu1 opt10 xw31:29" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 12 100 > $O/explore_4k_s8.log 2>&1
echo ALLDONE
