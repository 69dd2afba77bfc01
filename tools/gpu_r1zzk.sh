# cache-policy bits, repeat with more rounds (4 KiB product aux 2 / 3 / 18 / 19), two processes
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzk
mkdir -p $O
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31,nib G32 CH8 NBUF2 AUX18 wg/cu1 opt2 xw31,nib G32 CH8 NBUF2 AUX3 wg/cu1 opt2 xw31,nib G32 CH8 NBUF2 AUX19 wg/cu1 opt2 xw31" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 30 10 > $O/explore_4k_aux_a.log 2>&1
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX18 wg/cu1 opt2 xw31,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 30 10 > $O/explore_4k_aux_b.log 2>&1
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31,nib G32 CH8 NBUF2 AUX18 wg/cu1 opt2 xw31" timeout -k 10 300 ./tools/crc_explore 65536 $((1<<16)) 10 10 > $O/explore_64k_aux.log 2>&1
echo ALLDONE
