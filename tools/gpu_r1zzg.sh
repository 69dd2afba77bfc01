# static head + per-XCD pooled tail (explorer) vs the product split at 4 KiB
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzg
mkdir -p $O
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31:29,tail G32,roof G32 CH8 NBUF2 AUX2 wg/cu1 xw31:29" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 10 50 > $O/explore_4k_tail.log 2>&1
echo ALLDONE
