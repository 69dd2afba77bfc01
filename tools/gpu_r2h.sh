# progress-priority experiment (rows kernel OPT bit 8) on the 4 KiB plan, with per-wave timing
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2h
mkdir -p $O
F="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 xw31:29,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 | 256,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt10 xw31:29,nib G32 CH8 NBUF2 AUX2 wg/cu1 opt2 | 8 | 256"
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 16 10 > $O/explore_4k_prio.log 2>&1
EXPLORE_FILTER="$F" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 16 10 > $O/explore_4k_prio_b.log 2>&1
echo ALLDONE
