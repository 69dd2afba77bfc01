# progress-priority modes (rows kernel OPT bits 8-9) at 4 KiB, 8 KiB, 64 KiB, 1 MiB
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2i
mkdir -p $O
N4="nib G32 CH8 NBUF2 AUX2 wg/cu1"
EXPLORE_FILTER="$N4 opt2 xw31:29,$N4 opt2 | 256 xw,$N4 opt2 | 512 xw,$N4 opt2 | 768 xw" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 16 10 > $O/explore_4k_prio.log 2>&1
C64="crc G64 CH4 NBUF2 AUX2 wg/cu1"
EXPLORE_FILTER="$C64 opt0 xw31:29,$C64 opt256 xw,$C64 opt512 xw,$C64 opt768 xw" timeout -k 10 300 ./tools/crc_explore 65536 $((1<<16)) 16 10 > $O/explore_64k_prio.log 2>&1
EXPLORE_FILTER="$C64 opt0 xw31:29,$C64 opt256 xw,$C64 opt512 xw,$C64 opt768 xw" timeout -k 10 300 ./tools/crc_explore $((1<<20)) 4096 16 10 > $O/explore_1m_prio.log 2>&1
N64="nib G64 CH4 NBUF2 AUX2 wg/cu1"
EXPLORE_FILTER="$N64 opt0 xw31:29,$N64 opt256 xw,$N64 opt768 xw" timeout -k 10 300 ./tools/crc_explore 8192 $((1<<19)) 16 10 > $O/explore_8k_prio.log 2>&1
echo ALLDONE
