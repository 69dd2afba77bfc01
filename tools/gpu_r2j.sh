# progress-priority modes, second box, two runs per size
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2j
mkdir -p $O
N4="nib G32 CH8 NBUF2 AUX2 wg/cu1"
C64="crc G64 CH4 NBUF2 AUX2 wg/cu1"
N64="nib G64 CH4 NBUF2 AUX2 wg/cu1"
for r in a b; do
EXPLORE_FILTER="$N4 opt2 xw31:29,$N4 opt2 | 256 xw,$N4 opt2 | 512 xw31,$N4 opt2 | 768 xw" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 16 10 > $O/explore_4k_prio_$r.log 2>&1
EXPLORE_FILTER="$C64 opt0 xw31:29,$C64 opt256 xw,$C64 opt512 xw,$C64 opt768 xw" timeout -k 10 300 ./tools/crc_explore 65536 $((1<<16)) 16 10 > $O/explore_64k_prio_$r.log 2>&1
EXPLORE_FILTER="$C64 opt0 xw31:29,$C64 opt256 xw,$C64 opt512 xw,$C64 opt768 xw" timeout -k 10 300 ./tools/crc_explore $((1<<20)) 4096 16 10 > $O/explore_1m_prio_$r.log 2>&1
EXPLORE_FILTER="$N64 opt0 xw31:29,$N64 opt256 xw,$N64 opt512 xw,$N64 opt768 xw" timeout -k 10 300 ./tools/crc_explore 8192 $((1<<19)) 16 10 > $O/explore_8k_prio_$r.log 2>&1
done
echo ALLDONE
