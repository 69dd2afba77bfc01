# progress-priority modes for the 1 KiB (G16 pipelined), 3 KiB (G16 CH4) and 2 KiB (G64 CH2) plans
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2k
mkdir -p $O
N16="nib G16 CH4 NBUF2 AUX2 wg/cu2"
C16="crc G16 CH4 NBUF2 AUX2 wg/cu2"
C642="crc G64 CH2 NBUF2 AUX2 wg/cu1"
for r in a b; do
EXPLORE_FILTER="$N16 opt2 xw31:29,$N16 opt2 | 256,$N16 opt2 | 512,$N16 opt2 | 768" timeout -k 10 300 ./tools/crc_explore 1024 $((1<<22)) 16 10 > $O/explore_1k_prio_$r.log 2>&1
EXPLORE_FILTER="$C16 opt0 xw31:29,$C16 opt256,$C16 opt768" timeout -k 10 300 ./tools/crc_explore 3072 $((1<<20)) 16 10 > $O/explore_3k_prio_$r.log 2>&1
EXPLORE_FILTER="$C642 opt0 xw31:29,$C642 opt256,$C642 opt768" timeout -k 10 300 ./tools/crc_explore 2048 $((1<<21)) 16 10 > $O/explore_2k_prio_$r.log 2>&1
done
echo ALLDONE
