# 2-3 KiB plan (G16 CH4): one vs two 8-wave workgroups per CU, with and without priority
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2y
mkdir -p $O
for r in a b; do
EXPLORE_FILTER="crc G16 CH4 NBUF2 AUX2 wg/cu2 opt0 xw31:29,crc G16 CH4 NBUF2 AUX2 wg/cu2 opt256,crc G16 CH4 NBUF2 AUX2 wg/cu1 opt0,crc G16 CH4 NBUF2 AUX2 wg/cu1 opt256" timeout -k 10 300 ./tools/crc_explore 3072 $((1<<20)) 12 10 > $O/explore_3k_$r.log 2>&1
EXPLORE_FILTER="crc G16 CH4 NBUF2 AUX2 wg/cu2 opt0 xw31:29,crc G16 CH4 NBUF2 AUX2 wg/cu2 opt256,crc G16 CH4 NBUF2 AUX2 wg/cu1 opt0,crc G16 CH4 NBUF2 AUX2 wg/cu1 opt256" timeout -k 10 300 ./tools/crc_explore 2048 $((1<<21)) 12 10 > $O/explore_2k_$r.log 2>&1
done
echo ALLDONE
