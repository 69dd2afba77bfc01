# 1 KiB plan: one vs two 8-wave workgroups per CU, with and without priority (the prio image needs 64 B more LDS)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2x
mkdir -p $O
for r in a b; do
EXPLORE_FILTER="nib G16 CH4 NBUF2 AUX2 wg/cu2 opt2 xw31:29,nib G16 CH4 NBUF2 AUX2 wg/cu1 opt2 xw31:29,nib G16 CH4 NBUF2 AUX2 wg/cu1 opt2 | 256,nib G16 CH4 NBUF2 AUX2 wg/cu2 opt2 | 256" timeout -k 10 300 ./tools/crc_explore 1024 $((1<<22)) 12 10 > $O/explore_1k_$r.log 2>&1
done
echo ALLDONE
