# per-wave finish times: spread inside a workgroup (one CU) vs across workgroups, CRC and read roof
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzn
mkdir -p $O
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX2 wg/cu1 opt10 xw31:29,rooft G32 CH8 NBUF2 AUX2 wg/cu1 xw31:29" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 4 10 > $O/explore_4k_cu_spread.log 2>&1
echo ALLDONE
