# cache-policy bits of the streaming loads (aux 0/2/3/16/18/19) for the 4 KiB product and the read roof
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzj
mkdir -p $O
EXPLORE_FILTER="nib G32 CH8 NBUF2 AUX,roof G32 CH8 NBUF2 AUX" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 10 30 > $O/explore_4k_aux.log 2>&1
echo ALLDONE
