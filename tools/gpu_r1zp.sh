# nibble-table fold vs bit-matrix fold, NBUF depth (explorer, in-process A/B)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zp
mkdir -p $O
EXPLORE_FILTER="xw31:29" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 12 100 > $O/explore_4k_nib.log 2>&1
EXPLORE_FILTER="xw31:29" timeout -k 10 300 ./tools/crc_explore 65536 $((1<<16)) 8 100 > $O/explore_64k_nib.log 2>&1
echo ALLDONE
