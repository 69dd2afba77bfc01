set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1y
mkdir -p $O
timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 6 30 > $O/explore_4k.log 2>&1
timeout -k 10 300 ./tools/crc_explore 65536 $((1<<16)) 6 30 > $O/explore_64k.log 2>&1
echo ALLDONE
