set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1s
mkdir -p $O
timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 8 50 > $O/explore_4k.log 2>&1
echo ALLDONE
