set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zn
mkdir -p $O
timeout -k 10 300 ./tools/ranges_explore 8 > $O/ranges_explore.log 2>&1
echo ALLDONE
