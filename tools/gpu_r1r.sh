set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1r
mkdir -p $O
timeout -k 10 300 ./tools/ranges_explore 5 > $O/ranges_explore.log 2>&1
echo ALLDONE
