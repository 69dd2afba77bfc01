# extents kernel progress-priority modes (tools/ranges_explore), two runs; the rows explorer's 4 KiB product vs modes
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2n
mkdir -p $O
timeout -k 10 300 ./tools/ranges_explore 6 > $O/ranges_prio_a.log 2>&1
timeout -k 10 300 ./tools/ranges_explore 6 > $O/ranges_prio_b.log 2>&1
echo ALLDONE
