# extents kernel: nibble fold + distributed row apply, uniform mask skip (in-process A/B)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zr
mkdir -p $O
timeout -k 10 400 ./tools/ranges_explore 8 > $O/ranges_explore_nib.log 2>&1
echo ALLDONE
