# kernel trace of the segmented extents path's fixed cost (2048 small values)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzw
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/tools/seg_overhead.py > $O/ktrace.log 2>&1
echo ALLDONE
