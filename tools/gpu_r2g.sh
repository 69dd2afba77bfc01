# kernel-trace timeline of small segmented extents calls (32 and 2048 values)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt32 -o run --output-format csv -- python3 $R/tools/seg_overhead.py 32 > $O/kt32.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt2048 -o run --output-format csv -- python3 $R/tools/seg_overhead.py 2048 > $O/kt2048.log 2>&1
echo ALLDONE
