# kernel trace of a lone 256 MiB value through the segmented extents path
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/huge_value_trace.py > $O/kt.log 2>&1
echo ALLDONE
