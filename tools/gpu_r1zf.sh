set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zf
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
timeout -k 10 300 python tools/bench_paths.py memfile ranges > $O/paths.log 2>&1
EXPLORE_FILTER="opt2 xw0,roof G32" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 4 20 > $O/explore_4k.log 2>&1
echo ALLDONE
