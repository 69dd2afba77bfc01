# segmentation count limit re-measured on the current segmented path (one segment size per call, counted from the start)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g
mkdir -p $O
timeout -k 10 400 python tools/bench_paths.py seglimit > $O/seglimit.jsonl 2> $O/seglimit.err
echo ALLDONE
