# segmented extents for device lengths: count rule and minimum segment cap (PrisKV-shaped values, same process)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzs
mkdir -p $O
timeout -k 10 300 python tools/bench_paths.py seglimit > $O/seglimit.jsonl 2> $O/seglimit.err
echo ALLDONE
