# full path sweep at HEAD: every block size 16 B - 1 MiB, PrisKV-shaped values at 4 KiB / 64 KiB / 1 MiB blocks
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzq
mkdir -p $O
timeout -k 10 600 python tools/bench_paths.py blocks ranges > $O/paths.jsonl 2> $O/paths.err
echo ALLDONE
