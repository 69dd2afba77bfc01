# PrisKV-shaped values above the segmentation count rule (n = 4096, 8192): how far from the HBM rate
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzu
mkdir -p $O
timeout -k 10 400 python tools/bench_paths.py seglimit > $O/seglimit.jsonl 2> $O/seglimit.err
echo ALLDONE
