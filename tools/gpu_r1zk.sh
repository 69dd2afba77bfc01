set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zk
mkdir -p $O
timeout -k 10 300 ./tools/batch_bench 4 4096 16 2 16 > $O/batch_bench_16.jsonl 2>&1
timeout -k 10 300 ./tools/batch_bench 4 65536 16 2 16 > $O/batch_bench_64k.jsonl 2>&1
echo ALLDONE
