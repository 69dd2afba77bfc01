# N>1 rehearsal on one GPU (2 ranks, gloo barrier/max, both ranks on cuda:0) + default bench configs
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzh
mkdir -p $O
PRISKV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_2rank_gloo.log 2>&1
timeout -k 10 300 python bench.py --config sweep64k > $O/bench_64k.log 2>&1
timeout -k 10 300 python bench.py --config sweep1m > $O/bench_1m.log 2>&1
timeout -k 10 300 python bench.py --config streamed --steps 5 > $O/bench_streamed.log 2>&1
echo ALLDONE
