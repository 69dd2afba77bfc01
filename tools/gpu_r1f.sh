set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1f
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
PRISKV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_2rank_gloo.log 2>&1
timeout -k 10 400 python bench.py --config tib --steps 10 --warmup 3 > $O/bench_tib.log 2>&1
echo ALLDONE
