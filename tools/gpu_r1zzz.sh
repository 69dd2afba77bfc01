# small-call latency (eager and HIP-graph replay)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzz
mkdir -p $O
timeout -k 10 300 python tools/small_call_latency.py > $O/latency.jsonl 2> $O/latency.err
echo ALLDONE
