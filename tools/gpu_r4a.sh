# segment-size cost model in the segmented extents plan: parity, A/B of PRISKV_CRC_SEG_COST, lone-value kernel trace
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "segment or ranges" --timeout 200 --timeout-method thread > $O/pytest_seg.log 2>&1
timeout -k 10 300 python tools/bench_paths.py segcost > $O/segcost.jsonl 2> $O/segcost.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/huge_value_trace.py > $O/kt.log 2>&1
echo ALLDONE
