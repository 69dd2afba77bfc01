# workgroup-parallel segment reduce: segment tests, kernel trace of a lone 256 MiB value, few-values paths
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "segment or ranges" --timeout 200 --timeout-method thread > $O/pytest_seg.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python tools/bench_paths.py few > $O/few.jsonl 2> $O/few.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/tools/huge_value_trace.py > $O/kt.log 2>&1
echo ALLDONE
