# segmented extents: combine folded into the kernel (shifted segments + XOR reduce), one-wave plan; few-values timing + kernel trace
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zza
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python tools/bench_paths.py few > $O/few.jsonl 2> $O/few.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/tools/bench_paths.py few > $O/ktrace.log 2>&1
echo ALLDONE
