# nibble fold adopted for the 4 KiB plan: parity, bench, kernel trace; explorer at 1 / 8 / 16 KiB
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zq
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/ktrace.log 2>&1
cd $R
EXPLORE_FILTER="xw31:29" timeout -k 10 300 ./tools/crc_explore 1024 $((1<<22)) 8 50 > $O/explore_1k_nib.log 2>&1
EXPLORE_FILTER="xw31:29" timeout -k 10 300 ./tools/crc_explore 8192 $((1<<19)) 8 50 > $O/explore_8k_nib.log 2>&1
EXPLORE_FILTER="xw31:29" timeout -k 10 300 ./tools/crc_explore 16384 $((1<<18)) 8 50 > $O/explore_16k_nib.log 2>&1
echo ALLDONE
