# pipelined nibble-fold plans for 8 / 16 KiB blocks (G64 CH8, G64 CH16, G32 CH16); small kernel adopted: tests + path sweep
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zu
mkdir -p $O
EXPLORE_FILTER="xw31:29" timeout -k 10 300 ./tools/crc_explore 8192 $((1<<19)) 10 50 > $O/explore_8k_pipe.log 2>&1
EXPLORE_FILTER="xw31:29" timeout -k 10 300 ./tools/crc_explore 16384 $((1<<18)) 10 50 > $O/explore_16k_pipe.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 500 python tools/bench_paths.py blocks > $O/paths.jsonl 2> $O/paths.err
echo ALLDONE
