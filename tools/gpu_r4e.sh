# bench with the pipelined (2-stream) pass beside the one-stream value: default, 64 KiB, 1 MiB; kernel trace of the one-stream pass
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python bench.py --config sweep64k --no-cpu-baseline > $O/bench_64k.json 2> $O/bench_64k.err
timeout -k 10 200 python bench.py --config sweep1m --no-cpu-baseline > $O/bench_1m.json 2> $O/bench_1m.err
timeout -k 10 200 python bench.py --pipeline-streams 4 --no-cpu-baseline > $O/bench_ps4.json 2> $O/bench_ps4.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --pipeline-streams 0 > $O/bench_kt.json 2> $O/bench_kt.err
echo ALLDONE
