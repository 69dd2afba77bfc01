# bench A/B of the 4 KiB plan's XCD weights (8:7 default vs 31:29), interleaved; kernel trace; traffic
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2e
mkdir -p $O
for i in 1 2 3; do
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/bench_87_$i.log 2>&1
PRISKV_CRC_XCD_WEIGHTS=31:29 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/bench_3129_$i.log 2>&1
PRISKV_CRC_XCD_WEIGHTS=7:6 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/bench_76_$i.log 2>&1
done
timeout -k 10 300 python bench.py --block-size 1048576 --nblocks 4096 --no-cpu-baseline > $O/bench_1m.log 2>&1
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/ktrace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1
echo ALLDONE
