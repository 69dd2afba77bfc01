# round-end refresh with progress priority: gpu suite, smoke, bench (default + 64 KiB + 1 MiB),
# kernel-trace stats, HBM traffic passes (FETCH_SIZE, WRITE_SIZE, TCC_EA0_RDREQ)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --block-size 65536 --nblocks 65536 --no-cpu-baseline > $O/bench_64k.log 2>&1
timeout -k 10 300 python bench.py --block-size 1048576 --nblocks 4096 --no-cpu-baseline > $O/bench_1m.log 2>&1
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/ktrace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/pmc_rdreq -o run --output-format csv -- $B > $O/pmc_rdreq.log 2>&1
echo ALLDONE
