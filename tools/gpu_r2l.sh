# progress priority in the product plans: gpu suite, then bench A/B (PRISKV_CRC_PRIO=0 vs default), interleaved
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2 3; do
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/bench_prio_$i.log 2>&1
PRISKV_CRC_PRIO=0 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/bench_noprio_$i.log 2>&1
done
for bs in 1024 65536; do
timeout -k 10 120 python bench.py --no-cpu-baseline --block-size $bs --nblocks $((4294967296 / bs)) > $O/bench_prio_$bs.log 2>&1
PRISKV_CRC_PRIO=0 timeout -k 10 120 python bench.py --no-cpu-baseline --block-size $bs --nblocks $((4294967296 / bs)) > $O/bench_noprio_$bs.log 2>&1
done
timeout -k 10 120 python bench.py --no-cpu-baseline --block-size 1048576 --nblocks 4096 > $O/bench_prio_1048576.log 2>&1
PRISKV_CRC_PRIO=0 timeout -k 10 120 python bench.py --no-cpu-baseline --block-size 1048576 --nblocks 4096 > $O/bench_noprio_1048576.log 2>&1
echo ALLDONE
