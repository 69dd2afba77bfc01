# gpu suite with the priority on/off test; bench A/B of XCD weights under priority (31:29 vs 8:7)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2 3; do
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/bench_3129_$i.log 2>&1
PRISKV_CRC_XCD_WEIGHTS=8:7 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/bench_87_$i.log 2>&1
done
echo ALLDONE
