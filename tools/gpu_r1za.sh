set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1za
mkdir -p $O
EXPLORE_FILTER="opt2 xw,opt10,roof G32" timeout -k 10 300 ./tools/crc_explore 4096 $((1<<20)) 12 30 > $O/explore_4k.log 2>&1
for i in 1 2 3; do
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_w$i.log 2>&1
timeout -k 10 200 env PRISKV_CRC_XCD_WEIGHTS=1:1 python bench.py --no-cpu-baseline > $O/bench_e$i.log 2>&1
done
timeout -k 10 200 python bench.py --config sweep1m --no-cpu-baseline > $O/bench_1m.log 2>&1
timeout -k 10 200 python bench.py --config sweep64k --no-cpu-baseline > $O/bench_64k.log 2>&1
echo ALLDONE
