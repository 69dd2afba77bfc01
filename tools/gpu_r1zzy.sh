# PMC traffic (FETCH_SIZE / WRITE_SIZE) for the 64 KiB and 1 MiB plans and the extents kernel
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zzy
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in sweep64k sweep1m; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$cfg -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/fetch_$cfg.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write_$cfg -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/write_$cfg.log 2>&1
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_ranges -o run --output-format csv -- python3 $R/tools/bench_paths.py ranges > $O/fetch_ranges.log 2>&1
echo ALLDONE
