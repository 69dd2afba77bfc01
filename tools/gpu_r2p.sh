# extents shape choice (16-wave priority only for >= 32 extents per wave): gpu suite, ranges paths on/off
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
timeout -k 10 300 python tools/bench_paths.py ranges > $O/paths_$i.jsonl 2> $O/paths_$i.err
PRISKV_CRC_PRIO=0 timeout -k 10 300 python tools/bench_paths.py ranges > $O/paths_noprio_$i.jsonl 2> $O/paths_noprio_$i.err
done
echo ALLDONE
