# small kernel bit-matrix vs nibble fold (A/B per G); 1 KiB plan with conflict-free replicated tables; gpu tests
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1zt
mkdir -p $O
for bs in 32 64 128 256 512; do
  timeout -k 10 120 ./tools/crc_explore $bs $(( (1<<30) / bs )) 10 >> $O/explore_small_nib.log 2>&1
done
EXPLORE_FILTER="G16 CH4 NBUF2 AUX2 wg/cu2 opt2 xw31:29" timeout -k 10 300 ./tools/crc_explore 1024 $((1<<22)) 10 50 > $O/explore_1k_nibrep.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo ALLDONE
