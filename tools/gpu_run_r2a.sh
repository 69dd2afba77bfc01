set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "tib_config" > gpurun_out/r2_tibtest.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r2_bench_a.json 2> gpurun_out/r2_bench_a.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench_b.json 2> gpurun_out/r2_bench_b.err
