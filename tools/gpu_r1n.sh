set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1n
mkdir -p $O
timeout -k 10 500 python -m pytest tests -x -q -m "gpu" > $O/pytest.log 2>&1
timeout -k 10 400 python tools/bench_paths.py > $O/paths.log 2>&1
timeout -k 10 200 python bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_a -o run --output-format csv -- $B > $O/pmc_a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $O/pmc_b -o run --output-format csv -- $B > $O/pmc_b.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT -d $O/pmc_c -o run --output-format csv -- $B > $O/pmc_c.log 2>&1
echo ALLDONE
