#!/bin/bash
# tools/gpu_steps.sh -- the one GPU-box runner (it replaces round 1's 105
# one-off tools/gpu_r*.sh scripts; those stay in git history).
#
#   gpurun --timeout S -- 'bash tools/gpu_steps.sh TAG STEP [STEP ...]'
#
# Output goes to gpurun_out/TAG/.  Steps run in order, each under its own time
# limit; the script stops at the first failing step (set -e), so nothing runs
# on the GPU after a fault, an abort or a time limit.
#
#   tests                 pytest -m gpu over every GPU test (+ smoke, C executables)
#   tests:A,B             pytest -m gpu -k "A or B"
#   bench[:A,B,...]       python bench.py A B ...  (commas stand for spaces)
#   explore:BS:NB:R:F     tools/crc_explore BS NB R with EXPLORE_FILTER=F
#   ranges:ARGS           tools/ranges_explore ARGS (commas for spaces)
#   paths:ARGS            python tools/bench_paths.py ARGS (commas for spaces)
#   lib:ARGS              tools/lib_timing ARGS: blocks_dev through the C ABI, no torch
#   libenv:VAR=V:ARGS     the same with one environment variable set
#   py:SCRIPT[:ARGS]      python tools/SCRIPT ARGS (commas for spaces)
#   gloo2[:A,B,...]       2-rank rehearsal of bench.py's N>1 path on this one GPU (gloo)
#   gloo:N[:A,B,...]      the same with N ranks
#   ktrace[:A,B,...]      rocprofv3 --kernel-trace --stats over bench.py A B ...
#   ktracepy:SCRIPT[:A,B] rocprofv3 --kernel-trace --stats over python tools/SCRIPT A B ...
#   pmc:C1+C2[:A,B,...]   one rocprofv3 --pmc pass (counters C1 C2 ...) over bench.py A B ...
#   pmcpy:C1+C2:SCRIPT[:A,B]  one --pmc pass over python tools/SCRIPT A B ...
#   pmclib:C1+C2:ARGS     one --pmc pass over tools/lib_timing ARGS (no torch in the process)
#   pmclibenv:VAR=V:C1+C2:ARGS  the same with one environment variable exported first
#   probe:ENV2:ARGS       tools/alloc_probe ARGS, second context with ENV2 (A/B, same allocations)
#   pmcprobe:C1+C2:ARGS   one --pmc pass over tools/alloc_probe ARGS
#   ktracelib:ARGS        rocprofv3 --kernel-trace --stats over tools/lib_timing ARGS
#   oversub               bench.py as 2 ranks on this one GPU WITHOUT the rehearsal
#                         variable: must exit 3 (the device guard) -- the step fails otherwise
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
n=0
for step in "$@"; do
    n=$((n + 1))
    kind=${step%%:*}
    arg=""
    [[ "$step" == *:* ]] && arg=${step#*:}
    echo "[$n] $step" >&2
    case "$kind" in
    tests)
        k=()
        [[ -n "$arg" ]] && k=(-k "${arg//,/ or }")
        timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${k[@]}" \
            > "$O/pytest_$n.log" 2>&1
        if [[ -z "$arg" ]]; then
            timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
            timeout -k 10 120 ./tests/c/test_crc_gpu > "$O/c_gpu.log" 2>&1
        fi
        ;;
    bench)
        timeout -k 10 400 python -u bench.py ${arg//,/ } > "$O/bench_$n.json" 2> "$O/bench_$n.err"
        ;;
    explore)
        IFS=: read -r bs nb rounds filt <<< "$arg"
        EXPLORE_FILTER="$filt" timeout -k 10 300 ./tools/crc_explore "$bs" "$nb" "$rounds" > "$O/explore_$n.log" 2>&1
        ;;
    ranges)
        timeout -k 10 300 ./tools/ranges_explore ${arg//,/ } > "$O/ranges_$n.log" 2>&1
        ;;
    paths)
        timeout -k 10 400 python -u tools/bench_paths.py ${arg//,/ } > "$O/paths_$n.jsonl" 2> "$O/paths_$n.err"
        ;;
    lib)
        timeout -k 10 200 ./tools/lib_timing ${arg//,/ } > "$O/lib_$n.json" 2> "$O/lib_$n.err"
        ;;
    libenv)
        kv=${arg%%:*}
        largs=""
        [[ "$arg" == *:* ]] && largs=${arg#*:}
        env "$kv" timeout -k 10 200 ./tools/lib_timing ${largs//,/ } > "$O/lib_$n.json" 2> "$O/lib_$n.err"
        ;;
    py)
        script=${arg%%:*}
        pargs=""
        [[ "$arg" == *:* ]] && pargs=${arg#*:}
        timeout -k 10 400 python -u "tools/$script" ${pargs//,/ } > "$O/py_$n.out" 2> "$O/py_$n.err"
        ;;
    ktrace)
        (cd /tmp && export TMPDIR=/tmp &&
            timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/ktrace_$n" -o run --output-format csv \
                -- python3 "$R/bench.py" ${arg//,/ } > "$O/ktrace_$n.json" 2> "$O/ktrace_$n.err")
        ;;
    gloo2)
        PRISKV_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 ${arg//,/ } > "$O/gloo2_$n.json" \
            2> "$O/gloo2_$n.err"
        ;;
    gloo)
        # gloo:N[:A,B,...] -- N-rank rehearsal of bench.py's N>1 path on this one GPU (gloo)
        nr=${arg%%:*}
        bargs=""
        [[ "$arg" == *:* ]] && bargs=${arg#*:}
        PRISKV_BENCH_REHEARSAL=1 timeout -k 10 900 python -m torch.distributed.run --nnodes 1 --nproc-per-node "$nr" \
            --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus "$nr" ${bargs//,/ } > "$O/gloo${nr}_$n.json" \
            2> "$O/gloo${nr}_$n.err"
        ;;
    oversub)
        set +e
        timeout -k 10 120 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 2 --warmup 1 \
            > "$O/oversub_$n.out" 2> "$O/oversub_$n.err"
        rc=$?
        set -e
        echo "oversubscribed launch exit status $rc" >> "$O/oversub_$n.err"
        [[ $rc -ne 0 && $rc -ne 124 && $rc -ne 137 ]]
        grep -q "has no GPU of its own" "$O/oversub_$n.err"
        ;;
    ktracepy)
        script=${arg%%:*}
        pargs=""
        [[ "$arg" == *:* ]] && pargs=${arg#*:}
        (cd /tmp && export TMPDIR=/tmp &&
            timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/ktracepy_$n" -o run --output-format csv \
                -- python3 "$R/tools/$script" ${pargs//,/ } > "$O/ktracepy_$n.out" 2> "$O/ktracepy_$n.err")
        ;;
    pmc)
        ctrs=${arg%%:*}
        bargs=""
        [[ "$arg" == *:* ]] && bargs=${arg#*:}
        (cd /tmp && export TMPDIR=/tmp &&
            timeout -s KILL 180 rocprofv3 --pmc ${ctrs//+/ } -d "$O/pmc_$n" -o run --output-format csv \
                -- python3 "$R/bench.py" ${bargs//,/ } > "$O/pmc_$n.json" 2> "$O/pmc_$n.err")
        ;;
    pmcpy)
        # pmcpy:C1+C2:SCRIPT[:A,B] -- one --pmc pass over python tools/SCRIPT A B ...
        ctrs=${arg%%:*}
        rest=${arg#*:}
        script=${rest%%:*}
        pargs=""
        [[ "$rest" == *:* ]] && pargs=${rest#*:}
        (cd /tmp && export TMPDIR=/tmp &&
            timeout -s KILL 180 rocprofv3 --pmc ${ctrs//+/ } -d "$O/pmcpy_$n" -o run --output-format csv \
                -- python3 "$R/tools/$script" ${pargs//,/ } > "$O/pmcpy_$n.out" 2> "$O/pmcpy_$n.err")
        ;;
    pmclib)
        ctrs=${arg%%:*}
        largs=""
        [[ "$arg" == *:* ]] && largs=${arg#*:}
        (cd /tmp && export TMPDIR=/tmp LIB_TIMING_RAMP=20 &&
            timeout -s KILL 120 rocprofv3 --pmc ${ctrs//+/ } -d "$O/pmclib_$n" -o run --output-format csv \
                -- "$R/tools/lib_timing" ${largs//,/ } > "$O/pmclib_$n.out" 2> "$O/pmclib_$n.err")
        ;;
    pmclibenv)
        kv=${arg%%:*}
        rest=${arg#*:}
        ctrs=${rest%%:*}
        largs=""
        [[ "$rest" == *:* ]] && largs=${rest#*:}
        (cd /tmp && export TMPDIR=/tmp LIB_TIMING_RAMP=20 && export "$kv" &&
            timeout -s KILL 120 rocprofv3 --pmc ${ctrs//+/ } -d "$O/pmclib_$n" -o run --output-format csv \
                -- "$R/tools/lib_timing" ${largs//,/ } > "$O/pmclib_$n.out" 2> "$O/pmclib_$n.err")
        ;;
    probe)
        # probe:VAR=V[;VAR=V]:ARGS -- tools/alloc_probe ARGS with a second context (ALLOC_PROBE_ENV2): an A/B
        # on the same allocations in one process
        e2=${arg%%:*}
        largs=""
        [[ "$arg" == *:* ]] && largs=${arg#*:}
        ALLOC_PROBE_ENV2="$e2" timeout -k 10 300 ./tools/alloc_probe ${largs//,/ } > "$O/probe_$n.jsonl" \
            2> "$O/probe_$n.err"
        ;;
    pmcprobe)
        ctrs=${arg%%:*}
        largs=""
        [[ "$arg" == *:* ]] && largs=${arg#*:}
        (cd /tmp && export TMPDIR=/tmp &&
            timeout -s KILL 120 rocprofv3 --pmc ${ctrs//+/ } -d "$O/pmcprobe_$n" -o run --output-format csv \
                -- "$R/tools/alloc_probe" ${largs//,/ } > "$O/pmcprobe_$n.out" 2> "$O/pmcprobe_$n.err")
        ;;
    ktracelib)
        (cd /tmp && export TMPDIR=/tmp &&
            timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/ktracelib_$n" -o run --output-format csv \
                -- "$R/tools/lib_timing" ${arg//,/ } > "$O/ktracelib_$n.out" 2> "$O/ktracelib_$n.err")
        ;;
    *)
        echo "unknown step $step" >&2
        exit 2
        ;;
    esac
done
echo ALLDONE >&2
