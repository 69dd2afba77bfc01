#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r5j
AMD_LOG_LEVEL=4 timeout -k 10 120 python tools/dispatch_log_probe.py > gpurun_out/r5j/out.txt 2> gpurun_out/r5j/log.txt
rc=$?
grep -n "=== PHASE\|Dispatch Header\|BarrierAND\|BarrierValue\|Barrier packet" gpurun_out/r5j/log.txt | cut -c1-400 > gpurun_out/r5j/dispatch.txt
rm -f gpurun_out/r5j/log.txt
exit $rc
