#!/bin/bash
# round-5 one-off GPU steps: XCD offset probe, then steps of tools/gpu_steps.sh
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r5p}; mkdir -p $O
timeout -k 10 60 ./tools/xcd_offset_probe > $O/xcd_offset.jsonl 2> $O/xcd_offset.err || exit $?
[ $# -gt 0 ] && bash tools/gpu_steps.sh ${TAG:-r5p} "$@"
exit $?
