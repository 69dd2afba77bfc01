#!/bin/bash
# graph_race_probe.py (mixed, 1 round) under HIP runtime knobs, interleaved;
# stops at the first process that does not exit 0
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r5k}; mkdir -p $O
L=abbuild/r5base/libpriskv_crc.so
n=0
for rep in 1 2 3 4; do
  for kv in "NONE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1"; do
    n=$((n+1))
    env "$kv" timeout -k 10 200 python -u tools/graph_race_probe.py $L 1 mixed > $O/p_$n.json 2> $O/p_$n.err || exit $?
    echo "$kv $(python3 -c "import json;r=json.loads(open('$O/p_$n.json').read().splitlines()[-1]);print(r['bal_wrong_total'],[x['bal'] for x in r['mixed_wrong']])")" | tee -a $O/summary.txt
  done
done
