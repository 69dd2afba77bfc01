#!/bin/bash
# window mode for odd sizes near 4 KiB multiples: parity tests, then an A/B of the
# product library with the window mode on / off (PRISKV_CRC_WINDOW=0) in one process
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r5w}; mkdir -p $O
L=priskv_amd/lib/libpriskv_crc.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "window or stride or head_split or odd" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u tools/ab_libs.py $L $L@PRISKV_CRC_WINDOW=0 ${EXTRA:-} --rounds=3 --streams=2 \
  --cases=odd4097+odd4095+odd8193+odd8191+odd16383+odd4111+odd4200+base1+base8+8192xodd+1Mix4KiB \
  > $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); v = r["variant"]
    tag = v.split("@")[1] if "@" in v else (v.split("/")[1] if v.startswith("abbuild/") else "product")
    d[(r["case"], tag)].append(r["us_per_call"])
for k, v in sorted(d.items()):
    print(k, sorted(v)[len(v) // 2], min(v))
PY
# per-kernel durations (rows kernel in window mode vs crc_window_fix_kernel), one case per trace
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for c in odd4097 base1 odd8191; do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python3 tools/ab_libs.py $L --rounds=1 --cases=$c > $O/prof_$c.log 2>&1 || exit 1
  done
  for f in $O/prof_*/*/run_kernel_stats.csv $O/prof_*/run_kernel_stats.csv; do [ -f "$f" ] && { echo "== $f"; cut -d, -f1-6 "$f" | head -6; }; done
fi
