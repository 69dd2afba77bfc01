#!/bin/bash
# window mode on whole-KiB W (G = 16 plans): parity tests, then A/B against the previous build (abbuild/head)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r5wg}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "window or stride or head_split or odd or plan_strings" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/ab_libs.py priskv_amd/lib/libpriskv_crc.so abbuild/head/libpriskv_crc.so --rounds=3 \
  --cases=odd1023+odd1025+odd2047+odd2049+odd3073+odd5121+odd9217+base1+odd4097 \
  > $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 - $O/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); v = r["variant"]
    tag = v.split("/")[1] if v.startswith("abbuild/") else "product"
    d[(r["case"], tag)].append(r["us_per_call"])
for k, v in sorted(d.items()):
    print(k, sorted(v)[len(v) // 2], min(v))
PY
