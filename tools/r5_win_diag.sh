#!/bin/bash
# window mode: where the in-kernel version's time goes (diagnostic builds under abbuild/, --nocheck)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r5wd}; mkdir -p $O
L=priskv_amd/lib/libpriskv_crc.so
timeout -k 10 400 python -u tools/ab_libs.py $L ${VARIANTS} --rounds=2 --nocheck \
  --cases=${CASES:-odd4097+odd4095+odd16383+base1} > $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
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
