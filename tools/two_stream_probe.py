#!/usr/bin/env python3
"""Back-to-back value-block batches on one stream against batches alternating
over two or four streams (a batch's tail overlapping the next batch's head),
same process, interleaved repeats.  1 Mi x 4 KiB blocks per batch."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from priskv_amd import CrcContext  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
nb = (4 << 30) // bs
steps = 200
ctx = CrcContext(0)
region = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(region, 0x5EED, 0)
streams = [torch.cuda.Stream() for _ in range(4)]
outs = [torch.empty(nb, dtype=torch.int32, device="cuda") for _ in range(4)]


def run(k):
    ev = torch.cuda.Event()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ctx.blocks_dev(region, bs, out=outs[i % k], stream=streams[i % k])
    torch.cuda.synchronize()
    return time.perf_counter() - t0


for k in (1, 2, 4):  # ramp
    run(k)
res = {1: [], 2: [], 4: []}
for rep in range(3):
    for k in (1, 2, 4):
        res[k].append(bs * nb * steps / run(k) / 2**30)
ok = all(torch.equal(outs[0], o) for o in outs[1:])
print(json.dumps({"block_size": bs, "nblocks": nb, "steps": steps,
                  **{f"streams{k}_GiBs": [round(v, 1) for v in vs] for k, vs in res.items()},
                  "same_crcs": bool(ok)}), flush=True)
