#!/usr/bin/env python3
"""One call's blocks split into a head part on the caller's stream and a
small back part on a second stream forked from and joined back into it
(event fork/join per call, as a library call would do): can the back part
fill the head's tail?  Back-to-back calls, same process, interleaved repeats."""
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
steps = 100
ctx = CrcContext(0)
region = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(region, 0x5EED, 0)
s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()
out = torch.empty(nb, dtype=torch.int32, device="cuda")
ref = torch.empty(nb, dtype=torch.int32, device="cuda")
ctx.blocks_dev(region, bs, out=ref)
torch.cuda.synchronize()


def call(frac_den):
    if frac_den == 0:
        ctx.blocks_dev(region, bs, out=out, stream=s1)
        return
    nbk = nb // frac_den
    nh = nb - nbk
    e0 = torch.cuda.Event()
    e0.record(s1)
    s2.wait_event(e0)
    ctx.blocks_dev(region[: nh * bs], bs, out=out[:nh], stream=s1)
    ctx.blocks_dev(region[nh * bs:], bs, out=out[nh:], stream=s2)
    e1 = torch.cuda.Event()
    e1.record(s2)
    s1.wait_event(e1)


def run(d):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        call(d)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


dens = (0, 64, 32, 16, 8, 4)
for d in dens:
    run(d)
res = {d: [] for d in dens}
ok = True
for rep in range(3):
    for d in dens:
        out.zero_()
        res[d].append(bs * nb * steps / run(d) / 2**30)
        ok = ok and torch.equal(out, ref)
print(json.dumps({"block_size": bs, "nblocks": nb, "steps": steps,
                  **{("one_launch" if d == 0 else f"back_1_{d}") + "_GiBs": [round(v, 1) for v in vs]
                     for d, vs in res.items()}, "bit_identical": bool(ok)}), flush=True)
