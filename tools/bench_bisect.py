"""bench_bisect.py -- bench.py's steady-state kernel time vs the torch-free
harness (tools/lib_timing): the same library call measured under variations
of bench's sequence, interleaved in one process.  Tools only."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from priskv_amd import CrcContext  # noqa: E402

bs, nb, K = 4096, 1 << 20, 50
torch.cuda.set_device(0)
ctx = CrcContext(0)
region = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(region, 0x5EED5EED, word_offset=0)
out = torch.empty(nb, dtype=torch.int32, device="cuda")
null = torch.cuda.current_stream()
new = torch.cuda.Stream()


def timed(s, ramp_mode):
    def step():
        ctx.blocks_dev(region, bs, out=out, stream=s)
    if ramp_mode == "bursts":  # bench.ramp(): 4 launches + sync for 0.3 s
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            for _ in range(4):
                step()
            torch.cuda.synchronize()
    else:  # one long back-to-back run
        for _ in range(200):
            step()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(K):
        step()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


res = {}
for r in range(4):
    for sname, s in (("null", null), ("new", new)):
        for rm in ("bursts", "long"):
            res.setdefault(f"{sname}/{rm}", []).append(round(timed(s, rm), 4))
print(json.dumps(res))
