#!/usr/bin/env python3
"""Latency of small device calls (one stream, back to back, HIP events):
blocks_dev and ranges_dev for 1..4096 values of 4 KiB / 64 KiB, and the
same through a replayed HIP graph (no host launch cost)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from priskv_amd import CrcContext  # noqa: E402

ctx = CrcContext(0)
t = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(t, 3, 0)
s = torch.cuda.Stream()


def timed(fn, reps=200):
    with torch.cuda.stream(s):
        for _ in range(20):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def graphed(fn, reps=200):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        fn()
    torch.cuda.synchronize()
    return timed(g.replay, reps)


for bs in (4096, 65536):
    for n in (1, 16, 256, 4096):
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * bs
        lens = torch.full((n,), bs - 100, dtype=torch.int32, device="cuda")
        r = {"block_size": bs, "n": n}
        r["blocks_dev_us"] = round(timed(lambda: ctx.blocks_dev(t, bs, out=out, nblocks=n, stream=s)), 2)
        r["ranges_dev_us"] = round(timed(lambda: ctx.ranges_dev(t, offs, lens, out=out, stream=s)), 2)
        r["blocks_dev_graph_us"] = round(graphed(lambda: ctx.blocks_dev(t, bs, out=out, nblocks=n, stream=s)), 2)
        r["ranges_dev_graph_us"] = round(graphed(lambda: ctx.ranges_dev(t, offs, lens, out=out, stream=s)), 2)
        print(json.dumps(r), flush=True)
