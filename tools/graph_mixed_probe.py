#!/usr/bin/env python3
"""Which combination of calls in one HIP graph returns wrong CRCs (tools only)?

tests/test_gpu_graphs_pool.py::test_graph_mixed_split_and_fused_back_to_back
(round 5) found 9 of 1900 balanced split-mode blocks wrong when a graph held a
few-large-blocks split call, a fused ranges call, the balanced split call and
a fused lone odd block, replayed three times back to back.  This runs the
same calls in several groupings -- captured or not, replays back to back or
synchronised -- and prints the wrong-result count of every output per
configuration (one JSON line each); it asserts nothing.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _oracle as O  # noqa: E402
from priskv_amd import CrcContext, as_u32  # noqa: E402

MIB = 1 << 20
ctx = CrcContext(0)
region = 1900 * MIB
t = torch.empty(region, dtype=torch.uint8, device="cuda")
few = t[: 64 * MIB]
rng = np.random.default_rng(3)
lens = rng.integers(0, 10 * MIB + 1, 7).astype(np.uint32)
lens[:2] = [10 * MIB, 0]
offs = np.array([rng.integers(0, 64 * MIB - int(ln) + 1) for ln in lens], dtype=np.uint64)
d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
d_l = torch.from_numpy(lens.view(np.int32)).cuda()
odd = 12 * MIB + 1
outs = {"few": torch.empty(4, dtype=torch.int32, device="cuda"), "rng": torch.empty(7, dtype=torch.int32, device="cuda"),
        "bal": torch.empty(1900, dtype=torch.int32, device="cuda"), "odd": torch.empty(1, dtype=torch.int32, device="cuda")}
CALLS = {
    "few": lambda st: ctx.blocks_dev(few, 16 * MIB, out=outs["few"], nblocks=4, stream=st),
    "rng": lambda st: ctx.ranges_dev(few, d_o, d_l, out=outs["rng"], stream=st),
    "bal": lambda st: ctx.blocks_dev(t, MIB, out=outs["bal"], nblocks=1900, stream=st),
    "odd": lambda st: ctx.blocks_dev(t, odd, out=outs["odd"], nblocks=1, stream=st),
}


def want_of(host):
    return {"few": O.crc32_blocks(host[: 64 * MIB], 16 * MIB, nthreads=8),
            "rng": O.crc32_ranges(host[: 64 * MIB], offs, lens),
            "bal": O.crc32_blocks(host, MIB, nthreads=16),
            "odd": O.crc32_blocks(host[:odd], odd)}


def run(name, seq, graph=True, replays=3, sync_between=False, seeds=(61, 62, 63)):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for c in seq:
            CALLS[c](s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = None
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for c in seq:
                CALLS[c](torch.cuda.current_stream())
    res = []
    for seed in seeds:
        ctx.fill_splitmix(t, seed, 0)
        for o in outs.values():
            o.fill_(-1)
        torch.cuda.synchronize()
        for _ in range(replays):
            if graph:
                g.replay()
            else:
                with torch.cuda.stream(s):
                    for c in seq:
                        CALLS[c](s)
            if sync_between:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        w = want_of(t.cpu().numpy())
        bad = {c: int(np.count_nonzero(as_u32(outs[c]) != w[c])) for c in seq}
        res.append(bad)
    print(json.dumps({"config": name, "seq": seq, "graph": graph, "replays": replays, "sync_between": sync_between,
                      "wrong": res}), flush=True)
    del g


CONFIGS = [
    ("A all", ["few", "rng", "bal", "odd"], {}),
    ("A all, sync between replays", ["few", "rng", "bal", "odd"], {"sync_between": True}),
    ("A all, no graph", ["few", "rng", "bal", "odd"], {"graph": False}),
    ("B bal", ["bal"], {}),
    ("C few+bal", ["few", "bal"], {}),
    ("D rng+bal", ["rng", "bal"], {}),
    ("E odd+bal", ["odd", "bal"], {}),
    ("F bal first", ["bal", "few", "rng", "odd"], {}),
    ("G all, one replay", ["few", "rng", "bal", "odd"], {"replays": 1}),
]
only = sys.argv[1:]
for name, seq, kw in CONFIGS:
    if only and not any(name.startswith(o) for o in only):
        continue
    run(name, seq, **kw)
