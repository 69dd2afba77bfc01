#!/usr/bin/env python3
"""Odd block sizes and bases, ~4 GB per call, window mode on / off (tools only).

  python tools/odd_sweep.py [OUT.jsonl]

One process, one 4 GiB region filled on the device; for each (size, base
offset) the default context and one with PRISKV_CRC_WINDOW=0 each time 20
back-to-back blocks_dev calls (HIP events, after 5 warm-up calls), and
their CRCs must agree bit for bit (the oracle parity is the GPU tests').
One JSON line per case: the path and plan of each, us per call, TB/s and
the fraction of the 8 TB/s HBM spec.  A third context has the head split
off (PRISKV_CRC_HEADSPLIT=0).  ODD_SWEEP_CASES="bs:off,..." picks the cases.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from priskv_amd import CrcContext, blocks_path  # noqa: E402


def ctx_env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        return CrcContext(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


SIZES = [1000, 1009, 1023, 1025, 1072, 1500, 2000, 2047, 2049, 2100, 3000, 3071, 3073, 4000, 4081, 4095, 4097,
         4111, 4200, 5000, 5121, 6000, 6143, 6145, 7169, 8000, 8191, 8193, 9000, 9217, 10000, 12287, 12289, 16383,
         16385]
# (three aligned 4 KiB cases first: the first seconds of a process run slow, clocks ramping)
CASES = [(4096, 0)] * 3 + [(bs, 0) for bs in SIZES] + [(1024, 1), (2048, 1), (4096, 1), (4096, 8), (8192, 1),
                                                      (4100, 1), (4100, 0), (1088, 0), (12340, 0), (65540, 0)]
if os.environ.get("ODD_SWEEP_CASES"):  # "bs:off,bs:off,..."
    CASES = [tuple(int(x) for x in c.split(":")) for c in os.environ["ODD_SWEEP_CASES"].split(",")]
out = open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout
ctxs = {"window": CrcContext(0), "off": ctx_env(PRISKV_CRC_WINDOW="0"),
        "nohead": ctx_env(PRISKV_CRC_HEADSPLIT="0")}
region = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
ctxs["window"].fill_splitmix(region, 0x5EED, 0)
torch.cuda.synchronize()
for bs, mis in CASES:
    nb = ((4 << 30) - 64) // bs
    view = region[mis: mis + nb * bs]
    rec = {"block_size": bs, "base_offset": mis, "nblocks": nb, "bytes": nb * bs}
    got = {}
    for name, c in ctxs.items():
        o = torch.empty(nb, dtype=torch.int32, device="cuda")
        for _ in range(5):
            c.blocks_dev(view, bs, out=o, nblocks=nb)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            c.blocks_dev(view, bs, out=o, nblocks=nb)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        got[name] = o
        rec[name] = {"plan": c.blocks_plan(view.data_ptr(), nb, bs), "us": round(us, 2),
                     "TBps": round(nb * bs / us / 1e6, 3), "frac": round(nb * bs / us / 1e6 / 8.0, 4)}
    rec["path_default"] = blocks_path(view.data_ptr(), nb, bs)
    rec["bit_identical"] = bool(torch.equal(got["window"], got["off"]) and torch.equal(got["window"], got["nohead"]))
    assert rec["bit_identical"], rec
    out.write(json.dumps(rec) + "\n")
    out.flush()
