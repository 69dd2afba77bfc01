#!/usr/bin/env python3
"""Wrong-result rate of the mixed split + fused HIP graph (tools only).

  python tools/graph_race_probe.py LIB [ROUNDS] [MODE]

MODE: "mixed" (default: the four calls, 3 replays per refill), "first1" (the
same, but the graph's first launch is synchronised before the next), "syncfill"
(the same, but the refill is synchronised before the first replay), "check1" (the
same, but sync and check after every replay), "bal" (the balanced split call
alone in the graph), "nograph" (the four calls on a stream, no capture).

Round 5: tests/test_gpu_graphs_pool.py::test_graph_mixed_split_and_fused_
back_to_back returned 9-12 of 1900 balanced split-mode blocks wrong, on some
runs only, and only after the fused / verify graph tests had run in the same
process.  This replays that sequence -- the fused graphs of the three plan
shapes, the verify graph, then the mixed graph over 8 refills x 3 back-to-back
replays -- ROUNDS times with the library at LIB (the product or an A/B build
under abbuild/), and prints the wrong-block count per refill.  Asserts
nothing.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import priskv_amd.crc as C  # noqa: E402

C.LIB_PATH = sys.argv[1] if os.path.isabs(sys.argv[1]) else os.path.join(ROOT, sys.argv[1])
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
MODE = sys.argv[3] if len(sys.argv) > 3 else "mixed"
PRE = not MODE.endswith("+nopre")  # "+nopre": skip the fused / verify graphs before the mixed one
MODE = MODE.replace("+nopre", "")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _oracle as O  # noqa: E402
import test_gpu_graphs_pool as T  # noqa: E402
from priskv_amd import CrcContext, as_u32  # noqa: E402

MIB = 1 << 20
ctx = CrcContext(0)


def mixed(seeds):
    region = 1900 * MIB
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, 1, 0)
    few = t[: 64 * MIB]
    offs, lens = T._extents(7, 64 * MIB, 10 * MIB, 3)
    d_o, d_l = T._dev(torch, offs, lens)
    o = {k: torch.empty(n, dtype=torch.int32, device="cuda") for k, n in (("few", 4), ("bal", 1900), ("rng", 7),
                                                                           ("odd", 1))}
    odd = 12 * MIB + 1

    def calls(st):
        if MODE != "bal":
            ctx.blocks_dev(few, 16 * MIB, out=o["few"], nblocks=4, stream=st)
            ctx.ranges_dev(few, d_o, d_l, out=o["rng"], stream=st)
        ctx.blocks_dev(t, MIB, out=o["bal"], nblocks=1900, stream=st)
        if MODE != "bal":
            ctx.blocks_dev(t, odd, out=o["odd"], nblocks=1, stream=st)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        calls(s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = None
    if MODE != "nograph":
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            calls(torch.cuda.current_stream())
    res = []
    for seed in seeds:
        ctx.fill_splitmix(t, seed, 0)
        for x in o.values():
            x.fill_(-1)
        if MODE == "syncfill":
            torch.cuda.synchronize()
        host = None
        per = []
        for rep in range(3):
            if g is not None:
                g.replay()
                if MODE == "first1" and seed == seeds[0] and rep == 0:
                    torch.cuda.synchronize()
            else:
                calls(torch.cuda.current_stream())
            if MODE == "check1" or rep == 2:
                torch.cuda.synchronize()
                if host is None:
                    host = t.cpu().numpy()
                    want = {"few": O.crc32_blocks(host[: 64 * MIB], 16 * MIB, nthreads=8),
                            "rng": O.crc32_ranges(host[: 64 * MIB], offs, lens),
                            "bal": O.crc32_blocks(host, MIB, nthreads=16), "odd": O.crc32_blocks(host[:odd], odd)}
                ks = ["bal"] if MODE == "bal" else list(o)
                per.append({k: int(np.count_nonzero(as_u32(o[k]) != want[k])) for k in ks})
        r = dict(per[-1])
        if MODE == "check1":
            r["per_replay_bal"] = [x["bal"] for x in per]
        got = as_u32(o["bal"])
        bad = np.nonzero(got != want["bal"])[0]
        if len(bad):  # what the wrong CRCs are: stale data (the warm-up's seed 1), another block, ...
            info = []
            all_want = {w: i for i, w in enumerate(want["bal"].tolist())}
            for b in bad[:6].tolist():
                old1 = O.crc32_blocks(O.fill_splitmix(MIB, 1, b * MIB // 8), MIB)[0]
                info.append({"block": b, "got": hex(int(got[b])), "want": hex(int(want["bal"][b])),
                             "crc_seed1": hex(int(old1)), "equals_block": all_want.get(int(got[b]))})
            r["bad_info"] = info
            # one more replay after a sync: does it come out right?
            g.replay() if g is not None else calls(torch.cuda.current_stream())
            torch.cuda.synchronize()
            r["bal_after_extra_replay"] = int(np.count_nonzero(as_u32(o["bal"]) != want["bal"]))
        res.append(r)
    del g, t
    return res


for r in range(ROUNDS):
    pre = []
    for name, n, ml in (T._FUSED_SHAPES if PRE else []):
        try:
            T.test_graph_fused_back_to_back(torch, ctx, name, n, ml)
            pre.append("ok")
        except AssertionError as e:
            pre.append("FAIL " + str(e)[:80])
    try:
        if PRE:
            T.test_graph_verify_few_extents_back_to_back(torch, ctx)
            pre.append("ok")
    except AssertionError as e:
        pre.append("FAIL " + str(e)[:80])
    res = mixed(range(70 + 10 * r, 78 + 10 * r))
    print(json.dumps({"lib": sys.argv[1], "mode": MODE, "round": r, "pre": pre, "mixed_wrong": res,
                      "bal_wrong_total": sum(x["bal"] for x in res)}), flush=True)
