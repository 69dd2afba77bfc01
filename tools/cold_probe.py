#!/usr/bin/env python3
"""Attribute the cold first pass of bench.py's `cold` leg.

Every full pass here is one blocks_dev over 1 Mi x 4 KiB (the headline
workload, crc_rows_kernel), HIP-event timed on its own stream.  Scenarios:

  warm          back-to-back steady state on region R0 (the last of 24)
  fresh_hot     first CRC pass over a region only the fill kernel has
                touched, right after 24 warm passes (hot clocks, cold region)
  walked_idle   1 s idle, then a pass over R0 (hashed many times: cold
                clocks, walked region)
  fresh_idle    1 s idle, then the first pass over a filled region (bench.py's
                cold leg: cold clocks, cold region)
  prewarm_idle  1 s idle, then ~2 ms of small launches on a 256 B-block
                region (crc_small_kernel, L2-resident), then a pass over R0
  *_2nd         the pass right after the one named

Each scenario runs REPS times, interleaved.  Every crc_rows_kernel dispatch
of the process is one labelled pass, in the order printed under "order", so
a rocprofv3 --kernel-trace / --pmc run of this script maps dispatch i to its
scenario (tools/cold_attrib.py).  Prints one JSON object.
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BS, NB = 4096, 1 << 20
REPS = int(os.environ.get("COLD_PROBE_REPS", "3"))
IDLE_S = 1.0


def main():
    import torch
    from priskv_amd import CrcContext

    dev = torch.device("cuda", 0)
    ctx = CrcContext(0)
    s = torch.cuda.Stream(device=dev)
    out = torch.empty(NB, dtype=torch.int32, device=dev)
    r0 = torch.empty(BS * NB, dtype=torch.uint8, device=dev)
    ctx.fill_splitmix(r0, 0x5EED5EED)
    # fresh regions: filled now, first hashed in their scenario
    fresh = []
    for k in range(2 * REPS):
        t = torch.empty(BS * NB, dtype=torch.uint8, device=dev)
        ctx.fill_splitmix(t, 0xF00D + k)
        fresh.append(t)
    small = torch.empty(4 << 20, dtype=torch.uint8, device=dev)
    ctx.fill_splitmix(small, 7)
    small_out = torch.empty((4 << 20) // 256, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    order, res = [], {}

    def one(region, label):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ctx.blocks_dev(region, BS, out=out, stream=s)
        e1.record(s)
        e1.synchronize()
        order.append(label)
        res.setdefault(label, []).append(e0.elapsed_time(e1))

    def warm_up(n=24):
        for _ in range(n - 1):
            ctx.blocks_dev(r0, BS, out=out, stream=s)
            order.append("ramp")
        one(r0, "warm")

    # settle the process first (the first second of GPU work runs slow)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.5:
        ctx.blocks_dev(r0, BS, out=out, stream=s)
        order.append("ramp")
    torch.cuda.synchronize()
    fi = 0
    for _ in range(REPS):
        warm_up()
        one(fresh[fi], "fresh_hot")
        one(fresh[fi], "fresh_hot_2nd")
        fi += 1
        torch.cuda.synchronize()
        time.sleep(IDLE_S)
        one(r0, "walked_idle")
        one(r0, "walked_idle_2nd")
        torch.cuda.synchronize()
        time.sleep(IDLE_S)
        one(fresh[fi], "fresh_idle")
        one(fresh[fi], "fresh_idle_2nd")
        fi += 1
        torch.cuda.synchronize()
        time.sleep(IDLE_S)
        t1 = time.perf_counter()
        n = 0
        while time.perf_counter() - t1 < 0.002:
            ctx.blocks_dev(small, 256, out=small_out, stream=s)
            n += 1
        one(r0, "prewarm_idle")
        one(r0, "prewarm_idle_2nd")
    alg = NB * (BS + 4)
    summary = {k: {"ms": [round(x, 4) for x in v], "median_ms": round(statistics.median(v), 4),
                   "TBps": round(alg / (statistics.median(v) * 1e-3) / 1e12, 3)} for k, v in res.items()}
    rle = []  # dispatch order, run-length encoded: [label, count]
    for lab in order:
        if rle and rle[-1][0] == lab:
            rle[-1][1] += 1
        else:
            rle.append([lab, 1])
    print(json.dumps({"workload": f"{NB} x {BS} B", "idle_s": IDLE_S, "reps": REPS, "scenarios": summary,
                      "order": rle}))


if __name__ == "__main__":
    main()
