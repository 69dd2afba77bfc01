#!/usr/bin/env python3
"""Per-value (extent) paths through the library: GiB/s and the roofline
fraction of value bytes + 4 B per CRC, HIP events over back-to-back calls
after a warm ramp, every context interleaved round by round in one process
(VERDICT r2 item 4).  Cases:

  priskv4k   524 288 PrisKV-shaped values on 4 KiB blocks (1/2/4 blocks,
             ragged last block: server/buddy.c:134-140) over 4 GiB -- the
             memfile scrub (ranges_dev, the many-extents 16-wave shape)
  priskv64k  32 768 such values on 64 KiB blocks (byte-balanced split)
  one256m    one 256 MiB value (the fused few-extents kernel)
  blk256m    one 256 MiB block through blocks_dev (fused kernel, one length)

usage: values_bench.py [ROUNDS] [ENV=VALUE[:ENV=VALUE...] ...]   (each
argument adds a context created with those variables set, beside the
default one)
One JSON line per (case, context) with the median over rounds; every
context's CRCs are compared with the default context's and, on a sample,
with the CPU oracle.
"""
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import _oracle as O  # noqa: E402
import torch  # noqa: E402

from priskv_amd import CrcContext, as_u32  # noqa: E402

PEAK = 8.0e12


def extents(rng, n, region_bytes, bs):
    k = rng.integers(0, 3, n)
    span = (1 << k) * bs
    blk = rng.integers(0, region_bytes // bs - 4, n)
    offs = (blk * bs).astype(np.uint64)
    lens = np.minimum(span - rng.integers(0, bs, n), region_bytes - offs).astype(np.uint32)
    return offs, lens


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 7
    ctxs = [("default", CrcContext(0))]
    for a in sys.argv[1:]:
        if "=" in a:  # VAR=VALUE[:VAR=VALUE...]: one context with all of them set
            kv = [x.split("=", 1) for x in a.split(":")]
            for k, v in kv:
                os.environ[k] = v
            ctxs.append((a, CrcContext(0)))
            for k, _ in kv:
                del os.environ[k]
    region = 4 << 30
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctxs[0][1].fill_splitmix(t, 0x5EED5EED, 0)
    s = torch.cuda.Stream()
    rng = np.random.default_rng(1)
    cases = []
    for name, bs, n in (("priskv4k", 4096, 1 << 19), ("priskv64k", 65536, 1 << 15)):
        o, ln = extents(rng, n, region, bs)
        cases.append((name, "ranges", o, ln))
    cases.append(("one256m", "ranges", np.array([4096], np.uint64), np.array([256 << 20], np.uint32)))
    cases.append(("blk256m", "blocks", None, None))
    for name, kind, o, ln in cases:
        if kind == "ranges":
            d_o = torch.from_numpy(o.astype(np.int64)).cuda()
            d_l = torch.from_numpy(ln.view(np.int32)).cuda()
            nv, vb = o.size, int(ln.astype(np.uint64).sum())
        else:
            nv, vb = 1, 256 << 20
        outs = {c: torch.empty(nv, dtype=torch.int32, device="cuda") for c, _ in ctxs}

        def call(c, ctx):
            if kind == "ranges":
                ctx.ranges_dev(t, d_o, d_l, out=outs[c], stream=s)
            else:
                ctx.blocks_dev(t, 256 << 20, out=outs[c], stream=s, nblocks=1)

        per = max(3, min(200, int(2e-3 / max(vb / 6.5e12, 1e-6))))  # about 2 ms of calls per timing
        times = {c: [] for c, _ in ctxs}
        for r in range(rounds + 1):
            for c, ctx in ctxs:
                for _ in range(per):  # warm
                    call(c, ctx)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(per):
                    call(c, ctx)
                e1.record(s)
                e1.synchronize()
                if r:
                    times[c].append(e0.elapsed_time(e1) / per * 1e-3)
        ref = as_u32(outs["default"])
        if kind == "ranges":
            k = min(nv, 200)
            want = np.array([O.crc32(t[int(a):int(a) + int(b)].cpu().numpy()) for a, b in zip(o[:k], ln[:k])],
                            dtype=np.uint32)
        else:
            want = np.array([O.crc32(t[: 256 << 20].cpu().numpy())], dtype=np.uint32)
        for c, _ in ctxs:
            sec = statistics.median(times[c])
            got = as_u32(outs[c])
            print(json.dumps({"case": name, "ctx": c, "values": nv, "value_bytes": vb, "us": round(sec * 1e6, 2),
                              "GiBs": round(vb / sec / 2**30, 1), "TBs": round((vb + 4 * nv) / sec / 1e12, 3),
                              "frac": round((vb + 4 * nv) / sec / PEAK, 4), "calls_per_timing": per,
                              "same_as_default": bool(np.array_equal(got, ref)),
                              "oracle_sample_ok": bool(np.array_equal(got[:want.size], want))}), flush=True)


if __name__ == "__main__":
    main()
