#!/usr/bin/env python3
"""Measurement only: crc_stride_kernel (odd block sizes, unaligned bases)
against round 2's dispatch (PRISKV_CRC_STRIDE=0: extents kernel from 1 KiB,
generic kernel below) and against its own tuning variants (chunk shape,
forced G, two workgroups per CU), all contexts in one process, interleaved.

    python tools/stride_sweep.py [GiB per call=1] [rounds=2] [variants=all|tune|g|runs|funnel|oddlarge|base]

One JSON line per (round, size, context): HIP-event time per call over
`steps` back-to-back calls, TB/s of algorithmic bytes (block + 4 B CRC), and
whether the outputs equal the first context's (and the oracle's on a sample).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import _oracle as O  # noqa: E402
import torch  # noqa: E402

from priskv_amd import CrcContext, as_u32  # noqa: E402

SEED = 0x5EED5EED
# (block size, base misalignment)
CASES = [(19, 3), (100, 0), (200, 0), (520, 0), (1000, 0), (1500, 0), (3000, 0), (4100, 0), (4097, 0), (4096, 1),
         (4096, 4), (65537, 0), (100000, 0), ((1 << 20) - 1, 0), (256, 3)]


def ctx_env(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return CrcContext(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    which = sys.argv[3] if len(sys.argv) > 3 else "all"
    ctxs = {"stride": CrcContext(0), "round2": ctx_env(PRISKV_CRC_STRIDE="0")}
    if which == "all":
        for sh in (1, 2, 3):
            ctxs[f"shape{sh}"] = ctx_env(PRISKV_CRC_STRIDE_SHAPE=sh)
        ctxs["w1"] = ctx_env(PRISKV_CRC_STRIDE_WGS=1)
    elif which == "funnel":
        ctxs["nofunnel"] = ctx_env(PRISKV_CRC_STRIDE_FUNNEL=0)
    elif which == "runs":
        ctxs["noruns"] = ctx_env(PRISKV_CRC_STRIDE_RUNS=0)
        ctxs["noruns_sh3"] = ctx_env(PRISKV_CRC_STRIDE_RUNS=0, PRISKV_CRC_STRIDE_SHAPE=3)
        ctxs["runs_sh3"] = ctx_env(PRISKV_CRC_STRIDE_SHAPE=3)
    elif which == "tune":
        ctxs["w1"] = ctx_env(PRISKV_CRC_STRIDE_WGS=1)
        for sh in (1, 2, 3):
            ctxs[f"shape{sh}"] = ctx_env(PRISKV_CRC_STRIDE_SHAPE=sh)
    elif which == "g":
        for g in (16, 32, 64):
            ctxs[f"G{g}"] = ctx_env(PRISKV_CRC_STRIDE_G=g)
            ctxs[f"G{g}w1"] = ctx_env(PRISKV_CRC_STRIDE_G=g, PRISKV_CRC_STRIDE_WGS=1)
        ctxs["shape3"] = ctx_env(PRISKV_CRC_STRIDE_SHAPE=3)
    total = int(gib * (1 << 30))
    stream = torch.cuda.Stream()
    for rnd in range(rounds):
        cases = CASES
        if which == "oddlarge":  # odd sizes of 8 KiB-256 KiB: stride (funnel) against the extents kernel
            cases = [(8193, 0), (16385, 0), (32769, 0), (65537, 0), (131073, 0), (262145, 0), (16384, 1), (65536, 3)]
        for bs, mis in cases:
            nb = total // bs
            t = torch.empty(nb * bs + 64, dtype=torch.uint8, device="cuda")
            ctxs["stride"].fill_splitmix(t, SEED ^ bs, 0)
            view = t[mis: mis + nb * bs]
            ref = None
            for name, c in ctxs.items():
                out = torch.empty(nb, dtype=torch.int32, device="cuda")
                with torch.cuda.stream(stream):
                    for _ in range(3):
                        c.blocks_dev(view, bs, out=out, stream=stream)
                    steps = int(os.environ.get('SWEEP_STEPS', '20'))
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(steps):
                        c.blocks_dev(view, bs, out=out, stream=stream)
                    e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / steps
                if ref is None:
                    ref = out.clone()
                    samp = min(nb, max(1, (64 << 20) // bs))
                    ok = bool(np.array_equal(as_u32(out[:samp]),
                                             O.crc32_blocks(view[: samp * bs].cpu().numpy(), bs, nthreads=16)))
                else:
                    ok = bool(torch.equal(out, ref))
                print(json.dumps({"round": rnd, "block_size": bs, "misalign": mis, "nblocks": nb, "ctx": name,
                                  "plan": c.blocks_plan(view.data_ptr(), nb, bs), "ms": round(ms, 4),
                                  "TBs": round(nb * (bs + 4) / (ms * 1e-3) / 1e12, 3), "ok": ok}), flush=True)
                del out
            del t, view, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
