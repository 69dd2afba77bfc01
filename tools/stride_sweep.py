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
import time

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
    elif which == "retune":  # the stride kernel's knobs, unbiased (rotated order, warm-up)
        ctxs = {"default": ctxs["stride"]}
        ctxs["w1"] = ctx_env(PRISKV_CRC_STRIDE_WGS=1)
        ctxs["runs"] = ctx_env(PRISKV_CRC_STRIDE_RUNS=1)
        ctxs["w1_runs"] = ctx_env(PRISKV_CRC_STRIDE_WGS=1, PRISKV_CRC_STRIDE_RUNS=1)
        ctxs["w1_sh1"] = ctx_env(PRISKV_CRC_STRIDE_WGS=1, PRISKV_CRC_STRIDE_SHAPE=1)
        ctxs["g64"] = ctx_env(PRISKV_CRC_STRIDE_G=64)
    elif which == "runsab":  # lane groups side by side (default) against runs, at bench.py's batch size
        ctxs = {"default": ctxs["stride"], "runs": ctx_env(PRISKV_CRC_STRIDE_RUNS=1)}
    elif which == "large":  # G for multi-row blocks (the cost model's G = 64 threshold)
        ctxs = {"default": ctxs["stride"]}
        for g in (16, 32, 64):
            ctxs[f"G{g}"] = ctx_env(PRISKV_CRC_STRIDE_G=g)
    elif which in ("prio", "priorefine"):  # round 3: one 16-wave workgroup with progress priority (default) against two 8-wave
        ctxs = {"default": ctxs["stride"], "noprio": ctx_env(PRISKV_CRC_STRIDE_PRIO=0),
                "stride_big": ctx_env(PRISKV_CRC_STRIDE_MAX_KIB=1024)}
    elif which == "funnel":
        ctxs["nofunnel"] = ctx_env(PRISKV_CRC_STRIDE_FUNNEL=0)
    elif which == "runs":
        ctxs["runs"] = ctx_env(PRISKV_CRC_STRIDE_RUNS=1)
        ctxs["runs_sh3"] = ctx_env(PRISKV_CRC_STRIDE_RUNS=1, PRISKV_CRC_STRIDE_SHAPE=3)
        ctxs["sh3"] = ctx_env(PRISKV_CRC_STRIDE_SHAPE=3)
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
        if which == "refine":  # the stride / extents size limits, between the measured points
            cases = [(5121, 0), (6145, 0), (7169, 0), (8193, 0), (10244, 0), (12292, 0), (14340, 0), (16388, 0)]
        if which == "runsab":
            cases = [(4100, 0), (4097, 0), (3000, 0), (1000, 0), (520, 0)]
        if which == "cross":  # stride (default) against round 2's extents kernel on multi-row blocks
            cases = [(8196, 0), (16388, 0), (24580, 0), (32772, 0), (49156, 0), (65540, 0), (100000, 0),
                     (16384, 4), (65536, 4), (262148, 0)]
        if which == "large":
            cases = [(4100, 0), (8196, 0), (12292, 0), (16388, 0), (32772, 0), (65540, 0), (100000, 0),
                     (300004, 0), (1000004, 0), (65536, 4)]
        if which == "retune":
            cases = [(100, 0), (520, 0), (1000, 0), (3000, 0), (4100, 0), (4096, 4), (4097, 0), (100000, 0),
                     (19, 3), (256, 3)]
        if which == "prio":
            cases = [(19, 3), (100, 0), (200, 0), (520, 0), (1000, 0), (3000, 0), (4097, 0), (4096, 1), (4609, 0),
                     (6145, 0), (8193, 0), (9212, 0), (12289, 0), (12292, 0), (16385, 0), (24580, 0), (65537, 0)]
        if which == "priorefine":  # the stride / extents crossover with the prioritised stride kernel
            cases = [(8705, 0), (9217, 0), (9729, 0), (10241, 0), (10753, 0), (11265, 0), (10000, 0), (11000, 0),
                     (12000, 0), (14000, 0)]
        if which == "oddlarge":  # odd sizes of 8 KiB-256 KiB: stride (funnel) against the extents kernel
            cases = [(8193, 0), (16385, 0), (32769, 0), (65537, 0), (131073, 0), (262145, 0), (16384, 1), (65536, 3)]
        for bs, mis in cases:
            nb = total // bs
            t = torch.empty(nb * bs + 64, dtype=torch.uint8, device="cuda")
            next(iter(ctxs.values())).fill_splitmix(t, SEED ^ bs, 0)
            view = t[mis: mis + nb * bs]
            ref = None
            # Contexts in a rotated order each round, each after >= 0.25 s of
            # back-to-back warm-up calls: a context timed right after an idle
            # gap (the first one's oracle check) ran up to 17 % slow on the
            # same kernel (clock ramp), which biased the first
            # versions of this sweep.  The oracle check runs after all contexts.
            names = list(ctxs)
            k0 = rnd % len(names)
            for name in names[k0:] + names[:k0]:
                c = ctxs[name]
                out = torch.empty(nb, dtype=torch.int32, device="cuda")
                with torch.cuda.stream(stream):
                    t_w = time.perf_counter()
                    while time.perf_counter() - t_w < 0.25:
                        for _ in range(4):
                            c.blocks_dev(view, bs, out=out, stream=stream)
                        stream.synchronize()
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
                ok = bool(torch.equal(out, ref))
                print(json.dumps({"round": rnd, "block_size": bs, "misalign": mis, "nblocks": nb, "ctx": name,
                                  "plan": c.blocks_plan(view.data_ptr(), nb, bs), "ms": round(ms, 4),
                                  "TBs": round(nb * (bs + 4) / (ms * 1e-3) / 1e12, 3), "ok": ok}), flush=True)
                del out
            samp = min(nb, max(1, (64 << 20) // bs))
            if not np.array_equal(as_u32(ref[:samp]), O.crc32_blocks(view[: samp * bs].cpu().numpy(), bs, nthreads=16)):
                print(json.dumps({"round": rnd, "block_size": bs, "misalign": mis, "oracle_mismatch": True}), flush=True)
            del t, view, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
