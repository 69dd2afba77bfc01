#!/usr/bin/env python3
"""Few-values cases through ranges_dev with device-resident lengths, back to
back on one stream, for rocprofv3 --kernel-trace (where a call's time goes:
plan / extents / reduce kernels and the gaps between them), plus HIP-event
wall time per call.  Cases: 1 x 256 MiB, 32 x 1 MiB, 4096 x (4 KiB - 100),
4096 x 64 KiB, 16384 x 16 KiB, 1 / 64 / 65 x 4 KiB equal values (64 is the
largest wave-planned call).  --blocks: the rows kernel on 256 MiB for
comparison.  --noseg: also a context that never segments.  --ab: also through a context with
PRISKV_CRC_FUSED=0 (the three-launch plan / extents / reduce path).  Tools only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from priskv_amd import CrcContext  # noqa: E402

ctxs = [("fused", CrcContext(0))]
if "--ab" in sys.argv:
    os.environ["PRISKV_CRC_FUSED"] = "0"
    ctxs.append(("three-launch", CrcContext(0)))
    del os.environ["PRISKV_CRC_FUSED"]
if "--fused-ab" in sys.argv:  # the fused kernel's round-4 options, each off
    for var in ("PRISKV_CRC_FUSED_XW",):
        os.environ[var] = "0"
        ctxs.append((var.split("_")[-1].lower() + "=0", CrcContext(0)))
        del os.environ[var]
if "--noseg" in sys.argv:
    os.environ["PRISKV_CRC_SEG_MAX_EXTENTS"] = "0"
    ctxs.append(("unsegmented", CrcContext(0)))
    del os.environ["PRISKV_CRC_SEG_MAX_EXTENTS"]
ctx = ctxs[0][1]
s = torch.cuda.Stream()
t = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(t, 7, 0)
ROUNDS = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--rounds=")), "1"))  # whole sweeps
case_no = 0
for name, n, ln, stride in ROUNDS * (("1x256MiB", 1, 256 << 20, 0), ("32x1MiB", 32, 1 << 20, (1 << 20) + 4096),
                            ("4096x4KiB-100", 4096, 4096 - 100, 4096), ("4096x64KiB", 4096, 65536, 65536),
                            ("16384x16KiB", 16384, 16384, 16384), ("1x4KiB", 1, 4096, 0), ("64x4KiB", 64, 4096, 4096),
                            ("65x4KiB", 65, 4096, 4096), ("4x64MiB", 4, 64 << 20, 64 << 20),
                            ("16x16MiB", 16, 16 << 20, 16 << 20), ("1024x1MiB", 1024, 1 << 20, 1 << 20)):
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    lens = torch.full((n,), ln, dtype=torch.int32, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    case_no += 1
    for path, c in ctxs[case_no % len(ctxs):] + ctxs[:case_no % len(ctxs)]:  # order rotated per case
        with torch.cuda.stream(s):
            for _ in range(30):
                c.ranges_dev(t, offs, lens, out=out, stream=s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(100):
                c.ranges_dev(t, offs, lens, out=out, stream=s)
            e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / 100 * 1e3
        print(json.dumps({"case": name, "path": path, "us_per_call": round(us, 2),
                          "TBs": round(n * ln / (us * 1e-6) / 1e12, 3)}), flush=True)
if "--blocks" in sys.argv:  # the rows machinery on 256 MiB: one block (segments + combine), 16 KiB and 4 KiB blocks
    for bs, nb in ((256 << 20, 1), (64 << 20, 4), (16 << 20, 16), (1 << 20, 1024), (16384, 16384), (4096, 65536),
                   (65536, 4096)):
        out = torch.empty(nb, dtype=torch.int32, device="cuda")
        for path, c in ctxs:
            with torch.cuda.stream(s):
                for _ in range(30):
                    c.blocks_dev(t, bs, out=out, nblocks=nb, stream=s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(100):
                    c.blocks_dev(t, bs, out=out, nblocks=nb, stream=s)
                e1.record(s)
            e1.synchronize()
            print(json.dumps({"case": "blocks %dx%d" % (nb, bs), "path": path,
                              "plan": c.blocks_plan(t.data_ptr(), nb, bs)[:60],
                              "us_per_call": round(e0.elapsed_time(e1) / 100 * 1e3, 2)}), flush=True)
