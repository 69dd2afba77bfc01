#!/usr/bin/env python3
"""Few-values cases through ranges_dev with device-resident lengths, back to
back on one stream, for rocprofv3 --kernel-trace (where a call's time goes:
plan / extents / reduce kernels and the gaps between them), plus HIP-event
wall time per call.  Cases: 1 x 256 MiB, 32 x 1 MiB, 4096 x (4 KiB - 100),
4096 x 64 KiB equal values.  Tools only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from priskv_amd import CrcContext  # noqa: E402

ctx = CrcContext(0)
s = torch.cuda.Stream()
t = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(t, 7, 0)
for name, n, ln, stride in (("1x256MiB", 1, 256 << 20, 0), ("32x1MiB", 32, 1 << 20, (1 << 20) + 4096),
                            ("4096x4KiB-100", 4096, 4096 - 100, 4096), ("4096x64KiB", 4096, 65536, 65536)):
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    lens = torch.full((n,), ln, dtype=torch.int32, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(s):
        for _ in range(30):
            ctx.ranges_dev(t, offs, lens, out=out, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(100):
            ctx.ranges_dev(t, offs, lens, out=out, stream=s)
        e1.record(s)
    e1.synchronize()
    print(json.dumps({"case": name, "us_per_call": round(e0.elapsed_time(e1) / 100 * 1e3, 2),
                      "TBs": round(n * ln / (e0.elapsed_time(e1) / 100 * 1e-3) / 1e12, 3)}), flush=True)
