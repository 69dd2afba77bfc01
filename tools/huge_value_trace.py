#!/usr/bin/env python3
"""One huge value through ranges_dev (segmented), 50 calls back to back, for
rocprofv3 --kernel-trace: where the time of a lone 256 MiB extent goes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from priskv_amd import CrcContext  # noqa: E402

ln = int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 20
ctx = CrcContext(0)
t = torch.empty(ln + 4096, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(t, 7, 0)
d_o = torch.tensor([0], dtype=torch.int64, device="cuda")
d_l = torch.tensor([ln], dtype=torch.int32, device="cuda")
out = torch.empty(1, dtype=torch.int32, device="cuda")
for _ in range(50):
    ctx.ranges_dev(t, d_o, d_l, out=out)
torch.cuda.synchronize()
print("done")
