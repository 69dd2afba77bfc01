#!/usr/bin/env python3
"""Where the segmented extents path's fixed cost goes (run under rocprofv3
--kernel-trace): N PrisKV-shaped 4 KiB-block values (argv[1], default 2048),
segmented and not, 200 calls each, back to back on one stream."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from bench_paths import extents  # noqa: E402
from priskv_amd import CrcContext  # noqa: E402

region = 1 << 30
ctx = CrcContext(0)
os.environ["PRISKV_CRC_SEGMENT"] = "0"
ctx0 = CrcContext(0)
del os.environ["PRISKV_CRC_SEGMENT"]
t = torch.empty(region, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(t, 7, 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
offs, lens = extents(np.random.default_rng(5), n, region, 4096)
d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
d_l = torch.from_numpy(lens.view(np.int32)).cuda()
out = torch.empty(n, dtype=torch.int32, device="cuda")
for c in (ctx0, ctx, ctx0, ctx):
    for _ in range(200):
        c.ranges_dev(t, d_o, d_l, out=out)
    torch.cuda.synchronize()
print("done")
