#!/usr/bin/env python3
"""AQL dispatch headers of a split-mode call (zero kernel + split kernel),
outside and inside a HIP graph (tools only).  Run with AMD_LOG_LEVEL=4: the
HIP runtime logs every dispatch packet's barrier / acquire / release bits;
the markers printed here delimit the phases in that log."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from priskv_amd import CrcContext  # noqa: E402

MIB = 1 << 20
ctx = CrcContext(0)
t = torch.empty(64 * MIB, dtype=torch.uint8, device="cuda")
o = torch.empty(4, dtype=torch.int32, device="cuda")
ctx.fill_splitmix(t, 1, 0)
torch.cuda.synchronize()


def mark(m):
    torch.cuda.synchronize()
    print(f"=== PHASE {m}", file=sys.stderr, flush=True)


mark("stream: first call on a new stream (pool slot allocated and zeroed)")
s = torch.cuda.Stream()
ctx.blocks_dev(t, 16 * MIB, out=o, nblocks=4, stream=s)
mark("stream: second call (pooled slot, no zero kernel)")
ctx.blocks_dev(t, 16 * MIB, out=o, nblocks=4, stream=s)
mark("graph capture")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    ctx.blocks_dev(t, 16 * MIB, out=o, nblocks=4, stream=torch.cuda.current_stream())
mark("graph replay 1")
g.replay()
mark("graph replay 2")
g.replay()
mark("end")
