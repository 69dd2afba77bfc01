#!/usr/bin/env python3
"""Repeat split-mode calls and report every mismatch against the oracle
(tools only): plain calls on one stream, calls alternating two streams, and
a captured graph replayed back to back.

  python tools/split_stress.py [ITERS] [BS] [NB]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import _oracle as O  # noqa: E402
import priskv_amd.crc as C  # noqa: E402
from priskv_amd import CrcContext, as_u32  # noqa: E402

if os.environ.get("SPLIT_STRESS_LIB"):  # another build of the library
    C.LIB_PATH = os.path.abspath(os.environ["SPLIT_STRESS_LIB"])

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
BS = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
NB = int(sys.argv[3]) if len(sys.argv) > 3 else 1900
ctx = CrcContext(0)
print("plan", ctx.blocks_plan(0, NB, BS), flush=True)
n = BS * NB
t = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
bad = 0


def check(tag, out, want):
    global bad
    got = as_u32(out)
    idx = np.nonzero(got != want)[0]
    if len(idx):
        bad += 1
        print(tag, "mismatch", len(idx), idx[:16].tolist(), flush=True)


for seed in (21, 22):
    ctx.fill_splitmix(t, seed, 0)
    torch.cuda.synchronize()
    want = O.crc32_blocks(t[:n].cpu().numpy(), BS, nthreads=16)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    outs = []
    for i in range(ITERS):
        st = s1
        with torch.cuda.stream(st):
            outs.append(ctx.blocks_dev(t, BS, nblocks=NB, stream=st))
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        check(f"seed {seed} one-stream {i}", o, want)
    outs = []
    for i in range(ITERS):
        st = s1 if i % 2 else s2
        with torch.cuda.stream(st):
            outs.append(ctx.blocks_dev(t, BS, nblocks=NB, stream=st))
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        check(f"seed {seed} two-stream {i}", o, want)
    o1 = torch.empty(NB, dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ctx.blocks_dev(t, BS, out=o1, nblocks=NB, stream=torch.cuda.current_stream())
    for i in range(ITERS):
        g.replay()
        if i % 4 == 3:
            torch.cuda.synchronize()
            check(f"seed {seed} graph {i}", o1, want)
    torch.cuda.synchronize()
    check(f"seed {seed} graph end", o1, want)
# graphs captured over recycled stream-ordered memory: a pool-off context's
# per-call scratch (segment CRCs, non-zero) is freed into the default memory
# pool before every capture, then two split-mode calls are captured and
# replayed back to back (tests/test_gpu_parity.py::test_rows_split_mode_graph_capture)
os.environ["PRISKV_CRC_SCRATCH_POOL"] = "0"
junk_ctx = CrcContext(0)
del os.environ["PRISKV_CRC_SCRATCH_POOL"]
ctx.fill_splitmix(t, 23, 0)
torch.cuda.synchronize()
host = t[:n].cpu().numpy()
want = O.crc32_blocks(host, BS, nthreads=16)
want_big = O.crc32_blocks(host[: 256 << 20], 256 << 20, nthreads=16)
big = t[: 256 << 20]
rng = np.random.default_rng(5)
for it in range(ITERS):
    for _ in range(4):  # junk: segmented calls with per-call scratch
        lens = rng.integers(1 << 20, 12 << 20, 6).astype(np.uint32)
        offs = np.array([rng.integers(0, n - int(ln)) for ln in lens], dtype=np.uint64)
        junk_ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(),
                            torch.from_numpy(lens.view(np.int32)).cuda())
        junk_ctx.blocks_dev(t, 16 << 20, nblocks=3)
    torch.cuda.synchronize()
    o1 = torch.empty(NB, dtype=torch.int32, device="cuda")
    o2 = torch.empty(1, dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream()
        ctx.blocks_dev(t, BS, out=o1, nblocks=NB, stream=st)
        ctx.blocks_dev(big, 256 << 20, out=o2, nblocks=1, stream=st)
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        check(f"junk graph {it} replay {r}", o1, want)
        check(f"junk graph {it} replay {r} big", o2, want_big)
    del g
print("bad", bad, flush=True)
