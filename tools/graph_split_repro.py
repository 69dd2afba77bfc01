#!/usr/bin/env python3
"""Loop of tests/test_gpu_parity.py's two graph-capture tests in one process
(tools only), with diagnostics for split-mode mismatches: which blocks, and
whether a wrong value is the CRC of the data before the refill (the block was
never completed) or neither.

  python tools/graph_split_repro.py [ITERS]
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import _oracle as O  # noqa: E402
import priskv_amd.crc as C  # noqa: E402
from priskv_amd import CrcContext, as_u32  # noqa: E402

if os.environ.get("REPRO_LIB"):
    C.LIB_PATH = os.path.abspath(os.environ["REPRO_LIB"])
ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
SEED = 0x5EED
ctx = CrcContext(0)
bad = 0


def region(nbytes, seed, word_offset):
    t = torch.empty(nbytes + 16, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, seed, word_offset, nbytes=nbytes)
    return t


def prev_test():  # test_hip_graph_capture_and_replay
    n = 40 << 20
    t = region(n, SEED ^ 0x6A, 2)
    offs = np.array([5, 3 << 20, 20 << 20], dtype=np.uint64)
    lens = np.array([(3 << 20) - 9, 17 << 20, 100], dtype=np.uint32)
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    o1 = torch.empty(1000, dtype=torch.int32, device="cuda")
    o2 = torch.empty(2, dtype=torch.int32, device="cuda")
    o3 = torch.empty(3, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx.blocks_dev(t, 4096, out=o1, nblocks=1000, stream=s)
        ctx.blocks_dev(t, 16 << 20, out=o2, nblocks=2, stream=s)
        ctx.ranges_dev(t, d_o, d_l, out=o3, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream()
        ctx.blocks_dev(t, 4096, out=o1, nblocks=1000, stream=st)
        ctx.blocks_dev(t, 16 << 20, out=o2, nblocks=2, stream=st)
        ctx.ranges_dev(t, d_o, d_l, out=o3, stream=st)
    for seed in (11, 12):
        ctx.fill_splitmix(t, seed, 0)
        g.replay()
        torch.cuda.synchronize()


MODE = "b2b"  # b2b | sync | one | o1only (REPRO_MODES, comma-separated: each in turn)


def split_test(it):  # test_rows_split_mode_graph_capture
    global bad
    n = 1900 << 20
    t = region(n, SEED ^ 0x5B1, 3)
    torch.cuda.synchronize()
    before = O.crc32_blocks(t[:n].cpu().numpy(), 1 << 20, nthreads=16)
    big = t[: 256 << 20]
    o1 = torch.empty(1900, dtype=torch.int32, device="cuda")
    o2 = torch.empty(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx.blocks_dev(t, 1 << 20, out=o1, nblocks=1900, stream=s)
        ctx.blocks_dev(big, 256 << 20, out=o2, nblocks=1, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    warm = as_u32(o1)
    wb = np.nonzero(warm != before)[0]
    if len(wb):
        bad += 1
        print(f"it {it} warm-up mismatch {len(wb)} {wb[:12].tolist()}", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream()
        ctx.blocks_dev(t, 1 << 20, out=o1, nblocks=1900, stream=st)
        if MODE != "o1only":
            ctx.blocks_dev(big, 256 << 20, out=o2, nblocks=1, stream=st)
    prev = before
    for seed in (21, 22):
        ctx.fill_splitmix(t, seed, 0)
        g.replay()
        if MODE == "sync":
            torch.cuda.synchronize()
        if MODE != "one":
            g.replay()
        torch.cuda.synchronize()
        host = t[:n].cpu().numpy()
        want = O.crc32_blocks(host, 1 << 20, nthreads=16)
        got = as_u32(o1)
        idx = np.nonzero(got != want)[0]
        if len(idx):
            bad += 1
            stale = [int(i) for i in idx if got[i] == prev[i]]
            print(f"mode {MODE} it {it} seed {seed} mismatch {len(idx)} {idx[:12].tolist()} stale {stale[:12]} "
                  f"got {got[idx[:4]].tolist()} want {want[idx[:4]].tolist()}", flush=True)
        prev = want
    del g


import socket  # noqa: E402

print("host", socket.gethostname(), torch.cuda.get_device_properties(0).name,
      getattr(torch.cuda.get_device_properties(0), "uuid", ""), ctx.blocks_plan(0, 1900, 1 << 20), flush=True)
for MODE in os.environ.get("REPRO_MODES", "b2b").split(","):
    for it in range(ITERS):
        prev_test()
        split_test(it)
        print(f"mode {MODE} it {it} done bad {bad}", flush=True)
print("bad", bad, flush=True)
