#!/usr/bin/env python3
"""A/B of library builds on BASELINE configs[3]'s per-GPU shard (tools only).

  python tools/ab_tib.py LIB_A LIB_B [ROUNDS]

One process, one 128 GiB region (2 Mi x 64 KiB blocks, the block-cyclic
tile plan), both libraries loaded with ctypes (RTLD_LOCAL); each round
times 5 back-to-back calls of each library (order alternating) with HIP
events, and the two libraries' CRCs must agree bit for bit.  A 4 GiB
64 KiB batch (no tiles) is timed the same way as a control.  One JSON line
per (round, case, library).  For round 5's XCD-weighted tiles.
"""
import ctypes as C
import json
import os
import sys

import torch

libs = []
for path in sys.argv[1:3]:
    L = C.CDLL(os.path.abspath(path))
    L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.priskv_crc32_blocks_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
    libs.append((path, L, h))
ROUNDS = int(sys.argv[3]) if len(sys.argv) > 3 else 4
BS, NB = 65536, 2 << 20
region = torch.empty(BS * NB, dtype=torch.uint8, device="cuda")
g = torch.Generator(device="cuda").manual_seed(11)
region.random_(0, 256, generator=g)
s = torch.cuda.Stream()
outs = [torch.empty(NB, dtype=torch.int32, device="cuda") for _ in libs]
torch.cuda.synchronize()
for r in range(ROUNDS):
    for case, nb in (("tib 2Mi x 64KiB", NB), ("control 64Ki x 64KiB", 1 << 16)):
        order = libs if r % 2 == 0 else libs[::-1]
        for path, L, h in order:
            o = outs[libs.index((path, L, h))]
            for _ in range(2):
                assert L.priskv_crc32_blocks_dev(h, region.data_ptr(), nb, BS, o.data_ptr(), s.cuda_stream) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                assert L.priskv_crc32_blocks_dev(h, region.data_ptr(), nb, BS, o.data_ptr(), s.cuda_stream) == 0
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 5
            print(json.dumps({"round": r, "case": case, "lib": path, "ms_per_call": round(ms, 4),
                              "GBps": round(BS * nb / ms / 1e6, 1)}), flush=True)
        assert torch.equal(outs[0][:nb], outs[1][:nb]), (case, "libraries disagree")
