#!/usr/bin/env python3
"""Read roofs of several library builds on one region, in ONE process (tools only).

  python tools/roof_ab.py LIB[+LIB...] BS[+BS...] [ROUNDS]

For each block size (4096: the aligned rows pattern; odd sizes: the window
mode's pattern) and each library build (the product, or an A/B build whose
priskv_crc_read_roof_dev reads another pattern, e.g.
tools/patches/diag_roof_win_align.patch), every read-roof variant is timed
over ~4 GB of blocks (1 M blocks) with HIP events: the same short ramp each,
50 launches, order rotated per round.  One JSON line per (round, lib, bs,
variant), GB/s of the CRC's algorithmic bytes (block + 4 B).
"""
import ctypes as C
import json
import sys
import time

import torch

LIBS = sys.argv[1].split("+")
SIZES = [int(x) for x in sys.argv[2].split("+")]
ROUNDS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
NB = 1000000
K = 50


def load(path):
    L = C.CDLL(path)
    L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.priskv_crc_read_roof_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p,
                                           C.c_void_p]
    h = C.c_void_p()
    assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
    return L, h


libs = [(p, *load(p)) for p in LIBS]
s = torch.cuda.Stream()
sp = s.cuda_stream
region = torch.empty(max(SIZES) * NB + 4096, dtype=torch.uint8, device="cuda")
region.random_(0, 256, generator=torch.Generator(device="cuda").manual_seed(3))
sink = torch.zeros(8192, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
cases = [(p, L, h, bs, v) for (p, L, h) in libs for bs in SIZES for v in range(9)]
for r in range(ROUNDS):
    k = (r * 7) % len(cases)
    for p, L, h, bs, v in cases[k:] + cases[:k]:
        def fn():
            return L.priskv_crc_read_roof_dev(h, region.data_ptr(), NB, bs, v, sink.data_ptr(), sp)
        if fn() != 0:
            print(json.dumps({"round": r, "lib": p, "bs": bs, "variant": v, "error": "EINVAL"}), flush=True)
            continue
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.15:
            for _ in range(8):
                fn()
            s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(K):
            fn()
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / K * 1e3
        print(json.dumps({"round": r, "lib": p, "bs": bs, "variant": v, "us": round(us, 2),
                          "GBps": round(NB * (bs + 4) / (us * 1e-6) / 1e9, 1)}), flush=True)
