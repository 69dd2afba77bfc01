#!/usr/bin/env python3
"""What the 4 KiB plan's per-block fold costs (tools only).

  python tools/fold_bound_ab.py PRODUCT.so NOFOLD.so NOREDUCE.so [ROUNDS]

In ONE process, on one 4 GiB region (1 Mi x 4 KiB blocks, the headline
config): the product's crc_rows_kernel<64,4,4,2,818>, the same kernel with
the nibble fold removed (tools/patches/diag_4k_nofold.patch) and with the
fold and the DPP/readlane row reduction removed
(tools/patches/diag_4k_nofold_noreduce.patch) -- both timing-only builds
that return wrong CRCs -- and the product's read roof
(priskv_crc_read_roof_dev: the kernel's loads, ranges and XCD split without
hashing) in variants 0 (the plan's own shape) and 1-8.  Each is ramped the
same way, timed over 50 back-to-back launches with HIP events, the order
rotated per round.  One JSON line per (round, variant).
"""
import ctypes as C
import json
import sys
import time

import torch

PATHS = sys.argv[1:4]
ROUNDS = int(sys.argv[4]) if len(sys.argv) > 4 else 4
BS, NB = 4096, 1 << 20
K = 50


def load(path):
    L = C.CDLL(path)
    L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.priskv_crc32_blocks_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    L.priskv_crc_read_roof_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p,
                                           C.c_void_p]
    L.priskv_crc_fill_splitmix_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                               C.c_void_p]
    h = C.c_void_p()
    assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
    return L, h


libs = [load(p) for p in PATHS]
names = ["product", "nofold", "nofold_noreduce"]
s = torch.cuda.Stream()
sp = s.cuda_stream
region = torch.empty(BS * NB, dtype=torch.uint8, device="cuda")
out = torch.empty(NB, dtype=torch.int32, device="cuda")
sink = torch.zeros(8192, dtype=torch.int32, device="cuda")
L0, h0 = libs[0]
assert L0.priskv_crc_fill_splitmix_dev(h0, region.data_ptr(), BS * NB, 0x5EED, 0, sp) == 0
torch.cuda.synchronize()

variants = []
for (L, h), n in zip(libs, names):
    variants.append((n, (lambda L=L, h=h: L.priskv_crc32_blocks_dev(h, region.data_ptr(), NB, BS, out.data_ptr(), sp))))
for v in range(9):
    variants.append((f"roof{v}", (lambda v=v: L0.priskv_crc_read_roof_dev(h0, region.data_ptr(), NB, BS, v,
                                                                            sink.data_ptr(), sp))))

alg = NB * (BS + 4)
for r in range(ROUNDS):
    k = r % len(variants)
    for name, fn in variants[k:] + variants[:k]:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:  # the same ramp for every variant
            for _ in range(8):
                assert fn() == 0
            s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(K):
            fn()
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / K * 1e3
        print(json.dumps({"round": r, "variant": name, "us_per_launch": round(us, 2),
                          "TBps": round(alg / (us * 1e-6) / 1e12, 4), "frac": round(alg / (us * 1e-6) / 8e12, 4)}),
              flush=True)
