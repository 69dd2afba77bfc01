#!/usr/bin/env python3
"""A/B of two builds of libpriskv_crc.so in ONE process (tools only).

  python tools/ab_libs.py A.so B.so [rounds]

Both libraries are loaded side by side (ctypes, RTLD_LOCAL: separate symbol
namespaces), each with its own context on device 0; every case is timed with
HIP events over back-to-back calls on one stream, the two libraries
alternating (order rotated per round), on the same device buffers.  Prints
one JSON line per (round, case, library).  Used for kernel changes that have
no runtime switch (round 4: the fused kernel's wave plan before its tables).
"""
import ctypes
import json
import os
import sys

import torch

A, B = sys.argv[1], sys.argv[2]
ROUNDS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
C = ctypes


def load(path):
    L = C.CDLL(os.path.abspath(path))
    L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.priskv_crc32_ranges_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                          C.c_void_p]
    L.priskv_crc32_blocks_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
    return L, h


libs = {"A": load(A), "B": load(B)}
s = torch.cuda.Stream()
region = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
g = torch.Generator(device="cuda").manual_seed(7)
region.random_(0, 256, generator=g)
CASES = [("ranges 1x256MiB", 1, 256 << 20, 0), ("ranges 32x1MiB", 32, 1 << 20, (1 << 20) + 4096),
         ("ranges 4x64MiB", 4, 64 << 20, 64 << 20), ("ranges 1024x1MiB", 1024, 1 << 20, 1 << 20),
         ("ranges 65x4KiB", 65, 4096, 4096), ("ranges 4096x64KiB", 4096, 65536, 65536),
         ("blocks 1x256MiB", 1, 256 << 20, 0), ("blocks 16x16MiB", 16, 16 << 20, 0)]
ref = {}
for r in range(ROUNDS):
    for ci, (name, n, ln, stride) in enumerate(CASES):
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride
        lens = torch.full((n,), ln, dtype=torch.int32, device="cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        order = ["A", "B"] if (r + ci) % 2 == 0 else ["B", "A"]
        for tag in order:
            L, h = libs[tag]
            sp = s.cuda_stream

            def call():
                if name.startswith("ranges"):
                    rc = L.priskv_crc32_ranges_dev(h, region.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                                   out.data_ptr(), sp)
                else:
                    rc = L.priskv_crc32_blocks_dev(h, region.data_ptr(), n, ln, out.data_ptr(), sp)
                assert rc == 0, rc
            for _ in range(20):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(50):
                call()
            e1.record(s)
            e1.synchronize()
            got = out.cpu().numpy().tobytes()
            assert ref.setdefault(name, got) == got, (name, tag)  # A and B agree bit for bit
            print(json.dumps({"round": r, "case": name, "lib": tag, "us_per_call": round(e0.elapsed_time(e1) / 50 * 1e3, 2)}),
                  flush=True)
