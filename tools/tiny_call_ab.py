#!/usr/bin/env python3
"""GPU-side time of tiny calls, A/B of library builds in one process (tools only).

  python tools/tiny_call_ab.py LIB LIB ... [--rounds=R]

Host enqueue time is kept out of the measurement: each tiny call is queued
between two events behind a 256 MiB call (~50 us of GPU work), so the GPU
reaches event, call, event back to back and their distance is launch +
kernel only.  Medians over 200 calls per (round, case, variant); the
variants' CRCs must agree bit for bit.
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
ROUNDS = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--rounds=")), "3"))


def load(path):
    L = C.CDLL(os.path.abspath(path))
    L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.priskv_crc32_ranges_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                          C.c_void_p]
    L.priskv_crc32_blocks_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    if hasattr(L, "priskv_crc32_ranges_dev_bounded"):  # (round 6 on)
        L.priskv_crc32_ranges_dev_bounded.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                                      C.c_uint64, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
    return L, h


libs = {a: load(a) for a in ARGS}
tags = list(libs)
s = torch.cuda.Stream()
region = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
region.random_(0, 256, generator=torch.Generator(device="cuda").manual_seed(3))
big_out = torch.empty(1, dtype=torch.int32, device="cuda")
CASES = [("ranges", 1, 4096), ("ranges", 16, 4096), ("ranges", 64, 4096), ("ranges", 16, 65536),
         ("ranges", 64, 65536), ("ranges", 1, 1 << 20), ("blocks", 1, 4096), ("blocks", 64, 65536),
         # the same values with the host-known bound (priskv_crc32_ranges_dev_bounded, max_len = the length)
         ("rangesb", 1, 4096), ("rangesb", 16, 4096), ("rangesb", 64, 4096), ("rangesb", 16, 65536),
         ("rangesb", 64, 65536), ("rangesb", 1, 1 << 20)]
ref = {}
for r in range(ROUNDS):
    for ci, (kind, n, ln) in enumerate(CASES):
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * ln
        lens = torch.full((n,), ln, dtype=torch.int32, device="cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        k = (r + ci) % len(tags)
        for tag in tags[k:] + tags[:k]:
            L, h = libs[tag]
            sp = s.cuda_stream

            if kind == "rangesb" and not hasattr(L, "priskv_crc32_ranges_dev_bounded"):
                continue

            def tiny():
                if kind == "rangesb":
                    rc = L.priskv_crc32_ranges_dev_bounded(h, region.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                                           ln, out.data_ptr(), sp)
                elif kind == "ranges":
                    rc = L.priskv_crc32_ranges_dev(h, region.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                                   out.data_ptr(), sp)
                else:
                    rc = L.priskv_crc32_blocks_dev(h, region.data_ptr(), n, ln, out.data_ptr(), sp)
                assert rc == 0, rc

            def big():
                assert L.priskv_crc32_blocks_dev(h, region.data_ptr(), 1, 256 << 20, big_out.data_ptr(), sp) == 0

            for _ in range(20):
                big()
                tiny()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
            for e0, e1 in ev:
                big()
                e0.record(s)
                tiny()
                e1.record(s)
            torch.cuda.synchronize()
            us = [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
            got = out.cpu().numpy().tobytes()
            name = f"{kind} {n}x{ln}"
            assert ref.setdefault(name.replace("rangesb", "ranges"), got) == got, (name, tag)
            print(json.dumps({"round": r, "case": name, "variant": tag, "us_per_call": round(float(np.median(us)), 3),
                              "p10": round(float(np.percentile(us, 10)), 3),
                              "p90": round(float(np.percentile(us, 90)), 3)}), flush=True)
