#!/usr/bin/env python3
"""A/B of library builds and context options in ONE process (tools only).

  python tools/ab_libs.py VARIANT VARIANT ... [--rounds=R] [--cases=a+b]

VARIANT = path/to/libpriskv_crc.so[@VAR=V+VAR=V]: the library (loaded with
ctypes, RTLD_LOCAL: two builds keep separate symbol namespaces) and the
PRISKV_CRC_* environment its context is created with.  Every case is timed
with HIP events over back-to-back calls on one stream, the variants
alternating (order rotated per case and round), on the same device buffers,
and every variant's CRCs must agree bit for bit.  One JSON line per (round,
case, variant).  For kernel changes without a runtime switch (round 4: the
fused kernel's wave plan before its tables) and for tuning switches.
"""
import ctypes
import json
import os
import sys

import torch

ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
ROUNDS = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--rounds=")), "3"))
ONLY = next((a.split("=", 1)[1].split("+") for a in sys.argv if a.startswith("--cases=")), None)
# --streams=K: time every case on each of K created streams (HIP maps streams to
# hardware queues, whose first XCD differs: round 5), tagging lines with "stream"
NSTREAMS = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--streams=")), "1"))
C = ctypes


def load(spec):
    path, _, env = spec.partition("@")
    kv = [e.split("=", 1) for e in env.split("+") if e]
    for k, v in kv:
        os.environ[k] = v
    L = C.CDLL(os.path.abspath(path))
    L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.priskv_crc32_ranges_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                          C.c_void_p]
    L.priskv_crc32_blocks_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
    for k, _ in kv:
        del os.environ[k]
    return L, h


libs = {a: load(a) for a in ARGS}
TAGS = list(libs)
# each context's plan for the headline shape (its XCD probe result shows as
# "xcd-weighted" or not): a context whose probe found no round-robin dispatch
# runs equal shares, which differs by a percent or two
for _tag, (_L, _h) in libs.items():
    _L.priskv_crc32_blocks_plan.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_char_p, C.c_uint64]
    _buf = C.create_string_buffer(256)
    _L.priskv_crc32_blocks_plan(_h, C.c_void_p(1 << 20), 1 << 20, 4096, _buf, 256)
    print(json.dumps({"variant": _tag, "plan_1Mix4KiB": _buf.value.decode()}), flush=True)
STREAMS = [torch.cuda.Stream() for _ in range(NSTREAMS)]
s = STREAMS[0]
region = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
g = torch.Generator(device="cuda").manual_seed(7)
region.random_(0, 256, generator=g)
CASES = [("ranges 1x256MiB", 1, 256 << 20, 0), ("ranges 32x1MiB", 32, 1 << 20, (1 << 20) + 4096),
         ("ranges 4x64MiB", 4, 64 << 20, 64 << 20), ("ranges 1024x1MiB", 1024, 1 << 20, 1 << 20),
         ("ranges 65x4KiB", 65, 4096, 4096), ("ranges 4096x64KiB", 4096, 65536, 65536),
         ("blocks 1x256MiB", 1, 256 << 20, 0), ("blocks 16x16MiB", 16, 16 << 20, 0),
         ("blocks 65536x4KiB", 65536, 4096, 0), ("blocks 4096x64KiB", 4096, 65536, 0),
         ("blocks 1024x1MiB", 1024, 1 << 20, 0), ("blocks 4096x1MiB", 4096, 1 << 20, 0),
         ("blocks 1Mix4KiB", 1 << 20, 4096, 0),
         # odd sizes (the stride kernel), ~4 GiB per call
         ("blocks odd4097", 1000000, 4097, 0), ("blocks odd4095", 1000000, 4095, 0),
         ("blocks odd1000", 4000000, 1000, 0), ("blocks odd2047", 2000000, 2047, 0),
         ("blocks odd8193", 500000, 8193, 0), ("blocks odd100", 40000000, 100, 0),
         ("blocks odd8191", 500000, 8191, 0), ("blocks odd16383", 250000, 16383, 0),
         ("blocks odd4111", 1000000, 4111, 0), ("blocks odd4200", 1000000, 4200, 0),
         ("blocks odd2049", 2000000, 2049, 0), ("blocks odd3071", 1300000, 3071, 0),
         ("blocks odd3073", 1300000, 3073, 0), ("blocks odd5121", 800000, 5121, 0),
         ("blocks odd6143", 650000, 6143, 0), ("blocks odd10239", 400000, 10239, 0),
         ("blocks odd1023", 4000000, 1023, 0), ("blocks odd1025", 4000000, 1025, 0),
         ("blocks odd9217", 435000, 9217, 0), ("blocks odd15361", 260000, 15361, 0),
         ("blocks base1 2048", 2000000, 2048, 1),
         ("blocks al1024", 4000000, 1024, 0), ("blocks al2048", 2000000, 2048, 0),
         ("blocks al3072", 1300000, 3072, 0), ("blocks al6144", 650000, 6144, 0),
         # (blocks: the 4th field is a base offset) 4 KiB blocks on an odd base
         ("blocks base1 4096", 1000000, 4096, 1), ("blocks base8 4096", 1000000, 4096, 8),
         ("blocks base0 4096", 1000000, 4096, 0), ("blocks base16 4096", 1000000, 4096, 16),
         ("blocks base64 4096", 1000000, 4096, 64), ("blocks base128 4096", 1000000, 4096, 128),
         ("small32 blocks 8192xodd4097", 8192, 4097, 0), ("small32 blocks 8192xodd4095", 8192, 4095, 0),
         # 32 MiB calls: few large values / blocks against the rows kernel
         ("small32 ranges 32x1MiB", 32, 1 << 20, 1 << 20), ("small32 ranges 16x2MiB", 16, 2 << 20, 2 << 20),
         ("small32 blocks 32x1MiB", 32, 1 << 20, 0), ("small32 blocks 8192x4KiB", 8192, 4096, 0),
         ("small32 blocks 512x64KiB", 512, 65536, 0),
         # unbalanced batches below the split-few size: rows + combine (blocks) against the fused kernel (ranges)
         ("mid ranges 512x64KiB", 512, 65536, 65536), ("mid blocks 512x64KiB", 512, 65536, 0),
         ("mid ranges 100x1MiB", 100, 1 << 20, 1 << 20), ("mid blocks 100x1MiB", 100, 1 << 20, 0),
         ("mid ranges 1000x128KiB", 1000, 128 << 10, 128 << 10), ("mid blocks 1000x128KiB", 1000, 128 << 10, 0),
         ("mid ranges 200x512KiB", 200, 512 << 10, 512 << 10), ("mid blocks 200x512KiB", 200, 512 << 10, 0),
         ("mid ranges 1500x64KiB", 1500, 65536, 65536), ("mid blocks 1500x64KiB", 1500, 65536, 0),
         # tiny calls: launch and table-load latency (the fused kernel's wave plan up to 64 values)
         ("tiny ranges 1x4KiB", 1, 4096, 4096), ("tiny ranges 16x4KiB", 16, 4096, 4096),
         ("tiny ranges 64x4KiB", 64, 4096, 4096), ("tiny ranges 16x64KiB", 16, 65536, 65536),
         ("tiny ranges 64x64KiB", 64, 65536, 65536), ("tiny blocks 1x4KiB", 1, 4096, 0),
         ("tiny blocks 64x64KiB", 64, 65536, 0)]
# PrisKV-shaped scattered values (tools/values_bench.py extents(): 1-4 blocks,
# ragged ends, random blocks of the region)
import numpy as np  # noqa: E402
_rng = np.random.default_rng(1)
SCATTER = {}
for _name, _bs, _n in (("priskv4k", 4096, 1 << 19), ("priskv64k", 65536, 1 << 15)):
    _k = _rng.integers(0, 3, _n)
    _span = (1 << _k) * _bs
    _blk = _rng.integers(0, region.numel() // _bs - 4, _n)
    _o = (_blk * _bs).astype(np.uint64)
    _l = np.minimum(_span - _rng.integers(0, _bs, _n), region.numel() - _o).astype(np.uint32)
    SCATTER[_name] = (torch.from_numpy(_o.astype(np.int64)).cuda(), torch.from_numpy(_l.view(np.int32)).cuda())
    CASES.append(("ranges " + _name, _n, 0, 0))
ref = {}
for r in range(ROUNDS):
    for ci, (name, n, ln, stride) in enumerate(CASES):
        if name.split()[-1] in SCATTER:
            offs, lens = SCATTER[name.split()[-1]]
        else:
            offs = torch.arange(n, dtype=torch.int64, device="cuda") * stride
            lens = torch.full((n,), ln, dtype=torch.int32, device="cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        if ONLY and not any(o in name for o in ONLY):
            continue
        # offs / lens are written on torch's current stream; the calls run on
        # STREAMS[si]: wait for them (round 5: without this a call read the
        # arrays of a reused allocation before they were written -- garbage
        # offsets, an illegal-address fault in the tool)
        torch.cuda.synchronize()
        k = (r + ci) % len(TAGS)
        order = TAGS[k:] + TAGS[:k]
        for si, tag in [(si, tag) for si in range(NSTREAMS) for tag in order]:
            L, h = libs[tag]
            s = STREAMS[si]
            sp = s.cuda_stream

            def call():
                if name.split()[-2] == "ranges" or name.startswith("ranges"):
                    rc = L.priskv_crc32_ranges_dev(h, region.data_ptr(), offs.data_ptr(), lens.data_ptr(), n,
                                                   out.data_ptr(), sp)
                else:
                    rc = L.priskv_crc32_blocks_dev(h, region.data_ptr() + stride, n, ln, out.data_ptr(), sp)
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
            if "--nocheck" not in sys.argv:  # (--nocheck: timing-only probes of deliberately wrong builds)
                assert ref.setdefault(name, got) == got, (name, tag)  # A and B agree bit for bit
            rec = {"round": r, "case": name, "variant": tag, "us_per_call": round(e0.elapsed_time(e1) / 50 * 1e3, 2)}
            if NSTREAMS > 1:
                rec["stream"] = si
            print(json.dumps(rec), flush=True)
