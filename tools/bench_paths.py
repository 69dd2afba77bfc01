#!/usr/bin/env python3
"""Throughput of every API path of libpriskv_crc.so on one GPU.

Not the driver's benchmark (that is bench.py); this times the secondary
paths -- every block-size plan including sub-KiB and generic sizes, the
per-value extent kernel on device and host (zero-copy scrub), and the
host-streamed block path -- each checked against the CPU oracle on a sample.
One JSON line per case on stdout.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import _oracle as O  # noqa: E402
import torch  # noqa: E402

from priskv_amd import CrcContext, as_u32, blocks_path, host_register, host_unregister  # noqa: E402

SEED = 0x5EED5EED


def timeit(fn, steps, warm_s=0.2):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        fn()
        torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(steps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / steps * 1e-3


def emit(**kw):
    print(json.dumps(kw), flush=True)


def blocks_case(ctx, bs, total, steps=10):
    nb = total // bs
    t = torch.empty(nb * bs, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED ^ bs, 0)
    out = torch.empty(nb, dtype=torch.int32, device="cuda")
    sec = timeit(lambda: ctx.blocks_dev(t, bs, out=out), steps)
    samp = min(nb, max(1, (256 << 20) // bs))
    ok = np.array_equal(as_u32(out[:samp]), O.crc32_blocks(t[: samp * bs].cpu().numpy(), bs, nthreads=16))
    emit(path="blocks_dev", kernel=blocks_path(t.data_ptr(), nb, bs), plan=ctx.blocks_plan(t.data_ptr(), nb, bs)[:90],
         block_size=bs, nblocks=nb,
         ms=round(sec * 1e3, 4), GiBs=round(nb * bs / sec / 2**30, 1), TBs=round(nb * (bs + 4) / sec / 1e12, 3),
         checked=samp, bit_exact=bool(ok))
    del t, out


def extents(rng, n, region_bytes, bs):
    """Values as PrisKV stores them: start on a block, occupy 2^k blocks,
    valuelen ragged inside the last block (server/buddy.c:134-140)."""
    k = rng.integers(0, 3, n)
    span = (1 << k) * bs
    blk = rng.integers(0, region_bytes // bs - 4, n)
    offs = (blk * bs).astype(np.uint64)
    lens = np.minimum(span - rng.integers(0, bs, n), region_bytes - offs).astype(np.uint32)
    return offs, lens


def ranges_dev_case(ctx, bs=4096, region=4 << 30, n=1 << 19, steps=10):
    rng = np.random.default_rng(1)
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 0)
    offs, lens = extents(rng, n, region, bs)
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    sec = timeit(lambda: ctx.ranges_dev(t, d_o, d_l, out=out), steps)
    samp = 20000
    host = None
    got = as_u32(out[:samp])
    want = np.array([O.crc32(t[int(o):int(o) + int(ln)].cpu().numpy()) for o, ln in zip(offs[:200], lens[:200])],
                    dtype=np.uint32)
    ok = np.array_equal(got[:200], want)
    vb = int(lens.astype(np.uint64).sum())
    emit(path="ranges_dev", block_size=bs, values=n, value_bytes=vb, mean_len=round(vb / n), ms=round(sec * 1e3, 4),
         GiBs=round(vb / sec / 2**30, 1), checked=200, bit_exact=bool(ok))
    del t, host


def few_values_case(ctx, ctx_noseg):
    """Fewer values than resident waves (a GET batch to verify, a few huge
    values): device-segmented extents against one wave per value, same
    process, wall time per call including the plan and combine launches."""
    rng = np.random.default_rng(3)
    for count, ln in ((1, 256 << 20), (8, 16 << 20), (32, 1 << 20), (32, 4 << 20), (256, 1 << 20),
                      (1000, 64 << 10), (3000, 64 << 10), (32, 4096 * 4 - 100)):
        region = count * (ln + 4096) + 4096
        t = torch.empty(region, dtype=torch.uint8, device="cuda")
        ctx.fill_splitmix(t, SEED, 0)
        offs = (np.arange(count, dtype=np.uint64) * (ln + 4096) + rng.integers(0, 4096, count).astype(np.uint64))
        lens = np.full(count, ln, dtype=np.uint32)
        d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_l = torch.from_numpy(lens.view(np.int32)).cuda()
        res = {}
        outs = {}
        for name, c in (("segmented", ctx), ("one_wave_per_value", ctx_noseg)):
            out = torch.empty(count, dtype=torch.int32, device="cuda")
            sec = timeit(lambda: c.ranges_dev(t, d_o, d_l, out=out), 20)
            res[name] = (round(sec * 1e6, 1), round(count * ln / sec / 2**30, 1))
            outs[name] = as_u32(out)
        k = min(count, 8)
        want = O.crc32_ranges(t.cpu().numpy(), offs[:k], lens[:k])
        ok = np.array_equal(outs["segmented"], outs["one_wave_per_value"]) and np.array_equal(
            outs["segmented"][:k], want)
        emit(path="ranges_dev_few", values=count, value_len=ln, segmented_us=res["segmented"][0],
             segmented_GiBs=res["segmented"][1], unsegmented_us=res["one_wave_per_value"][0],
             unsegmented_GiBs=res["one_wave_per_value"][1], bit_exact=bool(ok))
        del t


def seg_limit_case(ctx_a, ctx_b, label_a, label_b):
    """PrisKV-shaped values at 4 KiB / 64 KiB / 1 MiB blocks, n = 1000..2048:
    two contexts with different PRISKV_CRC_SEG_MAX_EXTENTS, same process."""
    rng = np.random.default_rng(5)
    region = 4 << 30
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx_a.fill_splitmix(t, SEED, 0)
    for bs, n in ((4096, 2048), (4096, 8192), (4096, 16384), (65536, 2048), (65536, 8192), (65536, 16384),
                  (1 << 20, 1000), (1 << 20, 2048), (1 << 20, 4096), (1 << 20, 8192), (1 << 20, 16384)):
        offs, lens = extents(rng, n, region, bs)
        d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_l = torch.from_numpy(lens.view(np.int32)).cuda()
        res, outs = {}, {}
        for name, c in ((label_a, ctx_a), (label_b, ctx_b)):
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            sec = timeit(lambda: c.ranges_dev(t, d_o, d_l, out=out), 20)
            res[name] = round(sec * 1e6, 1)
            outs[name] = as_u32(out)
        vb = int(lens.astype(np.uint64).sum())
        ok = np.array_equal(outs[label_a], outs[label_b])
        emit(path="ranges_dev_seg_limit", block_size=bs, values=n, value_bytes=vb,
             **{label_a + "_us": res[label_a], label_b + "_us": res[label_b]},
             best_TBs=round(vb / min(res.values()) / 1e6, 3), bit_exact=bool(ok))
    del t


def few_blocks_case(ctx, ctx_noseg):
    """Few very large blocks (the rows path's segmentation + combine) against
    the unsegmented rows kernel, same process."""
    for count, bs in ((1, 256 << 20), (4, 64 << 20), (16, 16 << 20), (1024, 1 << 20)):
        t = torch.empty(count * bs, dtype=torch.uint8, device="cuda")
        ctx.fill_splitmix(t, SEED, 0)
        res, outs = {}, {}
        for name, c in (("segmented", ctx), ("unsegmented", ctx_noseg)):
            out = torch.empty(count, dtype=torch.int32, device="cuda")
            sec = timeit(lambda: c.blocks_dev(t, bs, out=out), 10)
            res[name] = (round(sec * 1e6, 1), round(count * bs / sec / 2**30, 1))
            outs[name] = as_u32(out)
        ok = np.array_equal(outs["segmented"], outs["unsegmented"]) and \
            outs["segmented"][0] == O.crc32(t[:bs].cpu().numpy())
        emit(path="blocks_dev_few_large", blocks=count, block_size=bs, segmented_us=res["segmented"][0],
             segmented_GiBs=res["segmented"][1], unsegmented_us=res["unsegmented"][0],
             unsegmented_GiBs=res["unsegmented"][1], bit_exact=bool(ok))
        del t


def ranges_host_case(ctx, bs=4096, region=2 << 30, n=1 << 17):
    rng = np.random.default_rng(2)
    host = O.fill_splitmix(region, SEED, 0)
    offs, lens = extents(rng, n, region, bs)
    host_register(host)
    try:
        ctx.ranges_host(host, offs, lens)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            got = ctx.ranges_host(host, offs, lens)
        sec = (time.perf_counter() - t0) / reps
    finally:
        host_unregister(host)
    ok = np.array_equal(got[:5000], O.crc32_ranges(host, offs[:5000], lens[:5000]))
    vb = int(lens.astype(np.uint64).sum())
    emit(path="ranges_host_zero_copy", values=n, value_bytes=vb, ms=round(sec * 1e3, 2),
         GiBs=round(vb / sec / 2**30, 2), checked=5000, bit_exact=bool(ok))


def blocks_host_case(ctx, bs=4096, total=2 << 30):
    host = O.fill_splitmix(total, SEED, 0)
    res = {}
    for mode in ("registered", "pageable"):
        if mode == "registered":
            host_register(host)
        ctx.blocks_host(host, bs)
        t0 = time.perf_counter()
        for _ in range(3):
            got = ctx.blocks_host(host, bs)
        res[mode] = total / ((time.perf_counter() - t0) / 3) / 2**30
        if mode == "registered":
            host_unregister(host)
    ok = np.array_equal(got[:65536], O.crc32_blocks(host[: 65536 * bs], bs, nthreads=16))
    emit(path="blocks_host_streamed", block_size=bs, bytes=total, registered_GiBs=round(res["registered"], 2),
         pageable_GiBs=round(res["pageable"], 2), checked=65536, bit_exact=bool(ok))


def memfile_case(ctx, bs=4096, total=2 << 30):
    """The memfile as the server maps it: a tmpfs file mapped MAP_SHARED
    (server/memory.c:351-457), registered once with hipHostRegister, then
    block-streamed and scrubbed per value zero-copy."""
    import mmap
    path = f"/dev/shm/priskv_crc_memfile_{os.getpid()}"
    try:
        with open(path, "w+b") as f:
            f.truncate(total)
            mm = mmap.mmap(f.fileno(), total, flags=mmap.MAP_SHARED, prot=mmap.PROT_READ | mmap.PROT_WRITE)
        host = np.frombuffer(mm, dtype=np.uint8)
        host[:] = O.fill_splitmix(total, SEED, 0)
        host_register(host)
        try:
            ctx.blocks_host(host, bs)
            t0 = time.perf_counter()
            for _ in range(3):
                got = ctx.blocks_host(host, bs)
            blk = total / ((time.perf_counter() - t0) / 3) / 2**30
            rng = np.random.default_rng(3)
            offs, lens = extents(rng, 1 << 17, total, bs)
            ctx.ranges_host(host, offs, lens)
            t0 = time.perf_counter()
            for _ in range(3):
                gr = ctx.ranges_host(host, offs, lens)
            sec = (time.perf_counter() - t0) / 3
        finally:
            host_unregister(host)
        ok = (np.array_equal(got[:65536], O.crc32_blocks(host[: 65536 * bs], bs, nthreads=16))
              and np.array_equal(gr[:5000], O.crc32_ranges(host, offs[:5000], lens[:5000])))
        vb = int(lens.astype(np.uint64).sum())
        emit(path="memfile_tmpfs_registered", bytes=total, blocks_host_GiBs=round(blk, 2),
             ranges_host_values=int(offs.size), ranges_host_GiBs=round(vb / sec / 2**30, 2), bit_exact=bool(ok))
        del host, got, gr
        mm.close()
    finally:
        if os.path.exists(path):
            os.unlink(path)


def main():
    which = sys.argv[1:] or ["blocks", "ranges", "host", "memfile"]
    ctx = CrcContext(0)
    if "blocks" in which:
        for bs in (16, 64, 256, 512, 1024, 2048, 3072, 4096, 8192, 16384, 20480, 32768, 65536, 131072, 262144,
                   524288, 1 << 20, 100, 4100):
            total = (1 << 30) if bs >= 1024 else (256 << 20)
            if bs in (100, 4100):
                total = 64 << 20
            blocks_case(ctx, bs, total)
    if "paths1g" in which:  # DESIGN §6 "Other paths": 1 GiB per call, every non-headline block plan
        for bs in (4096, 4096, 16, 32, 64, 128, 256, 512, 100, 1000, 1023, 2047, 4095, 4097, 4100, 12345, 65537):
            blocks_case(ctx, bs, 1 << 30)
    if "paths4g" in which:  # the same plans at the headline's ~4 GiB per call (fixed costs out of the way)
        for bs in (4096, 4096, 16, 32, 64, 128, 256, 512, 100, 1000, 1023, 1025, 2047, 2049, 4095, 4097, 4100,
                   8193, 12345, 65537):
            blocks_case(ctx, bs, 4 << 30)
    if "ranges" in which:
        ranges_dev_case(ctx)
        ranges_dev_case(ctx, bs=65536, n=1 << 15)
        ranges_dev_case(ctx, bs=1 << 20, n=1 << 11)
    if "host" in which:
        ranges_host_case(ctx)
        blocks_host_case(ctx)
    if "memfile" in which:
        memfile_case(ctx)
    if "few" in which or "ranges" in which:
        os.environ["PRISKV_CRC_SEGMENT"] = "0"
        ctx_noseg = CrcContext(0)
        del os.environ["PRISKV_CRC_SEGMENT"]
        few_values_case(ctx, ctx_noseg)
        few_blocks_case(ctx, ctx_noseg)
        ctx_noseg.close()
    if "seglimit" in which:
        os.environ["PRISKV_CRC_SEG_MAX_EXTENTS"] = "512"
        ctx_512 = CrcContext(0)
        os.environ["PRISKV_CRC_SEG_MAX_EXTENTS"] = "16384"
        ctx_16k = CrcContext(0)
        del os.environ["PRISKV_CRC_SEG_MAX_EXTENTS"]
        seg_limit_case(ctx_512, ctx_16k, "limit512", "limit16384")
        ctx_512.close()
        ctx_16k.close()


if __name__ == "__main__":
    main()
