#!/usr/bin/env python3
"""bench.py -- value-block CRC throughput on MI355X (BASELINE.json metric).

One "step" = one pass of priskv_crc32 (server/crc.c:90-109) over every value
block of this GPU's shard, device-resident (inputs already in HBM when the
timed region starts), through the library's C ABI
(priskv_crc32_blocks_dev, include/priskv_crc_gpu.h).

Headline workload (`value`, BASELINE.json configs[1]): 1 Mi x 4 KiB blocks =
4 GiB per GPU.  For N > 1 (launched by torch.distributed.run) each rank owns
its own 4 GiB shard -- the next 1 Mi blocks of one global region -- and
checksums it with no data-path collective ("weak" scaling); the barrier and
the max-over-ranks reduction are the benchmark contract, not part of the path.

Rank 0 prints ONE compact JSON line (~2.5 KB, compact_line: the contract's
keys, the headline roofline and cpu_baseline, and under "legs" each other
leg's value, ms_per_step, frac, frac_of_measured, traffic ratio and
bit_exact) and writes the full result below to the detail file
(gpurun_out/bench_detail.json, --detail).  The legs of the full result
(every BASELINE config that fits a GPU is measured in the same run, each
timed outside the headline's timed region, with barrier + max over ranks at
N > 1):
  sweep         configs[2]: 64 Ki x 64 KiB and 4 Ki x 1 MiB (4 GiB per GPU
                each), device-resident, each with its kernel's roofline and
                every block checked bit-exactly against the CPU oracle
  tib           configs[3]: each rank's 2 Mi x 64 KiB = 128 GiB shard of the
                16 Mi x 64 KiB (1 TiB at 8 GPUs) region; sampled parity
                (first, last, every 4096th block of every shard)
  odd           1 M x 4095 B and 1 M x 4097 B blocks per rank (odd sizes the
                server's -v accepts; the rows kernel's window mode), sampled
                parity, the window pattern's read roof, traffic from
                profiles/ when measured; run before tib (a region allocated
                after the 128 GiB leg reads slower)
  streamed      configs[4]: the headline's 1 Mi x 4 KiB blocks from HOST
                memory, end to end (H2D copies, kernels and D2H of the CRCs
                overlapped on 3 streams, priskv_crc32_blocks_host): pinned
                (registered) and pageable, roofline against PCIe Gen5 x16
  roofline      dominant kernel (crc_rows_kernel) vs the HBM roof: algorithmic
                bytes per launch / average launch time (HIP events on the launch
                stream); traffic = PMC-measured HBM bytes per launch for this
                workload when profiles/ holds a matching measurement, else null
  cold          the first full pass over a fresh region after the device has
                idled (clock ramp included), and the same after idle over an
                already-hashed region, beside the steady-state `value`
  ranks, dist   per-rank device identity (PCI address, UUID) and kernel time,
                process-group backend and world size: a line at N > 1 shows
                that N distinct GPUs did the work
  cpu_baseline  rank 0, every N, after all GPU work: the reference's own
                server/crc.c (compiled unmodified into oracle/_ref at -O2, its
                release flag, and -O0, the shipped default) timed on a bounded
                sample of the same blocks, 1 thread and every thread this
                process may use; the CRCs double as a bit-exact spot check
  parity        every headline block of every rank against the CPU oracle

Multi-rank launches must map ranks to distinct GPUs: a rank whose LOCAL_RANK
has no device of its own, or two ranks on one device, exit with status 3
before any measurement.  PRISKV_BENCH_REHEARSAL=1 lifts that for a
rehearsal of the N > 1 path on a one-GPU box (ranks share the device over
gloo), and the line then says so.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s CRC over device-resident value blocks at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
PCIE_PEAK_GBS = 63.0   # host link, PCIe Gen5 x16 (MI355X_MICROARCH.md chip table)
SEED = 0x5EED5EED
RAMP_MIN_S = 1.0
RAMP_MAX_S = 4.0
COLD_IDLE_S = 1.0
EXIT_DEVICES = 3
T_START = time.perf_counter()  # reset at main(); leg_wall_s counts from it

CONFIGS = {
    # name: (block_size, nblocks per GPU, description)
    "default": (4096, 1 << 20, "1Mi x 4KiB value blocks per GPU, device-resident (4 GiB/GPU; BASELINE configs[1])"),
    "sweep64k": (65536, 1 << 16, "64Ki x 64KiB value blocks per GPU, device-resident (4 GiB/GPU; BASELINE configs[2])"),
    "sweep1m": (1 << 20, 1 << 12, "4Ki x 1MiB value blocks per GPU, device-resident (4 GiB/GPU; BASELINE configs[2])"),
    "tib": (65536, 1 << 21, "2Mi x 64KiB value blocks per GPU (128 GiB/GPU; 1 TiB at 8 GPUs; BASELINE configs[3])"),
    # odd block sizes the server's -v also accepts (server/server.c:236-244): the window mode
    "odd4095": (4095, 1000000, "1M x 4095 B value blocks per GPU, device-resident (odd size: the window mode)"),
    "odd4097": (4097, 1000000, "1M x 4097 B value blocks per GPU, device-resident (odd size: the window mode)"),
}
SWEEP = (("64KiB", "sweep64k"), ("1MiB", "sweep1m"))
ODD = (("4095", "odd4095"), ("4097", "odd4097"))


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="default", choices=sorted(CONFIGS))
    p.add_argument("--block-size", type=int, default=None)
    p.add_argument("--nblocks", type=int, default=None)
    p.add_argument("--cpu-sample-bytes", type=int, default=2 << 30,
                   help="bytes of the shard the single-thread CPU baselines hash (about 4 s at -O2)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-tib", action="store_true", help="skip the configs[3] (128 GiB/GPU) leg")
    p.add_argument("--tib-steps", type=int, default=10)
    p.add_argument("--no-sweep", action="store_true", help="skip the configs[2] (64 KiB / 1 MiB) legs")
    p.add_argument("--sweep-steps", type=int, default=20)
    p.add_argument("--no-streamed", action="store_true", help="skip the configs[4] (host-resident) leg")
    p.add_argument("--no-odd", action="store_true", help="skip the odd block size legs (4095 / 4097 B)")
    p.add_argument("--streamed-steps", type=int, default=5)
    p.add_argument("--fresh-regions", action="store_true",
                   help="the 4 GiB legs (64 KiB, 1 MiB, odd sizes) each allocate their own region instead of "
                        "re-filling the headline's (rounds 1-6)")
    p.add_argument("--detail", default=None,
                   help="where the full result goes (default gpurun_out/bench_detail.json); stdout gets the compact line")
    return p.parse_args(argv)


# ---------------------------------------------------------------- rank <-> device
def device_guard(world: int, local: int, ndev: int, rehearsal: bool):
    """None if this rank may run, else the reason it must not.  One process
    per GPU: LOCAL_RANK must name a device of its own.  A rehearsal (several
    ranks on a one-GPU box, gloo) is allowed only when asked for."""
    if ndev < 1:
        return "no GPU visible to this process"
    if local < 0:
        return f"bad LOCAL_RANK {local}"
    if local >= ndev and not rehearsal:
        return (f"LOCAL_RANK {local} of WORLD_SIZE {world} has no GPU of its own ({ndev} visible): "
                f"ranks would share a device; set PRISKV_BENCH_REHEARSAL=1 only for a one-box rehearsal")
    return None


def duplicate_devices(infos):
    """Groups of ranks that report the same physical device (host + PCI
    address, or UUID when the PCI address is unknown)."""
    seen = {}
    for i in infos:
        key = (i["host"], i["pci"] or i["uuid"] or f"dev{i['device']}")
        seen.setdefault(key, []).append(i["rank"])
    return [r for r in seen.values() if len(r) > 1]


def device_info(torch, rank, local, gpu):
    p = torch.cuda.get_device_properties(gpu)
    dom, bus, dv = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    pci = f"{dom:04x}:{bus:02x}:{dv:02x}" if None not in (dom, bus, dv) else None
    uuid = str(getattr(p, "uuid", "") or "") or None
    return {"rank": rank, "local_rank": local, "host": socket.gethostname(), "device": gpu, "pci": pci,
            "uuid": uuid, "name": p.name}


def gather_obj(obj, world):
    import torch.distributed as dist
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


# ---------------------------------------------------------------- helpers
def load_traffic(block_size: int, nblocks: int):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if one matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(f"{block_size}x{nblocks}")
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def cpu_threads():
    """(threads used, CPUs in this process's affinity mask).  The box exports
    OMP_NUM_THREADS = its CPU share; the affinity mask may list the whole host."""
    avail = len(os.sched_getaffinity(0))
    try:
        cap = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        cap = 0
    return (min(avail, cap) if cap > 0 else avail), avail


def ramp(fn, stream, torch, window=16, min_s=RAMP_MIN_S, max_s=RAMP_MAX_S):
    """Untimed launches until the device is in its steady state.  A fresh
    process runs 5-8 % slow for about its first second of GPU work, and the
    first ~10 launches after idle up to 40 %: launch
    back-to-back windows of `window` steps and stop once two consecutive
    windows agree within 0.5 % (after at least min_s, at most max_s).
    Returns (launches, seconds)."""
    n = 0
    prev = None
    t0 = time.perf_counter()
    while True:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(window):
            fn()
            n += 1
        e1.record(stream)
        e1.synchronize()
        cur = e0.elapsed_time(e1)
        el = time.perf_counter() - t0
        if el >= max_s or (el >= min_s and prev is not None and abs(cur - prev) <= 0.005 * prev):
            return n, el
        prev = cur


def progress(rank, msg):
    """A progress line on stderr (rank 0): a multi-rank run with slow legs
    keeps showing signs of life; stdout carries only the JSON line."""
    if rank == 0:
        print(f"bench.py: {msg} ({time.perf_counter() - T_START:.1f} s since start)", file=sys.stderr, flush=True)


def per_launch_ms(fn, stream, torch, k):
    """k launches, one event pair around each (a second window after the
    timed one): per-launch kernel times in ms."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for e0, e1 in evs:
        e0.record(stream)
        fn()
        e1.record(stream)
    evs[-1][1].synchronize()
    return [e0.elapsed_time(e1) for e0, e1 in evs]


def launch_stats(ms):
    a = np.asarray(ms, dtype=np.float64)
    return {"launches": int(a.size), "median_ms": round(float(np.median(a)), 4), "min_ms": round(float(a.min()), 4),
            "max_ms": round(float(a.max()), 4)}


def read_roof(B, region, bs, nb, stream, alg, k, rotate=0):
    """The measured peak beside the CRC's roofline: priskv_crc_read_roof_dev
    (the CRC kernel's loads, per-wave ranges and XCD split, no hashing) over
    the same region in every variant -- the CRC plan's own pipeline depth and
    occupancy, and 2 / 3 / 4 chunks in flight at one or two workgroups per CU
    -- each ramped the same way, in an order rotated by `rotate` (so no
    variant always runs first or last), k launches each with one event pair
    per launch.  measured_peak is the best variant's mean rate (a roof of the
    pattern, not one sibling kernel's rate); measured_peak_v0, variant 0's
    alone (the CRC plan's own shape: the round-3 roof, comparable across
    rounds).  GB/s of the same algorithmic bytes."""
    from priskv_amd.crc import ROOF_SINK_WORDS, ROOF_VARIANTS
    torch = B.torch
    sink = torch.zeros(ROOF_SINK_WORDS, dtype=torch.int32, device=B.dev)
    per = {}
    order = [(v + rotate) % ROOF_VARIANTS for v in range(ROOF_VARIANTS)]
    for v in order:
        def step():
            B.ctx.read_roof_dev(region, bs, sink, stream=stream, nblocks=nb, variant=v)

        step()
        torch.cuda.synchronize()
        # the device is in its steady state after the CRC leg: the same short ramp for every variant
        ramp(step, stream, torch, window=8, min_s=0.15, max_s=2.0)
        ms = per_launch_ms(step, stream, torch, k)
        per[v] = (float(np.mean(ms)), launch_stats(ms))
    del sink
    best = min(per, key=lambda v: per[v][0])
    mean, st = per[best]
    return {"measured_peak": round(alg / (mean * 1e-3) / 1e9, 1),
            "measured_peak_best": round(alg / (st["min_ms"] * 1e-3) / 1e9, 1),
            "measured_peak_variant": best,
            "measured_peak_v0": round(alg / (per[0][0] * 1e-3) / 1e9, 1),
            "measured_peak_variants_GBps": {str(v): round(alg / (per[v][0] * 1e-3) / 1e9, 1) for v in sorted(per)},
            "measured_peak_order": order,
            "measured_peak_source": "priskv_crc_read_roof_dev on the same region in this process: the CRC kernel's "
                                    "loads, per-wave ranges and XCD split without hashing, best of "
                                    f"{ROOF_VARIANTS} variants (variant 0 = the CRC plan's own pipeline depth and "
                                    "occupancy; 1-6 = 2/2/3/3/4/4 chunks in flight at 1/2 workgroups per CU; 7-8 = "
                                    "the plan's shape with progress priority 1/3), each ramped alike, order rotated "
                                    f"per leg; mean of {k} launches each (one event pair per launch)",
            "roof_launch_ms": st}


class Bench:
    """Per-rank state shared by the legs."""

    def __init__(self, args, torch, dist, world, rank, dev, ctx):
        self.args, self.torch, self.dist = args, torch, dist
        self.world, self.rank, self.dev, self.ctx = world, rank, dev, ctx

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v):
        from priskv_amd.shard import max_over_ranks
        return max_over_ranks(v, device=self.dev)

    def all_ok(self, ok: bool) -> bool:
        return self.max(0.0 if ok else 1.0) == 0.0

    def timed(self, step, stream, k):
        """k back-to-back steps between barrier + synchronize on both sides:
        (max-over-ranks wall seconds, this rank's kernel ms per step).  Every
        rank starts its clock as the opening barrier releases it and stops
        it once its own device has drained; the max over ranks is the job's
        time, and the closing barrier's own latency (a collective, not the
        path) stays outside it."""
        torch = self.torch
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(k):
            step()
        ev1.record(stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        self.barrier()
        return self.max(el), ev0.elapsed_time(ev1) / k

    def alloc(self, nbytes):
        """A device region on every rank, or None on every rank when any rank
        cannot allocate (agreed before any other collective of the leg)."""
        torch = self.torch
        try:
            region, err = torch.empty(nbytes, dtype=torch.uint8, device=self.dev), None
        except torch.OutOfMemoryError as e:
            region, err = None, str(e)
        if not self.all_ok(region is not None):
            del region
            torch.cuda.empty_cache()
            return None, err or "another rank could not allocate"
        return region, None


def resident_leg(B: Bench, name, steps, parity="full", rotate=0, shared=None):
    """A device-resident config (CONFIGS[name]) at this N: each rank's shard
    of world x nb blocks, filled on the device, ramped, then `steps` timed
    passes.  parity "full": every block of every shard against the oracle;
    "sampled": first, last and every 4096th block.  shared: the headline's
    region, which the leg's blocks go into (re-filled with the leg's own
    pattern) when they fit -- one value region, as PrisKV's values live in
    one registered memfile region -- so that the legs do not each draw a fresh
    4 GiB allocation, whose read rate differs by a few percent from one
    allocation to the next; the leg's read roof is measured on
    the same region either way."""
    import _oracle as O
    from priskv_amd import as_u32
    from priskv_amd.shard import shard_blocks, shard_word_offset
    torch, ctx = B.torch, B.ctx
    bs, nb0, desc = CONFIGS[name]
    first, nb = shard_blocks(B.world * nb0, B.rank, B.world)
    # (every rank's shard has the same size, so every rank takes the same branch)
    if shared is not None and shared.numel() >= bs * nb:
        region, where = shared[: bs * nb], "the headline's region (shared)"
    else:
        region, err = B.alloc(bs * nb)
        if region is None:
            return {"workload": desc, "skipped": f"cannot allocate {bs * nb / 2**30:.0f} GiB: {err}"}
        where = "its own allocation"
    ctx.fill_splitmix(region, SEED, word_offset=shard_word_offset(first, bs))
    out = torch.empty(nb, dtype=torch.int32, device=B.dev)
    stream = torch.cuda.Stream(device=B.dev)

    def step():
        ctx.blocks_dev(region, bs, out=out, stream=stream)

    step()
    torch.cuda.synchronize()
    ramp(step, stream, torch, window=max(3, min(16, (64 << 30) // (bs * nb))), min_s=0.5)
    k = max(1, steps)
    el, kms = B.timed(step, stream, k)
    alg = nb * (bs + 4)
    lstats = launch_stats(per_launch_ms(step, stream, torch, k))
    try:  # (odd sizes: the window mode's roof, where the library mirrors its pattern)
        roof = read_roof(B, region, bs, nb, stream, alg, k, rotate)
    except OSError:
        roof = None
    if parity == "full":
        host = region.cpu().numpy()
        got = as_u32(out)
        want = O.crc32_blocks(host, bs, nthreads=8)
        nchk, what = nb, "every block"
        del host
    else:
        idx = np.unique(np.concatenate([np.arange(0, nb, 4096), [nb - 1]])).astype(np.int64)
        ti = torch.from_numpy(idx).to(B.dev)
        blocks = region.view(nb, bs).index_select(0, ti).cpu().numpy()
        got = as_u32(out.index_select(0, ti))
        want = O.crc32_blocks(blocks.reshape(-1), bs, nthreads=8)
        nchk, what = int(idx.size), "first, last, every 4096th block"
    ok = B.all_ok(bool(np.array_equal(got, want)))
    plan = ctx.blocks_plan(region.data_ptr(), nb, bs)
    del region, out
    torch.cuda.empty_cache()
    achieved = alg / (kms * 1e-3) / 1e9
    rl = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
          "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(bs, nb), "kernel_ms": round(kms, 4),
          "alg_bytes_per_launch": alg, "kernel_launch_ms": lstats}
    if roof:
        rl.update(roof)
        rl["frac_of_measured"] = round(achieved / roof["measured_peak"], 4)
        rl["frac_of_v0"] = round(achieved / roof["measured_peak_v0"], 4)
    return {"workload": desc, "value": round(bs * nb * B.world * k / el / 2**30, 2), "unit": "GiB/s",
            "n_gpus": B.world, "steps": k, "ms_per_step": round(el / k * 1e3, 4), "bytes_per_gpu": bs * nb,
            "region": where, "kernel": plan, "roofline": rl,
            "parity": {"checked_blocks_per_rank": nchk, "sample": what, "bit_exact": ok,
                       "oracle": "oracle/crc_oracle.c"}}


def streamed_leg(B: Bench, host, bs, want):
    """configs[4]: this rank's headline blocks from host memory, end to end
    through priskv_crc32_blocks_host (64 MiB chunks over 3 streams: H2D copy,
    kernel and D2H of the CRCs overlapped).  Pinned = the region registered
    with priskv_crc_host_register, as the server's RDMA-registered value
    buffer / memfile would be; pageable = bounced through pinned staging.
    `want` = the oracle's CRCs of `host`."""
    from priskv_amd import host_register, host_unregister
    nb = host.size // bs
    res = {}
    for mode in ("pinned", "pageable"):
        if mode == "pinned":
            host_register(host)
        try:
            out = B.ctx.blocks_host(host, bs)  # warm (allocates the staging buffers)
            k = max(1, B.args.streamed_steps if mode == "pinned" else max(1, B.args.streamed_steps // 2))
            B.barrier()
            t0 = time.perf_counter()
            for _ in range(k):
                out = B.ctx.blocks_host(host, bs, out=out)
            dt = B.max(time.perf_counter() - t0) / k
            B.barrier()
        finally:
            if mode == "pinned":
                host_unregister(host)
        ok = B.all_ok(bool(np.array_equal(out, want)))
        link = (nb * bs + nb * 4) / dt / 1e9  # bytes over this GPU's host link per second
        res[mode] = {"value": round(bs * nb * B.world / dt / 2**30, 2), "unit": "GiB/s", "steps": k,
                     "ms_per_step": round(dt * 1e3, 3),
                     "roofline": {"bound": "pcie", "achieved": round(link, 2), "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(link / PCIE_PEAK_GBS, 4),
                                  "peak_source": "PCIe Gen5 x16 host link spec, MI355X_MICROARCH.md"},
                     "bit_exact": ok}
    return {"workload": f"{nb} x {bs} B value blocks per GPU in host memory (BASELINE configs[4]): "
                        f"H2D + kernel + D2H of the CRCs, 64 MiB chunks on 3 streams",
            "n_gpus": B.world, **res,
            "parity": {"checked_blocks_per_rank": nb, "sample": "every block, against the oracle",
                       "bit_exact": res["pinned"]["bit_exact"] and res["pageable"]["bit_exact"]}}


def cold_leg(B: Bench, bs, nb, walked):
    """The first full pass after the device has idled COLD_IDLE_S: over a
    fresh region (filled on the device, never hashed -- what a one-off
    recovery scrub sees) and over `walked`, a region hashed many times
    already.  Rank-local, measured after all other GPU work."""
    torch, ctx = B.torch, B.ctx
    stream = torch.cuda.Stream(device=B.dev)
    out = torch.empty(nb, dtype=torch.int32, device=B.dev)
    region = torch.empty(bs * nb, dtype=torch.uint8, device=B.dev)
    ctx.fill_splitmix(region, SEED ^ 0xC01D)
    ctx.blocks_dev(region, bs, out=out, stream=stream, nblocks=min(nb, 64))
    res = {}
    for label, reg in (("fresh", region), ("walked", walked)):
        torch.cuda.synchronize()
        time.sleep(COLD_IDLE_S)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ctx.blocks_dev(reg, bs, out=out, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        res[label] = e0.elapsed_time(e1)
    del region, out
    torch.cuda.empty_cache()
    alg = nb * (bs + 4)
    f = res["fresh"]
    return {"ms": round(f, 4), "value": round(bs * nb / (f * 1e-3) / 2**30, 2), "unit": "GiB/s",
            "frac": round(alg / (f * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "walked_ms": round(res["walked"], 4),
            "walked_value": round(bs * nb / (res["walked"] * 1e-3) / 2**30, 2),
            "note": f"rank-local first pass after {COLD_IDLE_S:.1f} s idle over a fresh region (filled, never "
                    f"hashed) and, walked_*, over the headline region (hashed many times); kernel already loaded; "
                    f"measured after all other GPU work"}


def cpu_baseline(O, host, bs, gpu_crc):
    """The reference's server/crc.c at -O2 and -O0, 1 thread and every thread
    this process may use, on the same sample (rank 0, after all GPU work)."""
    nthr, avail = cpu_threads()
    n1 = host.size // bs
    variants, ok = [], True
    top = None
    for opt in ("O2", "O0"):
        for thr in (1, nthr):
            secs, crc, kind, label = O.time_cpu_baseline(host, bs, threads=thr, opt=opt)
            ok = ok and bool(np.array_equal(crc, gpu_crc))
            v = {"opt": f"-{opt}", "threads": thr, "value": round(n1 * bs / secs / 2**30, 4), "seconds": round(secs, 3),
                 "kind": kind}
            variants.append(v)
            if opt == "O2" and thr == 1:
                top = (v, kind, label)
    v, kind, label = top
    info = O.ref_build_info()
    return ({"value": v["value"], "unit": "GiB/s", "cores": 1, "kind": kind,
             "sample": f"first {n1} x {bs} B blocks ({n1 * bs / 2**30:.2f} GiB) of rank 0's shard; {label}; "
                       f"variants = -O2 (PRISKV_RELEASE, server/Makefile:23-24) and -O0 (shipped default, "
                       f"server/Makefile:25-26) at 1 and {nthr} threads (static block split)",
             "variants": variants, "threads_used": nthr, "cpus_in_affinity": avail, "cpu": cpu_model(),
             "compiler": info.get("compiler")}, ok)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _r(x, nd=4):
    return None if x is None else round(float(x), nd)


def compact_leg(leg: dict) -> dict:
    """One leg of the stdout line: value, ms_per_step, frac, frac_of_measured,
    traffic (measured HBM bytes / algorithmic bytes), bit_exact (or the
    leg's error / skip reason)."""
    if not isinstance(leg, dict):
        return {"error": str(leg)}
    if "error" in leg or "skipped" in leg:
        return {k: leg[k] for k in ("error", "skipped") if k in leg}
    rl = leg.get("roofline") or {}
    tr = rl.get("traffic")
    alg = rl.get("alg_bytes_per_launch")
    out = {"value": leg.get("value"), "ms_per_step": leg.get("ms_per_step"), "frac": rl.get("frac"),
           "frac_of_measured": rl.get("frac_of_measured"),
           "traffic": _r(tr / alg) if tr and alg else None,
           "bit_exact": (leg.get("parity") or {}).get("bit_exact")}
    return {k: v for k, v in out.items() if v is not None or k in ("traffic", "frac_of_measured")}


def compact_line(full: dict, detail_path: str) -> dict:
    """The ONE stdout line: the contract's keys, the headline roofline and
    cpu_baseline in short form, and every other leg as compact_leg -- short
    enough (~2.5 KB) that a driver keeping the last 3000 characters of stdout
    sees every leg.  Everything else (per-variant roofs, per-launch stats,
    sources, notes, per-rank identity) is in the detail file."""
    rl = full.get("roofline", {})
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in full}
    cfg = full.get("config", {})
    line["config"] = {k: cfg[k] for k in ("workload", "block_size", "nblocks_per_gpu", "parallelism", "kernel",
                                          "timed_launches") if k in cfg}
    line["roofline"] = {k: rl[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms",
                                           "alg_bytes_per_launch", "measured_peak", "measured_peak_v0",
                                           "frac_of_measured", "frac_of_v0") if k in rl}
    if "cpu_baseline" in full:
        cb = full["cpu_baseline"]
        line["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind") if k in cb}
        line["cpu_baseline"]["sample"] = (cb.get("sample", "").split(";")[0] + "; server/crc.c -O2 (oracle/_ref), "
                                          f"1 thread on {cb.get('cpu', '?')}")
        mt = [v for v in cb.get("variants", []) if v.get("opt") == "-O2" and v.get("threads", 1) > 1]
        if mt:
            line["cpu_baseline"]["multithread"] = {"threads": mt[0]["threads"], "value": mt[0]["value"]}
    par = full.get("parity", {})
    line["parity"] = {k: par[k] for k in ("bit_exact", "bit_exact_vs_reference_build", "checked_blocks_per_rank")
                      if k in par}
    d = full.get("dist", {})
    line["dist"] = {k: d[k] for k in ("backend", "world_size", "distinct_devices", "rehearsal") if k in d}
    legs = {}
    for k, v in (full.get("sweep") or {}).items():
        legs[k] = compact_leg(v)
    if "tib" in full:
        legs["tib"] = compact_leg(full["tib"])
    for k, v in (full.get("odd") or {}).items():
        legs[f"odd{k}"] = compact_leg(v)
    st = full.get("streamed")
    if isinstance(st, dict):
        for mode in ("pinned", "pageable"):
            if mode in st:
                m = st[mode]
                legs[f"streamed_{mode}"] = {"value": m.get("value"), "ms_per_step": m.get("ms_per_step"),
                                            "frac": (m.get("roofline") or {}).get("frac"),
                                            "bit_exact": m.get("bit_exact")}
        if "error" in st:
            legs["streamed"] = {"error": st["error"]}
    cold = full.get("cold")
    if isinstance(cold, dict):
        legs["cold"] = ({"value": cold.get("value"), "ms": cold.get("ms"), "frac": cold.get("frac"),
                         "walked_value": cold.get("walked_value")} if "error" not in cold else {"error": cold["error"]})
    line["legs"] = legs
    if "cold_ms" in full:
        line["cold_ms"] = full["cold_ms"]
    line["detail"] = detail_path
    return line


def main():
    global T_START
    T_START = time.perf_counter()
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = os.environ.get("PRISKV_BENCH_REHEARSAL", "") == "1"
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # device_count() does not initialise the GPU on this image: the guard
    # runs before any HIP call
    ndev = torch.cuda.device_count()
    why = device_guard(world, local, ndev, rehearsal)
    if why:
        print(f"bench.py: rank {rank}: {why}", file=sys.stderr, flush=True)
        sys.exit(EXIT_DEVICES)
    gpu = local % ndev if rehearsal else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    backend = os.environ.get("PRISKV_BENCH_BACKEND", "gloo" if rehearsal else "nccl")  # nccl == RCCL on ROCm
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    infos = gather_obj(device_info(torch, rank, local, gpu), world)
    dups = duplicate_devices(infos)
    if dups and not rehearsal:
        if rank == 0:
            print(f"bench.py: ranks share a physical device: {dups}", file=sys.stderr, flush=True)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(EXIT_DEVICES)

    from priskv_amd import CrcContext, as_u32
    from priskv_amd.shard import shard_blocks, shard_word_offset
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O

    bs, nb, desc = CONFIGS[args.config]
    if args.block_size:
        bs = args.block_size
    if args.nblocks:
        nb = args.nblocks
    walls = {"start_to_context": time.perf_counter() - T_START}
    t_leg = time.perf_counter()
    ctx = CrcContext(gpu)
    B = Bench(args, torch, dist, world, rank, dev, ctx)
    # weak scaling: the global region has world * nb blocks; this rank's shard
    # is its contiguous range of them (no data-path collective)
    first, nb = shard_blocks(world * nb, rank, world)
    region = torch.empty(bs * nb, dtype=torch.uint8, device=dev)
    ctx.fill_splitmix(region, SEED, word_offset=shard_word_offset(first, bs))
    out = torch.empty(nb, dtype=torch.int32, device=dev)
    # a created stream: torch's null stream costs ~1 % per launch (DESIGN.md
    # §6); the device-wide synchronize() around the timed region covers every
    # stream
    stream = torch.cuda.Stream(device=dev)

    def step():
        ctx.blocks_dev(region, bs, out=out, stream=stream)

    walls["setup"] = time.perf_counter() - t_leg
    t_leg = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    nramp, ramp_s = ramp(step, stream, torch)

    elapsed_max, kernel_ms = B.timed(step, stream, args.steps)
    walls["headline"] = time.perf_counter() - t_leg

    # a second window, one event pair per launch (median / min), then the
    # read roof of the same access pattern over the same region
    t_leg = time.perf_counter()
    alg_bytes = nb * (bs + 4)  # block read + 4-byte CRC written
    lstats = launch_stats(per_launch_ms(step, stream, torch, args.steps))
    roof = read_roof(B, region, bs, nb, stream, alg_bytes, args.steps) if bs % 4096 == 0 else None
    walls["launch_stats_and_roof"] = time.perf_counter() - t_leg

    total_bytes = bs * nb * world
    value = total_bytes * args.steps / elapsed_max / 2**30
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = load_traffic(bs, nb)
    path = ctx.blocks_plan(region.data_ptr(), nb, bs)  # the library reports its own plan

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 pattern filled on device)",
        "config": {"workload": desc, "block_size": bs, "nblocks_per_gpu": nb,
                   "bytes_per_gpu": bs * nb, "parallelism": f"shard{world} (contiguous block ranges, no collective)",
                   "kernel": path, "untimed_ramp_launches": nramp, "untimed_ramp_s": round(ramp_s, 2),
                   "timed_launches": f"dispatches {args.warmup + nramp + 1}..{args.warmup + nramp + args.steps} of "
                                     f"this kernel in the process (1-based; tools/ktrace_window.py)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel_ms": round(kernel_ms, 4),
                     "alg_bytes_per_launch": alg_bytes, "kernel_launch_ms": lstats},
    }
    if roof:
        result["roofline"].update(roof)
        result["roofline"]["frac_of_measured"] = round(achieved / roof["measured_peak"], 4)
        result["roofline"]["frac_of_v0"] = round(achieved / roof["measured_peak_v0"], 4)

    # the whole shard to host (untimed): every block is checked against the
    # oracle, rank 0's first cpu-sample-bytes time the CPU baseline, and the
    # streamed leg reads these same bytes from host memory
    t_leg = time.perf_counter()
    host = region.cpu().numpy()
    gpu_crc = as_u32(out)
    want = O.crc32_blocks(host, bs, nthreads=8)
    head_ok = B.all_ok(bool(np.array_equal(gpu_crc, want)))
    walls["parity"] = time.perf_counter() - t_leg
    progress(rank, f"headline {value:.1f} GiB/s, parity {'ok' if head_ok else 'FAILED'}")
    walked = region if args.config == "default" else None
    shared = None if args.fresh_regions else walked  # the 4 GiB legs' blocks go into this region
    if walked is None:
        del region
    del out
    torch.cuda.empty_cache()

    def leg(label, fn, *a, **kw):
        """A leg beside the headline, its wall time recorded under `label`.
        On one rank a failure is reported in the line instead of losing the
        headline; with several ranks it propagates (its collectives could no
        longer pair up)."""
        t0 = time.perf_counter()
        try:
            if world > 1:
                return fn(*a, **kw)
            try:
                return fn(*a, **kw)
            except Exception as e:  # noqa: BLE001 -- reported in the line
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
                return {"error": f"{type(e).__name__}: {e}"}
        finally:
            walls[label] = time.perf_counter() - t0
            progress(rank, f"{label} done in {walls[label]:.1f} s")

    if not args.no_sweep and args.config == "default":
        result["sweep"] = {k: leg(f"sweep_{k}", resident_leg, B, name, args.sweep_steps, rotate=1 + i, shared=shared)
                           for i, (k, name) in enumerate(SWEEP)}
    # the odd sizes before the 128 GiB leg: a region allocated after that
    # leg's free read 5-6 % slower, its read roof too (0.78 against 0.83 on one
    # box, profiles/r06/odd/): the state the benchmark's own largest leg
    # leaves, not the kernel
    if not args.no_odd and args.config == "default":
        result["odd"] = {k: leg(f"odd_{k}", resident_leg, B, name, args.sweep_steps, parity="sampled", rotate=4 + i,
                                shared=shared)
                         for i, (k, name) in enumerate(ODD)}
    if not args.no_tib and args.config == "default":
        result["tib"] = leg("tib", resident_leg, B, "tib", args.tib_steps, parity="sampled", rotate=3)
    if not args.no_streamed:
        result["streamed"] = leg("streamed", streamed_leg, B, host, bs, want)
    # cold passes LAST on the GPU: what a one-off recovery scrub sees (clock
    # ramp included); measured last so that the idle cannot leave its slower
    # first launches inside the other legs
    if walked is not None:
        result["cold"] = leg("cold", cold_leg, B, bs, nb, walked)
        if "ms" in result["cold"]:
            result["cold_ms"] = result["cold"]["ms"]
        del walked, shared
    torch.cuda.empty_cache()

    kms = gather_obj(round(kernel_ms, 4), world)
    result["ranks"] = [dict(i, kernel_ms=k) for i, k in zip(infos, kms)]
    result["dist"] = {"backend": dist.get_backend() if world > 1 else None, "world_size": world,
                      "distinct_devices": len({(i["host"], i["pci"] or i["uuid"]) for i in infos}),
                      "rehearsal": rehearsal}
    result["parity"] = {"checked_blocks_per_rank": nb, "sample": "every block", "bit_exact": head_ok,
                        "oracle": "oracle/crc_oracle.c"}
    if rank == 0 and not args.no_cpu_baseline:
        t_leg = time.perf_counter()
        nsamp = max(1, min(nb, args.cpu_sample_bytes // bs))
        result["cpu_baseline"], cpu_ok = cpu_baseline(O, host[: nsamp * bs], bs, gpu_crc[:nsamp])
        result["parity"]["bit_exact_vs_reference_build"] = cpu_ok
        walls["cpu_baseline"] = time.perf_counter() - t_leg
    t_leg = time.perf_counter()
    B.barrier()
    walls["final_barrier"] = time.perf_counter() - t_leg
    walls["total"] = time.perf_counter() - T_START
    if rank == 0:
        result["leg_wall_s"] = {k: round(v, 2) for k, v in walls.items()}
        result["leg_wall_s"]["note"] = ("rank 0's wall seconds per leg (process start to the line); the legs "
                                        "open and close with barriers, so rank 0's time is the job's")
        detail = args.detail or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(result, f, indent=1)
        except OSError as e:
            detail = f"not written: {e}"
        print(json.dumps(compact_line(result, os.path.relpath(detail, ROOT) if os.path.isabs(detail) else detail)),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
