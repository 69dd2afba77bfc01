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

Extra keys of the ONE JSON line rank 0 prints:
  tib           BASELINE.json configs[3] measured in the same run at every N:
                each rank's shard of the 16 Mi x 64 KiB (1 TiB at 8 GPUs)
                region, 2 Mi x 64 KiB = 128 GiB per GPU, filled on the device;
                aggregate GiB/s over the N ranks (barrier + max over ranks),
                with sampled blocks (first, last, every 4096th of every
                shard) checked bit-exactly against the CPU oracle
  roofline      dominant kernel (crc_rows_kernel) vs the HBM roof: algorithmic
                bytes per launch / average launch time (HIP events on the launch
                stream); traffic = PMC-measured HBM bytes per launch for this
                workload when profiles/ holds a matching measurement, else null
  cold_ms       the first full pass after the device has idled (clock ramp
                included), beside the steady-state `value`
  pipelined     the same K passes round-robin on 2 streams (reported beside,
                never instead of, `value`)
  cpu_baseline  rank 0, every N, after all GPU work: the reference's own
                server/crc.c (compiled unmodified into oracle/_ref at -O2, its
                release flag, and -O0, the shipped default) timed on a bounded
                sample of the same blocks, 1 thread and every thread this
                process may use; the CRCs double as a bit-exact spot check
  parity        result of comparing the GPU CRCs with those CPU samples
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s CRC over device-resident value blocks at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEED = 0x5EED5EED
RAMP_MIN_S = 1.0
RAMP_MAX_S = 4.0
COLD_IDLE_S = 1.0

CONFIGS = {
    # name: (block_size, nblocks per GPU, description)
    "default": (4096, 1 << 20, "1Mi x 4KiB value blocks per GPU, device-resident (4 GiB/GPU; BASELINE configs[1])"),
    "sweep64k": (65536, 1 << 16, "64Ki x 64KiB value blocks per GPU, device-resident (4 GiB/GPU)"),
    "sweep1m": (1 << 20, 1 << 12, "4Ki x 1MiB value blocks per GPU, device-resident (4 GiB/GPU)"),
    "tib": (65536, 1 << 21, "2Mi x 64KiB value blocks per GPU (128 GiB/GPU; 1 TiB at 8 GPUs; BASELINE configs[3])"),
}
TIB_BS, TIB_NB = CONFIGS["tib"][0], CONFIGS["tib"][1]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="default", choices=sorted(CONFIGS) + ["streamed"])
    p.add_argument("--block-size", type=int, default=None)
    p.add_argument("--nblocks", type=int, default=None)
    p.add_argument("--cpu-sample-bytes", type=int, default=2 << 30,
                   help="bytes of the shard the single-thread CPU baselines hash (about 4 s at -O2)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-tib", action="store_true", help="skip the configs[3] (128 GiB/GPU) leg")
    p.add_argument("--tib-steps", type=int, default=10)
    p.add_argument("--pipeline-streams", type=int, default=2,
                   help="streams for the reported-beside pipelined pass (0 = skip it)")
    return p.parse_args()


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
    first ~10 launches after idle up to 40 % (profiles/r01/clock_ramp.txt,
    profiles/r02/bench_bisect_*.json): launch back-to-back windows of
    `window` steps and stop once two consecutive windows agree within 0.5 %
    (after at least min_s, at most max_s).  Returns (launches, seconds)."""
    n = 0
    prev = None
    t0 = time.perf_counter()
    while True:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(window):
            fn(n)
            n += 1
        e1.record(stream)
        e1.synchronize()
        cur = e0.elapsed_time(e1)
        el = time.perf_counter() - t0
        if el >= max_s or (el >= min_s and prev is not None and abs(cur - prev) <= 0.005 * prev):
            return n, el
        prev = cur


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # one process per GPU; modulo only matters for a multi-rank rehearsal on a
    # one-GPU box (PRISKV_BENCH_BACKEND=gloo), never on the 8-GPU node
    gpu = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    backend = os.environ.get("PRISKV_BENCH_BACKEND", "nccl")  # nccl == RCCL on ROCm
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from priskv_amd import CrcContext, as_u32

    if args.config == "streamed":
        return streamed(args, torch, rank, world)

    bs, nb, desc = CONFIGS[args.config]
    if args.block_size:
        bs = args.block_size
    if args.nblocks:
        nb = args.nblocks
    from priskv_amd.shard import max_over_ranks, shard_blocks, shard_word_offset
    ctx = CrcContext(gpu)
    # weak scaling: the global region has world * nb blocks; this rank's shard
    # is its contiguous range of them (no data-path collective)
    first, nb = shard_blocks(world * nb, rank, world)
    region = torch.empty(bs * nb, dtype=torch.uint8, device=dev)
    ctx.fill_splitmix(region, SEED, word_offset=shard_word_offset(first, bs))
    out = torch.empty(nb, dtype=torch.int32, device=dev)
    # a created stream: torch's null stream costs ~1 % per launch
    # (profiles/r02/bench_bisect_*.json); the device-wide synchronize()
    # around the timed region covers every stream
    stream = torch.cuda.Stream(device=dev)
    sync = torch.cuda.synchronize

    def barrier():
        if world > 1:
            dist.barrier()

    def step(_i=0):
        ctx.blocks_dev(region, bs, out=out, stream=stream)

    for _ in range(args.warmup):
        step()
    sync()
    nramp, ramp_s = ramp(step, stream, torch)

    trace = os.environ.get("PRISKV_BENCH_TRACE")
    if trace:  # per-step kernel times of a separate, untimed pass (diagnostics only)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        evs[0].record(stream)
        for i in range(args.steps):
            step()
            evs[i + 1].record(stream)
        sync()
        print("per-step ms:", " ".join(f"{evs[i].elapsed_time(evs[i + 1]):.3f}" for i in range(args.steps)),
              file=sys.stderr)

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier()
    sync()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    sync()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # launches back-to-back on `stream`

    elapsed_max = max_over_ranks(elapsed, device=dev)

    total_bytes = bs * nb * world
    value = total_bytes * args.steps / elapsed_max / 2**30
    alg_bytes = nb * (bs + 4)  # block read + 4-byte CRC written
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
                   "also_measured": None if args.no_tib else CONFIGS["tib"][2] + " -> `tib`"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel_ms": round(kernel_ms, 4),
                     "alg_bytes_per_launch": alg_bytes},
    }

    if args.pipeline_streams > 1:
        # Reported beside `value`, never instead of it: the same K batch
        # passes, issued round-robin over independent streams as a server
        # with several scrub/verify batches in flight would.  Kernels on one
        # stream are serialized, so every batch pays its own tail;
        # on separate streams the next batch's workgroups take the CUs that
        # the previous one frees.  It gets the same untimed ramp as `value`.
        ns = args.pipeline_streams
        pstreams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(ns - 1)]
        pouts = [out] + [torch.empty(nb, dtype=torch.int32, device=dev) for _ in range(ns - 1)]

        def pstep(i):
            ctx.blocks_dev(region, bs, out=pouts[i % ns], stream=pstreams[i % ns])

        ramp(pstep, stream, torch, window=2 * ns * 8, min_s=0.3)
        sync()
        barrier()
        sync()
        tp0 = time.perf_counter()
        for i in range(args.steps):
            pstep(i)
        sync()
        barrier()
        p_elapsed = max_over_ranks(time.perf_counter() - tp0, device=dev)
        same = all(torch.equal(pouts[0], o) for o in pouts[1:])
        result["pipelined"] = {"streams": ns, "value": round(total_bytes * args.steps / p_elapsed / 2**30, 2),
                               "unit": "GiB/s", "ms_per_step": round(p_elapsed / args.steps * 1e3, 4),
                               "frac_of_peak": round(alg_bytes * args.steps / p_elapsed / 1e9 / HBM_PEAK_GBS, 4),
                               "outputs_identical": bool(same)}

    # every rank checks a sample of its own shard against the oracle
    # (untimed); the CPU baseline times the reference on rank 0's sample
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    want_cpu = rank == 0 and not args.no_cpu_baseline
    nsamp = max(1, min(nb, (args.cpu_sample_bytes if want_cpu else 64 << 20) // bs))
    host = region[: nsamp * bs].cpu().numpy()
    gpu_crc = as_u32(out[:nsamp])
    del region
    torch.cuda.empty_cache()

    if not args.no_tib:
        result["tib"] = tib_leg(args, torch, ctx, dev, rank, world, barrier, O)

    # cold pass, LAST on the GPU: the device idles COLD_IDLE_S and ONE full
    # pass over a fresh region of the same shape is timed -- what a one-off
    # recovery scrub sees (clock ramp included).  Measured last so that the
    # idle cannot leave its slower first launches inside the other legs.
    cold_ms = cold_pass(torch, ctx, dev, bs, nb, stream)
    result["cold_ms"] = round(cold_ms, 4)
    result["cold"] = {"ms": round(cold_ms, 4), "value": round(bs * nb / (cold_ms * 1e-3) / 2**30, 2), "unit": "GiB/s",
                      "note": f"rank-local first pass after {COLD_IDLE_S:.1f} s idle (kernel already loaded), "
                              f"measured after all other GPU work"}

    ok = bool(np.array_equal(O.crc32_blocks(host, bs, nthreads=8), gpu_crc))
    all_ok = max_over_ranks(0.0 if ok else 1.0, device=dev) == 0.0
    result["parity"] = {"checked_blocks_per_rank": nsamp, "bit_exact": bool(all_ok), "oracle": "oracle/crc_oracle.c"}
    if want_cpu:
        result["cpu_baseline"], cpu_ok = cpu_baseline(O, host, bs, gpu_crc)
        result["parity"]["bit_exact_vs_reference_build"] = cpu_ok
    barrier()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cold_pass(torch, ctx, dev, bs, nb, stream):
    """One full pass after the device has idled COLD_IDLE_S (fresh region of
    the same shape, so nothing is cache-warm)."""
    region = torch.empty(bs * nb, dtype=torch.uint8, device=dev)
    ctx.fill_splitmix(region, SEED ^ 0xC01D)
    out = torch.empty(nb, dtype=torch.int32, device=dev)
    ctx.blocks_dev(region, bs, out=out, stream=stream, nblocks=min(nb, 64))
    torch.cuda.synchronize()
    time.sleep(COLD_IDLE_S)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    ctx.blocks_dev(region, bs, out=out, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    del region, out
    torch.cuda.empty_cache()
    return e0.elapsed_time(e1)


def tib_leg(args, torch, ctx, dev, rank, world, barrier, O):
    """BASELINE configs[3]: this rank's 2 Mi x 64 KiB (128 GiB) shard of the
    16 Mi x 64 KiB region (world ranks x 2 Mi blocks), filled on the device."""
    from priskv_amd import as_u32
    from priskv_amd.shard import max_over_ranks, shard_blocks, shard_word_offset
    bs = TIB_BS
    first, nb = shard_blocks(world * TIB_NB, rank, world)
    try:
        region = torch.empty(bs * nb, dtype=torch.uint8, device=dev)
    except torch.OutOfMemoryError as e:  # reported, never silently shrunk
        return {"skipped": f"cannot allocate {bs * nb / 2**30:.0f} GiB: {e}"}
    ctx.fill_splitmix(region, SEED, word_offset=shard_word_offset(first, bs))
    out = torch.empty(nb, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def step(_i=0):
        ctx.blocks_dev(region, bs, out=out, stream=stream)

    step()
    torch.cuda.synchronize()
    ramp(step, stream, torch, window=3, min_s=0.5)
    k = max(1, args.tib_steps)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(k):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    el = max_over_ranks(time.perf_counter() - t0, device=dev)
    kms = ev0.elapsed_time(ev1) / k
    # sampled parity: first and last block of the shard and every 4096th
    # (the >2 GiB and >64 GiB ends of the shard included)
    idx = np.unique(np.concatenate([np.arange(0, nb, 4096), [nb - 1]])).astype(np.int64)
    ti = torch.from_numpy(idx).to(dev)
    blocks = region.view(nb, bs).index_select(0, ti).cpu().numpy()
    got = as_u32(out.index_select(0, ti))
    want = O.crc32_blocks(blocks.reshape(-1), bs, nthreads=8)
    ok = bool(np.array_equal(got, want))
    all_ok = max_over_ranks(0.0 if ok else 1.0, device=dev) == 0.0
    alg = nb * (bs + 4)
    plan = ctx.blocks_plan(region.data_ptr(), nb, bs)
    del region, out
    torch.cuda.empty_cache()
    return {"workload": CONFIGS["tib"][2], "value": round(bs * nb * world * k / el / 2**30, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": k, "ms_per_step": round(el / k * 1e3, 4), "bytes_per_gpu": bs * nb,
            "kernel": plan, "roofline": {"achieved": round(alg / (kms * 1e-3) / 1e9, 1),
                                                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                                      "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                                      "kernel_ms": round(kms, 4)},
            "parity": {"checked_blocks_per_rank": int(idx.size), "sample": "first, last, every 4096th block",
                       "bit_exact": bool(all_ok)}}


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


def streamed(args, torch, rank, world):
    """BASELINE config 5: 4 KiB blocks from pinned host memory, end to end."""
    from priskv_amd import CrcContext, host_register, host_unregister
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    bs = args.block_size or 4096
    nb = args.nblocks or (1 << 20)
    ctx = CrcContext(int(os.environ.get("LOCAL_RANK", "0")))
    host = O.fill_splitmix(bs * nb, SEED, rank * (bs * nb // 8))
    res = {}
    for mode in ("pinned", "pageable"):
        if mode == "pinned":
            host_register(host)
        out = ctx.blocks_host(host, bs)  # warm (allocates staging)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = ctx.blocks_host(host, bs)
        dt = (time.perf_counter() - t0) / args.steps
        if mode == "pinned":
            host_unregister(host)
        res[mode] = round(bs * nb / dt / 2**30, 2)
    samp = min(nb, 65536)
    ok = bool(np.array_equal(out[:samp], O.crc32_blocks(host[: samp * bs], bs, nthreads=8)))
    print(json.dumps({"metric": "GiB/s CRC of host-resident value blocks (PCIe-inclusive, streamed)",
                      "value": res["pinned"], "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
                      "pageable_GiBs": res["pageable"], "config": {"workload": f"{nb} x {bs} B host blocks",
                                                                   "block_size": bs},
                      "parity": {"checked_blocks": samp, "bit_exact": ok}}), flush=True)


if __name__ == "__main__":
    main()
