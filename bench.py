#!/usr/bin/env python3
"""bench.py -- value-block CRC throughput on MI355X (BASELINE.json metric).

One "step" = one pass of priskv_crc32 (server/crc.c:90-109) over every value
block of this GPU's shard, device-resident (inputs already in HBM when the
timed region starts), through the library's C ABI
(priskv_crc32_blocks_dev, include/priskv_crc_gpu.h).

Default workload (BASELINE.json configs[1]): 1 Mi x 4 KiB blocks = 4 GiB per
GPU.  For N > 1 (launched by torch.distributed.run) each rank owns its own
4 GiB shard -- the next 1 Mi blocks of one global region -- and checksums it
with no data-path collective ("weak" scaling); the barrier and the max-over-
ranks reduction are the benchmark contract, not part of the path.

Prints ONE JSON line on rank 0.  Extra keys:
  roofline      dominant kernel (crc_rows_kernel) vs the HBM roof: algorithmic
                bytes per launch / average launch time (HIP events on the launch
                stream); traffic = PMC-measured HBM bytes per launch for this
                workload when profiles/ holds a matching measurement, else null
  cpu_baseline  rank 0 at N=1: the reference's own server/crc.c (compiled -O2
                into oracle/_ref) timed single-threaded on a bounded sample of
                the same blocks, which also serves as a bit-exact spot check
  cpu_baseline_threads  the same sample split over 16 threads (the box's CPU share)
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
RAMP_S = 0.3

CONFIGS = {
    # name: (block_size, nblocks per GPU, description)
    "default": (4096, 1 << 20, "1Mi x 4KiB value blocks per GPU, device-resident (4 GiB/GPU)"),
    "sweep64k": (65536, 1 << 16, "64Ki x 64KiB value blocks per GPU, device-resident (4 GiB/GPU)"),
    "sweep1m": (1 << 20, 1 << 12, "4Ki x 1MiB value blocks per GPU, device-resident (4 GiB/GPU)"),
    "tib": (65536, 1 << 21, "2Mi x 64KiB value blocks per GPU (128 GiB/GPU; 1 TiB at 8 GPUs)"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="default", choices=sorted(CONFIGS) + ["streamed"])
    p.add_argument("--block-size", type=int, default=None)
    p.add_argument("--nblocks", type=int, default=None)
    p.add_argument("--cpu-sample-bytes", type=int, default=3 << 30,
                   help="bytes of the shard the CPU baseline hashes (about 10 s at -O2)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--pipeline-streams", type=int, default=2,
                   help="streams for the reported-beside pipelined pass (0 = skip it)")
    return p.parse_args()


def load_traffic(cfg_name: str, block_size: int, nblocks: int):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if one matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(f"{block_size}x{nblocks}")
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


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
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        ctx.blocks_dev(region, bs, out=out, stream=stream)
    torch.cuda.synchronize()
    # The first ~10 launches after idle run up to 40% slow while the device
    # leaves its idle power state (profiles/r01/clock_ramp.txt); keep stepping,
    # untimed, until >= RAMP_S seconds of back-to-back work have passed so the
    # timed steps see steady-state serving throughput.
    ramp = 0
    t_r = time.perf_counter()
    while time.perf_counter() - t_r < RAMP_S:
        for _ in range(8):
            ctx.blocks_dev(region, bs, out=out, stream=stream)
        torch.cuda.synchronize()
        ramp += 8

    def barrier():
        if world > 1:
            dist.barrier()

    trace = os.environ.get("PRISKV_BENCH_TRACE")
    if trace:  # per-step kernel times of a separate, untimed pass (diagnostics only)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        evs[0].record(stream)
        for i in range(args.steps):
            ctx.blocks_dev(region, bs, out=out, stream=stream)
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
        print("per-step ms:", " ".join(f"{evs[i].elapsed_time(evs[i + 1]):.3f}" for i in range(args.steps)),
              file=sys.stderr)

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        ctx.blocks_dev(region, bs, out=out, stream=stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # launches back-to-back on `stream`

    elapsed_max = max_over_ranks(elapsed, device=dev)

    total_bytes = bs * nb * world
    value = total_bytes * args.steps / elapsed_max / 2**30
    alg_bytes = nb * (bs + 4)  # block read + 4-byte CRC written
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = load_traffic(args.config, bs, nb)
    path = ctx_path(bs, region)

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
                   "kernel": path, "untimed_ramp_launches": ramp},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel_ms": round(kernel_ms, 4),
                     "alg_bytes_per_launch": alg_bytes},
    }

    if args.pipeline_streams > 1:
        # Reported beside `value`, never instead of it: the same K batch
        # passes, issued round-robin over independent streams as a server
        # with several scrub/verify batches in flight would.  Kernels on one
        # stream are serialized, so every batch pays its own tail (the last
        # ~50 us below the HBM rate); on separate streams the next
        # batch's workgroups take the CUs that the previous one frees.
        ns = args.pipeline_streams
        pstreams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(ns - 1)]
        pouts = [out] + [torch.empty(nb, dtype=torch.int32, device=dev) for _ in range(ns - 1)]
        for i in range(2 * ns):
            ctx.blocks_dev(region, bs, out=pouts[i % ns], stream=pstreams[i % ns])
        barrier()
        torch.cuda.synchronize()
        tp0 = time.perf_counter()
        for i in range(args.steps):
            ctx.blocks_dev(region, bs, out=pouts[i % ns], stream=pstreams[i % ns])
        torch.cuda.synchronize()
        barrier()
        p_elapsed = max_over_ranks(time.perf_counter() - tp0, device=dev)
        same = all(torch.equal(pouts[0], o) for o in pouts[1:])
        result["pipelined"] = {"streams": ns, "value": round(total_bytes * args.steps / p_elapsed / 2**30, 2),
                               "unit": "GiB/s", "ms_per_step": round(p_elapsed / args.steps * 1e3, 4),
                               "frac_of_peak": round(alg_bytes * args.steps / p_elapsed / 1e9 / HBM_PEAK_GBS, 4),
                               "outputs_identical": bool(same)}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        nsamp = max(1, min(nb, args.cpu_sample_bytes // bs))
        host = region[: nsamp * bs].cpu().numpy()
        secs, cpu_crc, kind, label = O.time_cpu_baseline(host, bs)
        gpu_crc = as_u32(out[:nsamp])
        ok = bool(np.array_equal(cpu_crc, gpu_crc))
        result["cpu_baseline"] = {"value": round(nsamp * bs / secs / 2**30, 4), "unit": "GiB/s", "cores": 1,
                                  "kind": kind,
                                  "sample": f"first {nsamp} x {bs} B blocks ({nsamp * bs / 2**30:.2f} GiB) of the "
                                            f"same shard, 1 thread, {label}; {secs:.1f} s",
                                  "cpu": cpu_model()}
        # the same sample split over the box's CPU share (SURVEY 8(d) config 1
        # asks for 1 thread and all threads); reported beside, not instead
        nthr = int(os.environ.get("PRISKV_BENCH_CPU_THREADS", "16"))
        secs_mt, cpu_crc_mt, _, _ = O.time_cpu_baseline(host, bs, threads=nthr)
        ok = ok and bool(np.array_equal(cpu_crc_mt, gpu_crc))
        result["cpu_baseline_threads"] = {"value": round(nsamp * bs / secs_mt / 2**30, 4), "unit": "GiB/s",
                                          "cores": nthr, "kind": kind,
                                          "sample": f"same sample, {nthr} threads (static block split); "
                                                    f"{secs_mt:.2f} s"}
        result["parity"] = {"checked_blocks": nsamp, "bit_exact": ok}
        if not ok:
            bad = np.nonzero(cpu_crc != gpu_crc)[0]
            result["parity"]["first_mismatch"] = int(bad[0])
    elif world > 1:
        # every rank spot-checks the start of its own shard against the oracle
        # (untimed); the flags are min-reduced so rank 0 reports all ranks
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        nsamp = max(1, min(nb, (64 << 20) // bs))
        ok = np.array_equal(O.crc32_blocks(region[: nsamp * bs].cpu().numpy(), bs, nthreads=8), as_u32(out[:nsamp]))
        all_ok = max_over_ranks(0.0 if ok else 1.0, device=dev) == 0.0
        result["parity"] = {"checked_blocks_per_rank": nsamp, "bit_exact": bool(all_ok)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def ctx_path(bs, region):
    """Kernel the library dispatches to (mirrors plan_for() in crc_gpu.hip)."""
    from priskv_amd import blocks_path
    p = blocks_path(region.data_ptr(), 1, bs)
    if p == "rows":
        pipe = bs in (1024, 4096)
        if bs == 4096:
            g, ch = 32, 8
        elif bs <= 16384 and bs % 4096:
            g, ch = 16, 4
        else:
            r = bs // 1024
            g, ch = 64, (4 if r % 4 == 0 else (2 if r % 2 == 0 else 1))
        w = os.environ.get("PRISKV_CRC_XCD_WEIGHTS", "31:29")
        split = "" if w.replace(" ", "") in ("1:1",) else f",xcd-weighted {w}"
        fold = ",pipelined-fold" if pipe else ""
        if bs in (1024, 4096, 8192):
            fold += ",nibble-table-fold"
        # progress-priority mode of the plan (kPlans in crc_gpu.hip)
        mode = 3 if bs == 4096 or (g == 64 and ch == 4 and bs >= 256 << 10) else (1 if ch == 4 or g == 16 else 0)
        if os.environ.get("PRISKV_CRC_PRIO") == "0":
            mode = 0
        prio = f",progress-priority {mode}" if mode else ""
        return f"crc_rows_kernel<G={g},CH={ch},NBUF=2,nt{fold}{split}{prio}>"
    return f"crc_{p}_kernel"


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
