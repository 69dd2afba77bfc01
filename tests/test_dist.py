"""Multi-process (N > 1) host logic on CPU with the gloo backend, world_size 2.

The GPU path shards a batch as contiguous block ranges with no data-path
collective; what these tests pin is the host side of that:
shard ranges tile the region, each rank's pattern window is the right slice
of one global region, per-rank results gather back in block order, and the
benchmark's max-over-ranks timing reduction.  The per-rank CRC here is the
CPU oracle standing in for the GPU (there is no GPU in this container); the
GPU parity of the per-rank computation itself is tests/test_gpu_parity.py.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import _oracle as O
from priskv_amd.shard import shard_blocks, shard_word_offset


def test_shard_blocks_tile_the_region():
    for n in (0, 1, 7, 64, 1 << 20, 1000003):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_blocks(n, r, world) for r in range(world)]
            assert spans[0][0] == 0
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    # power-of-two block counts (the reference's -b) split exactly
    assert {shard_blocks(1 << 24, r, 8)[1] for r in range(8)} == {1 << 21}
    with pytest.raises(ValueError):
        shard_blocks(10, 2, 2)


def test_shard_pattern_is_a_slice_of_the_global_region():
    bs, n, world = 512, 37, 3
    glob = O.fill_splitmix(bs * n, 0x1234, 0)
    for r in range(world):
        f, c = shard_blocks(n, r, world)
        part = O.fill_splitmix(bs * c, 0x1234, shard_word_offset(f, bs))
        assert np.array_equal(part, glob[f * bs:(f + c) * bs])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, bs, nblocks, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from priskv_amd.shard import gather_crcs, max_over_ranks
    first, count = shard_blocks(nblocks, rank, world)
    region = O.fill_splitmix(bs * count, 0x5EED, shard_word_offset(first, bs))
    local = O.crc32_blocks(region, bs)
    allc = gather_crcs(local, nblocks)
    t = max_over_ranks(0.5 + rank)
    dist.barrier()
    q.put((rank, allc, t))
    dist.destroy_process_group()


@pytest.mark.parametrize("nblocks", [64, 37])
def test_gloo_world2_shard_and_gather(nblocks):
    bs, world = 1024, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bs, nblocks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = O.crc32_blocks(O.fill_splitmix(bs * nblocks, 0x5EED, 0), bs)
    for rank, allc, t in res:
        assert np.array_equal(allc, want), rank
        assert t == 1.5  # max over ranks of 0.5 + rank


def _bench_worker(rank, world, port, fail_ranks, q):
    try:
        _bench_worker_body(rank, world, port, fail_ranks, q)
    except BaseException as e:  # report instead of leaving the test to time out
        q.put((rank, "error", repr(e), None, None, None, None, None))
        raise


def _bench_worker_body(rank, world, port, fail_ranks, q):
    """bench.py's Bench collectives at world 8 on CPU (gloo): the allocation
    agreement with some ranks failing, all_ok, max over ranks and the
    device-identity gather pair up in the order every leg issues them."""
    import sys as _sys

    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    class _Torch:  # torch with an allocator that fails on the chosen ranks (the tib leg's OOM)
        OutOfMemoryError = torch.OutOfMemoryError
        uint8 = torch.uint8

        @staticmethod
        def empty(n, dtype=None, device=None):
            if rank in fail_ranks:
                raise torch.OutOfMemoryError("simulated: cannot allocate")
            return torch.empty(n, dtype=dtype, device=device)

        class cuda:
            @staticmethod
            def empty_cache():
                pass

    B = bench.Bench(None, _Torch, dist, world, rank, "cpu", None)
    region, err = B.alloc(1 << 10)           # any failing rank: None everywhere
    ok_all = B.all_ok(True)
    ok_one = B.all_ok(rank != 3)
    mx = B.max(float(rank) * 0.25)
    infos = bench.gather_obj({"rank": rank}, world)
    region2, err2 = bench.Bench(None, torch, dist, world, rank, "cpu", None).alloc(1 << 10)  # none fail
    B.barrier()
    q.put((rank, region is None, err, ok_all, ok_one, mx, [i["rank"] for i in infos], region2 is not None))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_ranks", [(2, 5), (), (7,)])
def test_gloo_world8_bench_collectives(fail_ranks):
    """The N = 8 rehearsal of bench.py's per-leg collectives on CPU: every
    rank reaches the same decisions (skip on any rank's allocation failure,
    all_ok false when one rank fails) and the collectives pair up."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, fail_ranks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, skipped, err, ok_all, ok_one, mx, ranks, alloc2 in res:
        assert skipped != "error", (rank, err)
        assert skipped == bool(fail_ranks), (rank, err)
        if fail_ranks and rank not in fail_ranks:
            assert err == "another rank could not allocate"
        assert ok_all and not ok_one
        assert mx == 1.75
        assert ranks == list(range(world))
        assert alloc2


def _gpu_worker(rank, world, port, bs, nblocks, q):
    """One rank: its contiguous shard filled and hashed on the GPU (the
    product path, priskv_crc32_blocks_dev), every rank's CRCs gathered."""
    try:
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from priskv_amd import CrcContext, as_u32
        from priskv_amd.shard import gather_crcs
        first, count = shard_blocks(nblocks, rank, world)
        with CrcContext(0) as ctx:
            region = torch.empty(bs * count, dtype=torch.uint8, device="cuda:0")
            ctx.fill_splitmix(region, 0x5EED, shard_word_offset(first, bs))
            local = as_u32(ctx.blocks_dev(region, bs))
        allc = gather_crcs(local, nblocks)
        dist.barrier()
        q.put((rank, allc, None))
        dist.destroy_process_group()
    except BaseException as e:  # report instead of leaving the test to time out
        q.put((rank, None, repr(e)))
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("bs,nblocks", [(4096, 1 << 14), (1 << 20, 64)])
def test_gloo_world2_gpu_shards(bs, nblocks):
    """The N > 1 path with the GPU doing each rank's work: two ranks (one
    GPU on the test box, so both on device 0) hash their shards through the
    C ABI and gather; the result equals the oracle over the one global
    region."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, bs, nblocks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = O.crc32_blocks(O.fill_splitmix(bs * nblocks, 0x5EED, 0), bs)
    for rank, allc, err in res:
        assert err is None, (rank, err)
        assert np.array_equal(allc, want), rank
