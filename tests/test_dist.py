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
