"""Sharding of a value-block region across GPUs (one process per GPU).

SURVEY.md §8(e): each block's CRC depends only on its own bytes, so a batch
shards as contiguous block ranges -- GPU g takes [g*N/G, (g+1)*N/G) -- with no
data-path collective.  The value region's block count is a power of two
(server/server.c:246-256, server/memory.c:194,407), so G in {1,2,4,8}
divides it evenly; any other N is split with at most one block of imbalance.

Collectives appear only around the path: the benchmark's barrier and
max-over-ranks timing, and ``gather_crcs`` for callers that want every
rank's CRCs on every rank (verification / reporting).  On ROCm the "nccl"
backend is RCCL over xGMI; tests use "gloo" on CPU.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_blocks(nblocks: int, rank: int, world: int) -> Tuple[int, int]:
    """(first block, block count) of ``rank``'s contiguous shard."""
    if world < 1 or not 0 <= rank < world or nblocks < 0:
        raise ValueError(f"bad shard request nblocks={nblocks} rank={rank} world={world}")
    first = nblocks * rank // world
    return first, nblocks * (rank + 1) // world - first


def shard_word_offset(first_block: int, block_size: int) -> int:
    """Splitmix64 word index where a shard starting at ``first_block`` begins
    (test pattern of priskv_crc_fill_splitmix_dev), so the shards of all ranks
    are slices of one global region.  Needs the shard to start on an 8-byte
    boundary of that region (always true for rank 0, and for every rank when
    block_size % 8 == 0)."""
    if (first_block * block_size) % 8:
        raise ValueError("pattern word offsets need 8-byte aligned shard starts")
    return first_block * block_size // 8


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (timing) across the default process group."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = None
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_crcs(local: np.ndarray, nblocks: int, device=None) -> np.ndarray:
    """All ranks' shard CRCs concatenated in block order (uint32[nblocks]).

    Uses all_gather on int32 views padded to the largest shard; every rank's
    shard layout comes from shard_blocks, so no metadata is exchanged."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1:
        return np.asarray(local, dtype=np.uint32).copy()
    if dist.get_backend() == "gloo":
        device = None
    rank = dist.get_rank()
    first, count = shard_blocks(nblocks, rank, world)
    if len(local) != count:
        raise ValueError(f"rank {rank} holds {len(local)} CRCs, shard has {count}")
    width = max(shard_blocks(nblocks, r, world)[1] for r in range(world))
    buf = torch.zeros(width, dtype=torch.int32, device=device)
    if count:
        buf[:count] = torch.from_numpy(np.asarray(local, dtype=np.uint32).view(np.int32)).to(buf.device)
    parts = [torch.zeros(width, dtype=torch.int32, device=device) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = np.empty(nblocks, dtype=np.uint32)
    for r, p in enumerate(parts):
        f, c = shard_blocks(nblocks, r, world)
        out[f:f + c] = p[:c].cpu().numpy().view(np.uint32)
    return out
