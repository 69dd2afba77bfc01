#!/usr/bin/env python3
"""Is the extents kernel's static split (equal extent COUNTS per wave) what
holds PrisKV-shaped values below the rows kernel?  Same extents, same bytes,
three orders: as generated (random), dealt so that every wave's contiguous
range holds about the same number of chunks, and sorted by offset.  One JSON
line per case on stdout; each case checked against the oracle on a sample.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import _oracle as O  # noqa: E402
import torch  # noqa: E402
from bench_paths import SEED, extents, timeit  # noqa: E402

from priskv_amd import CrcContext, as_u32  # noqa: E402


def balanced_order(lens, waves):
    """Snake-deal extents (largest first) over `waves` bins, then lay the bins
    out back to back: wave w's static range [n w / W, n (w+1) / W) is bin w."""
    n = len(lens)
    per = n // waves
    cost = (lens.astype(np.int64) + 2047) // 2048
    order = np.argsort(-cost, kind="stable")
    bins = [[] for _ in range(waves)]
    for r in range(per):
        ids = order[r * waves:(r + 1) * waves]
        seq = range(waves) if r % 2 == 0 else range(waves - 1, -1, -1)
        for b, i in zip(seq, ids):
            bins[b].append(i)
    return np.concatenate([np.array(b, dtype=np.int64) for b in bins])


def wave_spread(lens, waves):
    e = (np.arange(waves + 1) * len(lens)) // waves
    c = np.add.reduceat(lens.astype(np.int64), e[:-1])
    return float(c.max() / c.mean())


def main():
    ctx = CrcContext(0)
    waves = torch.cuda.get_device_properties(0).multi_processor_count * 2 * 8
    region = 4 << 30
    n = 1 << 19
    assert n % waves == 0
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 0)
    rng = np.random.default_rng(1)
    offs, lens = extents(rng, n, region, 4096)
    perms = {
        "random": np.arange(n),
        "balanced": balanced_order(lens, waves),
        "sorted_offset": np.argsort(offs, kind="stable"),
    }
    cases = {}
    for name, p in perms.items():
        o, ln = offs[p], lens[p]
        cases[name] = (o, ln, torch.from_numpy(o.astype(np.int64)).cuda(), torch.from_numpy(ln.view(np.int32)).cuda())
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    vb = int(lens.astype(np.int64).sum())
    for rep in range(3):
        for name, (o, ln, d_o, d_l) in cases.items():
            sec = timeit(lambda: ctx.ranges_dev(t, d_o, d_l, out=out), 20)
            got = as_u32(out[:100])
            want = np.array([O.crc32(t[int(a):int(a) + int(b)].cpu().numpy()) for a, b in zip(o[:100], ln[:100])],
                            dtype=np.uint32)
            print(json.dumps(dict(case=name, rep=rep, values=n, value_bytes=vb, waves=waves,
                                  max_wave_bytes_over_mean=round(wave_spread(ln, waves), 4),
                                  us=round(sec * 1e6, 1), TBs=round(vb / sec / 1e12, 3),
                                  bit_exact=bool(np.array_equal(got, want)))), flush=True)


if __name__ == "__main__":
    main()
