"""In-process A/B of the rows-kernel XCD weights (tools, not product).

Two contexts on one device -- one with the default XCD weights, one with
PRISKV_CRC_XCD_WEIGHTS=1:1 (equal split) -- time the same 4 GiB batch of
4 KiB blocks, alternating which goes first each round; prints the medians.
usage: python tools/ab_xcd.py [weights=31:29] [rounds=12] [block_size=4096]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from priskv_amd import CrcContext  # noqa: E402


def make_ctx(weights):
    os.environ["PRISKV_CRC_XCD_WEIGHTS"] = weights
    c = CrcContext(0)
    del os.environ["PRISKV_CRC_XCD_WEIGHTS"]
    return c


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "31:29"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    bs = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    total = 4 << 30
    t = torch.empty(total, dtype=torch.uint8, device="cuda")
    cw, ce = make_ctx(w), make_ctx("1:1")
    cw.fill_splitmix(t, 1, 0)
    out = torch.empty(total // bs, dtype=torch.int32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {"weighted": [], "equal": []}

    def run(ctx, n=10):
        ev[0].record()
        for _ in range(n):
            ctx.blocks_dev(t, bs, out=out)
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / n

    for _ in range(30):  # ramp
        cw.blocks_dev(t, bs, out=out)
    torch.cuda.synchronize()
    for r in range(rounds):
        order = [("weighted", cw), ("equal", ce)] if r % 2 == 0 else [("equal", ce), ("weighted", cw)]
        for name, c in order:
            res[name].append(run(c))
    for name, v in res.items():
        med = statistics.median(v)
        print(f"{name:9s} {w if name == 'weighted' else '1:1':6s} bs {bs}: median {med:.4f} ms  "
              f"{total / med / 1e6:.1f} GB/s  (min {min(v):.4f}, max {max(v):.4f})")


if __name__ == "__main__":
    main()
