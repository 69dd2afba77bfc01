"""Coarse GPU time guards for the cross-workgroup finish (round 6).

A lone 256 MiB block or value has a part in every workgroup, all finishing
through one zero-at-rest word (finish_shared, crc_device.inc).  Round 6's
first single-word finish was a compare-and-swap loop: exact, but it
serialised the 256 workgroups' swaps and a lone block went from 49 to 302 us
per call -- no parity test could see that.  These tests time such calls
with HIP events (after a warm-up) and fail only on a regression of that
kind: the bounds are about twice the measured times, far
outside box-to-box spread.  Each result is also checked against the oracle.
"""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

MIB = 1 << 20


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ctx(torch_cuda):
    from priskv_amd import CrcContext
    c = CrcContext(0)
    yield c
    c.close()


def _median_us(torch, fn, stream, n=30):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in evs:
        e0.record(stream)
        fn()
        e1.record(stream)
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]))


# (name, blocks, block size, bound us): measured round 6 ~49 / ~48 / ~610 us
@pytest.mark.parametrize("name,nb,bs,bound", [("lone 256 MiB block", 1, 256 * MIB, 110.0),
                                              ("16 x 16 MiB", 16, 16 * MIB, 110.0),
                                              ("4096 x 1 MiB (split mode)", 4096, MIB, 1300.0)])
def test_few_large_blocks_not_serialised(torch_cuda, ctx, name, nb, bs, bound):
    torch = torch_cuda
    from priskv_amd import as_u32
    t = torch.empty(nb * bs, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, 0x9A4D + nb, 0)
    out = torch.full((nb,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    us = _median_us(torch, lambda: ctx.blocks_dev(t, bs, out=out, stream=s), s)
    print(f"{name}: {us:.1f} us per call ({ctx.blocks_plan(t.data_ptr(), nb, bs)[:70]})")
    assert np.array_equal(as_u32(out), O.crc32_blocks(t.cpu().numpy(), bs, nthreads=16)), name
    assert us < bound, f"{name}: {us:.1f} us per call (bound {bound}): the finish serialises?"


def test_lone_value_not_serialised(torch_cuda, ctx):
    """ranges_dev over one 256 MiB value (the fused few-extents kernel)."""
    torch = torch_cuda
    from priskv_amd import as_u32
    n = 256 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, 0x10E, 0)
    offs = np.array([5], dtype=np.uint64)
    lens = np.array([n - 3], dtype=np.uint32)
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    us = _median_us(torch, lambda: ctx.ranges_dev(t, d_o, d_l, out=out, stream=s), s)
    print(f"lone 256 MiB value: {us:.1f} us per call")
    assert np.array_equal(as_u32(out), O.crc32_ranges(t.cpu().numpy(), offs, lens))
    assert us < 120.0, f"lone 256 MiB value: {us:.1f} us per call: the finish serialises?"
