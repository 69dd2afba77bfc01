"""GPU parity: libpriskv_crc.so's HIP kernels vs the CPU oracle (bit-exact).

Every call goes through the C ABI (include/priskv_crc_gpu.h) via ctypes.
Inputs are seeded splitmix64 patterns produced on the device by the
library's fill kernel, whose bytes are themselves checked against the
oracle's generator; expected values come from the oracle
(oracle/crc_oracle.c, pinned to the reference in test_oracle.py) or
straight from the golden fixture produced by the reference.
"""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x5EED5EED


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


@pytest.fixture(scope="module")
def ctx_noseg(torch_cuda):
    """A context with segmentation off (PRISKV_CRC_SEGMENT=0, read at creation):
    every call takes the one-wave-per-extent / unsegmented rows path."""
    import os
    from priskv_amd import CrcContext
    old = os.environ.get("PRISKV_CRC_SEGMENT")
    os.environ["PRISKV_CRC_SEGMENT"] = "0"
    try:
        c = CrcContext(0)
    finally:
        if old is None:
            del os.environ["PRISKV_CRC_SEGMENT"]
        else:
            os.environ["PRISKV_CRC_SEGMENT"] = old
    yield c
    c.close()


@pytest.mark.parametrize("bs", [16, 32, 64, 128, 256, 512, 1024, 3072, 4096, 8192, 65536, 131072, 262144, 1 << 20])
def test_every_plan_at_48MiB(torch_cuda, ctx, bs):
    """Every rows plan and the sub-KiB kernel at ~48 MiB per call, a ragged
    count: the oracle's CRCs.  (Round 5 removed the no-priority variants,
    PRISKV_CRC_PRIO=0, measured slower in rounds 1-3.)"""
    torch = torch_cuda
    nb = max(1, (48 << 20) // bs) + 3
    t = _region(torch, ctx, bs * nb, SEED ^ (bs * 7), nb)
    want = O.crc32_blocks(t[: bs * nb].cpu().numpy(), bs, nthreads=8)
    got = _u32(ctx.blocks_dev(t, bs, nblocks=nb))
    torch.cuda.synchronize()
    assert np.array_equal(got, want), (bs, nb, np.nonzero(got != want)[0][:8])


@pytest.fixture(scope="module")
def ctx_seg16k(torch_cuda):
    """Segmentation for device-length calls of up to 16384 extents
    (PRISKV_CRC_SEG_MAX_EXTENTS, read at creation)."""
    import os
    from priskv_amd import CrcContext
    os.environ["PRISKV_CRC_SEG_MAX_EXTENTS"] = "16384"
    try:
        c = CrcContext(0)
    finally:
        del os.environ["PRISKV_CRC_SEG_MAX_EXTENTS"]
    yield c
    c.close()


def test_segmented_many_extents(torch_cuda, ctx_seg16k):
    """Thousands of extents through the segmented path (1024-thread plan, 64-way
    segment search): mixed lengths incl. empty and sub-16-B ones, ragged offsets."""
    torch = torch_cuda
    ctx = ctx_seg16k
    n_bytes = 256 << 20
    t = _region(torch, ctx, n_bytes, SEED ^ 0x99, 4)
    rng = np.random.default_rng(31)
    for k in (2049, 5000, 16384):
        lens = rng.integers(0, 200000, k).astype(np.uint32)
        lens[:8] = [0, 1, 15, 16, 17, 16384, 16385, 1 << 20]
        offs = np.array([rng.integers(0, n_bytes - int(ln)) for ln in lens], dtype=np.uint64)
        got = _u32(ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(),
                                  torch.from_numpy(lens.view(np.int32)).cuda()))
        torch.cuda.synchronize()
        want = O.crc32_ranges(t[:n_bytes].cpu().numpy(), offs, lens)
        assert np.array_equal(got, want), (k, np.nonzero(got != want)[0][:8])


def test_segmentation_limit_boundary(torch_cuda, ctx):
    """The default context segments device-length calls of up to 8192 extents
    and not above: both sides of the boundary, ragged lengths incl. empty and
    multi-MiB ones, give the oracle's CRCs."""
    torch = torch_cuda
    n_bytes = 128 << 20
    t = _region(torch, ctx, n_bytes, SEED ^ 0x8192, 4)
    host = t[:n_bytes].cpu().numpy()
    rng = np.random.default_rng(8192)
    for k in (8191, 8192, 8193):
        lens = rng.integers(0, 70000, k).astype(np.uint32)
        lens[:6] = [0, 1, 17, 3 << 20, 1 << 20, 65536]
        offs = np.array([rng.integers(0, n_bytes - int(ln)) for ln in lens], dtype=np.uint64)
        got = _u32(ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(),
                                  torch.from_numpy(lens.view(np.int32)).cuda()))
        torch.cuda.synchronize()
        want = O.crc32_ranges(host, offs, lens)
        assert np.array_equal(got, want), (k, np.nonzero(got != want)[0][:8])


@pytest.fixture(params=["segmented", "unsegmented"])
def any_ctx(request, ctx, ctx_noseg):
    """The default context and one with segmentation off."""
    return {"segmented": ctx, "unsegmented": ctx_noseg}[request.param]


def _region(torch, ctx, nbytes, seed=SEED, word_offset=0, pad=0):
    t = torch.empty(nbytes + pad + 16, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, seed, word_offset, nbytes=nbytes + pad)
    return t


def _u32(t):
    from priskv_amd import as_u32
    return as_u32(t)


def test_fill_matches_oracle_generator(torch_cuda, ctx):
    torch = torch_cuda
    for n, off in ((4096, 0), (1 << 20, 12345), (1000003, 7)):
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        ctx.fill_splitmix(t, SEED, off)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), O.fill_splitmix(n, SEED, off)), (n, off)


def test_golden_blocks_on_gpu(torch_cuda, ctx, golden):
    """The reference's own outputs (fixture) reproduced by the HIP kernels."""
    torch = torch_cuda
    for b in golden["blocks"]:
        bs, nb = b["block_size"], b["nblocks"]
        t = _region(torch, ctx, bs * nb, golden["seed"], b["word_offset"])
        out = ctx.blocks_dev(t, bs, nblocks=nb)
        torch.cuda.synchronize()
        assert [f"{v:08x}" for v in _u32(out)] == b["crcs"], bs


def test_golden_ranges_on_gpu(torch_cuda, ctx, golden):
    torch = torch_cuda
    r = golden["ranges"]
    t = _region(torch, ctx, r["region_bytes"], golden["seed"], r["word_offset"])
    offs = torch.tensor([it["offset"] for it in r["items"]], dtype=torch.int64, device="cuda")
    lens = torch.tensor([it["len"] for it in r["items"]], dtype=torch.int32, device="cuda")
    out = ctx.ranges_dev(t, offs, lens)
    torch.cuda.synchronize()
    assert [f"{v:08x}" for v in _u32(out)] == [it["crc"] for it in r["items"]]


# block sizes covering every dispatch path and rows-kernel plan
# (priskv_amd/csrc/crc_gpu.hip plan_for):
#   G32/CH8 pipelined nibble fold (4K), G16/CH4 pipelined nibble fold (1K),
#   G64/CH4 nibble fold (8K), G16/CH4 (2K, 3K, 5K, 6K),
#   G64/CH4 (12K, 16K, 20K, 64K, 128K; 256K and 1M with priority mode 3), G64/CH2 (18K), G64/CH1 (17K, 33K),
#   sub-KiB (16..512), extents (>= 1 KiB not a multiple of 1 KiB), generic (smaller odd sizes)
BLOCK_SIZES = [1024, 2048, 3072, 4096, 5120, 6144, 8192, 12288, 16384, 17408, 18432, 20480, 33792,
               65536, 131072, 262144, 1 << 20, 16, 32, 64, 128, 256, 512, 1, 3, 100, 1000, 4097, 4100, 48, 1025, 1040,
               65537, 70000]
NBLOCKS = [1, 2, 7, 63, 64, 65, 129, 1000, 4099]


@pytest.mark.parametrize("bs", BLOCK_SIZES)
def test_blocks_vs_oracle(torch_cuda, ctx, bs):
    torch = torch_cuda
    for nb in NBLOCKS:
        if bs * nb > (64 << 20):
            continue
        t = _region(torch, ctx, bs * nb, SEED ^ bs, nb)
        out = ctx.blocks_dev(t, bs, nblocks=nb)
        torch.cuda.synchronize()
        host = t[: bs * nb].cpu().numpy()
        want = O.crc32_blocks(host, bs, nthreads=8)
        got = _u32(out)
        assert np.array_equal(got, want), (bs, nb, np.nonzero(got != want)[0][:8])


def test_sub_kib_fold_tables(torch_cuda, ctx):
    """crc_small_kernel (byte-table fold for G = 2..16, nibble fold at G = 32,
    none at G = 1) against the oracle, every sub-KiB power of two, whole and
    ragged rows (the ragged tail takes the generic kernel)."""
    torch = torch_cuda
    c = ctx
    for bs in (16, 32, 64, 128, 256, 512):
        plan = c.blocks_plan(16, 4096, bs)
        assert plan.startswith(f"crc_small_kernel<G={bs // 16}"), plan
        assert ("byte-fold" in plan) == (32 <= bs <= 256), plan
        for nb in (1024 // bs * 3 * 2048 * 16 + 1, 1024 // bs * 40 + 3, 1024 // bs * 256 * 16 * 4 * 5 + 7):
            t = _region(torch, c, bs * nb, SEED ^ (bs * 7 + nb), nb)
            out = torch.full((nb,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
            got = _u32(c.blocks_dev(t, bs, out=out, nblocks=nb))
            torch.cuda.synchronize()
            want = O.crc32_blocks(t[: bs * nb].cpu().numpy(), bs, nthreads=8)
            assert np.array_equal(got, want), (bs, nb, np.nonzero(got != want)[0][:8])
            del t


@pytest.mark.parametrize("misalign", [1, 2, 4, 8, 12, 15])
@pytest.mark.parametrize("bs", [4096, 1000, 4100])
def test_unaligned_base(torch_cuda, ctx, misalign, bs):
    torch = torch_cuda
    nb = 97
    t = _region(torch, ctx, bs * nb + 64, SEED, 3)
    view = t[misalign: misalign + bs * nb]
    out = ctx.blocks_dev(view, bs, nblocks=nb)
    torch.cuda.synchronize()
    assert np.array_equal(_u32(out), O.crc32_blocks(view.cpu().numpy(), bs))


def test_zero_and_ff_blocks(torch_cuda, ctx):
    torch = torch_cuda
    for bs in (16, 512, 4096, 65536):
        z = torch.zeros(bs * 33, dtype=torch.uint8, device="cuda")
        out = ctx.blocks_dev(z, bs)
        torch.cuda.synchronize()
        assert not _u32(out).any()  # init 0 / xorout 0: zero data -> CRC 0
        f = torch.full((bs * 33,), 0xFF, dtype=torch.uint8, device="cuda")
        out = ctx.blocks_dev(f, bs)
        torch.cuda.synchronize()
        want = O.crc32(b"\xff" * bs)
        assert (_u32(out) == want).all()


def test_single_bit_flips_detected(torch_cuda, ctx):
    """Each flipped bit changes exactly its own block's CRC by crc(e_bit)."""
    torch = torch_cuda
    bs, nb = 4096, 256
    t = _region(torch, ctx, bs * nb)
    base = _u32(ctx.blocks_dev(t, bs, nblocks=nb)).copy()
    rng = np.random.default_rng(1)
    flips = rng.integers(0, bs * nb * 8, 64)
    for f in flips:
        byte, bit = int(f) // 8, int(f) % 8
        t[byte] ^= (1 << bit)
    out = _u32(ctx.blocks_dev(t, bs, nblocks=nb))
    torch.cuda.synchronize()
    want = O.crc32_blocks(t[: bs * nb].cpu().numpy(), bs)
    assert np.array_equal(out, want)
    touched = {int(f) // 8 // bs for f in flips}
    assert {i for i in range(nb) if out[i] != base[i]} <= touched


def test_ranges_vs_oracle(torch_cuda, any_ctx):
    ctx = any_ctx
    torch = torch_cuda
    n = 8 << 20
    t = _region(torch, ctx, n, SEED, 99)
    rng = np.random.default_rng(4)
    k = 3000
    lens = rng.integers(0, 70000, k).astype(np.uint32)
    lens[:10] = [0, 1, 2, 3, 4, 5, 15, 16, 17, 1 << 20]
    offs = np.array([rng.integers(0, n - int(ln)) for ln in lens], dtype=np.uint64)
    out = ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(),
                         torch.from_numpy(lens.view(np.int32)).cuda())
    torch.cuda.synchronize()
    want = O.crc32_ranges(t[:n].cpu().numpy(), offs, lens)
    assert np.array_equal(_u32(out), want)


def test_ranges_edges(torch_cuda, any_ctx):
    """Extents at every 16-B phase, lengths around 16 / 1 KiB boundaries, ranges
    starting at byte 0 (rows right-aligned before the region start) and ranges
    ending exactly at the end of an exactly-sized allocation."""
    ctx = any_ctx
    torch = torch_cuda
    n = 1 << 16
    t = torch.empty(n, dtype=torch.uint8, device="cuda")  # no padding after the end
    ctx.fill_splitmix(t, SEED, 7)
    offs, lens = [], []
    # (also run below through an unaligned view of the same bytes)
    for off in list(range(0, 34)) + [1000, 4095, 4096, 4097]:
        for ln in list(range(0, 41)) + [1000, 1023, 1024, 1025, 2047, 2048, 4095, 4096, 4097, 20000]:
            if off + ln <= n:
                offs.append(off)
                lens.append(ln)
    for ln in (0, 1, 15, 16, 17, 1023, 1024, 1025, 4096, 65535):  # flush with the end
        offs.append(n - ln)
        lens.append(ln)
    offs.append(0)
    lens.append(n)
    o = np.array(offs, dtype=np.uint64)
    ln = np.array(lens, dtype=np.uint32)
    out = ctx.ranges_dev(t, torch.from_numpy(o.astype(np.int64)).cuda(), torch.from_numpy(ln.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(_u32(out), O.crc32_ranges(t.cpu().numpy(), o, ln))
    # unaligned region base: the same extents relative to base + 5 (re-based in the library)
    keep = (o + ln.astype(np.uint64)) <= n - 5
    o2, l2 = o[keep], ln[keep]
    view = t[5:]
    out2 = ctx.ranges_dev(view, torch.from_numpy(o2.astype(np.int64)).cuda(),
                          torch.from_numpy(l2.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(_u32(out2), O.crc32_ranges(view.cpu().numpy(), o2, l2))


def test_ranges_chunk_boundaries(torch_cuda, any_ctx):
    """Extents whose row count crosses the extents kernel's 4-row chunk edges
    (lengths m*4 KiB +- 0..17 at every 16-B start phase): leading virtual rows,
    the trailing pad p = 0..15 undone by Z_-p, and head + tail masks in one row."""
    ctx = any_ctx
    torch = torch_cuda
    n = 1 << 17
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 21)
    offs, lens = [], []
    for phase in range(16):
        for m in range(4):
            for d in range(-17, 18):
                ln = m * 4096 + d
                if ln >= 0:
                    offs.append(4096 * (1 + m) + phase)
                    lens.append(ln)
    o = np.array(offs, dtype=np.uint64)
    ln = np.array(lens, dtype=np.uint32)
    out = ctx.ranges_dev(t, torch.from_numpy(o.astype(np.int64)).cuda(), torch.from_numpy(ln.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(_u32(out), O.crc32_ranges(t.cpu().numpy(), o, ln))


@pytest.mark.parametrize("bs,nb", [(1 << 20, 1), (1 << 20, 3), (1 << 20, 100), (2 << 20, 5), (4 << 20, 2),
                                   (48 << 10, 7), (3 << 20, 1), (1025 << 10, 3), (96 << 10, 1000),
                                   (64 << 20, 1), (48 << 20, 2), (3 << 24, 1)])
def test_segmented_large_blocks(torch_cuda, ctx, ctx_threelaunch, bs, nb):
    """Batches of few large blocks: the fused few-extents kernel (default) and,
    with PRISKV_CRC_FUSED=0, equal segments through the rows kernel combined
    with Z_seg (crc_combine_segments_kernel); results must not change."""
    torch = torch_cuda
    t = _region(torch, ctx, bs * nb, SEED ^ 0x51, nb)
    want = O.crc32_blocks(t[: bs * nb].cpu().numpy(), bs, nthreads=8)
    for c in (ctx, ctx_threelaunch):
        out = c.blocks_dev(t, bs, nblocks=nb)
        torch.cuda.synchronize()
        assert np.array_equal(_u32(out), want), (bs, nb)


@pytest.mark.parametrize("lens", [[64 << 20], [(1 << 20) + 5, 16 << 20, 0, 17], [1 << 20] * 32,
                                  [(4 << 20) - 1] * 3 + [12345] * 50, [1 << 14] * 7 + [(1 << 14) + 1] * 7,
                                  [(1 << 24) + (1 << 20)] * 2,
                                  [0, 1, 15, 16, 17, 1023, 1024, 1025, 16383, 16384, 16385, 65535, 65536, 65537]
                                  + list(np.random.default_rng(9).integers(0, 300000, 498))])
def test_few_large_extents(torch_cuda, ctx, ctx_noseg, lens):
    """Fewer extents than the resident waves: segmented on the device
    (crc_seg_plan / segment CRCs / crc_seg_combine); must equal the
    one-wave-per-extent path and the oracle, at ragged offsets."""
    torch = torch_cuda
    lens = np.array(lens, dtype=np.uint32)
    rng = np.random.default_rng(int(lens.sum()) & 0xFFFF)
    n = int(lens.sum()) + 4096 * len(lens) + 4096
    t = _region(torch, ctx, n, SEED ^ 0x77, 3)
    offs, pos = [], 0
    for ln in lens:
        pos += int(rng.integers(0, 4096))
        offs.append(pos)
        pos += int(ln)
    o = np.array(offs, dtype=np.uint64)
    d_o = torch.from_numpy(o.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    got = _u32(ctx.ranges_dev(t, d_o, d_l))
    ref = _u32(ctx_noseg.ranges_dev(t, d_o, d_l))
    torch.cuda.synchronize()
    want = O.crc32_ranges(t[:n].cpu().numpy(), o, lens)
    assert np.array_equal(ref, want)
    assert np.array_equal(got, want)


def test_read_roof_dev(torch_cuda, ctx):
    """priskv_crc_read_roof_dev (diagnostic read roof of the CRC kernel's
    access pattern): every variant (the plan's own depth and occupancy, and
    2 / 3 / 4 chunks in flight at one or two workgroups per CU) runs for the
    plans bench.py measures (4 KiB, 64 KiB, 1 MiB incl. the split mode, few
    large blocks); each launched wave stores the XOR of its words in its own
    sink slot, so the XOR of the zeroed sink equals the XOR of the whole
    region's 32-bit words; odd sizes of the window mode read their 4 KiB
    windows; it refuses what it cannot mirror (other block sizes, unaligned
    bases, unknown variants)."""
    import errno
    from priskv_amd.crc import ROOF_SINK_WORDS, ROOF_VARIANTS
    torch = torch_cuda
    t = _region(torch, ctx, 256 << 20, SEED ^ 0x2F, 17)
    words = t[:256 << 20].view(torch.int32)
    want = int(np.bitwise_xor.reduce(words.cpu().numpy().view(np.uint32)))
    sink = torch.zeros(ROOF_SINK_WORDS, dtype=torch.int32, device="cuda")
    for bs in (4096, 65536, 1 << 20, 64 << 20, 256 << 20):
        nb = (256 << 20) // bs
        for v in range(ROOF_VARIANTS):
            sink.zero_()
            ctx.read_roof_dev(t, bs, sink, nblocks=nb, variant=v)
            torch.cuda.synchronize()
            got = int(np.bitwise_xor.reduce(sink.cpu().numpy().view(np.uint32)))
            assert got == want, (bs, v, hex(got), hex(want))
    tiles = _ctx_env(PRISKV_CRC_TILE_MIN_GIB="0")  # the block-cyclic tile order at any size
    try:
        for bs in (4096, 65536):
            nb = (256 << 20) // bs
            sink.zero_()
            tiles.read_roof_dev(t, bs, sink, nblocks=nb)
            torch.cuda.synchronize()
            got = int(np.bitwise_xor.reduce(sink.cpu().numpy().view(np.uint32)))
            assert got == want, ("tiles", bs, hex(got), hex(want))
    finally:
        tiles.close()
    # odd sizes the window mode takes (4 KiB windows): the roof reads each
    # block's window, the 4096 bytes ending at the 16-B boundary at or after
    # the block's end, so the sink's XOR is the XOR of those windows' words
    host = t[:256 << 20].cpu().numpy()
    for bs in (4095, 4097, 4100, 4111):
        nb = 30000
        ends = ((np.arange(1, nb + 1, dtype=np.int64) * bs + 15) // 16) * 16
        idx = (ends[:, None] - 4096 + np.arange(0, 4096, 4)[None, :]).reshape(-1)
        wwant = int(np.bitwise_xor.reduce(host[idx[:, None] + np.arange(4)].reshape(-1).view(np.uint32)))
        for v in range(ROOF_VARIANTS):
            sink.zero_()
            ctx.read_roof_dev(t, bs, sink, nblocks=nb, variant=v)
            torch.cuda.synchronize()
            got = int(np.bitwise_xor.reduce(sink.cpu().numpy().view(np.uint32)))
            assert got == wwant, ("window", bs, v, hex(got), hex(wwant))
    from priskv_amd.crc import lib
    for bs, off, v in ((1024, 0, 0), (5000, 0, 0), (4096, 4, 0), (4096, 0, ROOF_VARIANTS), (4095, 4, 0)):
        assert lib().priskv_crc_read_roof_dev(ctx.handle, t[off:].data_ptr(), 4, bs, v, sink.data_ptr(),
                                              None) == -errno.EINVAL
    with pytest.raises(ValueError):
        ctx.read_roof_dev(t, 4096, sink[:16], nblocks=4)


def test_verify_dev(torch_cuda, ctx):
    """Device verify: CRC each value where it landed and compare with the
    expected CRCs (the oracle's); corrupted values are counted and the first
    one is reported."""
    torch = torch_cuda
    n_bytes = 16 << 20
    t = _region(torch, ctx, n_bytes, SEED, 5)
    rng = np.random.default_rng(8)
    k = 5000
    lens = rng.integers(0, 9000, k).astype(np.uint32)
    offs = np.array([rng.integers(0, n_bytes - int(ln)) for ln in lens], dtype=np.uint64)
    want = O.crc32_ranges(t[:n_bytes].cpu().numpy(), offs, lens)
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    d_e = torch.from_numpy(want.view(np.int32)).cuda()
    st = ctx.verify_dev(t, d_o, d_l, d_e)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0, -1]
    # corrupt one byte inside three chosen values (not shared with value 0..9)
    bad = [4999, 1234, 777]
    for i in bad:
        if lens[i] == 0:
            lens[i] = 1
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    want = O.crc32_ranges(t[:n_bytes].cpu().numpy(), offs, lens)
    d_e = torch.from_numpy(want.view(np.int32)).cuda()
    for i in bad:
        t[int(offs[i]) + int(lens[i]) // 2] ^= 0x40
    got = _u32(ctx.ranges_dev(t, d_o, d_l))
    mism = np.nonzero(got != want)[0]
    st = ctx.verify_dev(t, d_o, d_l, d_e).cpu().tolist()
    assert st == [len(mism), int(mism[0])] and set(bad) <= set(mism.tolist())
    # priskv_crc32_verify_dev_bounded: the same status with a tight, a wrong
    # (too small) and an unknown bound, and on a few small values
    for bound in (int(lens.max()), 100, 0):
        assert ctx.verify_dev(t, d_o, d_l, d_e, max_len=bound).cpu().tolist() == st, bound
    few = [i for i in bad if lens[i] <= 9000][:2] + [0, 1, 2]
    sel = torch.tensor(few, dtype=torch.int64, device="cuda")
    fst = ctx.verify_dev(t, d_o[sel], d_l[sel], d_e[sel], max_len=9000).cpu().tolist()
    wrong = [j for j, i in enumerate(few) if i in set(mism.tolist())]
    assert fst == [len(wrong), wrong[0] if wrong else -1]
    # empty batch
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    st = ctx.verify_dev(t, e, e.to(torch.int32), e.to(torch.int32)).cpu().tolist()
    assert st == [0, -1]
    st = ctx.verify_dev(t, e, e.to(torch.int32), e.to(torch.int32), max_len=4096).cpu().tolist()
    assert st == [0, -1]


def test_set_completion_batcher(torch_cuda, ctx):
    """SET-completion batcher: 4 submitting threads, every value called back
    exactly once with the oracle's CRC; the deadline path (no flush); close()
    drains; out-of-range extents are refused."""
    import threading
    import time
    from priskv_amd import CrcBatcher
    region = O.fill_splitmix(64 << 20, SEED, 17)
    rng = np.random.default_rng(23)
    k = 12000
    lens = rng.integers(0, 20000, k).astype(np.uint32)
    offs = np.array([rng.integers(0, region.size - int(ln)) for ln in lens], dtype=np.uint64)
    want = O.crc32_ranges(region, offs, lens)
    got, lock = {}, threading.Lock()

    def cb(cookie, crc, status):
        with lock:
            assert cookie not in got
            got[cookie] = (crc, status)

    with CrcBatcher(ctx, region, cb, max_batch=700, max_delay_us=300) as b:
        def worker(t):
            if t % 2:  # vectored: a CQ poll's worth of completions per call
                idx = np.arange(t, k, 4)
                for c in range(0, idx.size, 16):
                    j = idx[c:c + 16]
                    b.submitv(offs[j], lens[j], j)
            else:
                for i in range(t, k, 4):
                    b.submit(int(offs[i]), int(lens[i]), i)
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        b.flush()
        assert len(got) == k
        assert all(got[i] == (int(want[i]), 0) for i in range(k))
        # deadline path: a partial batch is hashed without a flush
        got.clear()
        for i in range(3):
            b.submit(int(offs[i]), int(lens[i]), i)
        t0 = time.time()
        while len(got) < 3 and time.time() - t0 < 10:
            time.sleep(0.001)
        assert got == {i: (int(want[i]), 0) for i in range(3)}
        with pytest.raises(OSError):
            b.submit(region.size - 10, 11, 99)
        got.clear()
        for i in range(100):
            b.submit(int(offs[i]), int(lens[i]), i)
    assert len(got) == 100  # close() drained the queue


def test_ranges_beyond_2GiB_and_many_per_wave(torch_cuda, ctx):
    """Extents at offsets with bit 31 (and bit 32) set, and far more extents
    than waves so each wave loops over many of them (a sign-extension of the
    low offset half once faulted here)."""
    torch = torch_cuda
    n = (5 << 30) + 4096
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 11)
    rng = np.random.default_rng(12)
    k = 40000
    offs = rng.integers(0, n - 20000, k).astype(np.uint64)
    offs[:8] = [(1 << 31) - 5, 1 << 31, (1 << 31) + 17, (3 << 30) + 1, 1 << 32, (1 << 32) + 4095,
                n - 20000, 0]
    lens = rng.integers(0, 20000, k).astype(np.uint32)
    out = ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(), torch.from_numpy(lens.view(np.int32)).cuda())
    torch.cuda.synchronize()
    got = _u32(out)
    check = list(range(8)) + list(rng.integers(8, k, 300))
    for i in check:
        o, ln = int(offs[i]), int(lens[i])
        assert got[i] == O.crc32(t[o:o + ln].cpu().numpy()), (i, o, ln)
    del t


@pytest.fixture(scope="module")
def ctx_nobal(torch_cuda):
    """A context with the byte-balanced extents split off (PRISKV_CRC_BALANCE=0)."""
    import os
    from priskv_amd import CrcContext
    os.environ["PRISKV_CRC_BALANCE"] = "0"
    try:
        c = CrcContext(0)
    finally:
        del os.environ["PRISKV_CRC_BALANCE"]
    yield c
    c.close()


@pytest.mark.parametrize("k", [4096, 4097, 20000, 65536, 131071])
def test_ranges_balanced_split(torch_cuda, ctx, ctx_nobal, k):
    """A few extents per wave with very uneven lengths (0 B to 256 KiB): the
    byte-balanced split (crc_ext_cost_kernel + ext_boundary) must give every
    extent to exactly one wave -- the output is pre-filled with a sentinel,
    so a gap would show -- and the same CRCs as the count split and the
    oracle.  k spans one extent per wave to just below the 16-wave shape."""
    torch = torch_cuda
    n = 512 << 20
    t = _region(torch, ctx, n, SEED, 31)
    rng = np.random.default_rng(k)
    big = rng.random(k) < 0.05
    lens = np.where(big, rng.integers(64 << 10, 256 << 10, k), rng.integers(0, 6000, k)).astype(np.uint32)
    if k > 131000:
        lens = np.minimum(lens, 12000).astype(np.uint32)  # keep the oracle pass short
    lens[:4] = [0, 1, 256 << 10, 17]
    offs = rng.integers(0, n - (256 << 10), k).astype(np.uint64)
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    want = O.crc32_ranges(t[:n].cpu().numpy(), offs, lens)
    sentinel = int(np.int32(np.uint32(0xA5A5A5A5).view(np.int32)))
    for c in (ctx, ctx_nobal):
        out = torch.full((k,), sentinel, dtype=torch.int32, device="cuda")
        c.ranges_dev(t, d_o, d_l, out=out)
        torch.cuda.synchronize()
        got = _u32(out)
        assert np.array_equal(got, want), (k, np.nonzero(got != want)[0][:8])
    del t


def test_ranges_many_per_wave_shapes(torch_cuda, any_ctx):
    """Enough extents (>= 32 per resident wave) for the extents kernel's
    16-wave progress-priority shape, with ragged offsets and lengths 0-9000 B,
    against the oracle on every extent; the no-priority context runs the same
    call in two 8-wave workgroups per CU."""
    torch = torch_cuda
    ctx = any_ctx
    n = 96 << 20
    t = _region(torch, ctx, n, SEED, 21)
    rng = np.random.default_rng(22)
    k = 200_000
    lens = rng.integers(0, 9000, k).astype(np.uint32)
    lens[:6] = [0, 1, 15, 16, 1024, 8999]
    offs = rng.integers(0, n - 9000, k).astype(np.uint64)
    out = ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(), torch.from_numpy(lens.view(np.int32)).cuda())
    torch.cuda.synchronize()
    want = O.crc32_ranges(t[:n].cpu().numpy(), offs, lens)
    got = _u32(out)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]


@pytest.mark.parametrize("bs", [1028, 1024 + 64, 4100, 4104, 4096 + 52, 4096 + 64, 8196, 8192 + 52, 9220,
                                (12 << 10) + 52, (16 << 10) + 52, (64 << 10) + 4, (1 << 20) + 4])
def test_head_split_blocks(torch_cuda, ctx, bs):
    """Block sizes of whole KiB rows plus a 4-64 B head on 4-byte aligned
    bases: the rows kernel hashes the bodies in place (stride = block size)
    and crc_head_kernel adds each head's shifted CRC.  Against the oracle on
    every block, output pre-filled with a sentinel, at base offsets 0, 4 and
    12, for ragged block counts (and few large blocks, which keep the other
    paths), and against a context with the head split off."""
    torch = torch_cuda
    off_ctx = _ctx_env(PRISKV_CRC_HEADSPLIT=0)
    sentinel = int(np.int32(np.uint32(0xA5A5A5A5).view(np.int32)))
    for nb in sorted({1, 3, 65, 2049, max(1, (64 << 20) // bs) + 7}):
        t = _region(torch, ctx, bs * nb + 16, SEED ^ (bs * 3 + nb), nb)
        for shift in (0, 4, 12):
            view = t[shift:shift + bs * nb]
            plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
            want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=8)
            for c in (ctx, off_ctx):
                out = torch.full((nb,), sentinel, dtype=torch.int32, device="cuda")
                c.blocks_dev(view, bs, out=out)
                torch.cuda.synchronize()
                got = _u32(out)
                assert np.array_equal(got, want), (bs, nb, shift, plan, np.nonzero(got != want)[0][:8])
        if nb >= 2049 and bs < (16 << 10):  # bodies too short to segment: the head split, unless windows
            from priskv_amd import blocks_path
            want_path = blocks_path(t.data_ptr(), nb, bs)
            plan = ctx.blocks_plan(t.data_ptr(), nb, bs)
            assert ("crc_head_kernel" in plan) == (want_path == "headsplit"), plan
            assert ("windows" in plan) == (want_path == "window"), plan
        del t
    off_ctx.close()


@pytest.mark.parametrize("bs", [(1023 << 10) + 4, (127 << 10) + 64, (96 << 10) + 12])
def test_head_split_few_large_odd_kib_bodies(torch_cuda, ctx, bs):
    """A few head + body blocks whose body is an odd number of KiB >= 64 KiB:
    the rows kernel cannot cut such bodies into whole-KiB segments, so the
    batch must not take the head split (one wave per block would stream at a
    few GB/s) but the extents path, which the fused kernel segments.  Plan
    and every CRC against the oracle (sentinel-filled output), for 1 to 9
    blocks; a balanced batch of the same size does take the head split."""
    torch = torch_cuda
    sentinel = int(np.int32(np.uint32(0xA5A5A5A5).view(np.int32)))
    for nb in (1, 2, 9):
        t = _region(torch, ctx, bs * nb + 16, SEED ^ (bs + nb), nb)
        view = t[4:4 + bs * nb]
        plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
        assert "crc_head_kernel" not in plan and plan.startswith("crc_ranges_fused_kernel"), plan
        out = torch.full((nb,), sentinel, dtype=torch.int32, device="cuda")
        ctx.blocks_dev(view, bs, out=out)
        torch.cuda.synchronize()
        want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=8)
        got = _u32(out)
        assert np.array_equal(got, want), (bs, nb, np.nonzero(got != want)[0][:8])
        del t
    nbal = 2 * torch.cuda.get_device_properties(0).multi_processor_count * 8  # two blocks per rows-kernel wave
    body = bs - bs % 1024  # (round 5: the head split only on bodies of whole 4 KiB chunks)
    assert ("crc_head_kernel" in ctx.blocks_plan(4096, nbal, bs)) == (body % 4096 == 0)


def test_ranges_many_shape_chunk_sizes(torch_cuda, ctx):
    """The 16-wave many-extents shape sizes each wave's chunks from its own
    extents (8, 4 or 2 rows: crc_device.inc OPT bit 14).  Three populations
    of 65 536 extents, each a contiguous index range so that its waves pick
    one size: values of 2 blocks with ragged ends (8-row chunks), aligned
    4096-B extents (4-row chunks) and short values of 0-1500 B (2-row
    chunks); lengths around every 1 KiB row and 8 KiB chunk edge at all 16
    start phases are spread over the first two.  Every extent against the
    oracle, output pre-filled with a sentinel."""
    torch = torch_cuda
    n = 256 << 20
    t = _region(torch, ctx, n, SEED, 51)
    rng = np.random.default_rng(51)
    m = 65536
    nblk = n // 4096 - 8
    o8 = rng.integers(0, nblk, m).astype(np.uint64) * 4096
    l8 = (8192 - rng.integers(0, 4096, m)).astype(np.uint32)
    edges = [(k * 1024 + d, ph) for k in (1, 2, 4, 7, 8, 9, 15, 16, 17) for d in (-17, -16, -1, 0, 1, 15, 16)
             for ph in range(16)]
    for j, (ln, ph) in enumerate(edges):  # chunk and row edges in the first population
        l8[7 * j] = max(0, ln)
        o8[7 * j] = o8[7 * j] + ph
    o4 = rng.integers(0, nblk, m).astype(np.uint64) * 4096
    l4 = np.full(m, 4096, dtype=np.uint32)
    o2 = rng.integers(0, n - 2000, m).astype(np.uint64)
    l2 = rng.integers(0, 1500, m).astype(np.uint32)
    l2[:4] = [0, 1, 1024, 1499]
    offs = np.concatenate([o8, o4, o2])
    lens = np.concatenate([l8, l4, l2])
    sentinel = int(np.int32(np.uint32(0xA5A5A5A5).view(np.int32)))
    out = torch.full((3 * m,), sentinel, dtype=torch.int32, device="cuda")
    ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(), torch.from_numpy(lens.view(np.int32)).cuda(),
                   out=out)
    torch.cuda.synchronize()
    want = O.crc32_ranges(t[:n].cpu().numpy(), offs, lens)
    got = _u32(out)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    del t


@pytest.mark.parametrize("register", [False, True])
def test_ranges_host_scrub(torch_cuda, ctx, register):
    """Memfile-scrub form: extents of a host region read zero-copy over PCIe."""
    from priskv_amd import host_register, host_unregister
    bs = 4096
    region = O.fill_splitmix(bs * 4096, SEED, 3)  # 16 MiB "value region"
    rng = np.random.default_rng(8)
    # values start on block boundaries and span 2^k blocks with a ragged valuelen
    nval = 1500
    k = rng.integers(0, 4, nval)
    blk = rng.integers(0, 4096 - 8, nval)
    offs = (blk * bs).astype(np.uint64)
    lens = np.minimum(rng.integers(1, (1 << k) * bs + 1), (4096 - blk) * bs).astype(np.uint32)
    lens[:4] = [0, 1, 16, bs]
    if register:
        host_register(region)
    try:
        got = ctx.ranges_host(region, offs, lens)
    finally:
        if register:
            host_unregister(region)
    assert np.array_equal(got, O.crc32_ranges(region, offs, lens))
    with pytest.raises(OSError):
        ctx.ranges_host(region, np.array([region.size - 1], np.uint64), np.array([2], np.uint32))


def test_multi_gpu_host_paths(torch_cuda, ctx):
    """Multi-GPU host-resident forms with 2-3 contexts (all on the visible
    device(s); on the 8-GPU node each context is its own GPU)."""
    from priskv_amd import CrcContext, blocks_host_multi, host_register, host_unregister, ranges_host_multi
    ndev = torch_cuda.cuda.device_count()
    ctxs = [CrcContext(i % ndev) for i in range(3)]
    try:
        bs = 4096
        host = O.fill_splitmix(bs * 20011, SEED, 9)
        want = O.crc32_blocks(host, bs, nthreads=8)
        assert np.array_equal(blocks_host_multi(ctxs, host, bs), want)
        host_register(host)
        try:
            assert np.array_equal(blocks_host_multi(ctxs[:2], host, bs), want)
            rng = np.random.default_rng(3)
            offs = (rng.integers(0, 20000, 5000) * bs).astype(np.uint64)
            lens = rng.integers(0, 3 * bs, 5000).astype(np.uint32)
            lens = np.minimum(lens, (host.size - offs)).astype(np.uint32)
            assert np.array_equal(ranges_host_multi(ctxs, host, offs, lens), O.crc32_ranges(host, offs, lens))
        finally:
            host_unregister(host)
        # unregistered region: registered once for all devices inside the call
        offs = np.array([0, 4096, 123], np.uint64)
        lens = np.array([4096, 100, 5000], np.uint32)
        assert np.array_equal(ranges_host_multi(ctxs[:2], host, offs, lens), O.crc32_ranges(host, offs, lens))
        with pytest.raises(OSError):
            blocks_host_multi([ctxs[0], ctxs[0]], host, bs)  # same context twice
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("pinned", [False, True])
def test_blocks_host_streamed(torch_cuda, ctx, pinned):
    from priskv_amd import host_register, host_unregister
    bs = 4096
    nb = (200 << 20) // bs + 3  # > 3 chunks of 64 MiB, ragged tail
    host = O.fill_splitmix(bs * nb, SEED, 5)
    if pinned:
        host_register(host)
    try:
        got = ctx.blocks_host(host, bs)
    finally:
        if pinned:
            host_unregister(host)
    assert np.array_equal(got, O.crc32_blocks(host, bs, nthreads=8))


def test_blocks_host_odd_sizes(torch_cuda, ctx):
    for bs, nb in ((100, 1000), (1 << 20, 5), (64, 7)):
        host = O.fill_splitmix(bs * nb, SEED, 1)
        assert np.array_equal(ctx.blocks_host(host, bs), O.crc32_blocks(host, bs))


def test_stream_argument(torch_cuda, ctx):
    torch = torch_cuda
    s = torch.cuda.Stream()
    bs, nb = 65536, 300
    with torch.cuda.stream(s):
        t = _region(torch, ctx, bs * nb)
        out = ctx.blocks_dev(t, bs, stream=s)
    s.synchronize()
    assert np.array_equal(_u32(out), O.crc32_blocks(t.cpu().numpy()[: bs * nb], bs, nthreads=8))


@pytest.mark.parametrize("pool,nstreams", [("1", 3), ("1", 12), ("0", 3)])
def test_scratch_pool_across_streams(torch_cuda, pool, nstreams):
    """Calls that need scratch (segmented extents, segmented large blocks,
    verify) enqueued back to back on several streams with no host sync between
    them, with growing sizes: each pooled slot serves the stream that took it
    first, in that stream's order; with 12 streams there are more streams
    than slots and the rest allocate per call (PRISKV_CRC_SCRATCH_POOL=0:
    per-call alloc/free always).  Every output must equal the oracle's."""
    import os
    torch = torch_cuda
    from priskv_amd import CrcContext
    os.environ["PRISKV_CRC_SCRATCH_POOL"] = pool
    try:
        c = CrcContext(0)
    finally:
        del os.environ["PRISKV_CRC_SCRATCH_POOL"]
    try:
        nbytes = 96 << 20
        region = _region(torch, c, nbytes, SEED ^ 0x9001, 2)
        torch.cuda.synchronize()
        host = region[:nbytes].cpu().numpy()
        rng = np.random.default_rng(9001)
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        calls = []
        for i in range(18):
            k = 1 + i % 6
            lens = rng.integers(1 << 20, 12 << 20, k).astype(np.uint32)
            offs = np.array([rng.integers(0, nbytes - int(ln)) for ln in lens], dtype=np.uint64)
            calls.append((offs, lens, torch.from_numpy(offs.astype(np.int64)).cuda(),
                          torch.from_numpy(lens.view(np.int32)).cuda()))
        want = [O.crc32_ranges(host, o, ln) for o, ln, _, _ in calls]
        bs_big = 16 << 20
        want_blocks = O.crc32_blocks(host[: bs_big * 4], bs_big, nthreads=4)
        torch.cuda.synchronize()
        outs = []
        for i, (o, ln, d_o, d_l) in enumerate(calls):
            st = streams[i % nstreams]
            with torch.cuda.stream(st):
                a = c.ranges_dev(region, d_o, d_l, stream=st)
                b = c.blocks_dev(region, bs_big, nblocks=1 + i % 4, stream=st)
                exp = torch.from_numpy(want[i].view(np.int32)).to("cuda", non_blocking=False)
                v = c.verify_dev(region, d_o, d_l, exp, stream=st)
            outs.append((a, b, v))
        torch.cuda.synchronize()
        for i, (a, b, v) in enumerate(outs):
            assert np.array_equal(_u32(a), want[i]), (pool, i)
            assert np.array_equal(_u32(b), want_blocks[: 1 + i % 4]), (pool, i)
            assert int(v[0]) == 0 and int(v[1]) == -1, (pool, i, v.tolist())
    finally:
        c.close()


def test_concurrent_streams_and_threads(torch_cuda, ctx):
    """One context shared by 4 host threads, each on its own stream, each
    mixing calls that need stream-ordered scratch (segmented extents, segmented
    large blocks) with plain ones; every result must equal the oracle's
    (contexts are immutable, *_dev calls may run concurrently)."""
    import threading
    torch = torch_cuda
    region = _region(torch, ctx, 48 << 20, SEED ^ 0xC0, 1)
    torch.cuda.synchronize()
    host = region[: 48 << 20].cpu().numpy()
    rng = np.random.default_rng(12)
    jobs = []
    for k in range(4):
        lens = rng.integers(1, 4 << 20, 6).astype(np.uint32)
        offs = np.array([rng.integers(0, (48 << 20) - int(ln)) for ln in lens], dtype=np.uint64)
        jobs.append((offs, lens, 1 << 20, 3 + k))
    want = [(O.crc32_ranges(host, o, ln), O.crc32_blocks(host[: bs * nb], bs, nthreads=4),
             O.crc32_blocks(host[:4096 * 1000], 4096, nthreads=4)) for o, ln, bs, nb in jobs]
    got = [None] * len(jobs)
    errs = []

    def run(k):
        try:
            o, ln, bs, nb = jobs[k]
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):  # inputs copied on the stream that reads them
                d_o = torch.from_numpy(o.astype(np.int64)).cuda()
                d_l = torch.from_numpy(ln.view(np.int32)).cuda()
            res = []
            for _ in range(5):
                with torch.cuda.stream(s):
                    a = ctx.ranges_dev(region, d_o, d_l, stream=s)
                    b = ctx.blocks_dev(region, bs, nblocks=nb, stream=s)
                    c = ctx.blocks_dev(region, 4096, nblocks=1000, stream=s)
                s.synchronize()
                res.append((_u32(a), _u32(b), _u32(c)))
            got[k] = res
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for k in range(len(jobs)):
        for a, b, c in got[k]:
            assert np.array_equal(a, want[k][0]) and np.array_equal(b, want[k][1]) and np.array_equal(c, want[k][2])


def test_threads_sharing_one_stream(torch_cuda, ctx):
    """4 host threads enqueue scratch-needing calls (segmented extents, split
    few large blocks, fused) on ONE shared stream with no host sync between
    them: pooled slots are owned per stream, so the calls in flight hold
    different slots of that stream (or allocate per call) and stream order
    keeps each slot's uses apart.  Every result must equal the oracle's."""
    import threading
    torch = torch_cuda
    region = _region(torch, ctx, 96 << 20, SEED ^ 0xD1, 1)
    torch.cuda.synchronize()
    host = region[: 96 << 20].cpu().numpy()
    rng = np.random.default_rng(31)
    shared = torch.cuda.Stream()
    shared.wait_stream(torch.cuda.current_stream())
    jobs = []
    for k in range(4):
        lens = rng.integers(1 << 20, 8 << 20, 3 + k).astype(np.uint32)
        offs = np.array([rng.integers(0, (96 << 20) - int(ln)) for ln in lens], dtype=np.uint64)
        jobs.append((offs, lens, torch.from_numpy(offs.astype(np.int64)).cuda(),
                     torch.from_numpy(lens.view(np.int32)).cuda()))
    torch.cuda.synchronize()
    want = [O.crc32_ranges(host, o, ln) for o, ln, _, _ in jobs]
    want_b = O.crc32_blocks(host[: 32 << 20], 16 << 20, nthreads=4)
    got, errs = [None] * len(jobs), []

    def run(k):
        try:
            _, _, d_o, d_l = jobs[k]
            res = []
            for _ in range(6):
                with torch.cuda.stream(shared):
                    res.append((ctx.ranges_dev(region, d_o, d_l, stream=shared),
                                ctx.blocks_dev(region, 16 << 20, nblocks=2, stream=shared)))
            got[k] = res
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    shared.synchronize()
    assert not errs, errs
    for k in range(len(jobs)):
        for a, b in got[k]:
            assert np.array_equal(_u32(a), want[k]) and np.array_equal(_u32(b), want_b), k


def test_hip_graph_capture_and_replay(torch_cuda, ctx):
    """The *_dev calls are pure stream work (kernels, stream-ordered scratch):
    they capture into a HIP graph and replay on new data with correct results --
    the rows plan, the segmented rows path (few large blocks: scratch + combine)
    and the segmented extents path (plan / segments / reduce)."""
    torch = torch_cuda
    n = 40 << 20
    t = _region(torch, ctx, n, SEED ^ 0x6A, 2)
    offs = np.array([5, 3 << 20, 20 << 20], dtype=np.uint64)
    lens = np.array([(3 << 20) - 9, 17 << 20, 100], dtype=np.uint32)
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    o1 = torch.empty(1000, dtype=torch.int32, device="cuda")
    o2 = torch.empty(2, dtype=torch.int32, device="cuda")
    o3 = torch.empty(3, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside capture
        ctx.blocks_dev(t, 4096, out=o1, nblocks=1000, stream=s)
        ctx.blocks_dev(t, 16 << 20, out=o2, nblocks=2, stream=s)
        ctx.ranges_dev(t, d_o, d_l, out=o3, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream()
        ctx.blocks_dev(t, 4096, out=o1, nblocks=1000, stream=st)
        ctx.blocks_dev(t, 16 << 20, out=o2, nblocks=2, stream=st)
        ctx.ranges_dev(t, d_o, d_l, out=o3, stream=st)
    for seed in (11, 12):
        ctx.fill_splitmix(t, seed, 0)
        g.replay()
        torch.cuda.synchronize()
        host = t[:n].cpu().numpy()
        assert np.array_equal(_u32(o1), O.crc32_blocks(host[: 4096 * 1000], 4096, nthreads=8))
        assert np.array_equal(_u32(o2), O.crc32_blocks(host[: 32 << 20], 16 << 20, nthreads=8))
        assert np.array_equal(_u32(o3), O.crc32_ranges(host, offs, lens))


def test_bad_args_on_gpu(torch_cuda, ctx):
    from priskv_amd.crc import lib
    L = lib()
    assert L.priskv_crc32_blocks_dev(ctx.handle, None, 5, 4096, None, None) == -22
    assert L.priskv_crc32_blocks_dev(ctx.handle, None, 0, 4096, None, None) == 0
    assert L.priskv_crc32_blocks_dev(ctx.handle, 16, 5, 0, 16, None) == -22
    import ctypes
    h = ctypes.c_void_p()
    assert L.priskv_crc_ctx_create(4096, ctypes.byref(h)) == -19
    # the binding refuses host or strided pointer arguments before they reach a kernel
    torch = torch_cuda
    t = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    o = torch.zeros(4, dtype=torch.int64)
    ln = torch.full((4,), 16, dtype=torch.int32)
    for bad in ((o, ln.cuda()), (o.cuda(), ln), (o.cuda()[::2], ln.cuda()[::2])):
        with pytest.raises(ValueError):
            ctx.ranges_dev(t, *bad)
    with pytest.raises(ValueError):
        ctx.verify_dev(t, o.cuda(), ln.cuda(), torch.zeros(4, dtype=torch.int32))
    with pytest.raises(ValueError):
        ctx.fill_splitmix(t, 1, nbytes=(1 << 16) + 1)
    with pytest.raises(ValueError):
        ctx.ranges_dev(t.cpu(), o.cuda(), ln.cuda())


@pytest.mark.slow
def test_full_size_properties(torch_cuda, ctx):
    """Size-independent properties at the BASELINE sizes, no CPU oracle:
    linearity (init 0 / xorout 0: crc(a ^ b) == crc(a) ^ crc(b)) over 1 Mi x
    4 KiB blocks, and combine consistency: the CRC of each 8 KiB block equals
    combine(crc(first 4 KiB), crc(second 4 KiB), 4096) from the 4 KiB batch of
    the same bytes (different kernel plans on each side)."""
    from priskv_amd import crc32_shift
    torch = torch_cuda
    bs, nb = 4096, 1 << 20
    a = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    ctx.fill_splitmix(a, SEED, 0)
    ctx.fill_splitmix(b, SEED + 1, 0)
    ca, cb = ctx.blocks_dev(a, bs), ctx.blocks_dev(b, bs)
    torch.bitwise_xor(a, b, out=b)
    cx = ctx.blocks_dev(b, bs)
    torch.cuda.synchronize()
    assert np.array_equal(_u32(cx), _u32(ca) ^ _u32(cb))
    # combine: Z_4096 applied to the first half's CRC as a GF(2) matrix on the host
    c4 = _u32(ca)
    c8 = _u32(ctx.blocks_dev(a, 2 * bs))
    torch.cuda.synchronize()
    cols = np.array([crc32_shift(1 << i, bs) for i in range(32)], dtype=np.uint32)
    first = c4[0::2]
    shifted = np.zeros_like(first)
    for i in range(32):
        shifted ^= np.where((first >> np.uint32(i)) & np.uint32(1), cols[i], np.uint32(0)).astype(np.uint32)
    assert np.array_equal(c8, shifted ^ c4[1::2])
    del a, b


@pytest.mark.slow
def test_full_config_1M_x_4K(torch_cuda, ctx):
    """BASELINE config 2: 1 Mi x 4 KiB = 4 GiB device-resident, every block
    checked against the oracle run on a D2H copy."""
    torch = torch_cuda
    bs, nb = 4096, 1 << 20
    t = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 0)
    out = ctx.blocks_dev(t, bs)
    torch.cuda.synchronize()
    host = t.cpu().numpy()
    want = O.crc32_blocks(host, bs, nthreads=16)
    assert np.array_equal(_u32(out), want)


# (block size, blocks): balanced batches with few blocks per wave; 1900 x
# 1 MiB gives fewer units per wave than units per block (waves whose whole
# range lies inside one block)
_SPLIT_CASES = [(1 << 20, 1900), (1 << 20, 4096), (512 << 10, 4000), (256 << 10, 6000), (1 << 20, 2048),
                # few large blocks: the 3-deep plan, units down to one 4 KiB chunk, 32 per wave
                (256 << 20, 1), (16 << 20, 16), (1 << 20, 1000), (32 << 20, 8),
                # ... or from 4 per wave, without the XCD weights (32-256 MiB batches)
                (64 << 10, 512), (128 << 10, 1000), (1 << 20, 100), (12 << 20, 3),
                # ... but not below 4 units per wave (the fused kernel)
                (4 << 20, 3), (12 << 20, 1)]


def test_verify_graph_capture(torch_cuda, ctx):
    """verify_dev captured into a HIP graph: its status words are set by a
    write-through init kernel and then only updated by atomics, so replays
    back to back report exactly the mismatches of the current data."""
    torch = torch_cuda
    n = 64 << 20
    t = _region(torch, ctx, n, SEED ^ 0x7E, 1)
    rng = np.random.default_rng(77)
    cnt = 5000  # many values: the plain extents path
    lens = rng.integers(1, 16 << 10, cnt).astype(np.uint32)
    offs = np.array([rng.integers(0, n - int(ln)) for ln in lens], dtype=np.uint64)
    d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    want = O.crc32_ranges(t[:n].cpu().numpy(), offs, lens)
    exp = torch.from_numpy(want.view(np.int32)).cuda()
    status = torch.empty(2, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx.verify_dev(t, d_o, d_l, exp, status=status, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ctx.verify_dev(t, d_o, d_l, exp, status=status, stream=torch.cuda.current_stream())
    for bad in ([], [4321], [17, 4000, 4999]):
        e = want.copy()
        for i in bad:
            e[i] ^= 1
        exp.copy_(torch.from_numpy(e.view(np.int32)))
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        st = status.tolist()
        assert st[0] == len(bad) and st[1] == (min(bad) if bad else -1), (bad, st)


def test_rows_split_mode_graph_capture(torch_cuda, ctx):
    """Split mode under HIP graph capture: its zero-at-rest counters come from
    stream-ordered scratch (allocated and zeroed inside the graph), and every
    replay on new data is exact -- a balanced 1 MiB batch and one 256 MiB block
    (the few-large-blocks plan), captured into one graph."""
    torch = torch_cuda
    n = 1900 << 20
    t = _region(torch, ctx, n, SEED ^ 0x5B1, 3)
    big = t[: 256 << 20]
    o1 = torch.empty(1900, dtype=torch.int32, device="cuda")
    o2 = torch.empty(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx.blocks_dev(t, 1 << 20, out=o1, nblocks=1900, stream=s)
        ctx.blocks_dev(big, 256 << 20, out=o2, nblocks=1, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream()
        ctx.blocks_dev(t, 1 << 20, out=o1, nblocks=1900, stream=st)
        ctx.blocks_dev(big, 256 << 20, out=o2, nblocks=1, stream=st)
    for seed in (21, 22):
        ctx.fill_splitmix(t, seed, 0)
        g.replay()
        g.replay()  # back to back: the counters are left zero by each launch
        torch.cuda.synchronize()
        host = t[:n].cpu().numpy()
        want = O.crc32_blocks(host, 1 << 20, nthreads=16)
        got = _u32(o1)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (seed, len(bad), bad[:16].tolist(), got[bad[:4]].tolist(), want[bad[:4]].tolist())
        assert np.array_equal(_u32(o2), O.crc32_blocks(host[: 256 << 20], 256 << 20, nthreads=16))


@pytest.mark.parametrize("bs,nb", _SPLIT_CASES)
def test_rows_split_mode(torch_cuda, ctx, bs, nb):
    """crc_rows_kernel's split mode (OPT bit 6): few blocks per wave cut into
    units so the XCD weights apply; parts of blocks combine through two
    zero-at-rest words per block inside the launch.  Every CRC against the
    oracle, sentinel-filled output, three launches back to back (the scratch
    must be left zero), and against a context with the split off."""
    torch = torch_cuda
    t = _region(torch, ctx, bs * nb, SEED ^ (bs + nb), 3)
    view = t[:bs * nb]
    plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
    xcd = "xcd-weighted" in ctx.blocks_plan(view.data_ptr(), 1 << 20, 4096)  # the probe saw round-robin XCDs
    waves = torch.cuda.get_device_properties(0).multi_processor_count * 8
    unbal = nb * 10 < 9 * waves
    S = 1  # units per block: power-of-two cuts of whole 4 KiB chunks, toward 32 per wave
    while nb * S < 32 * waves and (bs // 4096) % (2 * S) == 0:
        S *= 2
    few = unbal and nb * S >= 4 * waves  # unbalanced, and at least 4 units per wave
    assert ("split" in plan) == (few or (xcd and not unbal)), plan
    assert ("few large blocks" in plan) == few, plan
    want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=16)
    off = _ctx_env(PRISKV_CRC_SPLIT=0)
    try:
        assert "split" not in off.blocks_plan(view.data_ptr(), nb, bs)
        sentinel = int(np.int32(np.uint32(0xA5A5A5A5).view(np.int32)))
        for c in (ctx, ctx, ctx, off):
            out = torch.full((nb,), sentinel, dtype=torch.int32, device="cuda")
            c.blocks_dev(view, bs, out=out)
            torch.cuda.synchronize()
            got = _u32(out)
            assert np.array_equal(got, want), (bs, nb, plan, np.nonzero(got != want)[0][:8])
    finally:
        off.close()


@pytest.mark.slow
@pytest.mark.parametrize("bs", [65536, 1 << 20])
def test_full_sweep_4GiB(torch_cuda, ctx, bs):
    """BASELINE config 3 (sweep): 4 GiB of 64 KiB or 1 MiB blocks, all checked."""
    torch = torch_cuda
    nb = (4 << 30) // bs
    t = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED ^ bs, 0)
    out = ctx.blocks_dev(t, bs)
    torch.cuda.synchronize()
    want = O.crc32_blocks(t.cpu().numpy(), bs, nthreads=16)
    assert np.array_equal(_u32(out), want)


@pytest.mark.slow
def test_tib_config_per_gpu_shard(torch_cuda, ctx):
    """BASELINE configs[3]: one GPU's 2 Mi x 64 KiB = 128 GiB shard of the
    16 Mi x 64 KiB (1 TiB, 8-GPU) region, filled on the device exactly as
    bench.py's `tib` leg fills rank 7's shard (word offset of block 14 Mi).

    - sampled blocks vs the CPU oracle: first, last and every 4096th block
      (offsets up to 128 GiB, so bit 31 .. bit 36 of the byte offset are set);
    - full size, no oracle: combine consistency -- every 128 KiB block's CRC
      equals combine(crc(first 64 KiB), crc(second 64 KiB), 64 KiB) from the
      64 KiB batch of the same bytes (another plan, G64 over 128 rows);
    - full size, no oracle: linearity (init 0 / xorout 0) -- XOR-ing the same
      constant block C into every block XORs crc(C) into every CRC."""
    from priskv_amd import crc32_shift
    from priskv_amd.shard import shard_blocks, shard_word_offset
    torch = torch_cuda
    bs, per_gpu, world, rank = 65536, 1 << 21, 8, 7
    first, nb = shard_blocks(world * per_gpu, rank, world)
    t = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, shard_word_offset(first, bs))
    c64 = ctx.blocks_dev(t, bs)
    torch.cuda.synchronize()
    idx = np.unique(np.concatenate([np.arange(0, nb, 4096), [1, nb - 2, nb - 1]])).astype(np.int64)
    ti = torch.from_numpy(idx).cuda()
    blocks = t.view(nb, bs).index_select(0, ti).cpu().numpy()
    got = _u32(c64.index_select(0, ti))
    want = O.crc32_blocks(blocks.reshape(-1), bs, nthreads=8)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    # the sampled bytes are the oracle generator's (the fill is pinned too)
    assert np.array_equal(blocks[-1], O.fill_splitmix(bs, SEED, shard_word_offset(first + nb - 1, bs)))
    # combine consistency over the whole shard
    a = _u32(c64)
    c128 = _u32(ctx.blocks_dev(t, 2 * bs))
    torch.cuda.synchronize()
    cols = np.array([crc32_shift(1 << i, bs) for i in range(32)], dtype=np.uint32)
    lo = a[0::2]
    sh = np.zeros_like(lo)
    for i in range(32):
        sh ^= np.where((lo >> np.uint32(i)) & np.uint32(1), cols[i], np.uint32(0)).astype(np.uint32)
    assert np.array_equal(c128, sh ^ a[1::2])
    # linearity over the whole shard, in place
    C = O.fill_splitmix(bs, SEED ^ 0xC0FFEE, 3)
    crc_c = O.crc32(C)
    tv = t.view(nb, bs)
    cd = torch.from_numpy(C).cuda()
    for k in range(0, nb, 1 << 17):  # 8 GiB at a time keeps the temporaries small
        tv[k:k + (1 << 17)].bitwise_xor_(cd)
    cx = _u32(ctx.blocks_dev(t, bs))
    torch.cuda.synchronize()
    assert np.array_equal(cx, a ^ np.uint32(crc_c))
    del t, tv, c64
    torch.cuda.empty_cache()


def _ctx_env(**env):
    """A context created with the given PRISKV_CRC_* environment (read at creation)."""
    import os
    from priskv_amd import CrcContext
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return CrcContext(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("bs", [1024, 4096, 8192, 65536])
def test_xcd_weights_probe_fallback_and_tiles(torch_cuda, ctx, bs):
    """The XCD-weighted split (workgroup b assumed on XCD b % 8, checked by a
    probe at context creation), an override, equal shares, the probe's forced
    fallback, and block-cyclic tiles (forced on, small tiles so the last one
    is short) give the oracle's CRCs; the plan string says which split each
    context uses.  The batches hold >= 32 groups per resident wave, the size
    from which the library applies the weights."""
    torch = torch_cuda
    per = 64 // {1024: 16, 4096: 64, 8192: 64, 65536: 64}[bs]  # blocks per group of the plan
    nb = 32 * 2048 * per + 5 * per + (per if bs == 65536 else 0)
    if bs == 65536:
        nb = 16 * 2048 + 3  # 2 GiB: weights need 4 GiB here, tiles are the point
    t = _region(torch, ctx, bs * nb, SEED ^ bs ^ 0x3C, nb)
    want = O.crc32_blocks(t[: bs * nb].cpu().numpy(), bs, nthreads=16)
    ctxs = {"default": ctx, "1:1": _ctx_env(PRISKV_CRC_XCD_WEIGHTS="1:1"),
            "17:13": _ctx_env(PRISKV_CRC_XCD_WEIGHTS="17:13"), "fallback": _ctx_env(PRISKV_CRC_XCD_PROBE="0"),
            "tiles": _ctx_env(PRISKV_CRC_TILE_MIN_GIB="0", PRISKV_CRC_TILE_KIB=str(max(64, 4 * bs >> 10)))}
    plans = {}
    for name, c in ctxs.items():
        got = _u32(c.blocks_dev(t, bs, nblocks=nb))
        torch.cuda.synchronize()
        assert np.array_equal(got, want), (name, np.nonzero(got != want)[0][:8])
        plans[name] = c.blocks_plan(t.data_ptr(), nb, bs)
    assert "xcd-weighted" not in plans["1:1"] and "xcd-weighted" not in plans["fallback"], plans
    assert "block-cyclic" in plans["tiles"] and "xcd-weighted" not in plans["tiles"], plans
    if bs != 65536:
        assert "xcd-weighted 17:13" in plans["17:13"], plans
        # MI355X dispatches workgroups round-robin over its 8 XCDs: the probe agrees
        assert "xcd-weighted 31:29" in plans["default"], plans
    for name in ("1:1", "17:13", "fallback", "tiles"):
        ctxs[name].close()


def test_blocks_plan_strings(torch_cuda, ctx):
    """priskv_crc32_blocks_plan names the kernel blocks_dev launches."""
    base = 1 << 20  # any 16-B aligned address: the plan does not dereference it
    # 4 KiB: 4 chunks in flight from 1 GiB per call, 3 below
    assert ctx.blocks_plan(base, 1 << 20, 4096).startswith("crc_rows_kernel<G=64,CH=4,NBUF=4,nt,pipelined-fold,"
                                                             "nibble-fold,progress-priority 3")
    assert ctx.blocks_plan(base, 1 << 16, 4096).startswith("crc_rows_kernel<G=64,CH=4,NBUF=3,nt,pipelined-fold,"
                                                             "nibble-fold,progress-priority 3")
    assert ctx.blocks_plan(base, 1 << 16, 65536).startswith("crc_rows_kernel<G=64,CH=4,NBUF=2,nt,progress-priority 1")
    # the 128 GiB shard of BASELINE configs[3] runs in block-cyclic 1 MiB tiles
    assert "block-cyclic tiles of 16 groups" in ctx.blocks_plan(base, 1 << 21, 65536)
    assert ctx.blocks_plan(base, 1, 1 << 20).startswith("crc_ranges_fused_kernel")  # few large blocks
    assert ctx.blocks_plan(base + 1, 3, (3 << 20) + 5).startswith("crc_ranges_fused_kernel")
    assert ctx.blocks_plan(base, 20000, 1 << 20).startswith("crc_rows_kernel")  # balanced: whole blocks
    # unbalanced large blocks that can be cut into 32 units per wave: the
    # rows kernel's split mode on the 3-deep plan (one launch)
    assert "few large blocks" in ctx.blocks_plan(base, 1000, 1 << 20)
    assert "few large blocks" in ctx.blocks_plan(base, 1, 256 << 20)
    # ... else segments + combine
    assert "crc_combine_segments_kernel" in ctx.blocks_plan(base, 1000, (1 << 20) + 2048)
    assert ctx.blocks_plan(base, 100, 256) == "crc_small_kernel<G=16,byte-fold>"
    # odd sizes or bases near a multiple of 4 KiB: the rows kernel on windows
    for bs, mis in ((4096, 1), (4100, 1), (4095, 0), (4097, 8)):
        assert ctx.blocks_plan(base + mis, 100, bs) == (
            "crc_rows_kernel<G=64,CH=4,NBUF=3,nt,pipelined-fold,nibble-fold,progress-priority 3,window> (4096-B "
            "windows ending at the 16-B boundary after each block, corrected as each 64 CRCs are stored)"), (bs, mis)
    assert ctx.blocks_plan(base + 1, 100, 8193).startswith("crc_rows_kernel<G=64,CH=4,NBUF=2,nt,nibble-fold,"
                                                           "progress-priority 1,window> (8192-B windows")
    # other odd sizes and unaligned bases: the uniform-stride kernel
    assert ctx.blocks_plan(base + 1, 100, 4200).startswith("crc_stride_kernel<G=32,CH=8,NBUF=2,nt,progress-priority 3> "
                                                           "(9 rows of 512 B "
                                                           "per block, 408 B in front)")
    # whole KiB rows + a 49-64 B head on a 4-byte aligned base (4-48 B: the
    # window mode, above): rows kernel + head terms
    assert ctx.blocks_plan(base, 100, 12340) == ("crc_rows_kernel<G=64,CH=4,NBUF=2,nt,progress-priority 1> on the "
                                                 "12288-B bodies + crc_head_kernel (52-B heads)")
    assert "(4096-B windows" in ctx.blocks_plan(base, 100, 4100)
    assert ctx.blocks_plan(base, 100, 520).startswith("crc_stride_kernel<G=16,CH=8,NBUF=2,nt,progress-priority 3> (3 rows of 256 B")
    assert ctx.blocks_plan(base, 100, 100).startswith("crc_stride_kernel<G=8,CH=8,NBUF=2,nt,byte-fold,progress-priority 3> (1 rows of 128 B")
    # the extents kernel from 9 KiB, odd sizes and multiples of 4 alike
    assert ctx.blocks_plan(base, 100, 4609).startswith("crc_stride_kernel<G=32,CH=8,NBUF=2,nt,progress-priority 3>")
    assert ctx.blocks_plan(base, 100, 9100).startswith("crc_stride_kernel<")
    assert ctx.blocks_plan(base, 100, 9217) == "crc_ranges_kernel (extents)"
    assert ctx.blocks_plan(base, 100, 2049).startswith("crc_rows_kernel<G=16,CH=4,NBUF=2,nt,progress-priority 1,"
                                                      "window> (2048-B windows")
    assert ctx.blocks_plan(base, 100, 1025).startswith("crc_rows_kernel<G=16,CH=4,NBUF=2,nt,pipelined-fold,"
                                                      "nibble-fold,progress-priority 1,window> (1024-B windows")
    assert ctx.blocks_plan(base, 100, 9281) == "crc_ranges_kernel (extents)"
    assert ctx.blocks_plan(base, 100, 9212).startswith("crc_stride_kernel<G=32,CH=8,NBUF=2,nt,progress-priority 3> (18 rows of 512 B")
    assert ctx.blocks_plan(base, 100, 8700).startswith("crc_stride_kernel<G=32,CH=8,NBUF=2,nt,progress-priority 3> (17 rows of 512 B")
    assert ctx.blocks_plan(base, 100, 9300) == "crc_ranges_kernel (extents)"
    assert "crc_head_kernel (52-B heads)" in ctx.blocks_plan(base, 100, 16436)
    assert ctx.blocks_plan(base, 100, 9220) == "crc_ranges_kernel (extents)"
    assert ctx.blocks_plan(base, 100, 15) == "crc_generic_kernel"


def test_ranges_host_concurrent_temporary_registration(torch_cuda):
    """Two threads, two contexts, one region nobody registered: every call
    registers it temporarily through the library's shared registry, so one
    caller's unregister can never pull the mapping from under the other's
    kernel, and concurrent registrations never fail with -EEXIST.  The
    region is left unregistered afterwards."""
    import threading
    from priskv_amd import CrcContext, host_register, host_unregister
    region = O.fill_splitmix(32 << 20, SEED, 41)
    rng = np.random.default_rng(41)
    jobs = []
    for _ in range(2 * 12):
        lens = rng.integers(0, 300000, 400).astype(np.uint32)
        offs = np.array([rng.integers(0, region.size - int(ln)) for ln in lens], dtype=np.uint64)
        jobs.append((offs, lens, O.crc32_ranges(region, offs, lens)))
    ctxs = [CrcContext(0), CrcContext(0)]
    errors = []

    def worker(t):
        try:
            for j in range(t, len(jobs), 2):
                offs, lens, want = jobs[j]
                got = ctxs[t].ranges_host(region, offs, lens)
                if not np.array_equal(got, want):
                    errors.append((t, j, "mismatch"))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for c in ctxs:
        c.close()
    assert not errors, errors[:4]
    host_register(region)  # would raise EEXIST if a temporary registration had leaked
    host_unregister(region)


def test_ranges_host_overlapping_subranges(torch_cuda):
    """Three threads scrub views of one unregistered region: the whole
    region, its first 20 MiB and everything from 12 MiB on (views with other
    base pointers, which overlap each other without either containing the
    other).  A view inside a live temporary registration must take a
    reference on it (else the owner's unregister pulls the mapping from
    under the view's kernel), and an overlapping view must wait for it
    instead of failing.  No registration may leak."""
    import threading
    from priskv_amd import CrcContext, host_register, host_unregister
    region = O.fill_splitmix(32 << 20, SEED, 47)
    views = [(0, region.size), (0, 20 << 20), (12 << 20, region.size)]
    rng = np.random.default_rng(47)
    jobs = []
    for t, (a, b) in enumerate(views):
        v = region[a:b]
        for _ in range(10):
            lens = rng.integers(0, 200000, 300).astype(np.uint32)
            offs = np.array([rng.integers(0, v.size - int(ln)) for ln in lens], dtype=np.uint64)
            jobs.append((t, offs, lens, O.crc32_ranges(v, offs, lens)))
    ctxs = [CrcContext(0) for _ in views]
    errors = []

    def worker(t):
        a, b = views[t]
        v = region[a:b]
        try:
            for tt, offs, lens, want in jobs:
                if tt != t:
                    continue
                got = ctxs[t].ranges_host(v, offs, lens)
                if not np.array_equal(got, want):
                    errors.append((t, "mismatch"))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(len(views))]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th), "a scrub never returned (registry wait)"
    for c in ctxs:
        c.close()
    assert not errors, errors[:4]
    host_register(region)  # would raise EEXIST if a temporary registration had leaked
    host_unregister(region)


def test_batcher_flush_while_others_submit(torch_cuda, ctx):
    """flush() returns only after every value its thread submitted before it
    has been called back, while other threads keep submitting (the gather
    generation rule of crc_batch.cpp)."""
    import threading
    from priskv_amd import CrcBatcher
    region = O.fill_splitmix(16 << 20, SEED, 43)
    rng = np.random.default_rng(43)
    k = 4000
    lens = rng.integers(0, 9000, k).astype(np.uint32)
    offs = np.array([rng.integers(0, region.size - int(ln)) for ln in lens], dtype=np.uint64)
    want = O.crc32_ranges(region, offs, lens)
    got, lock, errors = {}, threading.Lock(), []

    def cb(cookie, crc, status):
        with lock:
            got[cookie] = (crc, status)

    with CrcBatcher(ctx, region, cb, max_batch=256, max_delay_us=5000) as b:
        def worker(t):
            mine = []
            for c in range(t * 1000, (t + 1) * 1000, 25):
                idx = np.arange(c, c + 25)
                b.submitv(offs[idx], lens[idx], idx)
                mine.extend(idx.tolist())
                if (c // 25) % 4 == t % 4:  # flush now and then, others keep submitting
                    b.flush()
                    with lock:
                        missing = [i for i in mine if i not in got]
                    if missing:
                        errors.append((t, len(missing)))
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        b.flush()
    assert not errors, errors[:4]
    assert len(got) == k and all(got[i] == (int(want[i]), 0) for i in range(k))


def test_blocks_host_partially_registered(torch_cuda, ctx):
    """A registration that covers only the first half of the batch: the
    streamed path must not DMA the unregistered half as if it were pinned
    (it takes the bounce path) -- same CRCs as the oracle."""
    from priskv_amd import host_register, host_unregister
    bs = 4096
    nb = (96 << 20) // bs
    host = O.fill_splitmix(bs * nb, SEED, 47)
    half = host[: (nb // 2) * bs]
    host_register(half)
    try:
        got = ctx.blocks_host(host, bs)
    finally:
        host_unregister(half)
    assert np.array_equal(got, O.crc32_blocks(host, bs, nthreads=8))


@pytest.fixture(scope="module")
def ctx_threelaunch(torch_cuda):
    """Few extents through the three-launch segmented path (plan kernel,
    extents kernel, reduce kernel): PRISKV_CRC_FUSED=0, read at creation."""
    c = _ctx_env(PRISKV_CRC_FUSED=0, PRISKV_CRC_SEG_MAX_EXTENTS=16384)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_fused16k(torch_cuda):
    c = _ctx_env(PRISKV_CRC_SEG_MAX_EXTENTS=16384)
    yield c
    c.close()


_FUSED_CASES = [
    [256 << 20],                                  # a lone huge value: every workgroup holds part of it
    [(1 << 14) + 1],                              # two segments, the last one byte
    [0],                                          # a lone empty extent
    [0] * 300,                                    # only empty extents
    [5 << 20, 0, 7, (3 << 20) + 1, 0],            # split and whole extents mixed
    [1 << 20] * 32,
    [(64 << 20) + 3] * 3 + [100] * 1000,          # few large among many small
    [4096] * 4096,                                # small values: kept whole
    [4100] * 8192,
    [(1 << 14) * 37 + 11] * 700,                  # extents straddling wave and workgroup edges
    [(1 << 20) + 1] * 64,                         # the largest wave-planned call, split
    [(1 << 20) + 1] * 65,                         # the smallest workgroup-planned one
]


@pytest.mark.parametrize("case", range(len(_FUSED_CASES) + 2))
def test_fused_few_extents(torch_cuda, ctx_fused16k, ctx_threelaunch, case):
    """The one-launch few-extents kernel (plan in LDS, per-extent counters,
    last-arriver combine) equals the oracle and the three-launch path, at
    ragged offsets on a 16-B-misaligned base, called repeatedly (the counters
    it leaves must read zero for the next call) -- and the counters survive
    alternating shapes."""
    torch = torch_cuda
    rng = np.random.default_rng(4242 + case)
    if case < len(_FUSED_CASES):
        lens = np.array(_FUSED_CASES[case], dtype=np.uint32)
    elif case == len(_FUSED_CASES):
        lens = rng.integers(0, 40000, 16384).astype(np.uint32)   # the extent limit
        lens[rng.integers(0, 16384, 50)] = 0
    else:
        lens = rng.integers(0, 3 << 19, 257).astype(np.uint32)
    n = int(lens.sum()) + 64 * len(lens) + 4096
    t = _region(torch, ctx_fused16k, n + 3, SEED ^ (0xF5 + case), 1)
    base = t[3:]                                  # 16-B misaligned base (shift 3)
    offs, pos = [], 0
    for ln in lens:
        pos += int(rng.integers(0, 64))
        offs.append(pos)
        pos += int(ln)
    o = np.array(offs, dtype=np.uint64)
    d_o = torch.from_numpy(o.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    want = O.crc32_ranges(base[:n].cpu().numpy(), o, lens)
    for c in [ctx_fused16k, ctx_threelaunch]:
        for _ in range(3):
            got = _u32(c.ranges_dev(base, d_o, d_l))
            torch.cuda.synchronize()
            assert np.array_equal(got, want), (case, np.nonzero(got != want)[0][:8])
    # a different shape in between, then the same call again
    small = _u32(ctx_fused16k.ranges_dev(base, d_o[:1], d_l[:1]))
    torch.cuda.synchronize()
    assert small[0] == want[0]
    got = _u32(ctx_fused16k.ranges_dev(base, d_o, d_l))
    torch.cuda.synchronize()
    assert np.array_equal(got, want)


_MANY_WG_CASES = [
    ("blocks", [48 << 20] * 5),                   # blocks straddling groups of 16 workgroups, XCD-weighted units
    ("blocks", [32 << 20] * 7),
    ("blocks", [256 << 20]),                      # every group shares the lone block
    ("ranges", [40 << 20, (3 << 20) + 5, 100 << 20, 1024, (77 << 20) + 1]),
    ("ranges", [(9 << 20) + 3] * 11),
    ("ranges", [256 << 20]),
]


def test_many_workgroup_finish(torch_cuda, ctx):
    """finish_shared (crc_device.inc) for items shared by many workgroups:
    blocks / values across groups of workgroups (partial at both ends), and
    lone items with a share in every workgroup, on the merging split plan and
    the fused kernel's wave plan.  Each call three times back to back and
    interleaved with the other shapes (the zero-at-rest words must be left
    zero), every CRC against the oracle.  (Round 6 also ran these cases on a
    two-level finish through per-group words, tools/patches/finish_two_level.patch:
    exact, and 0.3-0.5 us slower per call, so not kept.)"""
    torch = torch_cuda
    total = max(sum(ls) + 64 * len(ls) for _, ls in _MANY_WG_CASES) + 4096
    t = _region(torch, ctx, total + 5, SEED ^ 0x2F1, 1)
    host = t[:total + 5].cpu().numpy()
    rng = np.random.default_rng(77)
    calls = []
    for kind, ls in _MANY_WG_CASES:
        lens = np.array(ls, dtype=np.uint32)
        if kind == "blocks":
            bs, nb = int(lens[0]), len(lens)
            assert "few large blocks" in ctx.blocks_plan(t.data_ptr(), nb, bs)  # the merging split plan
            want = O.crc32_blocks(host[:bs * nb], bs, nthreads=16)
            calls.append((lambda bs=bs, nb=nb: ctx.blocks_dev(t, bs, nblocks=nb), want))
        else:
            offs, pos = [], 5
            for ln in lens:
                pos += int(rng.integers(0, 64))
                offs.append(pos)
                pos += int(ln)
            o = np.array(offs, dtype=np.uint64)
            d_o = torch.from_numpy(o.astype(np.int64)).cuda()
            d_l = torch.from_numpy(lens.view(np.int32)).cuda()
            want = O.crc32_ranges(host, o, lens)
            calls.append((lambda d_o=d_o, d_l=d_l: ctx.ranges_dev(t, d_o, d_l), want))
    for rnd in range(2):
        order = list(range(len(calls))) if rnd == 0 else list(reversed(range(len(calls))))
        for i in order:
            fn, want = calls[i]
            for _ in range(3):
                got = _u32(fn())
                torch.cuda.synchronize()
                assert np.array_equal(got, want), (_MANY_WG_CASES[i], np.nonzero(got != want)[0][:8])


@pytest.mark.parametrize("case", ["tiny", "small_mixed", "wrong_bound", "large_bound", "huge_bound", "unknown"])
def test_ranges_dev_bounded(torch_cuda, ctx, case):
    """priskv_crc32_ranges_dev_bounded: max_len steers the launch only, so
    every result equals the oracle whether the bound is tight, loose, wrong
    (smaller than some lengths), beyond u32 or 0 (unknown); a 16-B-misaligned
    base, zero lengths included, called twice."""
    torch = torch_cuda
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    if case == "tiny":
        lens, bound = np.full(16, 4096, np.uint32), 4096
    elif case == "small_mixed":
        lens = rng.integers(0, 5000, 300).astype(np.uint32)
        bound = int(lens.max())
    elif case == "wrong_bound":  # the bound says 1 KiB, two values are MiBs
        lens = rng.integers(0, 1024, 40).astype(np.uint32)
        lens[[3, 17]] = [(1 << 20) + 7, 3 << 20]
        bound = 1024
    elif case == "large_bound":  # few large values: the segmented (fused) path
        lens = np.array([(8 << 20) + 3, 0, 100, 5 << 20], np.uint32)
        bound = int(lens.max())
    elif case == "huge_bound":
        lens = rng.integers(0, 70000, 100).astype(np.uint32)
        bound = 1 << 40
    else:
        lens = rng.integers(0, 9000, 64).astype(np.uint32)
        bound = 0
    n = int(lens.sum()) + 64 * len(lens) + 4096
    t = _region(torch, ctx, n + 3, SEED ^ 0xB0, 1)
    base = t[3:]
    offs, pos = [], 0
    for ln in lens:
        pos += int(rng.integers(0, 64))
        offs.append(pos)
        pos += int(ln)
    o = np.array(offs, dtype=np.uint64)
    d_o = torch.from_numpy(o.astype(np.int64)).cuda()
    d_l = torch.from_numpy(lens.view(np.int32)).cuda()
    want = O.crc32_ranges(base[:n].cpu().numpy(), o, lens)
    for _ in range(2):
        got = _u32(ctx.ranges_dev(base, d_o, d_l, max_len=bound))
        torch.cuda.synchronize()
        assert np.array_equal(got, want), (case, np.nonzero(got != want)[0][:8])


@pytest.mark.parametrize("bs,nb", [((3 << 20) + 5, 3), (4100 * 64, 17), ((1 << 24) + 1, 1)])
def test_fused_constant_length_blocks(torch_cuda, ctx, bs, nb):
    """Blocks that are not whole 1 KiB rows (the extents path with one length
    and a stride): few large ones take the fused kernel with no lengths array."""
    torch = torch_cuda
    t = _region(torch, ctx, bs * nb, SEED ^ 0xC0, 1)
    got = _u32(ctx.blocks_dev(t, bs, nblocks=nb))
    torch.cuda.synchronize()
    want = O.crc32_blocks(t[: bs * nb].cpu().numpy(), bs, nthreads=8)
    assert np.array_equal(got, want), (bs, nb)


@pytest.mark.parametrize("kind", ["block_3GiB", "extent_2GiB_plus", "extent_near_4GiB"])
def test_fused_single_value_beyond_2GiB(torch_cuda, ctx, kind):
    """One value of 2-4 GiB through the fused kernel: a few-large-blocks call
    (3 GiB block), and ranges at offsets beyond 4 GiB with lengths past 2^31
    and up to 2^32 - 5 (u32 lengths, segment and shift arithmetic at the top
    of their range)."""
    torch = torch_cuda
    if kind == "block_3GiB":
        bs = 3 << 30
        t = _region(torch, ctx, bs, SEED ^ 0x3, 0)
        assert "few large blocks" in ctx.blocks_plan(t.data_ptr(), 1, bs)  # the rows kernel's split mode
        got = _u32(ctx.blocks_dev(t, bs, nblocks=1))
        torch.cuda.synchronize()
        want = O.crc32_blocks(t[:bs].cpu().numpy(), bs, nthreads=8)
        assert np.array_equal(got, want)
        del t
    else:
        ln = (2 << 30) + 4096 + 3 if kind == "extent_2GiB_plus" else (1 << 32) - 5
        off = (4 << 30) + 7
        n_bytes = off + ln + 64
        t = _region(torch, ctx, n_bytes, SEED ^ 0x4, 0)
        offs = np.array([off, 5], dtype=np.uint64)
        lens = np.array([ln, 100], dtype=np.uint32)
        got = _u32(ctx.ranges_dev(t, torch.from_numpy(offs.astype(np.int64)).cuda(),
                                  torch.from_numpy(lens.view(np.int32)).cuda()))
        torch.cuda.synchronize()
        host = t[: off + ln].cpu().numpy()
        want = O.crc32_ranges(host, offs, lens)
        assert np.array_equal(got, want), (kind, got, want)
        del t, host
    torch.cuda.empty_cache()


# (G, block sizes whose cost-model plan is G lanes per block): G < 16 only
# with one row per block; G = 64 never wins below the 9 KiB limit
_STRIDE_SIZES = {2: [16, 17, 23, 32], 4: [33, 48, 50, 64], 8: [65, 100, 127, 128],
                 16: [129, 255, 257, 520, 700], 32: [769, 1000, 1006, 4200, 8301, 9100]}


@pytest.mark.parametrize("G", sorted(_STRIDE_SIZES))
def test_stride_kernel_every_g_and_variant(torch_cuda, ctx, G):
    """crc_stride_kernel (odd block sizes, unaligned bases) for every lane
    count G the cost model picks, byte fold (G <= 8) or nibble fold, aligned
    or funnel-shift loads: the oracle's CRCs at base misalignments 0, 3 and
    4, for batches of 1 block, a ragged last group, and several groups per
    wave with a ragged end.  (Round 5 removed the forced-G and size-limit
    test hooks and the measured-slower variants they reached.)"""
    torch = torch_cuda
    per = 64 // G
    rng = np.random.default_rng(G)
    for bs in _STRIDE_SIZES[G]:
        big = max(per + 1, min((24 << 20) // bs, 3 * 2048 * per + per // 2 + 1))
        for nb in (1, per + 1, big):
            fast = bs % 1024 == 0 or (bs & (bs - 1) == 0 and bs <= 512)  # aligned: rows / sub-KiB kernels
            mis = int(rng.choice([3, 4] if fast else [0, 3, 4]))
            t = _region(torch, ctx, bs * nb + 16, SEED ^ (bs * 131 + nb), nb)
            view = t[mis: mis + bs * nb]
            want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=8)
            plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
            assert plan.startswith(f"crc_stride_kernel<G={G},"), plan
            # a sentinel-filled output: a CRC the kernel fails to store shows
            out = torch.full((nb,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
            got = _u32(ctx.blocks_dev(view, bs, out=out, nblocks=nb))
            torch.cuda.synchronize()
            assert np.array_equal(got, want), (G, bs, nb, mis, np.nonzero(got != want)[0][:8])
            del t


@pytest.mark.parametrize("misalign", [0, 1, 2, 3, 4, 8, 13])
def test_stride_kernel_cost_model_sizes(torch_cuda, ctx, misalign):
    """Odd sizes through the default plan (cost model), 16 B to 1 MiB - 1, at
    every kind of base misalignment: bit-exact with the oracle; blocks of 16 B
    and 4 KiB on unaligned bases (once extents / generic) included."""
    torch = torch_cuda
    sizes = [16, 31, 40, 96, 100, 200, 500, 520, 999, 1000, 1500, 2000, 3000, 4096, 4100, 5000, 9999,
             65535, 100000, (1 << 20) - 1]
    for bs in sizes:
        nb = max(3, min(4099, (16 << 20) // bs))
        t = _region(torch, ctx, bs * nb + 16, SEED ^ (bs + misalign), 7)
        view = t[misalign: misalign + bs * nb]
        out = torch.full((nb,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")  # unwritten CRCs show
        got = _u32(ctx.blocks_dev(view, bs, out=out, nblocks=nb))
        torch.cuda.synchronize()
        want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=8)
        assert np.array_equal(got, want), (bs, nb, misalign, np.nonzero(got != want)[0][:8])


# block sizes within W - 15 .. W + 48 B of W = 4, 8, 12, 16 KiB: window mode
_WINDOW_SIZES = [4081, 4095, 4096, 4097, 4099, 4111, 4112, 4127, 4144, 8177, 8191, 8193, 8240, 12287, 12300,
                 16369, 16383, 16385, 16432,
                 8239,
                 # other whole-KiB W up to 6 KiB (G = 16: four blocks per wave group), sizes
                 # or bases not multiples of 4, B > W or W = 1 KiB
                 1009, 1023, 1025, 1071, 1072, 2049, 3073, 5121, 6145]


@pytest.mark.parametrize("bs", _WINDOW_SIZES)
def test_window_blocks(torch_cuda, ctx, bs):
    """Odd sizes (or 4 KiB on odd bases) near a multiple W of 4 KiB: the rows
    kernel hashes each block's W-byte window ending at the 16-B boundary
    after the block, masking the window's bytes outside the block (front and
    tail) and hashing the block's bytes before the window (head) as one more
    row, then unshifts by the tail pad.  Against the oracle
    on every block, output pre-filled with a sentinel, at base offsets that
    put the first block's window start before the base, at it and after it,
    for 1, 2, 65 and 2049 blocks and a ~48 MiB batch; and against a context
    with the window mode off."""
    torch = torch_cuda
    off_ctx = _ctx_env(PRISKV_CRC_WINDOW=0)
    sentinel = int(np.int32(np.uint32(0xA5A5A5A5).view(np.int32)))
    W = (bs + 15) // 1024 * 1024
    G = 64 if W % 4096 == 0 else 16
    for nb in sorted({1, 2, 65, 2049, (48 << 20) // bs + 3}):
        t = _region(torch, ctx, bs * nb + 32, SEED ^ (bs * 5 + nb), nb)
        for shift in (1, 3, 8, 13, 15) if bs % 1024 == 0 else (0, 1, 7, 12, 15):
            view = t[shift:shift + bs * nb]
            plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
            from priskv_amd import blocks_path
            if blocks_path(view.data_ptr(), nb, bs) == "window":  # (else a multiple of 4 the stride kernel takes)
                assert plan.startswith(f"crc_rows_kernel<G={G},") and f"{W}-B windows" in plan, (bs, shift, plan)
            else:
                assert G == 16 and bs % 4 == 0 and (view.data_ptr() & 3) == 0, (bs, shift, plan)
            want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=8)
            for c in (ctx, off_ctx) if nb <= 2049 else (ctx,):
                out = torch.full((nb,), sentinel, dtype=torch.int32, device="cuda")
                c.blocks_dev(view, bs, out=out)
                torch.cuda.synchronize()
                got = _u32(out)
                assert np.array_equal(got, want), (bs, nb, shift, plan, np.nonzero(got != want)[0][:8])
        del t
    off_ctx.close()


@pytest.mark.parametrize("bs,shift,nb,kernel", [(4095, 3, (1 << 18) + 77, "crc_rows_kernel<G=64,CH=4,NBUF=4,"),
                                                (4097, 0, (1 << 18) + 77, "crc_rows_kernel<G=64,CH=4,NBUF=4,"),
                                                (4111, 9, (1 << 18) + 77, "crc_rows_kernel<G=64,CH=4,NBUF=4,"),
                                                (1025, 5, (1 << 18) + 78, "crc_rows_kernel<G=16,CH=4,NBUF=2,nt,pipelined"),
                                                (2049, 0, 300003, "crc_rows_kernel<G=16,CH=4,NBUF=2,nt,progress")])
def test_window_blocks_deep_plan(torch_cuda, ctx, bs, shift, nb, kernel):
    """Window mode on large batches: the deep 4 KiB plan (>= 2^18 blocks:
    four chunks in flight), and the G = 16 plans with >= 32 groups per
    resident wave, where the XCD weights split the groups; every CRC against
    the oracle -- every wave's range ends in a partial group of 64 blocks
    and starts from a carried granule loaded before its loop, and a ragged
    tail of < 4 blocks (G = 16) goes to the stride kernel."""
    torch = torch_cuda
    t = _region(torch, ctx, bs * nb + 32, SEED ^ (bs * 7 + shift), 3)
    view = t[shift:shift + bs * nb]
    plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
    W = (bs + 15) // 1024 * 1024
    assert plan.startswith(kernel) and f"{W}-B windows" in plan and ",window,xcd-weighted 31:29>" in plan, plan
    got = _u32(ctx.blocks_dev(view, bs, nblocks=nb))
    torch.cuda.synchronize()
    want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=16)
    assert np.array_equal(got, want), (bs, shift, np.nonzero(got != want)[0][:8])
    del t, view
    torch.cuda.empty_cache()


@pytest.mark.slow
@pytest.mark.parametrize("bs,nb,mis,kind", [(4607, 1000000, 1, "crc_stride_kernel<"),
                                             (4100, 1100000, 5, "window")])
def test_stride_and_window_beyond_4GiB(torch_cuda, ctx, bs, nb, mis, kind):
    """Batches past 4 GiB on odd bases, so group pointers pass 2^32: 4607-B
    blocks (the stride kernel) and 4100-B blocks (window mode since round 5):
    sampled blocks (first, last, every 4096th) against the oracle, and the
    batch equals the same batch run as two halves."""
    torch = torch_cuda
    t = _region(torch, ctx, bs * nb + 16, SEED ^ bs, 0)
    view = t[mis: mis + bs * nb]
    plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
    assert kind in plan, plan
    got = ctx.blocks_dev(view, bs, nblocks=nb)
    idx = np.unique(np.concatenate([np.arange(0, nb, 4096), [nb - 1]])).astype(np.int64)
    blocks = view.view(nb, bs).index_select(0, torch.from_numpy(idx).cuda()).cpu().numpy()
    want = O.crc32_blocks(blocks.reshape(-1), bs, nthreads=8)
    assert np.array_equal(_u32(got)[idx], want)
    h = nb // 2 + 1
    a = ctx.blocks_dev(view, bs, nblocks=h)
    b = ctx.blocks_dev(view[h * bs:], bs, nblocks=nb - h)
    torch.cuda.synchronize()
    assert torch.equal(got, torch.cat([a, b]))
    del t, view, got, a, b
    torch.cuda.empty_cache()


# noseg: segmentation off
@pytest.mark.parametrize("bs,nb,mis,kind,noseg", [((64 << 20) - 3, 3, 1, "crc_ranges_fused_kernel", False),
                                               ((64 << 20) - 4, 3, 4, "crc_ranges_kernel (extents)", True),
                                               ((64 << 20) + 5, 2, 0, "crc_ranges_fused_kernel", False),
                                               ((5 << 20) + 7, 400, 2, "crc_ranges_kernel (extents)", True),
                                               (4607, 6000, 1, "crc_stride_kernel<G=32,", False),
                                               (4609, 6000, 0, "crc_stride_kernel<G=32,", False),
                                               (9217, 3000, 0, "crc_ranges_kernel (extents)", False),
                                               (9400, 3000, 0, "crc_ranges_kernel (extents)", False),
                                               (16460, 3000, 0, "crc_ranges_kernel (extents)", False),
                                               (16388, 3000, 0, "crc_rows_kernel<G=64,", False),
                                               (4100, 2049, 4, "crc_rows_kernel<G=64,", False)])
def test_stride_kernel_large_and_limit_blocks(torch_cuda, ctx, ctx_noseg, bs, nb, mis, kind, noseg):
    """Blocks at both sides of the stride kernel's 9 KiB limit and far past
    it: 64 MiB (a few such blocks are cut into segments by the fused kernel,
    or with segmentation off hashed whole by the extents kernel), 2 GB
    batches of 5 MiB + 7 B blocks, and sizes of whole KiB rows + a 4-B
    head, which the head split hands to the rows kernel: the oracle's
    CRCs."""
    torch = torch_cuda
    ctx = ctx_noseg if noseg else ctx
    t = _region(torch, ctx, bs * nb + 16, SEED ^ (bs + nb), 5)
    view = t[mis: mis + bs * nb]
    plan = ctx.blocks_plan(view.data_ptr(), nb, bs)
    assert plan.startswith(kind), plan
    got = _u32(ctx.blocks_dev(view, bs, nblocks=nb))
    torch.cuda.synchronize()
    want = O.crc32_blocks(view.cpu().numpy(), bs, nthreads=16)
    assert np.array_equal(got, want), (bs, nb, np.nonzero(got != want)[0][:8])
    del t, view
    torch.cuda.empty_cache()
