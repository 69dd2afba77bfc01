"""GPU parity of the paths whose cross-workgroup finish uses zero-at-rest
scratch (the fused few-extents kernel, the rows kernel's split mode, verify's
status words, the three-launch segmented path) under HIP-graph replay, and of
the scratch pool under the stream shapes a server uses (hipStreamPerThread
from many threads, streams created and destroyed per connection).

Every replay is checked against the oracle (oracle/crc_oracle.c, pinned to
the reference's server/crc.c in test_oracle.py).  Graphs are replayed back to
back on new data: round 4's split-mode bug (4 of 1900 blocks wrong, dirty L2
lines of a plain-store zero kernel written back over the next launch's
memory-side atomics) was only visible that way.
"""
import ctypes
import threading

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x5EED0505
MIB = 1 << 20


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _ctx_env(**env):
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


@pytest.fixture(scope="module")
def ctx(torch_cuda):
    from priskv_amd import CrcContext
    c = CrcContext(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_threelaunch(torch_cuda):
    c = _ctx_env(PRISKV_CRC_FUSED=0)
    yield c
    c.close()


def _u32(t):
    from priskv_amd import as_u32
    return as_u32(t)


def _extents(n, region_bytes, max_len, seed):
    """n extents of 0 .. max_len bytes at random (any-alignment) offsets."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len + 1, n).astype(np.uint32)
    lens[: min(n, 2)] = [max_len, 0][: min(n, 2)]  # the longest and an empty one
    offs = np.array([rng.integers(0, region_bytes - int(ln) + 1) for ln in lens], dtype=np.uint64)
    return offs, lens


def _dev(torch, offs, lens):
    return (torch.from_numpy(offs.astype(np.int64)).cuda(), torch.from_numpy(lens.view(np.int32)).cuda())


# (name, extents, longest extent): the fused kernel's plans -- the wave plan
# up to 64 extents (a few large ones, and many smaller), the LDS prefix above
# (rounds 4-5 also ran an 8-wave shape up to 16 extents; round 6 dropped it)
_FUSED_SHAPES = [("fused<=16", 3, 24 * MIB), ("fused17-64", 40, 2 * MIB), ("fused>64", 300, 512 << 10)]


@pytest.mark.parametrize("name,n,max_len", _FUSED_SHAPES)
def test_graph_fused_back_to_back(torch_cuda, ctx, name, n, max_len):
    """ranges_dev on the fused kernel captured into a graph (scratch and its
    zeroing inside the graph), replayed three times back to back per refill."""
    torch = torch_cuda
    region = 64 * MIB
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 0)
    offs, lens = _extents(n, region, max_len, 7 + n)
    d_o, d_l = _dev(torch, offs, lens)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx.ranges_dev(t, d_o, d_l, out=out, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ctx.ranges_dev(t, d_o, d_l, out=out, stream=torch.cuda.current_stream())
    for seed in (31, 32, 33):
        ctx.fill_splitmix(t, seed, 0)
        out.fill_(-1)
        g.replay()
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        want = O.crc32_ranges(t.cpu().numpy(), offs, lens)
        got = _u32(out)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (name, seed, len(bad), bad[:8].tolist())


def test_graph_segmented_three_launch_back_to_back(torch_cuda, ctx_threelaunch):
    """The three-launch segmented extents path (plan, segments, reduce;
    PRISKV_CRC_FUSED=0) under graph replay, back to back."""
    torch = torch_cuda
    region = 64 * MIB
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx_threelaunch.fill_splitmix(t, SEED, 0)
    offs, lens = _extents(24, region, 6 * MIB, 99)
    d_o, d_l = _dev(torch, offs, lens)
    out = torch.empty(24, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx_threelaunch.ranges_dev(t, d_o, d_l, out=out, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ctx_threelaunch.ranges_dev(t, d_o, d_l, out=out, stream=torch.cuda.current_stream())
    for seed in (41, 42):
        ctx_threelaunch.fill_splitmix(t, seed, 0)
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(_u32(out), O.crc32_ranges(t.cpu().numpy(), offs, lens)), seed


def test_graph_verify_few_extents_back_to_back(torch_cuda, ctx):
    """verify_dev with few extents (the fused kernel into scratch, then the
    compare kernel's status atomics over agent-scope-initialised status
    words) under graph replay, back to back, matching and mismatching."""
    torch = torch_cuda
    region = 64 * MIB
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 0)
    offs, lens = _extents(5, region, 9 * MIB, 5)
    d_o, d_l = _dev(torch, offs, lens)
    expected = torch.empty(5, dtype=torch.int32, device="cuda")
    status = torch.empty(2, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx.verify_dev(t, d_o, d_l, expected, status=status, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ctx.verify_dev(t, d_o, d_l, expected, status=status, stream=torch.cuda.current_stream())
    for seed, flip in ((51, None), (52, 3), (53, 1)):
        ctx.fill_splitmix(t, seed, 0)
        want = O.crc32_ranges(t.cpu().numpy(), offs, lens)
        e = want.copy()
        if flip is not None:
            e[flip] ^= np.uint32(0x10)
        expected.copy_(torch.from_numpy(e.view(np.int32)))
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        st = status.cpu().numpy().view(np.uint64)
        if flip is None:
            assert st[0] == 0 and st[1] == np.uint64(2**64 - 1), st
        else:
            assert st[0] == 1 and st[1] == flip, (flip, st)


def test_graph_mixed_split_and_fused_back_to_back(torch_cuda, ctx):
    """One graph holding a split-mode call (few large blocks: zero-at-rest
    counters), a balanced split call (1 MiB blocks), a fused ranges call and a
    fused lone block, each drawing captured scratch; replayed back to back."""
    torch = torch_cuda
    region = 1900 * MIB
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    ctx.fill_splitmix(t, SEED, 0)
    few = t[: 64 * MIB]
    offs, lens = _extents(7, 64 * MIB, 10 * MIB, 3)
    d_o, d_l = _dev(torch, offs, lens)
    o_few = torch.empty(4, dtype=torch.int32, device="cuda")
    o_bal = torch.empty(1900, dtype=torch.int32, device="cuda")
    o_rng = torch.empty(7, dtype=torch.int32, device="cuda")
    o_odd = torch.empty(1, dtype=torch.int32, device="cuda")
    odd = (12 * MIB) + 1  # a lone odd-size block: the fused kernel
    plans = [ctx.blocks_plan(few.data_ptr(), 4, 16 * MIB), ctx.blocks_plan(t.data_ptr(), 1900, MIB),
             ctx.blocks_plan(t.data_ptr(), 1, odd)]
    assert "few large blocks" in plans[0] and "fused" in plans[2], plans

    def calls(st):
        ctx.blocks_dev(few, 16 * MIB, out=o_few, nblocks=4, stream=st)
        ctx.ranges_dev(few, d_o, d_l, out=o_rng, stream=st)
        ctx.blocks_dev(t, MIB, out=o_bal, nblocks=1900, stream=st)
        ctx.blocks_dev(t, odd, out=o_odd, nblocks=1, stream=st)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        calls(s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        calls(torch.cuda.current_stream())
    for seed in (61, 62):
        ctx.fill_splitmix(t, seed, 0)
        for o in (o_few, o_bal, o_rng, o_odd):
            o.fill_(-1)
        g.replay()
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        host = t.cpu().numpy()
        assert np.array_equal(_u32(o_few), O.crc32_blocks(host[: 64 * MIB], 16 * MIB, nthreads=8)), seed
        assert np.array_equal(_u32(o_rng), O.crc32_ranges(host[: 64 * MIB], offs, lens)), seed
        want = O.crc32_blocks(host, MIB, nthreads=16)
        got = _u32(o_bal)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (seed, len(bad), bad[:8].tolist(), [hex(x) for x in got[bad[:4]]],
                               [hex(x) for x in want[bad[:4]]])
        assert np.array_equal(_u32(o_odd), O.crc32_blocks(host[:odd], odd)), seed


HIP_STREAM_PER_THREAD = 2  # hip_runtime_api.h: hipStreamPerThread


def test_per_thread_default_stream_from_many_threads(torch_cuda, ctx):
    """Several host threads call split-mode and fused paths on
    hipStreamPerThread -- one handle naming a different stream on each
    thread.  The scratch pool keys its slots by (handle, thread), so no two
    threads' in-flight calls share zero-at-rest counters: every CRC exact."""
    torch = torch_cuda
    nthreads, iters = 6, 4
    region = 64 * MIB
    ts = [torch.empty(region, dtype=torch.uint8, device="cuda") for _ in range(nthreads)]
    outs = [(torch.empty(4, dtype=torch.int32, device="cuda"), torch.empty(5, dtype=torch.int32, device="cuda"))
            for _ in range(nthreads)]
    exts = [_extents(5, region, 8 * MIB, 70 + i) for i in range(nthreads)]
    dexts = [_dev(torch, *e) for e in exts]
    torch.cuda.synchronize()
    errors, results = [], {}
    barrier = threading.Barrier(nthreads)

    def worker(i):
        try:
            for it in range(iters):
                ctx.fill_splitmix(ts[i], 1000 * i + it, 0, stream=HIP_STREAM_PER_THREAD)
                barrier.wait()
                for _ in range(3):  # several launches in flight per thread
                    ctx.blocks_dev(ts[i], 16 * MIB, out=outs[i][0], nblocks=4, stream=HIP_STREAM_PER_THREAD)
                    ctx.ranges_dev(ts[i], *dexts[i], out=outs[i][1], stream=HIP_STREAM_PER_THREAD)
                barrier.wait()
                torch.cuda.synchronize()  # every thread's per-thread stream
                barrier.wait()
                results[(i, it)] = (ts[i].cpu().numpy(), _u32(outs[i][0]).copy(), _u32(outs[i][1]).copy())
                barrier.wait()
        except Exception as e:  # noqa: BLE001
            errors.append((i, repr(e)))
            barrier.abort()

    th = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errors, errors
    for (i, it), (host, blocks, ranges) in results.items():
        assert np.array_equal(blocks, O.crc32_blocks(host, 16 * MIB, nthreads=8)), (i, it)
        assert np.array_equal(ranges, O.crc32_ranges(host, *exts[i])), (i, it)
    for i in range(nthreads):  # hand the threads' slots back (here from the main thread: its own none)
        ctx.stream_release(HIP_STREAM_PER_THREAD)


def _hip():
    import torch  # noqa: F401  (the HIP runtime torch loaded)
    for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    pytest.skip("libamdhip64 not loadable")


def test_streams_created_and_destroyed_per_connection(torch_cuda, ctx):
    """A server that creates a stream per connection: 20 streams, more than
    the pool's slots, each created, used for split-mode and fused calls, and
    destroyed -- half of them after priskv_crc_stream_release, half without
    (their slots stay out of use: the pool was not contended when they were
    last released, so no event marks their end, and later streams fall back
    to per-call allocation).  Every CRC exact, then two live streams at once.
    The contended and in-flight cases: tests/test_gpu_pool_contention.py."""
    torch = torch_cuda
    hip = _hip()
    region = 64 * MIB
    t = torch.empty(region, dtype=torch.uint8, device="cuda")
    offs, lens = _extents(6, region, 8 * MIB, 11)
    d_o, d_l = _dev(torch, offs, lens)
    o1 = torch.empty(4, dtype=torch.int32, device="cuda")
    o2 = torch.empty(6, dtype=torch.int32, device="cuda")
    for k in range(20):
        ctx.fill_splitmix(t, 500 + k, 0)
        torch.cuda.synchronize()
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        for _ in range(2):
            ctx.blocks_dev(t, 16 * MIB, out=o1, nblocks=4, stream=s.value)
            ctx.ranges_dev(t, d_o, d_l, out=o2, stream=s.value)
        if k % 2:
            ctx.stream_release(s.value)
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0
        host = t.cpu().numpy()
        assert np.array_equal(_u32(o1), O.crc32_blocks(host, 16 * MIB, nthreads=8)), k
        assert np.array_equal(_u32(o2), O.crc32_ranges(host, offs, lens)), k
    # concurrent streams after the churn: two live streams at once, back to back
    ss = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.empty(4, dtype=torch.int32, device="cuda") for _ in ss]
    ctx.fill_splitmix(t, 999, 0)
    torch.cuda.synchronize()
    for _ in range(4):
        for st, o in zip(ss, outs):
            ctx.blocks_dev(t, 16 * MIB, out=o, nblocks=4, stream=st)
    torch.cuda.synchronize()
    want = O.crc32_blocks(t.cpu().numpy(), 16 * MIB, nthreads=8)
    for o in outs:
        assert np.array_equal(_u32(o), want)
