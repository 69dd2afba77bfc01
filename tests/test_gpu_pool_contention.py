"""GPU tests of the scratch pool under contention and of the XCD-weighted
split's coverage (round 6).

The pool (priskv_amd/csrc/crc_gpu.hip, Scratch) hands each stream its own
slots of zero-at-rest scratch (the split-mode and fused kernels' finish
words).  With more streams than slots a stream may take over another's slot
only after the library's own event, recorded at that slot's last release,
has completed -- never from a query of a handle the caller did not pass in
the current call.  These tests drive the two caller patterns a server has
(streams per connection, destroyed when the connection closes:
/root/reference/server/rdma.c:1860-1863; graph capture on one thread while
others submit) and check every CRC against the oracle (oracle/crc_oracle.c,
pinned to the reference's server/crc.c in test_oracle.py).

Some run on the test-only coverage build (priskv_amd/lib/cov/, `make cov`:
the product source with counters in the kernels' wave ranges and the pool),
which exports priskv_crc_cov_take / priskv_crc_cov_pool beside the product
ABI; the product library has neither.
"""
import ctypes
import os
import threading

import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROD_SO = os.path.join(ROOT, "priskv_amd", "lib", "libpriskv_crc.so")
COV_SO = os.path.join(ROOT, "priskv_amd", "lib", "cov", "libpriskv_crc_cov.so")
MIB = 1 << 20
NPOOL = 8  # crc_gpu.hip NPOOL: slots per pool


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _hip():
    import torch  # noqa: F401  (the HIP runtime torch loaded)
    for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    pytest.skip("libamdhip64 not loadable")


class Raw:
    """The C ABI of one library build, by ctypes (pointers as ints)."""

    def __init__(self, path, **env):
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built (make -C priskv_amd/csrc)")
        self.L = ctypes.CDLL(path)
        self.cov = hasattr(self.L, "priskv_crc_cov_take")
        L = self.L
        L.priskv_crc_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.priskv_crc_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.priskv_crc32_blocks_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_void_p, ctypes.c_void_p]
        L.priskv_crc32_ranges_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        L.priskv_crc32_blocks_plan.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.c_char_p, ctypes.c_uint64]
        L.priskv_crc_stream_release.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        if self.cov:
            L.priskv_crc_cov_take.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.priskv_crc_cov_pool.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        old = {k: os.environ.get(k) for k in env}
        os.environ.update({k: str(v) for k, v in env.items()})
        try:
            h = ctypes.c_void_p()
            assert L.priskv_crc_ctx_create(0, ctypes.byref(h)) == 0
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
        self.h = h

    def close(self):
        if self.h:
            self.L.priskv_crc_ctx_destroy(self.h)
            self.h = ctypes.c_void_p()

    def blocks(self, t, bs, n, out, stream):
        rc = self.L.priskv_crc32_blocks_dev(self.h, t.data_ptr(), n, bs, out.data_ptr(), stream)
        assert rc == 0, rc

    def ranges(self, t, d_o, d_l, out, stream):
        rc = self.L.priskv_crc32_ranges_dev(self.h, t.data_ptr(), d_o.data_ptr(), d_l.data_ptr(), d_o.numel(),
                                            out.data_ptr(), stream)
        assert rc == 0, rc

    def plan(self, t, n, bs):
        buf = ctypes.create_string_buffer(256)
        assert self.L.priskv_crc32_blocks_plan(self.h, t.data_ptr(), n, bs, buf, len(buf)) == 0
        return buf.value.decode()

    def cov_take(self):
        v = (ctypes.c_uint64 * 2)()
        assert self.L.priskv_crc_cov_take(self.h, v) == 0
        return int(v[0]), int(v[1])

    def cov_pool(self):
        v = (ctypes.c_uint64 * 3)()
        assert self.L.priskv_crc_cov_pool(self.h, v) == 0
        return {"calls": int(v[0]), "misses": int(v[1]), "takeovers": int(v[2])}


def _u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def _extents(n, region_bytes, max_len, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, max_len + 1, n).astype(np.uint32)
    offs = np.array([rng.integers(0, region_bytes - int(ln) + 1) for ln in lens], dtype=np.uint64)
    return offs, lens


def _fill(torch, t, seed):
    from priskv_amd import CrcContext
    with CrcContext(0) as c:
        c.fill_splitmix(t, seed, 0)
        torch.cuda.synchronize()


def _new_stream(hip, nonblocking=False):
    s = ctypes.c_void_p()
    if nonblocking:  # hipStreamNonBlocking: no implicit ordering with the legacy default stream
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
    else:
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    return s


@pytest.mark.parametrize("build", ["product", "cov"])
def test_destroyed_stream_in_flight_then_contended_pool(torch_cuda, build):
    """a split-mode call (4 x 16 MiB) and a fused call
    enqueued on stream X, X destroyed with NO sync, then 9 other live streams
    (more than the slots X left) drive split and fused calls until the pool
    is contended and slots change hands.  Every CRC -- X's included -- exact;
    on the coverage build the pool must report misses and at least one
    takeover."""
    torch = torch_cuda
    hip = _hip()
    R = Raw(PROD_SO if build == "product" else COV_SO)
    try:
        region = 64 * MIB
        t = torch.empty(region, dtype=torch.uint8, device="cuda")
        _fill(torch, t, 0xD0D0 + (build == "cov"))
        offs, lens = _extents(6, region, 8 * MIB, 21)
        d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_l = torch.from_numpy(lens.view(np.int32)).cuda()
        host = t.cpu().numpy()
        want_b = O.crc32_blocks(host, 16 * MIB, nthreads=8)
        want_r = O.crc32_ranges(host, offs, lens)
        assert "few large blocks" in R.plan(t, 4, 16 * MIB), R.plan(t, 4, 16 * MIB)
        torch.cuda.synchronize()

        def outs():
            return (torch.full((4,), -1, dtype=torch.int32, device="cuda"),
                    torch.full((6,), -1, dtype=torch.int32, device="cuda"))

        ox = outs()
        ss = [_new_stream(hip) for _ in range(NPOOL + 1)]
        os_ = [outs() for _ in ss]
        torch.cuda.synchronize()  # nothing below waits for the device until every call is in
        X = _new_stream(hip)
        for _ in range(3):
            R.blocks(t, 16 * MIB, 4, ox[0], X.value)
            R.ranges(t, d_o, d_l, ox[1], X.value)
        assert hip.hipStreamDestroy(X) == 0  # no sync: its kernels may still run
        for rnd in range(6):
            # round 3 starts with the streams that found no slot: the armed
            # slots of the streams synchronised after round 2 are complete
            order = list(zip(ss, os_))[::-1] if rnd == 3 else list(zip(ss, os_))
            for s, o in order:
                R.blocks(t, 16 * MIB, 4, o[0], s.value)
                R.ranges(t, d_o, d_l, o[1], s.value)
            if rnd == 2:  # let armed slots complete, so the next misses take them over
                for s in ss[: NPOOL - 1]:
                    assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipDeviceSynchronize() == 0
        for k, o in enumerate([ox] + os_):
            assert np.array_equal(_u32(o[0]), want_b), ("blocks", k)
            assert np.array_equal(_u32(o[1]), want_r), ("ranges", k)
        if R.cov:
            st = R.cov_pool()
            assert st["misses"] > 0 and st["takeovers"] > 0, st
        for s in ss:
            assert hip.hipStreamDestroy(s) == 0
    finally:
        R.close()


@pytest.mark.parametrize("kind", ["blocking", "nonblocking"])
def test_capture_on_one_thread_while_another_exhausts_pool(torch_cuda, kind):
    """stream X homes a pool slot; thread A begins a
    global-mode capture on X and captures split and fused calls; meanwhile
    thread B drives 9 other streams through split and fused calls until the
    pool is contended (misses, armed releases, takeovers, per-call
    allocations).  A's hipStreamEndCapture must succeed (round 5's takeover
    queried foreign streams, and querying a capturing stream invalidates its
    capture), and replays of A's graph and B's results are exact."""
    torch = torch_cuda
    hip = _hip()
    R = Raw(COV_SO)
    try:
        region = 64 * MIB
        t = torch.empty(region, dtype=torch.uint8, device="cuda")
        _fill(torch, t, 0xCAB)
        offs, lens = _extents(5, region, 8 * MIB, 31)
        d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_l = torch.from_numpy(lens.view(np.int32)).cuda()
        host = t.cpu().numpy()
        want_b = O.crc32_blocks(host, 16 * MIB, nthreads=8)
        want_r = O.crc32_ranges(host, offs, lens)
        oa = (torch.full((4,), -1, dtype=torch.int32, device="cuda"),
              torch.full((5,), -1, dtype=torch.int32, device="cuda"))
        ob = [(torch.full((4,), -1, dtype=torch.int32, device="cuda"),
               torch.full((5,), -1, dtype=torch.int32, device="cuda")) for _ in range(NPOOL + 1)]
        # blocking streams (hipStreamCreate): while a blocking stream is being
        # captured HIP refuses hipMallocAsync / hipFreeAsync on every stream,
        # so B's calls that need new scratch take the library's plain-malloc
        # fallback (tools/capture_blocking_probe.py)
        nb = kind == "nonblocking"
        X = _new_stream(hip, nonblocking=nb)
        R.blocks(t, 16 * MIB, 4, oa[0], X.value)  # X homes a slot
        assert hip.hipStreamSynchronize(X) == 0
        bs = [_new_stream(hip, nonblocking=nb) for _ in range(NPOOL + 1)]

        torch.cuda.synchronize()
        # no torch call below until both threads are done: torch's allocator
        # would itself be an illegal call under A's global-mode capture
        began, b_done = threading.Event(), threading.Event()
        errs, graph = [], ctypes.c_void_p()
        end_rc = []

        def thread_a():
            try:
                assert hip.hipStreamBeginCapture(X, 0) == 0  # hipStreamCaptureModeGlobal
                began.set()
                R.blocks(t, 16 * MIB, 4, oa[0], X.value)
                b_done.wait(60)
                R.ranges(t, d_o, d_l, oa[1], X.value)
                end_rc.append(hip.hipStreamEndCapture(X, ctypes.byref(graph)))
            except Exception as e:  # noqa: BLE001
                errs.append(("A", repr(e)))
                began.set()

        def thread_b():
            try:
                # B's own stream synchronisations below would be illegal under
                # A's global-mode capture (hipErrorStreamCaptureUnsupported,
                # and they invalidate A's capture): B runs in relaxed mode, as
                # a server thread beside a capturing one must.  The library's
                # own calls do not depend on it (its pool calls switch to
                # relaxed mode themselves): tools/capture_blocking_probe.py.
                mode = ctypes.c_int(2)  # hipStreamCaptureModeRelaxed
                assert hip.hipThreadExchangeStreamCaptureMode(ctypes.byref(mode)) == 0
                began.wait(60)
                for rnd in range(4):
                    for s, o in zip(bs, ob):
                        R.blocks(t, 16 * MIB, 4, o[0], s.value)
                        R.ranges(t, d_o, d_l, o[1], s.value)
                    if rnd == 1:
                        for s in bs[: NPOOL - 2]:
                            assert hip.hipStreamSynchronize(s) == 0
            except Exception as e:  # noqa: BLE001
                errs.append(("B", repr(e)))
            finally:
                b_done.set()

        th = [threading.Thread(target=thread_a), threading.Thread(target=thread_b)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=120)
        assert not errs, errs
        assert end_rc == [0], end_rc  # the capture survived B's contended pool
        st = R.cov_pool()
        assert st["misses"] > 0, st
        exe = ctypes.c_void_p()
        assert hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None, ctypes.c_size_t(0)) == 0
        assert hip.hipDeviceSynchronize() == 0
        for o in ob:
            assert np.array_equal(_u32(o[0]), want_b)
            assert np.array_equal(_u32(o[1]), want_r)
        for seed in (0xCAC, 0xCAD):
            _fill(torch, t, seed)
            host = t.cpu().numpy()
            for o in oa:
                o.fill_(-1)
            torch.cuda.synchronize()
            for _ in range(3):
                assert hip.hipGraphLaunch(exe, X) == 0
            assert hip.hipStreamSynchronize(X) == 0
            assert np.array_equal(_u32(oa[0]), O.crc32_blocks(host, 16 * MIB, nthreads=8)), seed
            assert np.array_equal(_u32(oa[1]), O.crc32_ranges(host, offs, lens)), seed
        assert hip.hipGraphExecDestroy(exe) == 0
        assert hip.hipGraphDestroy(graph) == 0
        for s in bs + [X]:
            assert hip.hipStreamDestroy(s) == 0
    finally:
        R.close()


def test_stream_destroy_waits_for_its_work(torch_cuda):
    """Without hipStreamGetId (the HIP runtime PyTorch ships is 7.0) the pool
    keys a slot by its stream's handle, and a stream created after another was
    destroyed may get the same handle.  That is safe only if hipStreamDestroy
    returns after the destroyed stream's work: then the new stream's calls
    cannot overlap the old one's.  ~5 ms of CRC work, an event recorded after
    it, the stream destroyed at once: the event must be complete when
    hipStreamDestroy returns."""
    import time
    torch = torch_cuda
    hip = _hip()
    R = Raw(PROD_SO)
    try:
        t = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        _fill(torch, t, 0xDE57)
        out = torch.empty(1 << 18, dtype=torch.int32, device="cuda")
        ev = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(ev), 2) == 0  # hipEventDisableTiming
        X = _new_stream(hip)
        torch.cuda.synchronize()
        for _ in range(30):  # 30 x 1 GiB, ~5 ms
            R.blocks(t, 4096, 1 << 18, out, X.value)
        assert hip.hipEventRecord(ev, X) == 0
        assert hip.hipEventQuery(ev) != 0, "the work finished before the destroy: the test proves nothing"
        t0 = time.perf_counter()
        assert hip.hipStreamDestroy(X) == 0
        dt = time.perf_counter() - t0
        q = hip.hipEventQuery(ev)
        print(f"hipStreamDestroy took {dt * 1e3:.2f} ms; event query after it: {q}")
        assert q == 0, f"hipStreamDestroy returned with the stream's work in flight ({dt * 1e3:.2f} ms)"
        assert hip.hipEventDestroy(ev) == 0
    finally:
        R.close()


# (name, block size, blocks, groups of the one launch or None): the plans
# whose static split the XCD weights move, each a single rows-kernel launch
_COV_CASES = [("4k_deep", 4096, 1 << 18, 1 << 18), ("window_4097", 4097, 1 << 17, 1 << 17),
              ("g16_2k", 2048, 1 << 18, 1 << 16), ("split_1m", MIB, 1900, None)]


def test_xcd_split_coverage(torch_cuda):
    """on the coverage build every wave adds its range
    (count, sum of indices) to device counters, and one launch's ranges must
    tile its n groups exactly: count n, index sum n(n-1)/2.  The deep 4 KiB,
    window, G = 16 and split plans run once alone, then twice on 8 streams at
    once (16 launches: 16 times the totals), on the context as the XCD probe
    set it up (weights where it found round-robin dispatch).  A context with
    PRISKV_CRC_XCD_PROBE=0 + PRISKV_CRC_XCD_WEIGHTS=17:13 must not apply the
    override (without round-robin dispatch the per-workgroup weight
    order is inconsistent) and stays exact.  Every CRC is checked against the
    oracle."""
    torch = torch_cuda
    wt = Raw(COV_SO)
    fb = Raw(COV_SO, PRISKV_CRC_XCD_PROBE="0", PRISKV_CRC_XCD_WEIGHTS="17:13")
    try:
        big = max(bs * n for _, bs, n, _ in _COV_CASES)
        t = torch.empty(big, dtype=torch.uint8, device="cuda")
        _fill(torch, t, 0xC0FE)
        host = t.cpu().numpy()
        streams = [torch.cuda.Stream() for _ in range(8)]
        wt.cov_take()
        plans = {}
        for name, bs, n, ng in _COV_CASES:
            want = O.crc32_blocks(host[: bs * n], bs, nthreads=16)
            outs = [torch.full((n,), -1, dtype=torch.int32, device="cuda") for _ in streams]
            plans[name] = wt.plan(t, n, bs)
            assert "xcd-weighted" not in fb.plan(t, n, bs), (name, fb.plan(t, n, bs))
            wt.cov_take()  # (the counters are one per library: drop the previous case's fallback calls)
            wt.blocks(t, bs, n, outs[0], streams[0].cuda_stream)
            N, idx = wt.cov_take()  # synchronises the device
            assert N > 0 and (ng is None or N == ng), (name, N, ng)
            assert N % n == 0 or ng is not None, (name, N)
            assert idx == (N * (N - 1) // 2) % (1 << 64), (name, N, idx)
            assert np.array_equal(_u32(outs[0]), want), name
            for o in outs:
                o.fill_(-1)
            torch.cuda.synchronize()
            for _ in range(2):
                for s, o in zip(streams, outs):
                    wt.blocks(t, bs, n, o, s.cuda_stream)
            got = wt.cov_take()
            assert got == (16 * N, (16 * idx) % (1 << 64)), (name, got, N, idx)
            for o in outs:
                assert np.array_equal(_u32(o), want), name
                o.fill_(-1)
            torch.cuda.synchronize()
            for s, o in zip(streams, outs):
                fb.blocks(t, bs, n, o, s.cuda_stream)
            torch.cuda.synchronize()
            for o in outs:
                assert np.array_equal(_u32(o), want), (name, "probe off + 17:13")
        print("plans:", plans)
    finally:
        for R in (wt, fb):
            R.close()


def test_per_thread_streams_contend_for_the_pool(torch_cuda):
    """More host threads on hipStreamPerThread than pool slots: with the HIP
    runtime PyTorch ships (no hipStreamGetId) each thread's slot is keyed by
    (handle, thread), so 12 threads contend for 8 slots, arm their releases
    and may take over each other's completed slots.  Every CRC exact; the
    coverage build must report misses; then every thread's slots go back
    through priskv_crc_stream_release on that thread."""
    torch = torch_cuda
    hip = _hip()
    R = Raw(COV_SO)
    HIP_STREAM_PER_THREAD = 2
    try:
        region = 64 * MIB
        t = torch.empty(region, dtype=torch.uint8, device="cuda")
        _fill(torch, t, 0x7E4D)
        offs, lens = _extents(4, region, 8 * MIB, 41)
        d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_l = torch.from_numpy(lens.view(np.int32)).cuda()
        host = t.cpu().numpy()
        want_b = O.crc32_blocks(host, 16 * MIB, nthreads=8)
        want_r = O.crc32_ranges(host, offs, lens)
        nthreads = NPOOL + 4
        outs = [(torch.full((4,), -1, dtype=torch.int32, device="cuda"),
                 torch.full((4,), -1, dtype=torch.int32, device="cuda")) for _ in range(nthreads)]
        torch.cuda.synchronize()
        errors, results = [], {}
        barrier = threading.Barrier(nthreads)

        def worker(i):
            try:
                for it in range(4):
                    for _ in range(2):
                        R.blocks(t, 16 * MIB, 4, outs[i][0], HIP_STREAM_PER_THREAD)
                        R.ranges(t, d_o, d_l, outs[i][1], HIP_STREAM_PER_THREAD)
                    assert hip.hipStreamSynchronize(ctypes.c_void_p(HIP_STREAM_PER_THREAD)) == 0
                    results[(i, it)] = (_u32(outs[i][0]).copy(), _u32(outs[i][1]).copy())
                    barrier.wait(timeout=60)
                assert R.L.priskv_crc_stream_release(R.h, HIP_STREAM_PER_THREAD) == 0
            except Exception as e:  # noqa: BLE001
                errors.append((i, repr(e)))
                barrier.abort()

        th = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=120)
        assert not errors, errors
        assert len(results) == nthreads * 4
        for (i, it), (b, r) in results.items():
            assert np.array_equal(b, want_b), (i, it)
            assert np.array_equal(r, want_r), (i, it)
        st = R.cov_pool()
        print("pool:", st)
        assert st["misses"] > 0, st  # (takeovers depend on the threads' timing; test (a) forces one)
    finally:
        R.close()


def test_mixed_paths_soak_many_threads(torch_cuda):
    """A short soak: 6 host threads on two contexts, each thread creating a
    stream per round (half of them destroyed without release or sync) and
    issuing the paths that draw pooled scratch -- split few large blocks,
    the balanced split, fused values -- beside plain rows, window and
    sub-KiB calls, on one read-only region; more live streams than slots.
    Every result against the oracle."""
    torch = torch_cuda
    hip = _hip()
    ctxs = [Raw(PROD_SO), Raw(PROD_SO)]
    try:
        region = 192 * MIB
        t = torch.empty(region, dtype=torch.uint8, device="cuda")
        _fill(torch, t, 0x50A4)
        offs, lens = _extents(5, 64 * MIB, 12 * MIB, 51)
        d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_l = torch.from_numpy(lens.view(np.int32)).cuda()
        host = t.cpu().numpy()
        # (block size, blocks): few large (split few), balanced 1 MiB split,
        # 4 KiB rows, 4095-B window, 256-B sub-KiB
        shapes = [(16 * MIB, 4), (MIB, 190), (4096, 40000), (4095, 40000), (256, 200000)]
        want = {bs: O.crc32_blocks(host[: bs * nb], bs, nthreads=16) for bs, nb in shapes}
        want_r = O.crc32_ranges(host[: 64 * MIB], offs, lens)
        nthreads, rounds = 6, 5
        outs = [{bs: torch.full((nb,), -1, dtype=torch.int32, device="cuda") for bs, nb in shapes}
                for _ in range(nthreads)]
        routs = [torch.full((5,), -1, dtype=torch.int32, device="cuda") for _ in range(nthreads)]
        torch.cuda.synchronize()
        errors, bad = [], []

        def worker(i):
            try:
                R = ctxs[i % 2]
                for r in range(rounds):
                    st = _new_stream(hip, nonblocking=bool((i + r) % 2))
                    for bs, nb in shapes:
                        R.blocks(t, bs, nb, outs[i][bs], st.value)
                    R.ranges(t, d_o, d_l, routs[i], st.value)
                    assert hip.hipStreamSynchronize(st) == 0
                    for bs, nb in shapes:
                        if not np.array_equal(_u32(outs[i][bs]), want[bs]):
                            bad.append((i, r, bs))
                    if not np.array_equal(_u32(routs[i]), want_r):
                        bad.append((i, r, "ranges"))
                    # the next round's calls on this thread's next stream; this
                    # one destroyed -- released first on even rounds only
                    if r % 2 == 0:
                        assert R.L.priskv_crc_stream_release(R.h, st.value) == 0
                    for bs, nb in shapes:
                        R.blocks(t, bs, nb, outs[i][bs], st.value)  # in flight at the destroy
                    assert hip.hipStreamDestroy(st) == 0
                    assert hip.hipDeviceSynchronize() == 0
                    for bs, nb in shapes:
                        if not np.array_equal(_u32(outs[i][bs]), want[bs]):
                            bad.append((i, r, bs, "after destroy"))
            except Exception as e:  # noqa: BLE001
                errors.append((i, repr(e)))

        th = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=300)
        assert not errors, errors
        assert not bad, bad[:10]
    finally:
        for R in ctxs:
            R.close()
