#!/usr/bin/env python3
"""Which launches HIP refuses while another stream is being captured (tools only).

  python tools/capture_blocking_probe.py

Round 6: thread B's library calls returned -EIO on blocking streams
(hipStreamCreate) while thread A captured a blocking stream X in global mode
(tests/test_gpu_pool_contention.py).  This separates HIP's rule from the
library: with X capturing, one plain library launch (priskv_crc_fill_splitmix_dev:
one kernel, no scratch, no pool) on (a) a blocking stream and (b) a
non-blocking stream, each from a second thread, then whether X's capture
still ends cleanly.  X itself blocking or non-blocking.  Prints one JSON line
per case; asserts nothing.
"""
import ctypes as C
import json
import os
import threading

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hip = C.CDLL("libamdhip64.so")
L = C.CDLL(os.path.join(ROOT, "priskv_amd", "lib", "libpriskv_crc.so"))
L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
L.priskv_crc_fill_splitmix_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p]
L.priskv_crc32_blocks_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
h = C.c_void_p()
assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
buf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
out = torch.empty(16, dtype=torch.int32, device="cuda")
cap = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()


def stream(nonblocking):
    s = C.c_void_p()
    assert (hip.hipStreamCreateWithFlags(C.byref(s), 1) if nonblocking else hip.hipStreamCreate(C.byref(s))) == 0
    return s


for x_nb in (False, True):
    for b_nb in (False, True):
        X, S = stream(x_nb), stream(b_nb)
        res = {"capturing_stream": "nonblocking" if x_nb else "blocking",
               "other_stream": "nonblocking" if b_nb else "blocking"}
        assert hip.hipStreamBeginCapture(X, 0) == 0  # global mode
        res["capture_launch_rc"] = L.priskv_crc_fill_splitmix_dev(h, cap.data_ptr(), cap.numel(), 2, 0, X.value)
        def other():
            res["fill_rc"] = L.priskv_crc_fill_splitmix_dev(h, buf.data_ptr(), buf.numel(), 1, 0, S.value)
            st = C.c_int(-1)
            res["is_capturing_rc"] = hip.hipStreamIsCapturing(S, C.byref(st))
            res["is_capturing"] = st.value
            # the split-mode path: pooled zero-at-rest scratch (16 MiB blocks: few large blocks)
            res["split_rc"] = L.priskv_crc32_blocks_dev(h, buf.data_ptr(), 4, 16 << 20, out.data_ptr(), S.value)
            res["split_rc_again"] = L.priskv_crc32_blocks_dev(h, buf.data_ptr(), 4, 16 << 20, out.data_ptr(),
                                                              S.value)
            mode = C.c_int(2)  # hipStreamCaptureModeRelaxed
            hip.hipThreadExchangeStreamCaptureMode(C.byref(mode))
            p = C.c_void_p()
            res["malloc_async_relaxed_rc"] = hip.hipMallocAsync(C.byref(p), C.c_size_t(1 << 16), S)
            if p:
                res["free_async_relaxed_rc"] = hip.hipFreeAsync(p, S)
            q = C.c_void_p()
            res["malloc_relaxed_rc"] = hip.hipMalloc(C.byref(q), C.c_size_t(1 << 16))
            ev = C.c_void_p()
            res["event_create_rc"] = hip.hipEventCreateWithFlags(C.byref(ev), 2)
            res["event_record_rc"] = hip.hipEventRecord(ev, S)
            res["event_query_rc"] = hip.hipEventQuery(ev)
            hip.hipThreadExchangeStreamCaptureMode(C.byref(mode))
            res["event_query_global_rc"] = hip.hipEventQuery(ev)
            res["stream_sync_global_rc"] = hip.hipStreamSynchronize(S)
            hip.hipGetLastError()

        th = threading.Thread(target=other)
        th.start()
        th.join()
        g = C.c_void_p()
        res["end_capture_rc"] = hip.hipStreamEndCapture(X, C.byref(g))
        # the same library calls from a second thread that makes no global-mode
        # call of its own: the capture must survive them
        assert hip.hipStreamBeginCapture(X, 0) == 0
        L.priskv_crc_fill_splitmix_dev(h, cap.data_ptr(), cap.numel(), 2, 0, X.value)
        rc2 = []
        th = threading.Thread(target=lambda: rc2.extend(
            [L.priskv_crc32_blocks_dev(h, buf.data_ptr(), 4, 16 << 20, out.data_ptr(), S.value) for _ in range(3)]))
        th.start()
        th.join()
        res["clean_split_rcs"] = rc2
        g2 = C.c_void_p()
        res["clean_end_capture_rc"] = hip.hipStreamEndCapture(X, C.byref(g2))
        if g2:
            hip.hipGraphDestroy(g2)
        if g:
            hip.hipGraphDestroy(g)
        hip.hipDeviceSynchronize()
        hip.hipGetLastError()
        for s in (X, S):
            hip.hipStreamDestroy(s)
        print(json.dumps(res), flush=True)
