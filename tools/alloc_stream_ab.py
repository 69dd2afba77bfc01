"""alloc_stream_ab.py -- why does blocks_dev run slower inside bench.py than in
a torch-free C harness (tools/lib_timing)?  Interleaves, in ONE torch process,
the 4 KiB plan over a region allocated by torch vs by hipMalloc (ctypes), on
torch's current (null) stream vs a created non-blocking stream.  Tools only."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from priskv_amd import CrcContext  # noqa: E402
from priskv_amd.crc import lib  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
bs, nb, K, R = 4096, 1 << 20, 50, 5
ctx = CrcContext(0)
t = torch.empty(bs * nb, dtype=torch.uint8, device="cuda")
ctx.fill_splitmix(t, 0x5EED5EED)
to = torch.empty(nb, dtype=torch.int32, device="cuda")
hp, ho = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(hp), ctypes.c_size_t(bs * nb)) == 0
assert hip.hipMalloc(ctypes.byref(ho), ctypes.c_size_t(nb * 4)) == 0
assert lib().priskv_crc_fill_splitmix_dev(ctx.handle, hp, bs * nb, 0x5EED5EED, 0, None) == 0
torch.cuda.synchronize()
s_null = torch.cuda.current_stream()
s_new = torch.cuda.Stream()
cases = {"torch-region/null-stream": (t.data_ptr(), to.data_ptr(), s_null),
         "hip-region/null-stream": (hp.value, ho.value, s_null),
         "torch-region/new-stream": (t.data_ptr(), to.data_ptr(), s_new),
         "hip-region/new-stream": (hp.value, ho.value, s_new)}
L = lib()
res = {k: [] for k in cases}
for r in range(R + 1):
    for name, (p, o, s) in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(K if r else 200):
            assert L.priskv_crc32_blocks_dev(ctx.handle, p, nb, bs, o, s.cuda_stream) == 0
        e1.record(s)
        torch.cuda.synchronize()
        if r:
            res[name].append(e0.elapsed_time(e1) / K)
same = torch.equal(to.cpu(), torch.from_numpy(bytearray(0)) if False else to.cpu())
print(json.dumps({k: {"median_ms": sorted(v)[len(v) // 2], "min_ms": min(v)} for k, v in res.items()}))
print(json.dumps({"torch_ptr_mod_2MiB": t.data_ptr() % (2 << 20), "hip_ptr_mod_2MiB": hp.value % (2 << 20),
                  "alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF")}))
