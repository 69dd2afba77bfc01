#!/usr/bin/env python3
"""Per-wave and per-XCD timing of one rows-kernel launch (tools only).

  python tools/wave_times.py [BS] [NB] [REPS] [XW]

Runs the coverage build (priskv_amd/lib/cov/, `make cov`), whose
crc_rows_kernel stores each wave's XCD, group count and start / end
s_memrealtime (100 MHz) stamps, over NB x BS blocks (default the headline
1 Mi x 4 KiB), REPS launches after a ramp, and prints per launch: the spread
of wave end times, each XCD's mean / max end (µs after the launch's first
wave start) and mean rate per wave, and how long the last wave outlasts the
mean -- the tail the static (XCD-weighted) split leaves.  XW: an XCD weight
override (PRISKV_CRC_XCD_WEIGHTS, e.g. 1:1) for comparison.  JSON lines.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BS = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 5
if len(sys.argv) > 4:
    os.environ["PRISKV_CRC_XCD_WEIGHTS"] = sys.argv[4]

L = C.CDLL(os.path.join(ROOT, "priskv_amd", "lib", "cov", "libpriskv_crc_cov.so"))
L.priskv_crc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
L.priskv_crc32_blocks_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
L.priskv_crc_cov_waves.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
L.priskv_crc_fill_splitmix_dev.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p]
L.priskv_crc32_blocks_plan.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_char_p, C.c_uint64]
h = C.c_void_p()
assert L.priskv_crc_ctx_create(0, C.byref(h)) == 0
s = torch.cuda.Stream()
sp = s.cuda_stream
region = torch.empty(BS * NB, dtype=torch.uint8, device="cuda")
out = torch.empty(NB, dtype=torch.int32, device="cuda")
assert L.priskv_crc_fill_splitmix_dev(h, region.data_ptr(), BS * NB, 7, 0, sp) == 0
buf = C.create_string_buffer(256)
L.priskv_crc32_blocks_plan(h, C.c_void_p(region.data_ptr()), NB, BS, buf, 256)
print(json.dumps({"plan": buf.value.decode()}), flush=True)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:
    for _ in range(8):
        L.priskv_crc32_blocks_dev(h, region.data_ptr(), NB, BS, out.data_ptr(), sp)
    s.synchronize()
rec = np.zeros((8192, 4), dtype=np.uint64)
for r in range(REPS):
    rec[:] = 0
    assert L.priskv_crc32_blocks_dev(h, region.data_ptr(), NB, BS, out.data_ptr(), sp) == 0
    assert L.priskv_crc_cov_waves(h, rec.ctypes.data, 8192) == 0
    live = rec[:, 3] != 0
    w = rec[live]
    xcc = (w[:, 0] & 0xFF).astype(int)
    ng = w[:, 1].astype(np.float64)
    t_s, t_e = w[:, 2].astype(np.float64), w[:, 3].astype(np.float64)
    base = t_s.min()
    end_us = (t_e - base) / 100.0  # 100 MHz ticks -> us
    dur_us = (t_e - t_s) / 100.0
    per = {}
    for x in range(8):
        m = xcc == x
        if m.any():
            per[x] = {"waves": int(m.sum()), "mean_end_us": round(float(end_us[m].mean()), 2),
                      "max_end_us": round(float(end_us[m].max()), 2),
                      "GBps_per_wave": round(float((ng[m] * BS / (dur_us[m] * 1e-6) / 1e9).mean()), 3),
                      "groups_per_wave": round(float(ng[m].mean()), 1)}
    print(json.dumps({"rep": r, "waves": int(live.sum()), "end_min_us": round(float(end_us.min()), 2),
                      "end_mean_us": round(float(end_us.mean()), 2), "end_max_us": round(float(end_us.max()), 2),
                      "tail_us": round(float(end_us.max() - end_us.mean()), 2),
                      "start_spread_us": round(float((t_s.max() - base) / 100.0), 2), "xcd": per}), flush=True)
