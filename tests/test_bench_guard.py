"""bench.py's rank -> device guard (CPU; no GPU needed).

A multi-GPU line must come from N distinct GPUs: a rank whose LOCAL_RANK
has no device of its own, or two ranks reporting one physical device, exit
with status 3 before any measurement, unless PRISKV_BENCH_REHEARSAL=1 asks
for a one-box rehearsal (the gloo path).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_device_guard_rules():
    g = bench.device_guard
    assert g(1, 0, 1, False) is None
    assert g(8, 7, 8, False) is None
    assert g(2, 1, 8, False) is None
    assert "no GPU" in g(1, 0, 0, False)
    assert "no GPU" in g(2, 0, 0, True)          # a rehearsal still needs one device
    assert "no GPU of its own" in g(8, 3, 1, False)
    assert "no GPU of its own" in g(2, 1, 1, False)
    assert g(2, 1, 1, True) is None               # rehearsal: ranks share the device
    assert g(2, -1, 8, False)


def _info(rank, host="h", pci="0000:05:00", uuid=None, device=0):
    return {"rank": rank, "host": host, "pci": pci, "uuid": uuid, "device": device}


def test_duplicate_devices():
    d = bench.duplicate_devices
    assert d([_info(0, pci="0000:05:00"), _info(1, pci="0000:15:00")]) == []
    assert d([_info(0), _info(1), _info(2, pci="0000:25:00")]) == [[0, 1]]
    assert d([_info(0), _info(1, host="other")]) == []  # same bus id on two hosts
    # no PCI address: the UUID decides
    assert d([_info(0, pci=None, uuid="a"), _info(1, pci=None, uuid="a")]) == [[0, 1]]
    assert d([_info(0, pci=None, uuid="a"), _info(1, pci=None, uuid="b")]) == []


@pytest.mark.parametrize("local", ["0", "1"])
def test_bench_exits_3_without_a_device_of_its_own(local):
    """In this container no GPU is visible: every rank must stop with status
    3 and say why, before any HIP call or collective."""
    env = dict(os.environ, WORLD_SIZE="2", RANK=local, LOCAL_RANK=local, MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29533")
    env.pop("PRISKV_BENCH_REHEARSAL", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == bench.EXIT_DEVICES, p.stderr[-2000:]
    assert "no GPU visible" in p.stderr
    assert p.stdout.strip() == ""  # no JSON line


def _canned_resident(value, frac, with_roof=True):
    """A resident leg shaped as bench.resident_leg returns it, long strings included."""
    rl = {"bound": "hbm", "achieved": frac * 8000, "peak": 8000.0, "unit": "GB/s", "frac": frac,
          "traffic": 4303306084.03, "kernel_ms": 0.6296, "alg_bytes_per_launch": 4299161600,
          "kernel_launch_ms": {"launches": 20, "median_ms": 0.63, "min_ms": 0.62, "max_ms": 0.64}}
    if with_roof:
        rl.update({"measured_peak": 7080.3, "measured_peak_best": 7215.8, "measured_peak_variant": 1,
                   "measured_peak_v0": 7000.1, "measured_peak_variants_GBps": {str(v): 7000.0 + v for v in range(9)},
                   "measured_peak_order": list(range(9)), "measured_peak_source": "x" * 600,
                   "roof_launch_ms": {"launches": 20, "median_ms": 0.6, "min_ms": 0.59, "max_ms": 0.61},
                   "frac_of_measured": 0.9644, "frac_of_v0": 0.97})
    return {"workload": "w" * 120, "value": value, "unit": "GiB/s", "n_gpus": 1, "steps": 20, "ms_per_step": 0.63,
            "bytes_per_gpu": 1 << 32, "kernel": "k" * 150, "roofline": rl,
            "parity": {"checked_blocks_per_rank": 1 << 20, "sample": "every block", "bit_exact": True,
                       "oracle": "oracle/crc_oracle.c"}}


def test_compact_line_shows_every_leg_in_the_last_3000_chars():
    """the driver keeps the tail of stdout, so the line
    must carry every leg's value and frac near its end.  A canned full
    result (as main() builds it, with every verbose field) through
    compact_line: the whole line stays under 3000 characters and its last
    3000 hold each leg's value and frac."""
    import json
    full = _canned_resident(6342.07, 0.8535)
    full.update({"metric": bench.METRIC, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                 "dtype": "u8", "data": "synthetic", "warmup": 5,
                 "config": {"workload": "w" * 100, "block_size": 4096, "nblocks_per_gpu": 1 << 20,
                            "bytes_per_gpu": 1 << 32, "parallelism": "shard1", "kernel": "k" * 130,
                            "untimed_ramp_launches": 1600, "untimed_ramp_s": 1.0, "timed_launches": "t" * 90}})
    full["sweep"] = {"64KiB": _canned_resident(6300.5, 0.86), "1MiB": _canned_resident(6400.25, 0.8758)}
    full["tib"] = _canned_resident(6500.75, 0.8789)
    full["odd"] = {"4095": _canned_resident(6100.5, 0.8237, False), "4097": _canned_resident(6080.5, 0.8199, False)}
    full["streamed"] = {"workload": "s" * 100, "n_gpus": 1,
                        "pinned": {"value": 52.2, "unit": "GiB/s", "steps": 5, "ms_per_step": 80.0,
                                   "roofline": {"frac": 0.89, "peak_source": "p" * 80}, "bit_exact": True},
                        "pageable": {"value": 47.94, "unit": "GiB/s", "steps": 2, "ms_per_step": 90.0,
                                     "roofline": {"frac": 0.81}, "bit_exact": True},
                        "parity": {"bit_exact": True}}
    full["cold"] = {"ms": 0.74, "value": 5400.5, "unit": "GiB/s", "frac": 0.7282, "walked_ms": 0.7,
                    "walked_value": 5600.0, "note": "n" * 200}
    full["cold_ms"] = 0.74
    full["ranks"] = [{"rank": 0, "host": "h" * 30, "pci": "0000:05:00", "uuid": "u" * 36, "kernel_ms": 0.63}]
    full["dist"] = {"backend": None, "world_size": 1, "distinct_devices": 1, "rehearsal": False}
    full["parity"] = {"checked_blocks_per_rank": 1 << 20, "sample": "every block", "bit_exact": True,
                      "oracle": "oracle/crc_oracle.c", "bit_exact_vs_reference_build": True}
    full["cpu_baseline"] = {"value": 0.5849, "unit": "GiB/s", "cores": 1, "kind": "reference",
                            "sample": "first 524288 x 4096 B blocks (2.00 GiB) of rank 0's shard; " + "s" * 300,
                            "variants": [{"opt": "-O2", "threads": 1, "value": 0.58},
                                         {"opt": "-O2", "threads": 16, "value": 8.9}],
                            "threads_used": 16, "cpus_in_affinity": 256, "cpu": "AMD EPYC 9575F 64-Core Processor"}
    full["leg_wall_s"] = {"total": 30.0, "note": "n" * 150}
    text = json.dumps(bench.compact_line(full, "gpurun_out/bench_detail.json"))
    assert len(text) < 3000, len(text)
    tail = json.loads(text)
    for k in ("metric", "value", "roofline", "cpu_baseline", "legs"):
        assert k in tail
    assert tail["roofline"]["frac"] == 0.8535 and tail["roofline"]["frac_of_measured"] == 0.9644
    legs = tail["legs"]
    want = {"64KiB": (6300.5, 0.86), "1MiB": (6400.25, 0.8758), "tib": (6500.75, 0.8789),
            "odd4095": (6100.5, 0.8237), "odd4097": (6080.5, 0.8199), "streamed_pinned": (52.2, 0.89),
            "streamed_pageable": (47.94, 0.81), "cold": (5400.5, 0.7282)}
    for k, (v, f) in want.items():
        assert legs[k]["value"] == v and legs[k]["frac"] == f, (k, legs.get(k))
        assert f'"{k}": {{"value": {v}' in text[-3000:], k
    assert legs["tib"]["traffic"] == round(4303306084.03 / 4299161600, 4)
    assert legs["odd4095"]["frac_of_measured"] is None and legs["64KiB"]["bit_exact"] is True
    assert tail["cpu_baseline"]["cores"] == 1 and tail["cpu_baseline"]["multithread"]["threads"] == 16
