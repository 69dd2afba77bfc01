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
