"""RCCL ("nccl" backend on ROCm) under the collectives bench.py issues at N > 1.

The driver's N > 1 runs are the only multi-GPU measurement and no 8-GPU node
is ours to use; the world-2 / world-8 rehearsals run over gloo
(tests/test_dist.py).  This runs the RCCL side once on the box's one GPU at
world size 1, in a child process so no process group leaks into the test
session: ``init_process_group("nccl", device_id=...)`` exactly as bench.py
calls it, then the collectives bench.py and priskv_amd.shard issue -- a
barrier, an all_reduce(MAX) of a float64 device tensor (max_over_ranks), an
all_gather of int32 device tensors (gather_crcs), all_gather_object
(per-rank device identity) -- and checks their results.  A world of one
cannot show that N GPUs pair up; it shows the RCCL code path itself runs on
MI355X with these tensors.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["PRISKV_ROOT"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)  # bench.py's RCCL branch
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
dist.barrier()
t = torch.tensor([3.25], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert float(t.item()) == 3.25
crc = torch.arange(10, dtype=torch.int32, device=dev)
parts = [torch.zeros(10, dtype=torch.int32, device=dev)]
dist.all_gather(parts, crc)
assert torch.equal(parts[0], crc)
obj = [None]
dist.all_gather_object(obj, {"rank": 0, "pci": "x"})
assert obj == [{"rank": 0, "pci": "x"}]
from priskv_amd.shard import max_over_ranks
assert max_over_ranks(1.5, device=dev) == 1.5
dist.destroy_process_group()
print("rccl world-1 collectives: ok")
"""


def test_rccl_world1_collectives():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29531", RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", PRISKV_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert "rccl world-1 collectives: ok" in r.stdout
