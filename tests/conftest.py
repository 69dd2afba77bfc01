import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: multi-GiB cases")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(HERE, "golden", "crc_golden.json")) as f:
        return json.load(f)
