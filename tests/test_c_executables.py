"""The C test executables (tests/c/), in PrisKV's own unit-test style
(server/test/test_kv.c: standalone binaries, "[OK]"/"[FAILED]", exit status).

test_crc_host runs here: the drop-in priskv_crc32 linked from
libpriskv_crc_host.a the way the server links crc.o; so does test_lds_images
(the byte-fold LDS image layout).  test_crc_gpu drives the
batched C ABI from plain C with HIP's C runtime API; it is built by
__graft_entry__.build() (make -C tests/c) and runs on the GPU box.
"""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c")


def _binary(name):
    path = os.path.join(HERE, name)
    if not os.path.exists(path):
        subprocess.run(["make", "-C", HERE, name], check=True, capture_output=True)
    return path


def test_c_host_executable():
    r = subprocess.run([_binary("test_crc_host")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "test_crc_host: OK" in r.stdout and "[FAILED]" not in r.stdout


def test_c_lds_image_layout():
    """The sub-KiB byte-fold LDS image against the kernels' lookup addresses
    and the bank-conflict-free property, on the CPU (tests/c/test_lds_images.c)."""
    r = subprocess.run([_binary("test_lds_images")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "test_lds_images: OK" in r.stdout and "[FAILED]" not in r.stdout


@pytest.mark.gpu
def test_c_gpu_executable():
    path = os.path.join(HERE, "test_crc_gpu")
    assert os.path.exists(path), "tests/c/test_crc_gpu is built by __graft_entry__.build()"
    r = subprocess.run([path], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "test_crc_gpu: OK" in r.stdout and "[FAILED]" not in r.stdout
