"""Pin the CPU oracle (oracle/crc_oracle.c) before trusting it.

Mirrors the executable-per-check style of server/test/ (assert + [OK]) in
pytest form.  Sources of truth, in order:
  1. tests/golden/crc_golden.json -- produced by the reference's server/crc.c
     compiled unmodified (tests/golden/gen_golden.py, oracle/Makefile);
  2. the reference build itself (oracle/_ref), when present;
  3. zlib's independent identity crc(b) == zlib.crc32(b, ~0) ^ ~0.
"""
import numpy as np
import pytest

import _oracle as O


def _pattern(kind, n, seed, word_offset=0):
    if kind == "zero":
        return b"\x00" * n
    if kind == "ff":
        return b"\xff" * n
    if kind == "counter":
        return bytes(i & 0xFF for i in range(n))
    return O.fill_splitmix(n, seed, word_offset).tobytes()


def test_table_matches_reference(golden):
    # server/crc.c:31-68 -- our generated table == the reference's, as read back
    ours = [f"{v:08x}" for v in O.table()]
    assert ours == golden["table"]


def test_known_answers(golden):
    for s in golden["strings"]:
        data = bytes.fromhex(s["hex"]) if s["hex"] is not None else bytes([s["repeat"]["byte"]]) * s["repeat"]["n"]
        assert O.crc32(data) == int(s["crc"], 16), data[:16]
    assert O.crc32(b"123456789") == 0x2DFD2D88  # check value of this CRC variant


def test_lengths(golden):
    for c in golden["lengths"]:
        data = _pattern(c["pattern"], c["len"], golden["seed"])
        assert O.crc32(data) == int(c["crc"], 16), (c["pattern"], c["len"])


def test_ranges(golden):
    r = golden["ranges"]
    region = O.fill_splitmix(r["region_bytes"], golden["seed"], r["word_offset"])
    offs = [it["offset"] for it in r["items"]]
    lens = [it["len"] for it in r["items"]]
    got = O.crc32_ranges(region, offs, lens)
    assert [f"{v:08x}" for v in got] == [it["crc"] for it in r["items"]]


def test_blocks(golden):
    for b in golden["blocks"]:
        region = O.fill_splitmix(b["block_size"] * b["nblocks"], golden["seed"], b["word_offset"])
        for nt in (1, 3):
            got = O.crc32_blocks(region, b["block_size"], nthreads=nt)
            assert [f"{v:08x}" for v in got] == b["crcs"], b["block_size"]


def test_splitmix_generator_two_implementations():
    c = O.fill_splitmix(8 * 1000 + 5, 0x1234, 77)
    n = O.splitmix_numpy(1001, 0x1234, 77).view(np.uint8)[: 8 * 1000 + 5]
    assert np.array_equal(c, n)


def test_zlib_identity_random():
    rng = np.random.default_rng(7)
    for _ in range(300):
        n = int(rng.integers(0, 5000))
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.crc32(data) == O.zlib_identity(data)


@pytest.mark.parametrize("opt", ["O2", "O0"])
def test_against_reference_build(opt):
    if O.ref_lib(opt) is None:
        pytest.skip("oracle/_ref not built (reference sources absent)")
    rng = np.random.default_rng(11)
    for _ in range(300):
        n = int(rng.integers(0, 9000))
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.crc32(data) == O.ref_crc32(data, opt)


def test_zero_and_linearity():
    # init 0 / xorout 0 => any all-zero input has CRC 0 and crc(a^b) = crc(a)^crc(b)
    assert O.crc32(b"\x00" * 12345) == 0
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, 999, dtype=np.uint8)
    b = rng.integers(0, 256, 999, dtype=np.uint8)
    assert O.crc32(a ^ b) == O.crc32(a) ^ O.crc32(b)
