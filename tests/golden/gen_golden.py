#!/usr/bin/env python3
"""Generate tests/golden/crc_golden.json from the REFERENCE itself.

The reference's server/crc.c is compiled unmodified by oracle/Makefile into
oracle/_ref/libpriskv_ref_crc_O2.so; this script calls its priskv_crc32
(server/crc.c:90-109) on fully specified inputs and records the outputs.
Every vector is cross-checked against zlib's identity
crc(b) == zlib.crc32(b, ~0) ^ ~0 before it is written.  Inputs are stored as
generator specs (splitmix64 seed + word offset, constant fills, literal
strings), not as raw data, so the fixture stays small.

Run in the survey/dev container (needs /root/reference):
    make -C oracle && python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle as O  # noqa: E402

SEED = 0x5EED5EED
LENGTHS = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129,
           255, 256, 1023, 1024, 4095, 4096, 4097, 65535, 65536, 1048576]
STRINGS = [b"", b"a", b"abc", b"123456789",
           b"The quick brown fox jumps over the lazy dog", b"\x00" * 4096, b"\xff" * 16]


def ref(data: bytes) -> int:
    v = O.ref_crc32(data, "O2")
    z = O.zlib_identity(data)
    if v != z:
        raise SystemExit(f"reference/zlib disagree on len={len(data)}: {v:#x} vs {z:#x}")
    return v


def pattern(kind: str, n: int, seed: int = SEED, word_offset: int = 0) -> bytes:
    if kind == "zero":
        return b"\x00" * n
    if kind == "ff":
        return b"\xff" * n
    if kind == "counter":
        return bytes(i & 0xFF for i in range(n))
    if kind == "splitmix":
        return O.fill_splitmix(n, seed, word_offset).tobytes()
    raise ValueError(kind)


def main() -> None:
    if O.ref_lib("O2") is None:
        raise SystemExit("oracle/_ref/libpriskv_ref_crc_O2.so missing: run `make -C oracle`")
    g = {
        "about": "golden vectors for priskv_crc32 (server/crc.c:90-109), produced by the "
                 "reference compiled unmodified (oracle/_ref, -O2) and cross-checked against "
                 "zlib.crc32(b, 0xFFFFFFFF) ^ 0xFFFFFFFF",
        "generator": "tests/golden/gen_golden.py",
        "pattern_spec": "splitmix: 64-bit LE word i = mix64(seed + (word_offset + i + 1) * "
                        "0x9E3779B97F4A7C15), mix64 = splitmix64 finaliser; counter: byte i = i & 0xff",
        "seed": SEED,
    }
    # the Sarwate table, read back through the reference (crc of one byte b == T[b])
    g["table"] = [f"{ref(bytes([b])):08x}" for b in range(256)]
    g["strings"] = [{"hex": s.hex() if len(s) <= 64 else None,
                     "repeat": None if len(s) <= 64 else {"byte": s[0], "n": len(s)},
                     "crc": f"{ref(s):08x}"} for s in STRINGS]
    lens = []
    for kind in ("zero", "ff", "counter", "splitmix"):
        for n in LENGTHS:
            lens.append({"pattern": kind, "len": n, "crc": f"{ref(pattern(kind, n)):08x}"})
    # unaligned starts: splitmix region, slices at odd offsets
    region = pattern("splitmix", 1 << 16, SEED, 1000)
    rng = np.random.default_rng(1234)
    ranges = []
    for _ in range(64):
        off = int(rng.integers(0, 4096))
        ln = int(rng.integers(0, 1 << 14))
        ranges.append({"offset": off, "len": ln, "crc": f"{ref(region[off:off + ln]):08x}"})
    g["lengths"] = lens
    g["ranges"] = {"pattern": "splitmix", "word_offset": 1000, "region_bytes": 1 << 16,
                   "items": ranges}
    # whole value blocks (server/memory.h:87-91: block i at base + i*block_size);
    # the region is one splitmix stream starting at word 0.
    blocks = []
    for bs, nb in ((1024, 64), (4096, 64), (65536, 8), (1 << 20, 2), (512, 16), (16, 64)):
        reg = pattern("splitmix", bs * nb, SEED, 0)
        crcs = [f"{ref(reg[i * bs:(i + 1) * bs]):08x}" for i in range(nb)]
        blocks.append({"block_size": bs, "nblocks": nb, "word_offset": 0, "crcs": crcs})
    g["blocks"] = blocks
    out = os.path.join(HERE, "crc_golden.json")
    with open(out, "w") as f:
        json.dump(g, f, indent=1)
    print(f"wrote {out}: {len(lens)} length cases, {len(ranges)} ranges, "
          f"{sum(b['nblocks'] for b in blocks)} blocks")


if __name__ == "__main__":
    main()
