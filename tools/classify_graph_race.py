#!/usr/bin/env python3
"""Classify round 5's graph wrong results from the probe records (CPU only).

  python tools/classify_graph_race.py [RECORD.jsonl ...] [--json OUT]

Input: the `bad_info` entries of tools/graph_race_probe.py's records
(profiles/r05/graph_memnode/*.jsonl).  Each names a 1 MiB block of the
balanced split-mode call (1900 x 1 MiB, crc_rows_kernel split mode), the CRC
the graph returned (`got`) and the right one (`want`); the fill is
splitmix64(seed, word offset block * 2^17) and the seed is 70 + 10 * round +
the refill index (tools/graph_race_probe.py:137).

For each entry, with d = got ^ want (CRC linearity, init 0, no xorout: the CRC
of a block is the XOR of its units' CRCs each moved to the block end, Z_dist):
  - `lost_run`: d equals Z(crc(units i..j)) of one contiguous run of units of
    some power-of-two unit size (4 KiB .. 512 KiB) -- a part's share that the
    finish did not include (or included twice);
  - `stale_run`: d equals Z(crc_new(run)) ^ Z(crc_old(run)) for the previous
    refill's seed or the warm-up's seed 1 -- a part hashed from old data;
  - none: d is not a function of this block's data in those shapes (counters
    or accumulators not zero when the launch started).

Self-contained (zlib + numpy), so the classification does not depend on the
library or the oracle build.  The seed of each entry is checked first: the
recomputed CRC must equal `want`.
"""
import glob
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIB = 1 << 20
POLY = 0xEDB88320


def crc(b: bytes) -> int:
    """priskv_crc32 (server/crc.c:90-109): zlib with the init and xorout undone."""
    return zlib.crc32(b, 0xFFFFFFFF) ^ 0xFFFFFFFF


def splitmix(nwords: int, seed: int, word_offset: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        i = np.arange(word_offset + 1, word_offset + nwords + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def block_bytes(seed: int, block: int) -> bytes:
    return splitmix(MIB // 8, seed, block * MIB // 8).tobytes()


def multmodp(a: int, b: int) -> int:
    """a * b mod P in the reflected domain (x^0 is bit 31)."""
    m, p = 1 << 31, 0
    while True:
        if a & m:
            p ^= b
            if (a & (m - 1)) == 0:
                return p
        m >>= 1
        b = (b >> 1) ^ POLY if b & 1 else b >> 1


_X2N = [1 << 30]  # x^(2^k) mod P, k = 0..
for _ in range(63):
    _X2N.append(multmodp(_X2N[-1], _X2N[-1]))


def zshift(v: int, nbytes: int) -> int:
    """Z_nbytes(v): the register after nbytes zero bytes (crc(M || 0^n) from crc(M))."""
    p, k, n = 1 << 31, 3, nbytes  # x^(8n)
    while n:
        if n & 1:
            p = multmodp(_X2N[k], p)
        n >>= 1
        k += 1
    return multmodp(p, v)


def unit_contribs(data: bytes, u: int) -> list:
    m = len(data) // u
    return [zshift(crc(data[k * u:(k + 1) * u]), len(data) - (k + 1) * u) for k in range(m)]


def runs(c: list) -> dict:
    """XOR of contributions over every contiguous run (i, j) -> value."""
    px = [0]
    for x in c:
        px.append(px[-1] ^ x)
    out = {}
    for i in range(len(c)):
        for j in range(i, len(c)):
            out.setdefault(px[j + 1] ^ px[i], (i, j))
    return out


UNITS = [4096 << k for k in range(8)]  # 4 KiB .. 512 KiB


def classify(seed: int, prev_seed, block: int, got: int, want: int) -> dict:
    new = block_bytes(seed, block)
    check = crc(new)
    r = {"seed": seed, "block": block, "got": hex(got), "want": hex(want), "seed_ok": check == want,
         "d": hex(got ^ want)}
    if check != want:
        return r
    d = got ^ want
    olds = {s: block_bytes(s, block) for s in {1, prev_seed} if s is not None}
    for u in UNITS:
        cn = unit_contribs(new, u)
        hit = runs(cn).get(d)
        if hit:
            r.setdefault("lost_run", []).append({"unit": u, "units": hit, "of": MIB // u})
        for s, ob in olds.items():
            co = unit_contribs(ob, u)
            hit = runs([a ^ b for a, b in zip(cn, co)]).get(d)
            if hit:
                r.setdefault("stale_run", []).append({"unit": u, "units": hit, "old_seed": s})
            hit = runs(co).get(d)
            if hit:
                r.setdefault("old_run", []).append({"unit": u, "units": hit, "old_seed": s})
    r["class"] = ("lost_run" if "lost_run" in r else "stale_run" if "stale_run" in r
                  else "old_run" if "old_run" in r else "none")
    return r


def main(argv):
    out_json = None
    if "--json" in argv:
        i = argv.index("--json")
        out_json = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    files = argv or sorted(glob.glob(os.path.join(ROOT, "profiles/r05/graph_memnode/*.jsonl")))
    results = []
    for f in files:
        for line in open(f):
            rec = json.loads(line)
            base = 70 + 10 * rec["round"]
            for k, refill in enumerate(rec["mixed_wrong"]):
                for b in refill.get("bad_info", []):
                    r = classify(base + k, base + k - 1 if k else None, b["block"], int(b["got"], 16),
                                 int(b["want"], 16))
                    r["file"] = os.path.relpath(f, ROOT)
                    r["refill"] = k
                    results.append(r)
                    print(json.dumps(r), flush=True)
    summary = {}
    for r in results:
        c = r.get("class", "seed_mismatch")
        summary[c] = summary.get(c, 0) + 1
    print(json.dumps({"entries": len(results), "classes": summary}))
    if out_json:
        with open(out_json, "w") as f:
            json.dump({"entries": results, "classes": summary}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
