"""ctypes access to the TEST-ONLY checkers under oracle/.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (priskv_amd/ and libpriskv_crc.so) never does.

  oracle/liboracle_crc.so          our restatement of server/crc.c:90-109
  oracle/_ref/libpriskv_ref_crc_*  the reference's server/crc.c compiled
                                    unmodified (oracle/Makefile); optional
"""
from __future__ import annotations

import ctypes
import os
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_crc.so")
REF_SO = {
    "O2": os.path.join(ORACLE_DIR, "_ref", "libpriskv_ref_crc_O2.so"),
    "O0": os.path.join(ORACLE_DIR, "_ref", "libpriskv_ref_crc_O0.so"),
}

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)

_lib = None
_ref = {}


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"oracle not built: {ORACLE_SO} (run `make -C oracle`)")
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_crc32.restype = ctypes.c_uint32
        L.oracle_crc32.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_crc32_blocks.restype = ctypes.c_int
        L.oracle_crc32_blocks.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_int]
        L.oracle_crc32_ranges.restype = None
        L.oracle_crc32_ranges.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_fill_splitmix.restype = None
        L.oracle_fill_splitmix.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_uint64]
        L.oracle_splitmix_word.restype = ctypes.c_uint64
        L.oracle_splitmix_word.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_table.restype = None
        L.oracle_table.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def ref_lib(opt: str = "O2"):
    """The reference's own server/crc.c (compiled by oracle/Makefile), or None."""
    if opt not in _ref:
        path = REF_SO[opt]
        if os.path.exists(path):
            L = ctypes.CDLL(path)
            L.priskv_crc32.restype = ctypes.c_uint32
            L.priskv_crc32.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
            _ref[opt] = L
        else:
            _ref[opt] = None
    return _ref[opt]


def _ptr(a) -> int:
    if isinstance(a, (bytes, bytearray)):
        a = np.frombuffer(a, dtype=np.uint8)
    return a.ctypes.data


def crc32(data) -> int:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a).view(np.uint8)
    return int(lib().oracle_crc32(a.ctypes.data if a.size else None, a.size))


def ref_crc32(data, opt: str = "O2") -> int:
    L = ref_lib(opt)
    if L is None:
        raise RuntimeError("reference build absent (oracle/_ref)")
    a = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
    buf = (ctypes.c_uint8 * max(1, a.size)).from_buffer_copy(a.tobytes() or b"\0")
    return int(L.priskv_crc32(ctypes.addressof(buf), a.size))


def zlib_identity(data) -> int:
    """Second, independent oracle: crc(b) == zlib.crc32(b, ~0) ^ ~0."""
    return zlib.crc32(bytes(data), 0xFFFFFFFF) ^ 0xFFFFFFFF


def crc32_blocks(region: np.ndarray, block_size: int, nthreads: int = 1) -> np.ndarray:
    region = np.ascontiguousarray(region).view(np.uint8)
    assert region.size % block_size == 0
    n = region.size // block_size
    out = np.empty(n, dtype=np.uint32)
    if n:
        rc = lib().oracle_crc32_blocks(region.ctypes.data, n, block_size, out.ctypes.data, nthreads)
        assert rc == 0
    return out


def crc32_ranges(region: np.ndarray, offsets, lengths) -> np.ndarray:
    region = np.ascontiguousarray(region).view(np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.empty(offs.size, dtype=np.uint32)
    if offs.size:
        lib().oracle_crc32_ranges(region.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                  offs.size, out.ctypes.data)
    return out


def fill_splitmix(nbytes: int, seed: int, word_offset: int = 0) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        lib().oracle_fill_splitmix(out.ctypes.data, nbytes, seed & (2**64 - 1), word_offset)
    return out


def table() -> np.ndarray:
    t = np.empty(256, dtype=np.uint32)
    lib().oracle_table(t.ctypes.data)
    return t


def splitmix_numpy(nwords: int, seed: int, word_offset: int = 0) -> np.ndarray:
    """Independent numpy restatement of oracle_fill_splitmix (uint64 wraps)."""
    with np.errstate(over="ignore"):
        i = np.arange(word_offset + 1, word_offset + nwords + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def ref_build_info() -> dict:
    """oracle/_ref/BUILDINFO.json (compiler and flags of the reference build), or {}."""
    import json
    try:
        with open(os.path.join(ORACLE_DIR, "_ref", "BUILDINFO.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def time_cpu_baseline(region: np.ndarray, block_size: int, prefer: str = "reference", threads: int = 1,
                      opt: str = "O2"):
    """Time a CPU pass over region's blocks in C (threads > 1: static split).

    prefer="reference": the reference's own server/crc.c (oracle/_ref, built at
    -O2, its release flag, or -O0, its shipped default) when it was built;
    otherwise our restatement ("port").  Returns (seconds, crcs uint32[], kind, label)."""
    L = lib()
    L.oracle_time_blocks_fn.restype = ctypes.c_double
    L.oracle_time_blocks_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_void_p]
    region = np.ascontiguousarray(region).view(np.uint8)
    n = region.size // block_size
    out = np.empty(n, dtype=np.uint32)
    R = ref_lib(opt) if prefer == "reference" else None
    if R is not None:
        fn = ctypes.cast(R.priskv_crc32, ctypes.c_void_p).value
        kind, label = "reference", f"server/crc.c priskv_crc32 compiled -{opt} (oracle/_ref)"
    else:
        fn = ctypes.cast(L.oracle_crc32_u32len, ctypes.c_void_p).value
        kind, label = "port", "oracle/crc_oracle.c byte-serial restatement -O2"
    if threads > 1:
        L.oracle_time_blocks_fn_mt.restype = ctypes.c_double
        L.oracle_time_blocks_fn_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_int]
        secs = L.oracle_time_blocks_fn_mt(fn, region.ctypes.data, n, block_size, out.ctypes.data, threads)
    else:
        secs = L.oracle_time_blocks_fn(fn, region.ctypes.data, n, block_size, out.ctypes.data)
    return secs, out, kind, label
