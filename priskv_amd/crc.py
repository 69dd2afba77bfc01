"""Python mirror of the value-block CRC C ABI (include/crc.h, include/priskv_crc_gpu.h).

PrisKV's own interface for this path is the C function
``uint32_t priskv_crc32(uint8_t *buf, uint32_t len)`` (server/crc.h:37,
server/crc.c:90-109).  This module binds the in-tree ``libpriskv_crc.so``
with ctypes -- exactly the binding a PrisKV maintainer would write (see
INTEGRATION.md) -- and adds torch-tensor conveniences for tests and the
benchmark.  torch is plumbing here (device memory, streams); every checksum
is computed by the library's HIP kernels (or, for ``priskv_crc32`` itself,
by its host C code).

Errors follow the reference's 0 / -errno convention at the C boundary and
surface here as ``OSError(errno, ...)``.  There is no CPU fallback for the
batched calls: if the library or the GPU is missing they raise.
"""
from __future__ import annotations

import ctypes
import errno as _errno
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libpriskv_crc.so")

PATH_ROWS, PATH_EXTENTS, PATH_SMALL, PATH_GENERIC, PATH_STRIDE, PATH_HEAD, PATH_WINDOW = 1, 2, 3, 4, 5, 6, 7
PATH_NAMES = {PATH_ROWS: "rows", PATH_EXTENTS: "extents", PATH_SMALL: "small", PATH_GENERIC: "generic",
              PATH_STRIDE: "stride", PATH_HEAD: "headsplit", PATH_WINDOW: "window"}

_lib: Optional[ctypes.CDLL] = None

# include/priskv_crc_gpu.h: read-roof variants and sink size
ROOF_VARIANTS = 9
ROOF_SINK_WORDS = 8192

# (name, restype, argtypes) for every symbol the two headers declare
_C = ctypes
SIGNATURES = [
    ("priskv_crc32", _C.c_uint32, [_C.c_void_p, _C.c_uint32]),
    ("priskv_crc_ctx_create", _C.c_int, [_C.c_int, _C.POINTER(_C.c_void_p)]),
    ("priskv_crc_ctx_destroy", None, [_C.c_void_p]),
    ("priskv_crc_ctx_device", _C.c_int, [_C.c_void_p]),
    ("priskv_crc_stream_release", _C.c_int, [_C.c_void_p, _C.c_void_p]),
    ("priskv_crc32_blocks_dev", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint32, _C.c_void_p, _C.c_void_p]),
    ("priskv_crc32_ranges_dev", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_void_p, _C.c_void_p]),
    ("priskv_crc32_ranges_dev_bounded", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint64, _C.c_void_p, _C.c_void_p]),
    ("priskv_crc32_verify_dev", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_void_p, _C.c_void_p, _C.c_void_p]),
    ("priskv_crc32_verify_dev_bounded", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint64, _C.c_void_p, _C.c_void_p,
      _C.c_void_p]),
    ("priskv_crc32_blocks_host", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint32, _C.c_void_p]),
    ("priskv_crc32_ranges_host", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_void_p]),
    ("priskv_crc32_blocks_host_multi", _C.c_int,
     [_C.c_void_p, _C.c_int, _C.c_void_p, _C.c_uint64, _C.c_uint32, _C.c_void_p]),
    ("priskv_crc32_ranges_host_multi", _C.c_int,
     [_C.c_void_p, _C.c_int, _C.c_void_p, _C.c_uint64, _C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_void_p]),
    ("priskv_crc_batch_create", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint32, _C.c_uint32, _C.c_void_p, _C.c_void_p,
      _C.POINTER(_C.c_void_p)]),
    ("priskv_crc_batch_submit", _C.c_int, [_C.c_void_p, _C.c_uint64, _C.c_uint32, _C.c_uint64]),
    ("priskv_crc_batch_submitv", _C.c_int, [_C.c_void_p, _C.c_uint64, _C.c_void_p, _C.c_void_p, _C.c_void_p]),
    ("priskv_crc_batch_flush", _C.c_int, [_C.c_void_p]),
    ("priskv_crc_batch_destroy", None, [_C.c_void_p]),
    ("priskv_crc_host_register", _C.c_int, [_C.c_void_p, _C.c_uint64]),
    ("priskv_crc_host_unregister", _C.c_int, [_C.c_void_p]),
    ("priskv_crc32_shift", _C.c_uint32, [_C.c_uint32, _C.c_uint64]),
    ("priskv_crc32_combine", _C.c_uint32, [_C.c_uint32, _C.c_uint32, _C.c_uint64]),
    ("priskv_crc32_host_impl", _C.c_char_p, []),
    ("priskv_crc_fill_splitmix_dev", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint64, _C.c_uint64, _C.c_void_p]),
    ("priskv_crc32_blocks_path", _C.c_int, [_C.c_void_p, _C.c_uint64, _C.c_uint32]),
    ("priskv_crc32_blocks_plan", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint32, _C.c_char_p, _C.c_uint64]),
    ("priskv_crc_read_roof_dev", _C.c_int,
     [_C.c_void_p, _C.c_void_p, _C.c_uint64, _C.c_uint32, _C.c_uint32, _C.c_void_p, _C.c_void_p]),
    ("priskv_crc_version", _C.c_char_p, []),
]


def lib() -> ctypes.CDLL:
    """Load libpriskv_crc.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` or `make -C priskv_amd/csrc`")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        e = -rc
        raise OSError(e, f"{what}: {_errno.errorcode.get(e, e)} ({os.strerror(e)})")


# ---------------------------------------------------------------- host-side ABI
def priskv_crc32(buf) -> int:
    """server/crc.h:37 -- the drop-in host symbol (keys; synchronous, CPU)."""
    a = np.frombuffer(memoryview(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    a = np.ascontiguousarray(a).view(np.uint8)
    if a.size >= 2**32:
        raise ValueError("priskv_crc32 takes a uint32_t length (server/crc.h:37)")
    return int(lib().priskv_crc32(a.ctypes.data if a.size else None, a.size))


def crc32_shift(crc: int, nbytes: int) -> int:
    return int(lib().priskv_crc32_shift(crc & 0xFFFFFFFF, nbytes))


def crc32_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return int(lib().priskv_crc32_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b))


def blocks_path(ptr: int, nblocks: int, block_size: int) -> str:
    rc = lib().priskv_crc32_blocks_path(ptr, nblocks, block_size)
    _check(rc if rc < 0 else 0, "priskv_crc32_blocks_path")
    return PATH_NAMES[rc]


def version() -> str:
    return lib().priskv_crc_version().decode()


def host_impl() -> str:
    """Host path priskv_crc32 folds long inputs with: vclmul / clmul / slice8."""
    return lib().priskv_crc32_host_impl().decode()


def host_register(arr: np.ndarray) -> None:
    _check(lib().priskv_crc_host_register(arr.ctypes.data, arr.nbytes), "priskv_crc_host_register")


def host_unregister(arr: np.ndarray) -> None:
    _check(lib().priskv_crc_host_unregister(arr.ctypes.data), "priskv_crc_host_unregister")


# ---------------------------------------------------------------- context
def _device_args(region, *tensors) -> None:
    """The C ABI takes raw device pointers: a host tensor, another device or a
    strided view would be read as garbage (or fault), so refuse them here."""
    if not region.is_cuda:
        raise ValueError("region must be a device tensor (use the *_host calls for host memory)")
    for t in tensors:
        if not t.is_cuda or t.device != region.device or not t.is_contiguous():
            raise ValueError("offsets / lengths / out must be contiguous tensors on the region's device")


def _host_out(out: Optional[np.ndarray], n: int) -> np.ndarray:
    """A host result array the C code may write n uint32 entries into."""
    if out is None:
        return np.empty(n, dtype=np.uint32)
    if not isinstance(out, np.ndarray) or out.dtype != np.uint32 or not out.flags.c_contiguous or out.size < n:
        raise ValueError(f"out must be a C-contiguous uint32 numpy array of >= {n} entries")
    return out


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


class CrcContext:
    """One libpriskv_crc context (device tables + streamed-path staging)."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().priskv_crc_ctx_create(device, ctypes.byref(self._h)), "priskv_crc_ctx_create")
        self.device = device

    def close(self) -> None:
        if self._h:
            lib().priskv_crc_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def stream_release(self, stream) -> None:
        """Hand `stream`'s scratch-pool slots back (priskv_crc_stream_release;
        waits for the stream).  Call before destroying a stream that ran
        *_dev calls, while no other thread submits to it."""
        _check(lib().priskv_crc_stream_release(self._h, _stream_ptr(stream)), "priskv_crc_stream_release")

    def blocks_plan(self, region_ptr: int, nblocks: int, block_size: int) -> str:
        """The kernel plan blocks_dev would launch (priskv_crc32_blocks_plan)."""
        buf = ctypes.create_string_buffer(256)
        _check(lib().priskv_crc32_blocks_plan(self._h, region_ptr, nblocks, block_size, buf, len(buf)),
               "priskv_crc32_blocks_plan")
        return buf.value.decode()

    # ---- device-resident
    def blocks_dev(self, region, block_size: int, out=None, stream=None, nblocks: Optional[int] = None):
        """d_out[i] = priskv_crc32(region + i*block_size, block_size); returns an int32 cuda
        tensor holding the uint32 bit patterns (asynchronous on `stream`)."""
        import torch
        if not region.is_cuda:
            raise ValueError("region must be a device tensor (use blocks_host for host memory)")
        nbytes = region.numel() * region.element_size()
        n = nbytes // block_size if nblocks is None else nblocks
        if n * block_size > nbytes:
            raise ValueError("nblocks * block_size exceeds the region")
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=region.device)
        if out.numel() < n or out.element_size() != 4 or not out.is_contiguous():
            raise ValueError("out must be a contiguous 4-byte tensor of >= nblocks entries")
        _device_args(region, out)
        _check(lib().priskv_crc32_blocks_dev(self._h, region.data_ptr(), n, block_size, out.data_ptr(),
                                             _stream_ptr(stream)), "priskv_crc32_blocks_dev")
        return out

    def ranges_dev(self, region, offsets, lengths, out=None, stream=None, max_len=None):
        """priskv_crc32_ranges_dev; with max_len (a host-known upper bound on
        the lengths, a launch hint only) priskv_crc32_ranges_dev_bounded."""
        import torch
        n = offsets.numel()
        if lengths.numel() != n or offsets.dtype != torch.int64 or lengths.dtype != torch.int32:
            raise ValueError("offsets must be int64 and lengths int32 device tensors of equal length")
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=region.device)
        if out.numel() < n or out.element_size() != 4:
            raise ValueError("out must be a 4-byte tensor of >= len(offsets) entries")
        _device_args(region, offsets, lengths, out)
        if max_len is not None:
            _check(lib().priskv_crc32_ranges_dev_bounded(self._h, region.data_ptr(), offsets.data_ptr(),
                                                         lengths.data_ptr(), n, int(max_len), out.data_ptr(),
                                                         _stream_ptr(stream)),
                   "priskv_crc32_ranges_dev_bounded")
            return out
        _check(lib().priskv_crc32_ranges_dev(self._h, region.data_ptr(), offsets.data_ptr(),
                                             lengths.data_ptr(), n, out.data_ptr(), _stream_ptr(stream)),
               "priskv_crc32_ranges_dev")
        return out

    def verify_dev(self, region, offsets, lengths, expected, status=None, stream=None, max_len=None):
        """Device verify (priskv_crc32_verify_dev): returns the 2-entry int64
        status tensor {mismatches, first mismatching index or -1 (UINT64_MAX)},
        filled asynchronously on `stream`.  max_len: a host-known bound on the
        lengths (priskv_crc32_verify_dev_bounded, a launch hint only)."""
        import torch
        n = offsets.numel()
        if (lengths.numel() != n or expected.numel() != n or offsets.dtype != torch.int64
                or lengths.dtype != torch.int32 or expected.element_size() != 4):
            raise ValueError("offsets int64, lengths int32 and expected 4-byte device tensors of equal length")
        if status is None:
            status = torch.empty(2, dtype=torch.int64, device=region.device)
        if status.numel() < 2 or status.element_size() != 8:
            raise ValueError("status must be an 8-byte tensor of >= 2 entries")
        _device_args(region, offsets, lengths, expected, status)
        if max_len is not None:
            _check(lib().priskv_crc32_verify_dev_bounded(self._h, region.data_ptr(), offsets.data_ptr(),
                                                         lengths.data_ptr(), n, int(max_len), expected.data_ptr(),
                                                         status.data_ptr(), _stream_ptr(stream)),
                   "priskv_crc32_verify_dev_bounded")
            return status
        _check(lib().priskv_crc32_verify_dev(self._h, region.data_ptr(), offsets.data_ptr(), lengths.data_ptr(),
                                             n, expected.data_ptr(), status.data_ptr(), _stream_ptr(stream)),
               "priskv_crc32_verify_dev")
        return status

    def fill_splitmix(self, region, seed: int, word_offset: int = 0, stream=None, nbytes=None) -> None:
        size = region.numel() * region.element_size()
        nb = size if nbytes is None else nbytes
        if nb > size:
            raise ValueError("nbytes exceeds the region")
        _device_args(region)
        _check(lib().priskv_crc_fill_splitmix_dev(self._h, region.data_ptr(), nb, seed & (2**64 - 1),
                                                  word_offset, _stream_ptr(stream)),
               "priskv_crc_fill_splitmix_dev")

    def read_roof_dev(self, region, block_size: int, sink, stream=None, nblocks: Optional[int] = None,
                      variant: int = 0) -> None:
        """Diagnostic read roof of the CRC kernel's access pattern over `region`
        (priskv_crc_read_roof_dev): variant 0 in the CRC plan's own pipeline
        depth and occupancy, 1 .. ROOF_VARIANTS - 1 in others; sink:
        ROOF_SINK_WORDS 4-byte entries, one per launched wave."""
        nbytes = region.numel() * region.element_size()
        n = nbytes // block_size if nblocks is None else nblocks
        if (n * block_size > nbytes or sink.numel() < ROOF_SINK_WORDS or sink.element_size() != 4
                or not sink.is_contiguous()):
            raise ValueError("nblocks * block_size must fit the region and sink hold ROOF_SINK_WORDS 4-byte entries")
        _device_args(region, sink)
        _check(lib().priskv_crc_read_roof_dev(self._h, region.data_ptr(), n, block_size, variant, sink.data_ptr(),
                                              _stream_ptr(stream)), "priskv_crc_read_roof_dev")

    # ---- host-resident (streamed over PCIe)
    def blocks_host(self, region: np.ndarray, block_size: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        region = np.ascontiguousarray(region).view(np.uint8).reshape(-1)
        n = region.size // block_size
        out = _host_out(out, n)
        _check(lib().priskv_crc32_blocks_host(self._h, region.ctypes.data, n, block_size, out.ctypes.data),
               "priskv_crc32_blocks_host")
        return out


def _ranges_host(self, region: np.ndarray, offsets, lengths, out: Optional[np.ndarray] = None) -> np.ndarray:
    """Per-value extents of a host region (memfile scrub), zero-copy over PCIe."""
    region = np.ascontiguousarray(region).view(np.uint8).reshape(-1)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lengths, dtype=np.uint32)
    if offs.shape != lens.shape:
        raise ValueError("offsets and lengths must have the same length")
    out = _host_out(out, offs.size)
    _check(lib().priskv_crc32_ranges_host(self._h, region.ctypes.data, region.size, offs.ctypes.data,
                                          lens.ctypes.data, offs.size, out.ctypes.data),
           "priskv_crc32_ranges_host")
    return out


CrcContext.ranges_host = _ranges_host


def _ctx_array(ctxs):
    arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    return arr


def blocks_host_multi(ctxs, region: np.ndarray, block_size: int, out: Optional[np.ndarray] = None) -> np.ndarray:
    """Host-resident blocks split across several contexts (one GPU each)."""
    region = np.ascontiguousarray(region).view(np.uint8).reshape(-1)
    n = region.size // block_size
    out = _host_out(out, n)
    _check(lib().priskv_crc32_blocks_host_multi(_ctx_array(ctxs), len(ctxs), region.ctypes.data, n, block_size,
                                                out.ctypes.data), "priskv_crc32_blocks_host_multi")
    return out


def ranges_host_multi(ctxs, region: np.ndarray, offsets, lengths, out: Optional[np.ndarray] = None) -> np.ndarray:
    """Host extents (memfile scrub) split across several contexts (one GPU each)."""
    region = np.ascontiguousarray(region).view(np.uint8).reshape(-1)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lengths, dtype=np.uint32)
    if offs.shape != lens.shape:
        raise ValueError("offsets and lengths must have the same length")
    out = _host_out(out, offs.size)
    _check(lib().priskv_crc32_ranges_host_multi(_ctx_array(ctxs), len(ctxs), region.ctypes.data, region.size,
                                                offs.ctypes.data, lens.ctypes.data, offs.size, out.ctypes.data),
           "priskv_crc32_ranges_host_multi")
    return out


BATCH_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int)


class CrcBatcher:
    """SET-completion batcher (priskv_crc_batch_*): submit (value_off,
    valuelen, cookie) from any thread; callback(cookie, crc, status) runs on
    the library's worker thread once the value's batch has been hashed."""

    def __init__(self, ctx: "CrcContext", region: np.ndarray, callback, max_batch: int = 1024,
                 max_delay_us: int = 200):
        self._region = region  # keep the mapping alive
        self._cb = BATCH_CB(lambda _arg, cookie, crc, status: callback(cookie, crc, status))
        self._h = ctypes.c_void_p()
        _check(lib().priskv_crc_batch_create(ctx.handle, region.ctypes.data, region.nbytes, max_batch, max_delay_us,
                                             self._cb, None, ctypes.byref(self._h)), "priskv_crc_batch_create")

    def submit(self, value_off: int, valuelen: int, cookie: int) -> None:
        _check(lib().priskv_crc_batch_submit(self._h, value_off, valuelen, cookie), "priskv_crc_batch_submit")

    def submitv(self, value_offs, valuelens, cookies) -> None:
        o = np.ascontiguousarray(value_offs, dtype=np.uint64)
        ln = np.ascontiguousarray(valuelens, dtype=np.uint32)
        c = np.ascontiguousarray(cookies, dtype=np.uint64)
        if not (o.size == ln.size == c.size):
            raise ValueError("value_offs, valuelens and cookies must have the same length")
        _check(lib().priskv_crc_batch_submitv(self._h, o.size, o.ctypes.data, ln.ctypes.data, c.ctypes.data),
               "priskv_crc_batch_submitv")

    def flush(self) -> None:
        _check(lib().priskv_crc_batch_flush(self._h), "priskv_crc_batch_flush")

    def close(self) -> None:
        if self._h:
            lib().priskv_crc_batch_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def as_u32(t) -> np.ndarray:
    """int32 tensor of CRC bit patterns -> numpy uint32."""
    return t.detach().cpu().numpy().view(np.uint32)
