"""priskv_amd -- MI355X-native value-block CRC for PrisKV.

The product is the C-ABI library priskv_amd/lib/libpriskv_crc.so
(include/crc.h + include/priskv_crc_gpu.h); this package binds it.
"""
from .crc import (CrcBatcher, CrcContext, as_u32, blocks_host_multi, blocks_path, crc32_combine, crc32_shift,  # noqa: F401
                  host_impl, host_register, host_unregister, lib, priskv_crc32, ranges_host_multi, version)

__all__ = ["CrcBatcher", "CrcContext", "as_u32", "blocks_host_multi", "ranges_host_multi", "blocks_path", "crc32_combine", "crc32_shift", "host_impl", "host_register",
           "host_unregister", "lib", "priskv_crc32", "version"]
