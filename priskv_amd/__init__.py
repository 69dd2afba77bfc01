"""priskv_amd -- MI355X-native value-block CRC for PrisKV.

The product is the C-ABI library priskv_amd/lib/libpriskv_crc.so
(include/crc.h + include/priskv_crc_gpu.h); this package binds it.
"""
from .crc import (CrcContext, as_u32, blocks_path, crc32_combine, crc32_shift, host_register,  # noqa: F401
                  host_unregister, lib, priskv_crc32, version)

__all__ = ["CrcContext", "as_u32", "blocks_path", "crc32_combine", "crc32_shift", "host_register",
           "host_unregister", "lib", "priskv_crc32", "version"]
