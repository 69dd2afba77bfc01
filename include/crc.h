/*
 * crc.h -- drop-in for PrisKV's server/crc.h.
 *
 * Replaces: server/crc.h:37  `uint32_t priskv_crc32(uint8_t *buf, uint32_t len);`
 * (same include guard, server/crc.h:27-28; same extern "C" guards, :30-41).
 * Callers that link it unchanged: server/kv.c:314 (priskv_find_key),
 * server/kv.c:408 (priskv_insert_keynode), server/rdma.c:764
 * (priskv_tiering_req_new).
 *
 * Implemented on the host in priskv_amd/csrc/crc_host.c, bit-exact with
 * server/crc.c:90-109 (reflected 0xEDB88320, init 0, no final xor): a
 * VPCLMULQDQ or PCLMULQDQ fold for longer inputs where the CPU has it
 * (crc_host_clmul.c, chosen once from cpuid), slice-by-8 tables otherwise
 * and for short inputs.  This
 * symbol hashes keys (<= 1 KiB, server/rdma.h:49) synchronously on the RDMA
 * completion path, where a GPU launch would cost more than the work; the
 * batched value-block checksum runs on the GPU through priskv_crc_gpu.h.
 */
#ifndef __PRISKV_SERVER_CRC__
#define __PRISKV_SERVER_CRC__

#if defined(__cplusplus)
extern "C"
{
#endif

#include <stdint.h>

uint32_t priskv_crc32(uint8_t *buf, uint32_t len);

#if defined(__cplusplus)
}
#endif

#endif /* __PRISKV_SERVER_CRC__ */
