/* crc_internal.h -- hidden helpers shared by crc_host.c and crc_gpu.hip. */
#ifndef PRISKV_CRC_INTERNAL_H
#define PRISKV_CRC_INTERNAL_H

#include <stdint.h>

#if defined(__cplusplus)
extern "C"
{
#endif

#define PRV_HIDDEN __attribute__((visibility("hidden")))

/* LDS image: 256 rows x 64 words (256 B): words [0,32) = set A (Z_4),
 * words [32,64) = set B (Z_(4+gap)); word 4k+t of a half = table for byte
 * position t, copy k (k = 0..7).  64 KiB total. */
#define PRV_LDS_WORDS (256 * 64)

/* wave row: 64 lanes x 16 B */
#define PRV_ROW_BYTES 1024u
#define PRV_ROW_GAP (PRV_ROW_BYTES - 16u)

PRV_HIDDEN void prv_lds_image(uint32_t out[PRV_LDS_WORDS], uint32_t gap_bytes);
PRV_HIDDEN void prv_lds_image_step(uint32_t out[PRV_LDS_WORDS], uint32_t step, uint32_t gap_bytes);
PRV_HIDDEN void prv_fold_columns(uint32_t out[32 * 64], uint32_t group);
/* nibble fold tables, 8*16*width words (crc_device.inc nib_fold) */
PRV_HIDDEN void prv_fold_nibbles(uint32_t *out, uint32_t group, uint32_t width);
PRV_HIDDEN void prv_shift_columns(uint32_t out[32], uint64_t nbytes);
/* sub-KiB byte-fold image for G = 2..16 lanes per block (crc_device.inc
 * byte_fold): set A of prv_lds_image in words [0,32) of each 64-word row,
 * the byte fold tables in words [32,64); G = 16 adds a second 64 KiB region
 * (tables of bytes 2, 3).  PRV_SMALL_WORDS(G) words. */
#define PRV_SMALL_WORDS(G) ((G) == 16 ? 2 * PRV_LDS_WORDS : PRV_LDS_WORDS)
PRV_HIDDEN void prv_small_image(uint32_t *out, uint32_t group);
PRV_HIDDEN void prv_sarwate_table(uint32_t out[256]);
/* host CRC register update (init = crc, no xor): tables; clmul folding for
 * len >= 64 / vclmul for len >= 256 (x86-64, after prv_clmul_init) */
PRV_HIDDEN uint32_t prv_crc32_table(uint32_t crc, const uint8_t *p, uint64_t len);
PRV_HIDDEN void prv_clmul_init(void);
PRV_HIDDEN uint32_t prv_crc32_clmul(uint32_t crc, const uint8_t *p, uint64_t len);
PRV_HIDDEN uint32_t prv_crc32_vclmul(uint32_t crc, const uint8_t *p, uint64_t len);
/* out[p*32 + i] = column i of Z_-p (p = 0..15): undoes p trailing zero bytes */
PRV_HIDDEN void prv_unshift_columns(uint32_t out[16 * 32]);
/* out[(4p + k)*32 + j] = column j of Z_-p o Z_(256(3-k)) (extents nibble fold) */
PRV_HIDDEN void prv_rowshift_columns(uint32_t out[16 * 4 * 32]);

#if defined(__cplusplus)
}
#endif

#endif
