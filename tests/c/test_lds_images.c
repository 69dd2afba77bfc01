/*
 * test_lds_images.c -- the sub-KiB byte-fold LDS image (prv_small_image,
 * crc_host.c) against the addresses the kernels compute (crc_device.inc
 * lane_const / fold_const), on the CPU.  For every G = 2..16, lane, lookup
 * i and byte value b:
 *   - the main set-A lookup at byte b*256 + 16k + 4t holds Z_4(b << 8t);
 *   - the fold lookup at (column byte) | b << 8 | plane << 16 holds
 *     Z_(4 + 16(G-1-c))(b << 8j), c = lane % G, for the byte j the lane reads;
 *   - each lane reads every byte j of the register once over i = 0..3;
 *   - the 32 lanes of each ds_read half hit 32 distinct banks (word % 32)
 *     in every lookup, whatever the data.
 * Z_n is checked through the library's own priskv_crc32_shift, which
 * tests/test_host_abi.py pins against the oracle.  Links
 * libpriskv_crc_host.a (prv_small_image is a hidden, internal symbol).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "priskv_crc_gpu.h"

#define LDS_WORDS (256 * 64)
void prv_small_image(uint32_t *out, uint32_t group); /* crc_internal.h */

static int failures;
#define CHECK(cond, ...)                                                                                   \
    do {                                                                                                   \
        if (!(cond)) {                                                                                     \
            if (failures++ < 10)                                                                           \
                printf("[FAILED] " __VA_ARGS__);                                                           \
        }                                                                                                  \
    } while (0)

/* the kernel's fold_const: column byte and register byte j of lookup i */
static void fold_lookup(uint32_t G, uint32_t lane, uint32_t i, uint32_t *colbyte, uint32_t *j, uint32_t *plane)
{
    const uint32_t h = (lane & 31) / G, cc = lane % G;
    if (G == 16) {
        *j = 2 * (i >> 1) + ((i + h) & 1);
        *colbyte = 128 + 4 * (16 * (*j & 1) + cc);
        *plane = i >= 2;
    } else {
        *j = (i + h) & 3;
        *colbyte = 128 + 4 * ((h >> 2) * 4 * G + *j * G + cc);
        *plane = 0;
    }
}

int main(void)
{
    static uint32_t img[2 * LDS_WORDS];
    for (uint32_t G = 2; G <= 16; G *= 2) {
        prv_small_image(img, G);
        /* main set A: copy k, table t (lane_const: byte i of the register at 16k + 4t) */
        for (uint32_t b = 0; b < 256; b++)
            for (uint32_t k = 0; k < 8; k++)
                for (uint32_t t = 0; t < 4; t++)
                    CHECK(img[(b * 256 + 16 * k + 4 * t) / 4] == priskv_crc32_shift(b << (8 * t), 4),
                          "G=%u set A b=%u k=%u t=%u\n", G, b, k, t);
        for (uint32_t lane = 0; lane < 64; lane++) {
            const uint32_t c = lane % G;
            uint32_t seen = 0;
            for (uint32_t i = 0; i < 4; i++) {
                uint32_t cb, j, pl;
                fold_lookup(G, lane, i, &cb, &j, &pl);
                CHECK(cb < 256, "G=%u lane %u lookup %u: column byte %u\n", G, lane, i, cb);
                seen |= 1u << j;
                for (uint32_t b = 0; b < 256; b++) {
                    const uint32_t addr = cb | (b << 8) | (pl << 16);
                    CHECK(img[addr / 4] == priskv_crc32_shift(b << (8 * j), 4 + 16 * (G - 1 - c)),
                          "G=%u lane %u lookup %u b=%u\n", G, lane, i, b);
                }
            }
            CHECK(seen == 15, "G=%u lane %u reads bytes %x\n", G, lane, seen);
        }
        for (uint32_t half = 0; half < 2; half++)
            for (uint32_t i = 0; i < 4; i++) {
                uint32_t banks = 0;
                for (uint32_t l = 32 * half; l < 32 * half + 32; l++) {
                    uint32_t cb, j, pl;
                    fold_lookup(G, l, i, &cb, &j, &pl);
                    banks |= 1u << ((cb / 4) % 32); /* b*64 and plane*16384 words are 0 mod 32 */
                }
                CHECK(banks == 0xFFFFFFFFu, "G=%u half %u lookup %u: banks %08x\n", G, half, i, banks);
            }
    }
    printf(failures ? "test_lds_images: FAILED (%d)\n" : "test_lds_images: OK\n", failures);
    return failures ? 1 : 0;
}
