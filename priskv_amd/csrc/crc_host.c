/*
 * crc_host.c -- host side of the PrisKV value-block CRC (C, no HIP).
 *
 * 1. priskv_crc32(): the drop-in for server/crc.c:90-109 / server/crc.h:37.
 *    Bit-exact with the reference (reflected 0xEDB88320, init 0 at :92, no
 *    final xor at :108) but processes 8 bytes per step with eight tables
 *    (slice-by-8) instead of the reference's byte-serial table walk
 *    (:70-88), and folds inputs of >= 64 B with carry-less multiplies
 *    (crc_host_clmul.c: PCLMULQDQ, or VPCLMULQDQ/AVX-512 from 256 B).  Reentrant: the tables are built once under pthread_once
 *    (SURVEY §8b threading row) and only read afterwards; buf is never
 *    written or retained.  It stays on the CPU because its callers hash keys
 *    of <= 1 KiB synchronously on the RDMA completion path
 *    (server/kv.c:314,408, server/rdma.c:764).
 *
 * 2. GF(2) algebra for the GPU path.  With init 0 and no xorout the CRC is a
 *    linear map, so "advance the register over n zero bytes" (Z_n) is a 32x32
 *    bit matrix and crc(A||B) = Z_|B|(crc(A)) ^ crc(B).  The GPU kernels need
 *      - the 64 KiB LDS image of slice-by-4 tables for Z_4 (set A) and for
 *        Z_(4+row gap) (set B), in the rotated 8-copy layout described in
 *        DESIGN.md §3 (conflict-free ds_read_b32 for any index pattern);
 *      - per-lane fold columns: lane l's partial is advanced by
 *        Z_(16*(G-1-l%G)) before the cross-lane XOR;
 *      - shift columns Z_(2^k) for combining segment partials.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/crc.h"
#include "../../include/priskv_crc_gpu.h"
#include "crc_internal.h"

#define POLY 0xEDB88320u

static uint32_t g_slice[8][256];     /* g_slice[k][b]: byte b followed by k zero bytes */
static uint32_t g_zpow[64][32];      /* columns of Z_(2^k) */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
/* host path of priskv_crc32 for inputs long enough to fold (crc_host_clmul.c);
 * picked once from cpuid, capped by PRISKV_CRC_HOST_IMPL=slice8|clmul|vclmul */
enum { IMPL_SLICE8, IMPL_CLMUL, IMPL_VCLMUL };
static int g_impl = IMPL_SLICE8;

static uint32_t mat_apply(const uint32_t m[32], uint32_t v)
{
    uint32_t r = 0;
    while (v) {
        int i = __builtin_ctz(v);
        r ^= m[i];
        v &= v - 1;
    }
    return r;
}

/* out = a o b (apply b first); out may alias neither input */
static void mat_compose(uint32_t out[32], const uint32_t a[32], const uint32_t b[32])
{
    for (int i = 0; i < 32; i++)
        out[i] = mat_apply(a, b[i]);
}

static void host_init(void)
{
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++)
            c = (c & 1) ? (c >> 1) ^ POLY : (c >> 1);
        g_slice[0][b] = c;
    }
    for (int k = 1; k < 8; k++)
        for (int b = 0; b < 256; b++) {
            uint32_t p = g_slice[k - 1][b];
            g_slice[k][b] = (p >> 8) ^ g_slice[0][p & 0xff];
        }
    /* Z_1: one zero byte through the register */
    for (int i = 0; i < 32; i++) {
        uint32_t v = 1u << i;
        g_zpow[0][i] = g_slice[0][v & 0xff] ^ (v >> 8);
    }
    for (int k = 1; k < 64; k++)
        mat_compose(g_zpow[k], g_zpow[k - 1], g_zpow[k - 1]);
#if defined(__x86_64__)
    prv_clmul_init();
    __builtin_cpu_init();
    if (__builtin_cpu_supports("pclmul"))
        g_impl = IMPL_CLMUL;
    if (g_impl == IMPL_CLMUL && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("vpclmulqdq"))
        g_impl = IMPL_VCLMUL;
    const char *want = getenv("PRISKV_CRC_HOST_IMPL");
    if (want) {
        const int cap = !strcmp(want, "slice8") ? IMPL_SLICE8 : (!strcmp(want, "clmul") ? IMPL_CLMUL : IMPL_VCLMUL);
        if (cap < g_impl)
            g_impl = cap;
    }
#endif
}

static inline uint32_t load_le32(const uint8_t *p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return v; /* x86-64 / aarch64-le hosts */
}

/* slice-by-8 over whole 8-byte steps, then byte steps (server/crc.c:70-73) */
uint32_t prv_crc32_table(uint32_t crc, const uint8_t *p, uint64_t len)
{
    while (len >= 8) {
        uint32_t lo = load_le32(p) ^ crc;
        uint32_t hi = load_le32(p + 4);
        crc = g_slice[7][lo & 0xff] ^ g_slice[6][(lo >> 8) & 0xff] ^
              g_slice[5][(lo >> 16) & 0xff] ^ g_slice[4][lo >> 24] ^ g_slice[3][hi & 0xff] ^
              g_slice[2][(hi >> 8) & 0xff] ^ g_slice[1][(hi >> 16) & 0xff] ^ g_slice[0][hi >> 24];
        p += 8;
        len -= 8;
    }
    while (len--)
        crc = g_slice[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
    return crc;
}

uint32_t priskv_crc32(uint8_t *buf, uint32_t len)
{
    pthread_once(&g_once, host_init);
#if defined(__x86_64__)
    if (len >= 256 && g_impl >= IMPL_VCLMUL)
        return prv_crc32_vclmul(0, buf, len);
    if (len >= 64 && g_impl >= IMPL_CLMUL)
        return prv_crc32_clmul(0, buf, len);
#endif
    return prv_crc32_table(0, buf, len);
}

const char *priskv_crc32_host_impl(void)
{
    pthread_once(&g_once, host_init);
    static const char *const names[] = {"slice8", "clmul", "vclmul"};
    return names[g_impl];
}

uint32_t priskv_crc32_shift(uint32_t crc, uint64_t nbytes)
{
    pthread_once(&g_once, host_init);
    for (int k = 0; nbytes && crc; k++, nbytes >>= 1)
        if (nbytes & 1)
            crc = mat_apply(g_zpow[k], crc);
    return crc;
}

uint32_t priskv_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    return priskv_crc32_shift(crc_a, len_b) ^ crc_b;
}

/* ---- internal (hidden) builders for the HIP shim ---------------------- */

void prv_shift_columns(uint32_t out[32], uint64_t nbytes)
{
    for (int i = 0; i < 32; i++)
        out[i] = priskv_crc32_shift(1u << i, nbytes);
}

void prv_lds_image(uint32_t out[PRV_LDS_WORDS], uint32_t gap_bytes)
{
    prv_lds_image_step(out, 4, gap_bytes);
}

void prv_lds_image_step(uint32_t out[PRV_LDS_WORDS], uint32_t step, uint32_t gap_bytes)
{
    /* as prv_lds_image with Z_step / Z_(step+gap) (step 8: slice-by-8 pairs) */
    uint32_t za[32], zb[32];
    prv_shift_columns(za, step);
    prv_shift_columns(zb, step + (uint64_t)gap_bytes);
    for (uint32_t idx = 0; idx < 256; idx++)
        for (uint32_t k = 0; k < 8; k++)
            for (uint32_t t = 0; t < 4; t++) {
                /* slot t of copy k holds the table for byte position t of the
                 * 32-bit register: E_t[idx] = Z(idx << 8t) */
                out[idx * 64 + 4 * k + t] = mat_apply(za, idx << (8 * t));
                out[idx * 64 + 32 + 4 * k + t] = mat_apply(zb, idx << (8 * t));
            }
}

void prv_fold_columns(uint32_t out[32 * 64], uint32_t group)
{
    /* out[i*64 + l] = column i of Z_(16*(G-1-(l%G))), G = group (1..64) */
    for (uint32_t l = 0; l < 64; l++) {
        uint64_t dist = 16ull * (group - 1 - (l % group));
        for (int i = 0; i < 32; i++)
            out[i * 64 + l] = priskv_crc32_shift(1u << i, dist);
    }
}

void prv_fold_nibbles(uint32_t *out, uint32_t group, uint32_t width)
{
    /* out[(16n + v)*width + s] = Z_(4 + 16(G-1-s%G))(v << 4n), G = group
     * (2..64), width a multiple of G: the nibble tables of nib_fold
     * (crc_device.inc), one slot per lane of a ds_read half */
    for (uint32_t sl = 0; sl < width; sl++) {
        const uint64_t dist = 4ull + 16ull * (group - 1 - sl % group);
        for (uint32_t n = 0; n < 8; n++)
            for (uint32_t v = 0; v < 16; v++)
                out[(16 * n + v) * width + sl] = priskv_crc32_shift(v << (4 * n), dist);
    }
}

void prv_small_image(uint32_t *out, uint32_t group)
{
    /* set A (Z_4) as prv_lds_image; fold entry F_j[b][c] = Z_(4 + 16(G-1-c))(b << 8j)
     * at word region(j)*PRV_LDS_WORDS + b*64 + 32 + e (layout: crc_device.inc fold_const) */
    const uint32_t G = group;
    uint32_t za[32];
    prv_shift_columns(za, 4);
    memset(out, 0, sizeof(uint32_t) * PRV_SMALL_WORDS(G));
    for (uint32_t b = 0; b < 256; b++)
        for (uint32_t k = 0; k < 8; k++)
            for (uint32_t t = 0; t < 4; t++)
                out[b * 64 + 4 * k + t] = mat_apply(za, b << (8 * t));
    for (uint32_t c = 0; c < G; c++) {
        uint32_t zc[32];
        prv_shift_columns(zc, 4ull + 16ull * (G - 1 - c));
        for (uint32_t j = 0; j < 4; j++)
            for (uint32_t b = 0; b < 256; b++) {
                const uint32_t v = mat_apply(zc, b << (8 * j));
                if (G == 16) {
                    out[(j >> 1) * PRV_LDS_WORDS + b * 64 + 32 + 16 * (j & 1) + c] = v;
                } else {
                    for (uint32_t cp = 0; cp < 8 / G; cp++)
                        out[b * 64 + 32 + cp * 4 * G + j * G + c] = v;
                }
            }
    }
}

/* one zero byte backwards: c' = T[c & 0xff] ^ (c >> 8) has top byte
 * T[c & 0xff] >> 24, and the top bytes of the 256 table entries are distinct,
 * so c & 0xff = b with T[b] >> 24 == c' >> 24 and c = ((c' ^ T[b]) << 8) | b */
static uint32_t unshift_byte(uint32_t c, const uint8_t inv_top[256])
{
    const uint32_t b = inv_top[c >> 24];
    return ((c ^ g_slice[0][b]) << 8) | b;
}

void prv_unshift_columns(uint32_t out[16 * 32])
{
    pthread_once(&g_once, host_init);
    uint8_t inv_top[256];
    for (uint32_t b = 0; b < 256; b++)
        inv_top[g_slice[0][b] >> 24] = (uint8_t)b;
    for (int i = 0; i < 32; i++) {
        uint32_t v = 1u << i;
        for (int p = 0; p < 16; p++) {
            out[p * 32 + i] = v; /* column i of Z_-p */
            v = unshift_byte(v, inv_top);
        }
    }
}

void prv_rowshift_columns(uint32_t out[16 * 4 * 32])
{
    /* out[(4p + k)*32 + j] = Z_-p(Z_(256(3-k))(1 << j)): row k's total of the
     * extents kernel's nibble fold, shifted to the extent end and back over p
     * pad bytes */
    uint32_t un[16 * 32];
    prv_unshift_columns(un);
    for (int p = 0; p < 16; p++)
        for (int k = 0; k < 4; k++)
            for (int j = 0; j < 32; j++) {
                uint32_t cols[32];
                for (int i = 0; i < 32; i++)
                    cols[i] = un[p * 32 + i];
                out[(4 * p + k) * 32 + j] = mat_apply(cols, priskv_crc32_shift(1u << j, 256u * (3 - k)));
            }
}

void prv_sarwate_table(uint32_t out[256])
{
    pthread_once(&g_once, host_init);
    memcpy(out, g_slice[0], sizeof(g_slice[0]));
}
