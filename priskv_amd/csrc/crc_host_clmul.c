/*
 * crc_host_clmul.c -- carry-less-multiply folding for the host priskv_crc32
 * (a faster CPU path for keys, bit-exact with
 * server/crc.c:90-109 -- reflected 0xEDB88320, init 0, no final xor).
 *
 * The message is consumed 16 bytes (one 128-bit lane) at a time.  Read in
 * the reflected bit order of server/crc.c, a lane is a polynomial of degree
 * < 128; "folding" lane X over the next D bits of the message replaces it by
 *     X_lo * k(D + 32)  ^  X_hi * k(D - 32)        (two 64x64 clmuls)
 * and XORs the lane D bits further on, where k(e) = reflect32(x^e mod P) << 1
 * (P = 0x104C11DB7, the normal form of 0xEDB88320).  Folding keeps the
 * invariant "CRC of the bytes consumed so far == CRC of the 16 bytes of the
 * running lane with register 0", so the last lane is finished with two
 * slice-by-8 steps instead of a Barrett reduction, and the < 16-byte tail
 * with byte steps -- no reduction constants at all.  The constants are
 * computed at init from the polynomial (host_init in crc_host.c), not
 * tabulated.
 *
 *   prv_crc32_clmul   PCLMULQDQ, 4 x 128-bit lanes (64 B per turn), len >= 64
 *   prv_crc32_vclmul  VPCLMULQDQ + AVX-512, 4 x 512-bit lanes (256 B per
 *                     turn), len >= 256
 * Both are compiled with function target attributes: the library builds for
 * any x86-64 and crc_host.c picks the path at run time (cpuid).
 */
#if defined(__x86_64__)
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include "crc_internal.h"

static uint64_t g_k[2 * 2048 / 64 + 2]; /* g_k[e/32] = k(e), e a multiple of 32, 0 <= e <= 2080 */

static uint64_t xpow_mod(unsigned e)
{
    uint64_t r = 1;
    for (unsigned i = 0; i < e; i++) {
        r <<= 1;
        if (r & (1ull << 32))
            r ^= 0x104C11DB7ull;
    }
    return r;
}

static uint64_t reflect32(uint64_t v)
{
    uint64_t r = 0;
    for (int i = 0; i < 32; i++)
        if (v & (1ull << i))
            r |= 1ull << (31 - i);
    return r;
}

void prv_clmul_init(void)
{
    for (unsigned e = 0; e <= 2080; e += 32)
        g_k[e / 32] = reflect32(xpow_mod(e)) << 1;
}

static inline uint64_t k(unsigned e) { return g_k[e / 32]; }

/* fold constant for a distance of D bits: {lo qword: k(D + 32), hi: k(D - 32)} */
__attribute__((target("pclmul,sse2"))) static inline __m128i kfold(unsigned D)
{
    return _mm_set_epi64x((long long)k(D - 32), (long long)k(D + 32));
}

__attribute__((target("pclmul,sse2"))) static inline __m128i fold128(__m128i x, __m128i kk, __m128i next)
{
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, kk, 0x00), _mm_clmulepi64_si128(x, kk, 0x11)),
                         next);
}

__attribute__((target("pclmul,sse2"))) static inline __m128i ld(const uint8_t *p)
{
    return _mm_loadu_si128((const __m128i *)p);
}

/* 16-byte lanes from the running lane x: fold in the remaining whole lanes,
 * then finish x and the tail with table steps */
__attribute__((target("pclmul,sse2"))) static uint32_t finish(__m128i x, const uint8_t *p, uint64_t len)
{
    const __m128i k1 = kfold(128);
    while (len >= 16) {
        x = fold128(x, k1, ld(p));
        p += 16;
        len -= 16;
    }
    uint8_t b[16];
    _mm_storeu_si128((__m128i *)b, x);
    return prv_crc32_table(prv_crc32_table(0, b, 16), p, len);
}

__attribute__((target("pclmul,sse2"))) uint32_t prv_crc32_clmul(uint32_t crc, const uint8_t *p, uint64_t len)
{
    const __m128i k4 = kfold(512), k1 = kfold(128);
    __m128i x0 = _mm_xor_si128(ld(p), _mm_cvtsi32_si128((int)crc));
    __m128i x1 = ld(p + 16), x2 = ld(p + 32), x3 = ld(p + 48);
    p += 64;
    len -= 64;
    while (len >= 64) {
        x0 = fold128(x0, k4, ld(p));
        x1 = fold128(x1, k4, ld(p + 16));
        x2 = fold128(x2, k4, ld(p + 32));
        x3 = fold128(x3, k4, ld(p + 48));
        p += 64;
        len -= 64;
    }
    x1 = fold128(x0, k1, x1);
    x2 = fold128(x1, k1, x2);
    x3 = fold128(x2, k1, x3);
    return finish(x3, p, len);
}

#define TGT512 __attribute__((target("avx512f,vpclmulqdq,pclmul,sse2")))

TGT512 static inline __m512i fold512(__m512i x, __m512i kk, __m512i next)
{
    return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, kk, 0x00), _mm512_clmulepi64_epi128(x, kk, 0x11),
                                     next, 0x96);
}

TGT512 static inline __m512i kfold512(unsigned D)
{
    return _mm512_broadcast_i32x4(_mm_set_epi64x((long long)k(D - 32), (long long)k(D + 32)));
}

TGT512 uint32_t prv_crc32_vclmul(uint32_t crc, const uint8_t *p, uint64_t len)
{
    const __m512i k16 = kfold512(2048), k4 = kfold512(512);
    __m512i z0 = _mm512_xor_si512(_mm512_loadu_si512(p),
                                  _mm512_inserti32x4(_mm512_setzero_si512(), _mm_cvtsi32_si128((int)crc), 0));
    __m512i z1 = _mm512_loadu_si512(p + 64), z2 = _mm512_loadu_si512(p + 128), z3 = _mm512_loadu_si512(p + 192);
    p += 256;
    len -= 256;
    while (len >= 256) {
        z0 = fold512(z0, k16, _mm512_loadu_si512(p));
        z1 = fold512(z1, k16, _mm512_loadu_si512(p + 64));
        z2 = fold512(z2, k16, _mm512_loadu_si512(p + 128));
        z3 = fold512(z3, k16, _mm512_loadu_si512(p + 192));
        p += 256;
        len -= 256;
    }
    z1 = fold512(z0, k4, z1);
    z2 = fold512(z1, k4, z2);
    z3 = fold512(z2, k4, z3);
    while (len >= 64) {
        z3 = fold512(z3, k4, _mm512_loadu_si512(p));
        p += 64;
        len -= 64;
    }
    /* the four lanes of z3 into one: lane j (0..2) folds over (3 - j) * 128
     * bits onto lane 3 (whose constant is 0) */
    const __m512i kl = _mm512_set_epi64(0, 0, (long long)k(96), (long long)k(160), (long long)k(224),
                                        (long long)k(288), (long long)k(352), (long long)k(416));
    const __m512i t = _mm512_xor_si512(_mm512_clmulepi64_epi128(z3, kl, 0x00), _mm512_clmulepi64_epi128(z3, kl, 0x11));
    __m128i x = _mm_xor_si128(_mm_xor_si128(_mm512_extracti32x4_epi32(t, 0), _mm512_extracti32x4_epi32(t, 1)),
                              _mm_xor_si128(_mm512_extracti32x4_epi32(t, 2), _mm512_extracti32x4_epi32(z3, 3)));
    return finish(x, p, len);
}
#endif
