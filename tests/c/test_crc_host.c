/*
 * test_crc_host.c -- the drop-in priskv_crc32 (include/crc.h) exercised the way
 * PrisKV's own unit tests are written (server/test/test_kv.c, test_kv_mt.c):
 * a standalone C executable, assert-style checks, "[OK]"/"[FAILED]" lines and
 * a non-zero exit status on failure.  Links libpriskv_crc_host.a exactly as
 * the server would link crc.o (server/Makefile:32-35).
 *
 *  - known answers (the reference's outputs, zlib-cross-checked);
 *  - every length 0..4200 at every alignment 0..63 against a byte-serial
 *    Sarwate restatement of server/crc.c:70-73,90-109 kept in this file;
 *  - 4 threads hashing concurrently with no lock (test_kv_mt.c:42-44 style),
 *    which covers the first-call table initialisation race.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crc.h"

static uint32_t T[256];

static void sarwate_init(void)
{
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++)
            c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        T[i] = c;
    }
}

static uint32_t sarwate(const uint8_t *p, uint32_t n)
{
    uint32_t crc = 0; /* init 0, no final xor (server/crc.c:92,108) */
    while (n--)
        crc = T[(crc ^ *p++) & 0xff] ^ (crc >> 8);
    return crc;
}

static int failures;
#define CHECK(cond, ...)                                                                                      \
    do {                                                                                                      \
        if (!(cond)) {                                                                                        \
            printf("  check failed at %s:%d: ", __FILE__, __LINE__);                                        \
            printf(__VA_ARGS__);                                                                              \
            printf("\n");                                                                                     \
            failures++;                                                                                       \
        }                                                                                                     \
    } while (0)

static void test_known_answers(void)
{
    const int before = failures;
    static const struct {
        const char *s;
        uint32_t crc;
    } ka[] = {{"", 0x00000000u},
              {"a", 0x3ab551ceu},
              {"abc", 0xca6598d0u},
              {"123456789", 0x2dfd2d88u},
              {"The quick brown fox jumps over the lazy dog", 0xb9c60808u}};
    for (size_t i = 0; i < sizeof(ka) / sizeof(ka[0]); i++) {
        const uint32_t got = priskv_crc32((uint8_t *)ka[i].s, (uint32_t)strlen(ka[i].s));
        CHECK(got == ka[i].crc, "\"%s\": 0x%08x != 0x%08x", ka[i].s, got, ka[i].crc);
    }
    uint8_t z[4096], f[16];
    memset(z, 0, sizeof(z));
    memset(f, 0xff, sizeof(f));
    CHECK(priskv_crc32(z, sizeof(z)) == 0u, "4096 zero bytes");
    CHECK(priskv_crc32(f, sizeof(f)) == 0xd3088d4fu, "16 x 0xff: 0x%08x", priskv_crc32(f, sizeof(f)));
    CHECK(priskv_crc32(NULL, 0) == 0u, "len 0 with NULL");
    printf("known answers [%s]\n", failures == before ? "OK" : "FAILED");
}

static uint8_t *pattern(size_t n, uint64_t seed)
{
    uint8_t *b = malloc(n);
    uint64_t x = seed;
    for (size_t i = 0; i < n; i++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b[i] = (uint8_t)(x >> 24);
    }
    return b;
}

static void test_lengths_and_alignments(void)
{
    const int before = failures;
    uint8_t *buf = pattern(4200 + 64, 0x5EED5EEDull);
    for (uint32_t off = 0; off < 64; off++)
        for (uint32_t n = 0; n <= 4200; n += (n < 300 ? 1 : 37)) {
            const uint32_t want = sarwate(buf + off, n), got = priskv_crc32(buf + off, n);
            if (got != want) {
                CHECK(0, "off %u len %u: 0x%08x != 0x%08x", off, n, got, want);
                break;
            }
        }
    free(buf);
    printf("lengths 0..4200 x alignments 0..63 vs byte-serial restatement [%s]\n",
           failures == before ? "OK" : "FAILED");
}

#define NTHREADS 4
#define NBUFS 256
static uint8_t *g_bufs[NBUFS];
static uint32_t g_lens[NBUFS], g_want[NBUFS];
static int g_bad[NTHREADS];

static void *hammer(void *arg)
{
    const int t = (int)(intptr_t)arg;
    for (int rep = 0; rep < 200; rep++)
        for (int i = 0; i < NBUFS; i++) {
            const int k = (i * 7 + t * 13 + rep) % NBUFS;
            if (priskv_crc32(g_bufs[k], g_lens[k]) != g_want[k])
                g_bad[t]++;
        }
    return NULL;
}

static void test_threads(void)
{
    const int before = failures;
    for (int i = 0; i < NBUFS; i++) {
        g_lens[i] = (uint32_t)(i * 37 % 1100) + 1; /* keys <= 1 KiB (server/rdma.h:49) and a little more */
        g_bufs[i] = pattern(g_lens[i], 1000u + (uint64_t)i);
        g_want[i] = sarwate(g_bufs[i], g_lens[i]);
    }
    pthread_t th[NTHREADS];
    for (int t = 0; t < NTHREADS; t++)
        pthread_create(&th[t], NULL, hammer, (void *)(intptr_t)t);
    for (int t = 0; t < NTHREADS; t++) {
        pthread_join(th[t], NULL);
        CHECK(g_bad[t] == 0, "thread %d: %d wrong checksums", t, g_bad[t]);
    }
    for (int i = 0; i < NBUFS; i++)
        free(g_bufs[i]);
    printf("%d threads, no lock [%s]\n", NTHREADS, failures == before ? "OK" : "FAILED");
}

int main(void)
{
    sarwate_init();
    /* threads first: the library's tables are built on the first call */
    test_threads();
    test_known_answers();
    test_lengths_and_alignments();
    printf("test_crc_host: %s\n", failures ? "FAILED" : "OK");
    return failures ? 1 : 0;
}
