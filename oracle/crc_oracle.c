/*
 * crc_oracle.c -- CPU restatement of PrisKV's priskv_crc32.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (priskv_amd/, the
 * libpriskv_crc.so C-ABI) links, loads or calls this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and
 * only as the checker / the timed CPU baseline, never as the thing measured
 * on the GPU.
 *
 * What it restates (reference = aibrix/PrisKV snapshot at /root/reference):
 *   - server/crc.c:31-68  priskv_crc_table[256]: the Sarwate table of the
 *     reflected polynomial 0xEDB88320.  Restated here by *generating* it
 *     from the polynomial (oracle_table), not by copying the literal.
 *   - server/crc.c:70-73  the byte step
 *         crc = T[(crc ^ *buf++) & 0xff] ^ (crc >> 8)
 *   - server/crc.c:90-109 priskv_crc32(): init 0 (:92), the byte step over
 *     all len bytes (the x8 / x4 / x1 unrolls at :93-106 are only unrolling),
 *     and no final XOR (:108).
 *
 * Pinning: tests/test_oracle.py checks this restatement against
 *   (1) the golden vectors in tests/golden/crc_golden.json, which
 *       tests/golden/gen_golden.py produced by calling the reference's own
 *       server/crc.c compiled unmodified into oracle/_ref/ (oracle/Makefile);
 *   (2) when oracle/_ref/libpriskv_ref_crc.so is present, the reference
 *       itself on fresh random buffers;
 *   (3) the independent identity crc(b) == zlib.crc32(b, 0xFFFFFFFF) ^ 0xFFFFFFFF.
 *
 * Also here (test-data plumbing, shared with the GPU fill kernel's spec):
 *   oracle_fill_splitmix: byte pattern = little-endian splitmix64 stream,
 *   64-bit word i of the buffer = mix64(seed + (i + 1) * 0x9E3779B97F4A7C15)
 *   where i counts from the *start of the whole value region* (word_offset),
 *   so every block of a large region is distinct.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_POLY 0xEDB88320u

/* server/crc.c:31-68 restated: T[i] = i pushed through 8 reflected
 * shift/xor steps of the polynomial. */
void oracle_table(uint32_t out[256])
{
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++)
            c = (c & 1) ? (c >> 1) ^ ORACLE_POLY : (c >> 1);
        out[i] = c;
    }
}

static uint32_t g_tab[256];
static pthread_once_t g_tab_once = PTHREAD_ONCE_INIT;
static void tab_init(void) { oracle_table(g_tab); }

/* server/crc.c:90-109 restated.  The reference takes a uint32_t len; the
 * oracle takes 64-bit so it can also check > 4 GiB regions piecewise. */
uint32_t oracle_crc32(const uint8_t *buf, uint64_t len)
{
    pthread_once(&g_tab_once, tab_init);
    uint32_t crc = 0; /* server/crc.c:92 */
    for (uint64_t i = 0; i < len; i++)
        crc = g_tab[(crc ^ buf[i]) & 0xff] ^ (crc >> 8); /* server/crc.c:70-73 */
    return crc; /* server/crc.c:108: no final xor */
}

/* --- batched form over a value region (server/memory.h:87-91 layout:
 *     block i at base + i*block_size) with a static contiguous partition
 *     over nthreads pthreads (the reference's threaded-memset partition
 *     style, server/memory.c:152-177). --------------------------------- */
typedef struct {
    const uint8_t *base;
    uint64_t first, last, block_size;
    uint32_t *out;
} blocks_job;

static void *blocks_worker(void *arg)
{
    blocks_job *j = (blocks_job *)arg;
    for (uint64_t b = j->first; b < j->last; b++)
        j->out[b] = oracle_crc32(j->base + b * j->block_size, j->block_size);
    return NULL;
}

int oracle_crc32_blocks(const uint8_t *base, uint64_t nblocks, uint64_t block_size,
                        uint32_t *out, int nthreads)
{
    pthread_once(&g_tab_once, tab_init);
    if (nthreads < 1)
        nthreads = 1;
    if ((uint64_t)nthreads > nblocks)
        nthreads = nblocks ? (int)nblocks : 1;
    pthread_t th[256];
    blocks_job jobs[256];
    if (nthreads > 256)
        nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        jobs[t].base = base;
        jobs[t].first = nblocks * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].last = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
        jobs[t].block_size = block_size;
        jobs[t].out = out;
    }
    for (int t = 1; t < nthreads; t++)
        if (pthread_create(&th[t], NULL, blocks_worker, &jobs[t]))
            return -1;
    blocks_worker(&jobs[0]);
    for (int t = 1; t < nthreads; t++)
        pthread_join(th[t], NULL);
    return 0;
}

/* Arbitrary (offset, length) extents inside one region -- the per-value
 * form (priskv_key.value_off / .valuelen, server/memory.h:50-51). */
void oracle_crc32_ranges(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
                         uint64_t n, uint32_t *out)
{
    for (uint64_t i = 0; i < n; i++)
        out[i] = oracle_crc32(base + offsets[i], lengths[i]);
}

/* --- test-data generator -------------------------------------------- */
static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t oracle_splitmix_word(uint64_t seed, uint64_t word_index)
{
    return mix64(seed + (word_index + 1) * 0x9E3779B97F4A7C15ull);
}

/* Fill nbytes (multiple of 8 not required) starting at 64-bit word
 * word_offset of the pattern.  Little-endian byte order. */
void oracle_fill_splitmix(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t word_offset)
{
    uint64_t nw = nbytes / 8;
    for (uint64_t i = 0; i < nw; i++) {
        uint64_t v = oracle_splitmix_word(seed, word_offset + i);
        memcpy(dst + 8 * i, &v, 8); /* x86 and gfx950 are both little-endian */
    }
    uint64_t rem = nbytes - 8 * nw;
    if (rem) {
        uint64_t v = oracle_splitmix_word(seed, word_offset + nw);
        memcpy(dst + 8 * nw, &v, rem);
    }
}

/* --- CPU baseline timing helper -------------------------------------
 * Runs fn (e.g. the reference's own priskv_crc32 from oracle/_ref, looked
 * up by the caller) over nblocks blocks so that the timed loop is C, not
 * Python-per-call.  Returns elapsed seconds. */
#include <time.h>
typedef uint32_t (*crc_fn)(uint8_t *, uint32_t);
double oracle_time_blocks_fn(crc_fn fn, const uint8_t *base, uint64_t nblocks, uint32_t block_size,
                             uint32_t *out)
{
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (uint64_t i = 0; i < nblocks; i++)
        out[i] = fn((uint8_t *)base + i * (uint64_t)block_size, block_size);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* the same pass split over nthreads (static contiguous block ranges, the
 * SURVEY 8(d) "nproc threads" CPU reference); returns wall seconds */
struct time_mt_arg {
    crc_fn fn;
    const uint8_t *base;
    uint64_t lo, hi;
    uint32_t bs;
    uint32_t *out;
};

static void *time_mt_worker(void *p)
{
    struct time_mt_arg *a = (struct time_mt_arg *)p;
    for (uint64_t i = a->lo; i < a->hi; i++)
        a->out[i] = a->fn((uint8_t *)a->base + i * (uint64_t)a->bs, a->bs);
    return NULL;
}

double oracle_time_blocks_fn_mt(crc_fn fn, const uint8_t *base, uint64_t nblocks, uint32_t block_size,
                                uint32_t *out, int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    struct time_mt_arg args[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int t = 0; t < nthreads; t++) {
        args[t] = (struct time_mt_arg){fn, base, nblocks * (uint64_t)t / (uint64_t)nthreads,
                                       nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads, block_size, out};
        pthread_create(&th[t], NULL, time_mt_worker, &args[t]);
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

uint32_t oracle_crc32_u32len(uint8_t *buf, uint32_t len) { return oracle_crc32(buf, len); }
