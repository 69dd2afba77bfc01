/*
 * host_key_bench.c -- single-thread throughput of a host priskv_crc32 over
 * key-sized inputs (keys <= 1 KiB, server/rdma.h:49, are
 * hashed on the RDMA completion path by server/kv.c:314,408).
 *
 *   host_key_bench LIB.so [sizes...]
 * dlopens LIB (any library exporting uint32_t priskv_crc32(uint8_t *,
 * uint32_t)), hashes a rotating set of 4096 distinct buffers of each size
 * (L1/L2-resident, like keys in a hot request path) for ~0.2 s per size and
 * prints one JSON line per size: ns per call and GB/s, plus a checksum of
 * one pass's results so two libraries can be compared for equality.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

typedef uint32_t (*crc_fn)(uint8_t *, uint32_t);

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s LIB.so [sizes...]\n", argv[0]);
        return 2;
    }
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen %s: %s\n", argv[1], dlerror());
        return 2;
    }
    crc_fn crc = (crc_fn)dlsym(h, "priskv_crc32");
    const char *(*impl)(void) = (const char *(*)(void))dlsym(h, "priskv_crc32_host_impl");
    if (!crc) {
        fprintf(stderr, "no priskv_crc32 in %s\n", argv[1]);
        return 2;
    }
    static const uint32_t dflt[] = {16, 32, 64, 128, 256, 512, 1024, 4096, 65536};
    const int nsz = argc > 2 ? argc - 2 : (int)(sizeof(dflt) / sizeof(dflt[0]));
    const int nbuf = 4096;
    for (int si = 0; si < nsz; si++) {
        const uint32_t sz = argc > 2 ? (uint32_t)strtoul(argv[2 + si], 0, 0) : dflt[si];
        const uint64_t stride = (sz + 63) & ~63u;
        const int nb = sz >= 4096 ? 64 : nbuf;
        uint8_t *mem = aligned_alloc(64, stride * nb + 64);
        uint64_t x = 0x5EED5EEDull;
        for (uint64_t i = 0; i < stride * nb; i++) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            mem[i] = (uint8_t)(x >> 56);
        }
        uint32_t chk = 0, acc = 0;
        uint64_t calls = 0;
        for (int i = 0; i < nb; i++) /* warm-up pass; its XOR identifies the results */
            chk ^= crc(mem + i * stride, sz) * (2u * i + 1u);
        const double t0 = now();
        double t1 = t0;
        while (t1 - t0 < 0.2) {
            for (int i = 0; i < nb; i++)
                acc ^= crc(mem + i * stride, sz);
            calls += nb;
            t1 = now();
        }
        const double ns = (t1 - t0) * 1e9 / calls;
        printf("{\"lib\": \"%s\", \"impl\": \"%s\", \"bytes\": %u, \"ns_per_call\": %.2f, \"GBps\": %.3f, "
               "\"check\": \"0x%08x\"}\n",
               argv[1], impl ? impl() : "reference", sz, ns, sz / ns, chk);
        if (acc == 0x12345678u) /* keeps the timed calls live */
            fputc(' ', stderr);
        free(mem);
    }
    return 0;
}
