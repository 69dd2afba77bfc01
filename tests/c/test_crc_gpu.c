/*
 * test_crc_gpu.c -- the batched C ABI (include/priskv_crc_gpu.h) driven from
 * plain C, as PrisKV's server (C) would call it: HIP's C runtime API for
 * device memory and streams, no C++ and no Python.  PrisKV's test style
 * (server/test/test_kv.c): standalone executable, "[OK]"/"[FAILED]" lines,
 * non-zero exit on failure.  Every GPU result is checked against the host
 * priskv_crc32 from the same library, which test_crc_host.c and the pytest
 * suite pin to the reference server/crc.c, and every block and value result
 * also against the test-only oracle (oracle/liboracle_crc.so, the CPU
 * restatement of server/crc.c:90-109, loaded with dlopen: a checker, not
 * linked into anything the product ships).
 *
 *   blocks_dev    4 KiB / 64 KiB / 1 MiB / 4100-B / 256-B blocks, and 4 and 1 large
 *                 blocks (split across workgroups), on a stream
 *   ranges_dev    PrisKV-shaped values (value_off on a 4 KiB block, valuelen ragged)
 *   verify_dev    the same values, clean and with one corrupted byte
 *   ranges_host   the zero-copy memfile scrub over a registered host region
 *   blocks_host   the host-streamed block path
 *   errors        -EINVAL for bad arguments, -ENODEV for a missing device
 */
#include <dlfcn.h>
#include <errno.h>
#include <libgen.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "crc.h"
#include "priskv_crc_gpu.h"

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
#define HIPOK(x)                                                                                              \
    do {                                                                                                      \
        hipError_t e_ = (x);                                                                                  \
        if (e_ != hipSuccess) {                                                                               \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);                   \
            exit(2);                                                                                          \
        }                                                                                                     \
    } while (0)

static void report(const char *name, int before)
{
    printf("%s [%s]\n", name, failures == before ? "OK" : "FAILED");
}

#define REGION (64u << 20)

/* the test-only oracle, next to this executable's tree: ../../oracle/ */
static uint32_t (*oracle_crc32)(const void *, uint64_t);

static void load_oracle(void)
{
    char exe[PATH_MAX], so[PATH_MAX + 64];
    const ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
    if (n <= 0) {
        printf("cannot resolve /proc/self/exe\n");
        exit(2);
    }
    exe[n] = 0;
    snprintf(so, sizeof(so), "%s/../../oracle/liboracle_crc.so", dirname(exe));
    void *h = dlopen(so, RTLD_NOW | RTLD_LOCAL);
    if (!h || !(*(void **)&oracle_crc32 = dlsym(h, "oracle_crc32"))) {
        printf("oracle not loadable (%s): %s\n", so, dlerror());
        exit(2);
    }
}

int main(void)
{
    load_oracle();
    priskv_crc_ctx *ctx = NULL;
    int rc = priskv_crc_ctx_create(0, &ctx);
    if (rc) {
        printf("priskv_crc_ctx_create: %d\n", rc);
        return 2;
    }
    hipStream_t s;
    HIPOK(hipStreamCreate(&s));
    uint8_t *d_region, *h_region;
    HIPOK(hipMalloc((void **)&d_region, REGION));
    h_region = malloc(REGION);
    rc = priskv_crc_fill_splitmix_dev(ctx, d_region, REGION, 0x5EED5EEDull, 0, s);
    CHECK(rc == 0, "fill: %d", rc);
    HIPOK(hipMemcpyAsync(h_region, d_region, REGION, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));

    /* ---- blocks_dev */
    {
        const int before = failures;
        /* (REGION / 4 and REGION: few large blocks, whose parts finish
         * across workgroups through the zero-at-rest word) */
        static const uint32_t sizes[] = {4096, 65536, 1u << 20, 4100, 256, REGION / 4, REGION};
        uint32_t *d_out, *h_out = malloc(sizeof(uint32_t) * (REGION / 256));
        HIPOK(hipMalloc((void **)&d_out, sizeof(uint32_t) * (REGION / 256)));
        for (size_t k = 0; k < sizeof(sizes) / sizeof(sizes[0]); k++) {
            const uint32_t bs = sizes[k];
            const uint64_t nb = REGION / bs;
            rc = priskv_crc32_blocks_dev(ctx, d_region, nb, bs, d_out, s);
            CHECK(rc == 0, "blocks_dev bs %u: %d", bs, rc);
            HIPOK(hipMemcpyAsync(h_out, d_out, nb * 4, hipMemcpyDeviceToHost, s));
            HIPOK(hipStreamSynchronize(s));
            for (uint64_t i = 0; i < nb; i += (nb > 4096 ? 7 : 1))
                if (h_out[i] != priskv_crc32(h_region + i * bs, bs)) {
                    CHECK(0, "blocks_dev bs %u block %llu", bs, (unsigned long long)i);
                    break;
                }
            for (uint64_t i = 0; i < nb; i++) /* every block against the oracle */
                if (h_out[i] != oracle_crc32(h_region + i * bs, bs)) {
                    CHECK(0, "blocks_dev bs %u block %llu vs oracle", bs, (unsigned long long)i);
                    break;
                }
        }
        HIPOK(hipFree(d_out));
        free(h_out);
        report("blocks_dev 4 KiB / 64 KiB / 1 MiB / 4100 B / 256 B / 4 and 1 large blocks", before);
    }

    /* PrisKV-shaped values: start on a 4 KiB block, occupy 1/2/4 blocks, ragged length */
    enum { NV = 3000 };
    uint64_t *offs = malloc(sizeof(uint64_t) * NV);
    uint32_t *lens = malloc(sizeof(uint32_t) * NV), *want = malloc(sizeof(uint32_t) * NV);
    uint64_t x = 12345;
    for (int i = 0; i < NV; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t span = 4096u << ((x >> 33) % 3);
        offs[i] = ((x >> 40) % (REGION / 4096 - 4)) * 4096;
        lens[i] = span - (uint32_t)((x >> 20) % 4096);
        want[i] = priskv_crc32(h_region + offs[i], lens[i]);
        CHECK(want[i] == oracle_crc32(h_region + offs[i], lens[i]), "host vs oracle, value %d", i);
    }
    uint64_t *d_offs;
    uint32_t *d_lens, *d_crc, *d_want;
    uint64_t *d_status, h_status[2];
    HIPOK(hipMalloc((void **)&d_offs, sizeof(uint64_t) * NV));
    HIPOK(hipMalloc((void **)&d_lens, sizeof(uint32_t) * NV));
    HIPOK(hipMalloc((void **)&d_crc, sizeof(uint32_t) * NV));
    HIPOK(hipMalloc((void **)&d_want, sizeof(uint32_t) * NV));
    HIPOK(hipMalloc((void **)&d_status, sizeof(h_status)));
    HIPOK(hipMemcpy(d_offs, offs, sizeof(uint64_t) * NV, hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(d_lens, lens, sizeof(uint32_t) * NV, hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(d_want, want, sizeof(uint32_t) * NV, hipMemcpyHostToDevice));

    /* ---- ranges_dev (3000 values: one wave each) and a 20-value batch (segmented) */
    {
        const int before = failures;
        uint32_t *got = malloc(sizeof(uint32_t) * NV);
        static const uint64_t counts[] = {NV, 20};
        uint32_t maxl = 0;
        for (uint64_t i = 0; i < NV; i++)
            maxl = lens[i] > maxl ? lens[i] : maxl;
        /* c = 2, 3: the same through ranges_dev_bounded with the host-known
         * longest length, and with a bound below it (a hint only: exact) */
        for (int c = 0; c < 4; c++) {
            const uint64_t cnt = counts[c & 1];
            HIPOK(hipMemsetAsync(d_crc, 0xA5, sizeof(uint32_t) * cnt, s)); /* sentinel: every CRC is written */
            if (c < 2)
                rc = priskv_crc32_ranges_dev(ctx, d_region, d_offs, d_lens, cnt, d_crc, s);
            else
                rc = priskv_crc32_ranges_dev_bounded(ctx, d_region, d_offs, d_lens, cnt, c == 2 ? maxl : 16, d_crc,
                                                     s);
            CHECK(rc == 0, "ranges_dev: %d", rc);
            HIPOK(hipMemcpyAsync(got, d_crc, sizeof(uint32_t) * cnt, hipMemcpyDeviceToHost, s));
            HIPOK(hipStreamSynchronize(s));
            for (uint64_t i = 0; i < cnt; i++)
                if (got[i] != want[i]) {
                    CHECK(0, "ranges_dev%s n %llu value %llu", c < 2 ? "" : "_bounded", (unsigned long long)cnt,
                          (unsigned long long)i);
                    break;
                }
        }
        free(got);
        report("ranges_dev / ranges_dev_bounded PrisKV-shaped values", before);
    }

    /* ---- verify_dev: clean, then one corrupted byte in value 1234 */
    {
        const int before = failures;
        rc = priskv_crc32_verify_dev(ctx, d_region, d_offs, d_lens, NV, d_want, d_status, s);
        CHECK(rc == 0, "verify_dev: %d", rc);
        HIPOK(hipMemcpyAsync(h_status, d_status, sizeof(h_status), hipMemcpyDeviceToHost, s));
        HIPOK(hipStreamSynchronize(s));
        CHECK(h_status[0] == 0 && h_status[1] == UINT64_MAX, "clean: %llu %llu", (unsigned long long)h_status[0],
              (unsigned long long)h_status[1]);
        uint8_t b;
        const uint64_t at = offs[1234] + lens[1234] / 2;
        HIPOK(hipMemcpy(&b, d_region + at, 1, hipMemcpyDeviceToHost));
        b ^= 0x10;
        HIPOK(hipMemcpy(d_region + at, &b, 1, hipMemcpyHostToDevice));
        rc = priskv_crc32_verify_dev(ctx, d_region, d_offs, d_lens, NV, d_want, d_status, s);
        HIPOK(hipMemcpyAsync(h_status, d_status, sizeof(h_status), hipMemcpyDeviceToHost, s));
        HIPOK(hipStreamSynchronize(s));
        /* values overlap at random: count every value that covers the byte */
        uint64_t hit = 0, first = UINT64_MAX;
        for (int i = 0; i < NV; i++)
            if (at >= offs[i] && at < offs[i] + lens[i]) {
                hit++;
                first = first < (uint64_t)i ? first : (uint64_t)i;
            }
        CHECK(rc == 0 && h_status[0] == hit && h_status[1] == first, "corrupt: %llu %llu want %llu %llu",
              (unsigned long long)h_status[0], (unsigned long long)h_status[1], (unsigned long long)hit,
              (unsigned long long)first);
        b ^= 0x10;
        HIPOK(hipMemcpy(d_region + at, &b, 1, hipMemcpyHostToDevice));
        report("verify_dev clean / one corrupted byte", before);
    }

    /* ---- host-resident: zero-copy scrub and streamed blocks */
    {
        const int before = failures;
        uint32_t *got = malloc(sizeof(uint32_t) * (REGION / 4096));
        rc = priskv_crc_host_register(h_region, REGION);
        CHECK(rc == 0, "host_register: %d", rc);
        rc = priskv_crc32_ranges_host(ctx, h_region, REGION, offs, lens, NV, got);
        CHECK(rc == 0 && memcmp(got, want, sizeof(uint32_t) * NV) == 0, "ranges_host: %d", rc);
        rc = priskv_crc32_blocks_host(ctx, h_region, REGION / 4096, 4096, got);
        CHECK(rc == 0, "blocks_host: %d", rc);
        for (uint64_t i = 0; i < REGION / 4096; i += 13)
            if (got[i] != priskv_crc32(h_region + i * 4096, 4096)) {
                CHECK(0, "blocks_host block %llu", (unsigned long long)i);
                break;
            }
        CHECK(priskv_crc_host_unregister(h_region) == 0, "host_unregister");
        free(got);
        report("ranges_host (zero-copy scrub) / blocks_host (streamed)", before);
    }

    /* ---- error conventions (0 / -errno, nothing aborts) */
    {
        const int before = failures;
        priskv_crc_ctx *bad = NULL;
        CHECK(priskv_crc_ctx_create(1 << 20, &bad) == -ENODEV && bad == NULL, "missing device");
        CHECK(priskv_crc32_blocks_dev(ctx, NULL, 5, 4096, d_crc, s) == -EINVAL, "NULL base");
        CHECK(priskv_crc32_blocks_dev(ctx, d_region, 5, 0, d_crc, s) == -EINVAL, "block_size 0");
        CHECK(priskv_crc32_blocks_dev(ctx, NULL, 0, 4096, NULL, s) == 0, "empty batch");
        const uint64_t bad_off = 4000;
        const uint32_t bad_len = 200;
        uint32_t bad_out;
        CHECK(priskv_crc32_ranges_host(ctx, h_region, 4096, &bad_off, &bad_len, 1, &bad_out) == -EINVAL,
              "extent outside the region");
        report("error conventions", before);
    }

    HIPOK(hipFree(d_offs));
    HIPOK(hipFree(d_lens));
    HIPOK(hipFree(d_crc));
    HIPOK(hipFree(d_want));
    HIPOK(hipFree(d_status));
    HIPOK(hipFree(d_region));
    HIPOK(hipStreamDestroy(s));
    priskv_crc_ctx_destroy(ctx);
    free(h_region);
    free(offs);
    free(lens);
    free(want);
    printf("test_crc_gpu: %s\n", failures ? "FAILED" : "OK");
    return failures ? 1 : 0;
}
