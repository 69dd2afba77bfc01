// alloc_probe.cpp -- does the rate of one batch depend on WHICH allocation
// holds it?  (tools only; round 3: lib_timing runs of the same plan came out
// 0.66 or 0.75 ms per 4 GiB in different processes on one box.)
// Allocates K regions of `bytes` each with hipMalloc (plus optional padding
// allocations between them to shift virtual addresses), fills each, then
// times priskv_crc32_blocks_dev over every region for every block size in
// turn, R rounds round-robin, and prints one JSON line per (region, size)
// with the region's virtual address and its alignment.  ALLOC_PROBE_ENV2=
// "VAR=V[:VAR=V]" adds a second context created with those variables set,
// timed right after the first on every (region, size): an A/B that holds
// the allocation fixed.
// Usage: alloc_probe [K=4] [GiB=4] [rounds=3] [pad_MiB=0] [bs,bs,...=256,4096]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>

#include "../include/priskv_crc_gpu.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

int main(int argc, char **argv)
{
    const int K = argc > 1 ? atoi(argv[1]) : 4;
    const uint64_t bytes = (argc > 2 ? strtoull(argv[2], 0, 0) : 4) << 30;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const uint64_t pad = (argc > 4 ? strtoull(argv[4], 0, 0) : 0) << 20;
    std::vector<uint32_t> sizes;
    {
        char buf[256];
        snprintf(buf, sizeof(buf), "%s", argc > 5 ? argv[5] : "256,4096");
        for (char *t = strtok(buf, ","); t; t = strtok(nullptr, ","))
            sizes.push_back((uint32_t)atoi(t));
    }
    priskv_crc_ctx *ctx = nullptr, *ctxs[2] = {nullptr, nullptr};
    if (priskv_crc_ctx_create(0, &ctx))
        return 2;
    ctxs[0] = ctx;
    int nctx = 1;
    if (const char *e2 = getenv("ALLOC_PROBE_ENV2")) {
        char buf[512];
        snprintf(buf, sizeof(buf), "%s", e2);
        std::vector<std::string> names;
        for (char *t = strtok(buf, ":"); t; t = strtok(nullptr, ":")) {
            char *eq = strchr(t, '=');
            if (!eq)
                continue;
            *eq = 0;
            setenv(t, eq + 1, 1);
            names.push_back(t);
        }
        if (priskv_crc_ctx_create(0, &ctxs[1]))
            return 2;
        for (auto &n : names)
            unsetenv(n.c_str());
        nctx = 2;
    }
    std::vector<void *> reg(K), pads;
    uint32_t *o = nullptr;
    CK(hipMalloc((void **)&o, bytes / 16 * 4));
    // ALLOC_PROBE_FLAGS=N: odd regions from hipExtMallocWithFlags(N) (e.g. 4 =
    // hipDeviceMallocContiguous), even ones from hipMalloc
    const char *fl = getenv("ALLOC_PROBE_FLAGS");
    for (int k = 0; k < K; k++) {
        if (fl && (k & 1))
            CK(hipExtMallocWithFlags(&reg[k], bytes, (unsigned)atoi(fl)));
        else
            CK(hipMalloc(&reg[k], bytes));
        if (priskv_crc_fill_splitmix_dev(ctx, reg[k], bytes, 0x5EED5EEDull + k, 0, nullptr))
            return 2;
        if (pad) {
            void *p = nullptr;
            CK(hipMalloc(&p, pad));
            pads.push_back(p);
        }
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int kLaunch = 20;
    std::vector<std::vector<std::vector<float>>> ms(K * nctx, std::vector<std::vector<float>>(sizes.size()));
    for (int i = 0; i < 300; i++) // ramp
        priskv_crc32_blocks_dev(ctx, reg[0], bytes / 4096, 4096, o, s);
    for (int r = 0; r < rounds; r++)
        for (int k = 0; k < K; k++)
            for (size_t z = 0; z < sizes.size(); z++)
                for (int c = 0; c < nctx; c++) {
                    const uint32_t bs = sizes[z];
                    const uint64_t nb = bytes / bs;
                    priskv_crc32_blocks_dev(ctxs[c], reg[k], nb, bs, o, s); // untimed: switch region / size
                    CK(hipEventRecord(e0, s));
                    for (int i = 0; i < kLaunch; i++)
                        if (priskv_crc32_blocks_dev(ctxs[c], reg[k], nb, bs, o, s))
                            return 3;
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    ms[k * nctx + c][z].push_back(t / kLaunch);
                }
    for (int k = 0; k < K; k++)
        for (size_t z = 0; z < sizes.size(); z++)
            for (int c = 0; c < nctx; c++) {
            std::vector<float> v = ms[k * nctx + c][z];
            std::sort(v.begin(), v.end());
            const uintptr_t a = (uintptr_t)reg[k];
            int align = 0;
            while (align < 40 && !(a & (1ull << align)))
                align++;
            printf("{\"tool\": \"alloc_probe\", \"region\": %d, \"ctx\": %d, \"va\": \"0x%llx\", \"va_align_log2\": %d, "
                   "\"block_size\": %u, \"median_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, \"TBps\": %.3f}\n",
                   k, c, (unsigned long long)a, align, sizes[z], v[v.size() / 2], v[0], v.back(),
                   (double)bytes / sizes[z] * (sizes[z] + 4) / v[v.size() / 2] / 1e9);
        }
    for (int c = 0; c < nctx; c++)
        priskv_crc_ctx_destroy(ctxs[c]);
    return 0;
}
