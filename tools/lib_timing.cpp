// lib_timing.cpp -- times priskv_crc32_blocks_dev through the library's C ABI
// with plain hipMalloc'd memory and no torch in the process (tools only):
// separates "the kernel" from "bench.py's process" when their numbers differ.
// Usage: lib_timing [block_size] [nblocks] [launches] [rounds]
// LIB_TIMING_ROOF=v+1: time priskv_crc_read_roof_dev variant v (the plan's
// loads, no hashing) instead; LIB_TIMING_RAMP=N: N ramp launches (default 400; fewer
// under rocprofv3 --pmc, which serialises every dispatch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
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
    const uint32_t bs = argc > 1 ? (uint32_t)atoi(argv[1]) : 4096;
    const uint64_t nb = argc > 2 ? strtoull(argv[2], 0, 0) : (1ull << 32) / bs;
    const int k = argc > 3 ? atoi(argv[3]) : 50;
    const int rounds = argc > 4 ? atoi(argv[4]) : 7;
    priskv_crc_ctx *ctx = nullptr;
    if (int rc = priskv_crc_ctx_create(0, &ctx)) {
        fprintf(stderr, "ctx_create %d\n", rc);
        return 2;
    }
    void *d = nullptr;
    uint32_t *o = nullptr;
    CK(hipMalloc(&d, (size_t)bs * nb));
    CK(hipMalloc((void **)&o, nb * 4));
    if (priskv_crc_fill_splitmix_dev(ctx, d, (uint64_t)bs * nb, 0x5EED5EEDull, 0, nullptr))
        return 2;
    char plan[256];
    priskv_crc32_blocks_plan(ctx, d, nb, bs, plan, sizeof(plan));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int roof = getenv("LIB_TIMING_ROOF") ? atoi(getenv("LIB_TIMING_ROOF")) : 0;
    uint32_t *sink = nullptr;
    CK(hipMalloc((void **)&sink, PRISKV_CRC_ROOF_SINK_WORDS * 4));
    // default ramp: 400 launches up to 4 GiB per call, ~1.6 TiB of reads above
    const uint64_t nbytes = (uint64_t)bs * nb;
    const int ramp_default = nbytes <= (4ull << 30) ? 400 : (int)std::max<uint64_t>(20, (400ull << 32) / nbytes);
    const int ramp = getenv("LIB_TIMING_RAMP") ? atoi(getenv("LIB_TIMING_RAMP")) : ramp_default;
    auto call = [&]() {
        return roof ? priskv_crc_read_roof_dev(ctx, d, nb, bs, (uint32_t)(roof - 1), sink, s)
                    : priskv_crc32_blocks_dev(ctx, d, nb, bs, o, s);
    };
    for (int i = 0; i < ramp; i++) // ramp
        call();
    CK(hipStreamSynchronize(s));
    std::vector<float> ms;
    for (int r = 0; r < rounds; r++) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < k; i++)
            if (call())
                return 3;
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t / k);
    }
    std::sort(ms.begin(), ms.end());
    const double alg = (double)nb * (bs + 4);
    printf("{\"tool\": \"lib_timing\", \"roof\": %d, \"block_size\": %u, \"nblocks\": %llu, \"plan\": \"%s\", \"launches\": %d, "
           "\"median_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, \"TBps_median\": %.3f}\n",
           roof, bs, (unsigned long long)nb, plan, k, ms[ms.size() / 2], ms[0], ms.back(), alg / ms[ms.size() / 2] / 1e9);
    priskv_crc_ctx_destroy(ctx);
    return 0;
}
