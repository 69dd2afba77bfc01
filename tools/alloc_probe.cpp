// alloc_probe.cpp -- does the rate of one batch depend on WHICH allocation
// holds it?  (tools only; round 3: lib_timing runs of the same plan came out
// 0.66 or 0.75 ms per 4 GiB in different processes on one box.)
// Allocates K regions of `bytes` each with hipMalloc (plus optional padding
// allocations between them to shift virtual addresses), fills each, then
// times priskv_crc32_blocks_dev over every region for every block size in
// turn, R rounds round-robin, and prints one JSON line per (region, size)
// with the region's virtual address and its alignment.  ALLOC_PROBE_ENV2=
// "VAR=V[;VAR=V]" adds a second context created with those variables set,
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

// Pure read roof of one region: each wave streams its own contiguous range
// of 1 KiB rows (the sub-KiB and rows kernels' pattern, no hashing), R rows
// in flight, NW waves per workgroup, one workgroup per CU.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
template <int NW, int R>
__global__ __launch_bounds__(64 * NW, 1) void read_roof(const uint8_t *__restrict__ base, uint64_t nrows,
                                                      uint32_t *__restrict__ sink)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t W = (uint64_t)gridDim.x * NW, wid = (uint64_t)blockIdx.x * NW + wave;
    const uint64_t r0 = nrows * wid / W, r1 = nrows * (wid + 1) / W;
    v4u acc = {0, 0, 0, 0};
    for (uint64_t r = r0; r + R <= r1; r += R) {
        v4u x[R];
#pragma unroll
        for (int k = 0; k < R; k++)
            x[k] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(base + (r + k) * 1024) + lane);
#pragma unroll
        for (int k = 0; k < R; k++)
            acc ^= x[k];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
        sink[threadIdx.x] = acc.x;
}

// the same with raw buffer loads (the product kernels' load form: wave-uniform
// descriptor per chunk of R rows, VGPR offset, nt)
template <int NW, int R>
__global__ __launch_bounds__(64 * NW, 1) void read_roof_buf(const uint8_t *__restrict__ base, uint64_t nrows,
                                                          uint32_t *__restrict__ sink)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t W = (uint64_t)gridDim.x * NW, wid = (uint64_t)blockIdx.x * NW + wave;
    const uint64_t r0 = nrows * wid / W, r1 = nrows * (wid + 1) / W;
    v4u acc = {0, 0, 0, 0};
    for (uint64_t r = r0; r + R <= r1; r += R) {
        const uint64_t a = (uint64_t)(uintptr_t)(base + r * 1024);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(uintptr_t)(((uint64_t)hi << 32) | lo), 0, R * 1024, 0x00020000);
        v4u x[R];
#pragma unroll
        for (int k = 0; k < R; k++)
            x[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane + k * 1024, 0, 2));
#pragma unroll
        for (int k = 0; k < R; k++)
            acc ^= x[k];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
        sink[threadIdx.x] = acc.x;
}

int main(int argc, char **argv)
{
    const int K = argc > 1 ? atoi(argv[1]) : 4;
    // ALLOC_PROBE_MIB=M: regions of M MiB instead of GiB
    const uint64_t bytes = getenv("ALLOC_PROBE_MIB") ? strtoull(getenv("ALLOC_PROBE_MIB"), 0, 0) << 20
                                                     : (argc > 2 ? strtoull(argv[2], 0, 0) : 4) << 30;
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
        for (char *t = strtok(buf, ";"); t; t = strtok(nullptr, ";")) {
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
    // ALLOC_PROBE_OUTS=M: M more output buffers; every (region, size) is
    // also timed writing its CRCs into each of them (ctx 0 only)
    const int nouts = getenv("ALLOC_PROBE_OUTS") ? atoi(getenv("ALLOC_PROBE_OUTS")) : 0;
    std::vector<uint32_t *> outs(1, o);
    for (int j = 0; j < nouts; j++) {
        uint32_t *p = nullptr;
        CK(hipMalloc((void **)&p, bytes / 16 * 4));
        outs.push_back(p);
    }
    // ALLOC_PROBE_FLAGS=N: odd regions from hipExtMallocWithFlags(N) (e.g. 4 =
    // hipDeviceMallocContiguous), even ones from hipMalloc
    const char *fl = getenv("ALLOC_PROBE_FLAGS");
    for (int k = 0; k < K; k++) {
        if (fl && (k & 1))
            CK(hipExtMallocWithFlags(&reg[k], bytes, (unsigned)atoi(fl)));
        else
            CK(hipMalloc(&reg[k], bytes));
        // ALLOC_PROBE_SAMESEED=1: every region holds the same bytes
        const uint64_t seed = getenv("ALLOC_PROBE_SAMESEED") ? 0x5EED5EEDull : 0x5EED5EEDull + k;
        if (priskv_crc_fill_splitmix_dev(ctx, reg[k], bytes, seed, 0, nullptr))
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
    const int NO = (int)outs.size();
    if (NO > 1)
        nctx = 1;
    std::vector<std::vector<std::vector<float>>> ms(K * nctx * NO, std::vector<std::vector<float>>(sizes.size()));
    for (int i = 0; i < 300; i++) // ramp
        priskv_crc32_blocks_dev(ctx, reg[0], bytes / 4096, 4096, o, s);
    for (int r = 0; r < rounds; r++)
        for (int k = 0; k < K; k++)
            for (size_t z = 0; z < sizes.size(); z++)
                for (int c = 0; c < nctx * NO; c++) {
                    const uint32_t bs = sizes[z];
                    const uint64_t nb = bytes / bs;
                    priskv_crc_ctx *cx = ctxs[NO > 1 ? 0 : c];
                    uint32_t *oc = outs[NO > 1 ? c : 0];
                    priskv_crc32_blocks_dev(cx, reg[k], nb, bs, oc, s); // untimed: switch region / size
                    CK(hipEventRecord(e0, s));
                    for (int i = 0; i < kLaunch; i++)
                        if (priskv_crc32_blocks_dev(cx, reg[k], nb, bs, oc, s))
                            return 3;
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    ms[k * nctx * NO + c][z].push_back(t / kLaunch);
                }
    // ALLOC_PROBE_SPLIT=P: time every region's P equal pieces on their own
    // (first block size only): is a slow region slow everywhere or in places?
    if (const char *sp = getenv("ALLOC_PROBE_SPLIT")) {
        const int P = atoi(sp);
        const uint32_t bs = sizes[0];
        const uint64_t pb = bytes / P;
        for (int k = 0; k < K; k++) {
            printf("{\"tool\": \"alloc_probe\", \"region\": %d, \"block_size\": %u, \"piece_ms\": [", k, bs);
            for (int p = 0; p < P; p++) {
                std::vector<float> t3;
                for (int r = 0; r < 3; r++) {
                    CK(hipEventRecord(e0, s));
                    for (int i = 0; i < kLaunch; i++)
                        priskv_crc32_blocks_dev(ctx, (const uint8_t *)reg[k] + p * pb, pb / bs, bs, o, s);
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    t3.push_back(t / kLaunch);
                }
                std::sort(t3.begin(), t3.end());
                printf("%s%.4f", p ? ", " : "", t3[1]);
            }
            printf("]}\n");
        }
    }
    // ALLOC_PROBE_ROOF=1: the pure read roof of every region, 16 and 8 waves per CU
    if (getenv("ALLOC_PROBE_ROOF")) {
        int ncu = 0;
        CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
        for (int k = 0; k < K; k++)
            for (int v = 0; v < 4; v++) {
                std::vector<float> t3;
                for (int r = 0; r < 3; r++) {
                    CK(hipEventRecord(e0, s));
                    for (int i = 0; i < kLaunch; i++) {
                        if (v == 0)
                            hipLaunchKernelGGL((read_roof<16, 8>), dim3(ncu), dim3(1024), 0, s, (const uint8_t *)reg[k],
                                               bytes / 1024, o);
                        else if (v == 1)
                            hipLaunchKernelGGL((read_roof<8, 8>), dim3(ncu), dim3(512), 0, s, (const uint8_t *)reg[k],
                                               bytes / 1024, o);
                        else if (v == 2)
                            hipLaunchKernelGGL((read_roof_buf<16, 8>), dim3(ncu), dim3(1024), 0, s,
                                               (const uint8_t *)reg[k], bytes / 1024, o);
                        else
                            hipLaunchKernelGGL((read_roof_buf<16, 4>), dim3(ncu), dim3(1024), 0, s,
                                               (const uint8_t *)reg[k], bytes / 1024, o);
                    }
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    t3.push_back(t / kLaunch);
                }
                std::sort(t3.begin(), t3.end());
                static const char *names[] = {"global 16w R8", "global 8w R8", "buffer 16w R8", "buffer 16w R4"};
                printf("{\"tool\": \"alloc_probe\", \"region\": %d, \"roof\": \"%s\", \"median_ms\": %.4f, "
                       "\"TBps\": %.3f}\n",
                       k, names[v], t3[1], (double)bytes / t3[1] / 1e9);
            }
    }
    for (int k = 0; k < K; k++)
        for (size_t z = 0; z < sizes.size(); z++)
            for (int c = 0; c < nctx * NO; c++) {
            std::vector<float> v = ms[k * nctx * NO + c][z];
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
