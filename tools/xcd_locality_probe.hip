// xcd_locality_probe.hip -- does it matter which XCD reads which bytes?
// (measurement tool, not product)
//
// A read-only stream over 4 GiB in the rows kernel's shape (256 workgroups x
// 8 waves, 4 KiB chunks, two chunks in flight per wave, non-temporal
// dwordx4 loads).  The region is cut into granules of GZ bytes, and granule g
// is in class g % 8.  Mode "contig": every wave reads one contiguous share
// of all granules (the rows kernel's pattern).  Mode "shift s": the waves of
// XCD x (workgroup b runs on XCD b % 8, checked below) read only the
// granules of class (x + s) % 8.  If some physical address bits tie HBM
// channels / stacks to XCDs, one shift reads faster than the others at the
// granule size where that happens.
// Usage: xcd_locality_probe [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void xcc_kernel(uint32_t *out)
{
    if (threadIdx.x == 0) {
        uint32_t x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
        out[blockIdx.x] = x;
    }
}

// shift < 8: class mode; shift == 8: contiguous shares
__global__ __launch_bounds__(512) void read_kernel(const uint8_t *__restrict__ base, uint64_t total, uint64_t gz,
                                                   uint32_t shift, uint32_t *__restrict__ sink)
{
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t ngr = total / gz;     // granules
    const uint64_t cpg = gz / 4096;      // 4 KiB chunks per granule
    uint64_t i0, i1, stride_g, first_g;  // the wave's granules: first_g + i * stride_g, i in [i0, i1)
    if (shift >= 16) {
        // shift = 16 + I: groups of I consecutive waves of a workgroup share
        // one contiguous range, wave k of a group reading its 4 KiB chunks
        // k, k + I, k + 2I, ... (2048 / I concurrent streams, every wave
        // busy); shift = 32: only even waves read, each two waves' share
        // (1024 streams, half the waves idle)
        const uint64_t W = (uint64_t)gridDim.x * 8, w = (uint64_t)blockIdx.x * 8 + wave;
        const uint64_t nch_all = total / 4096;
        uint64_t c0, c1, step = 1;
        if (shift == 32) {
            if (w & 1)
                return;
            c0 = nch_all * (w / 2) / (W / 2);
            c1 = nch_all * (w / 2 + 1) / (W / 2);
        } else {
            const uint64_t I = shift - 16, grp = w / I, k = w % I;
            const uint64_t g0 = nch_all * grp / (W / I), g1 = nch_all * (grp + 1) / (W / I);
            c0 = g0 + k;
            c1 = g1;
            step = I;
        }
        uint32_t u = 0;
        v4u A[4], B[4];
        auto ad = [&](uint64_t c) { return reinterpret_cast<const v4u *>(base + c * 4096) + lane; };
        uint64_t c = c0;
        if (c < c1) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                A[k] = __builtin_nontemporal_load(ad(c) + 64 * k);
        }
        for (; c + step < c1; c += 2 * step) {
            const v4u *pb = ad(c + step);
#pragma unroll
            for (int k = 0; k < 4; k++)
                B[k] = __builtin_nontemporal_load(pb + 64 * k);
#pragma unroll
            for (int k = 0; k < 4; k++)
                u ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
            if (c + 2 * step < c1) {
                const v4u *pa = ad(c + 2 * step);
#pragma unroll
                for (int k = 0; k < 4; k++)
                    A[k] = __builtin_nontemporal_load(pa + 64 * k);
            }
#pragma unroll
            for (int k = 0; k < 4; k++)
                u ^= B[k].x ^ B[k].y ^ B[k].z ^ B[k].w;
        }
        if (c < c1) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                u ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
        }
        sink[blockIdx.x * 512 + threadIdx.x] = u;
        return;
    }
    if (shift < 8) {
        const uint32_t x = blockIdx.x % 8, wx = (blockIdx.x / 8) * 8 + wave, WX = (gridDim.x / 8) * 8;
        const uint64_t m = ngr / 8;      // granules per class
        i0 = m * wx / WX;
        i1 = m * (wx + 1) / WX;
        first_g = (x + shift) % 8;
        stride_g = 8;
    } else {
        const uint64_t W = (uint64_t)gridDim.x * 8, w = (uint64_t)blockIdx.x * 8 + wave;
        i0 = ngr * w / W;
        i1 = ngr * (w + 1) / W;
        first_g = 0;
        stride_g = 1;
    }
    const uint64_t nch = (i1 - i0) * cpg;
    auto addr = [&](uint64_t t) {
        const uint64_t i = i0 + t / cpg, g = first_g + i * stride_g;
        return reinterpret_cast<const v4u *>(base + g * gz + (t % cpg) * 4096) + lane;
    };
    uint32_t u = 0;
    v4u A[4], B[4];
    uint64_t t = 0;
    if (nch) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            A[k] = __builtin_nontemporal_load(addr(t) + 64 * k);
    }
    for (; t + 2 <= nch; t += 2) {
        const v4u *pb = addr(t + 1);
#pragma unroll
        for (int k = 0; k < 4; k++)
            B[k] = __builtin_nontemporal_load(pb + 64 * k);
#pragma unroll
        for (int k = 0; k < 4; k++)
            u ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
        if (t + 2 < nch) {
            const v4u *pa = addr(t + 2);
#pragma unroll
            for (int k = 0; k < 4; k++)
                A[k] = __builtin_nontemporal_load(pa + 64 * k);
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
            u ^= B[k].x ^ B[k].y ^ B[k].z ^ B[k].w;
    }
    if (t < nch) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            u ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
    }
    sink[blockIdx.x * 512 + threadIdx.x] = u;
}

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t total = 4ull << 30;
    uint8_t *d;
    uint32_t *sink, *xcc;
    CK(hipMalloc(&d, total));
    CK(hipMemset(d, 0x5A, total));
    const uint32_t grid = (uint32_t)ncu;
    CK(hipMalloc(&sink, (size_t)grid * 512 * 4));
    CK(hipMalloc(&xcc, 4096 * 4));
    hipLaunchKernelGGL(xcc_kernel, dim3(grid), dim3(64), 0, 0, xcc);
    std::vector<uint32_t> h(grid);
    CK(hipMemcpy(h.data(), xcc, grid * 4, hipMemcpyDeviceToHost));
    int rr = 1;
    for (uint32_t b = 0; b < grid; b++)
        rr &= h[b] == b % 8;
    printf("CUs %d, workgroup b on XCD b %% 8: %s\n", ncu, rr ? "yes" : "NO");
    const uint64_t gzs[] = {4096, 16384, 65536, 262144, 1 << 20, 4 << 20};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // warm up
    for (int i = 0; i < 200; i++)
        hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(512), 0, 0, d, total, (uint64_t)65536, 8u, sink);
    CK(hipDeviceSynchronize());
    if (getenv("PROBE_STREAMS")) { // concurrent streams: interleave 1, 2, 4, 8 waves; half the waves
        const uint32_t modes[] = {17, 18, 20, 24, 32};
        std::vector<std::vector<float>> ms(5);
        for (int r = 0; r < rounds; r++)
            for (int m = 0; m < 5; m++) {
                for (int i = 0; i < 3; i++)
                    hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(512), 0, 0, d, total, (uint64_t)4096, modes[m], sink);
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < 10; i++)
                    hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(512), 0, 0, d, total, (uint64_t)4096, modes[m], sink);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms[m].push_back(t / 10);
            }
        const char *nm[5] = {"1 wave per stream", "2 waves interleaved", "4 waves interleaved", "8 waves interleaved",
                             "half the waves, 1 per stream"};
        for (int m = 0; m < 5; m++) {
            std::sort(ms[m].begin(), ms[m].end());
            const double med = ms[m][ms[m].size() / 2];
            printf("%-30s median %.4f ms  %.3f TB/s  (best %.3f)\n", nm[m], med, total / med / 1e9,
                   total / ms[m][0] / 1e9);
        }
        return 0;
    }
    for (uint64_t gz : gzs) {
        std::vector<std::vector<float>> ms(9);
        for (int r = 0; r < rounds; r++)
            for (uint32_t s = 0; s < 9; s++) {
                for (int i = 0; i < 3; i++)
                    hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(512), 0, 0, d, total, gz, s, sink);
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < 10; i++)
                    hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(512), 0, 0, d, total, gz, s, sink);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms[s].push_back(t / 10);
            }
        printf("granule %7llu B:", (unsigned long long)gz);
        for (uint32_t s = 0; s < 9; s++) {
            std::sort(ms[s].begin(), ms[s].end());
            const double med = ms[s][ms[s].size() / 2];
            printf("  %s%u %.3f ms %.2f TB/s", s == 8 ? "contig" : "shift", s == 8 ? 0 : s, med, total / med / 1e9);
        }
        printf("\n");
        fflush(stdout);
    }
    return 0;
}
