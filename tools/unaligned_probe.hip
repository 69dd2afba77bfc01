// tools/unaligned_probe.hip -- measurement only (not product code).
//
// Questions for a uniform-stride kernel whose 16-B windows start at any byte
// (block size not a multiple of 16, or an unaligned base):
//   1. does raw_buffer_load_b128 at a byte offset that is not a multiple of
//      4 (or 16) return the bytes at that offset?
//   2. a load that straddles num_records: zero for the whole load, or only for
//      the dwords past the end?
//   3. streaming rate of per-wave contiguous 1 KiB rows at offsets 0, 4, 1 ...
//
//   ./unaligned_probe [GiB=4] [rounds=5]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t *p, uint32_t bytes)
{
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

// lane i: 16 B at offset off + 16 i of a descriptor of `bytes` bytes
__global__ void probe_copy(const uint8_t *base, uint32_t bytes, uint32_t off, v4u *out)
{
    const __amdgpu_buffer_rsrc_t r = rsrc(base, bytes);
    out[threadIdx.x] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off + 16 * threadIdx.x), 0, 2));
}

// each wave streams its contiguous range of 1 KiB rows starting at base + off,
// NB rows in flight; XOR of everything per lane to out
template <int NB>
__global__ __launch_bounds__(512) void probe_stream(const uint8_t *base, uint64_t rows, uint32_t off, v4u *out)
{
    const int lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 8, wid = (uint64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
    const uint64_t r0 = rows * wid / W, r1 = rows * (wid + 1) / W;
    v4u acc = {0, 0, 0, 0};
    for (uint64_t r = r0; r < r1; r += NB) {
        const uint32_t n = (uint32_t)(r1 - r < NB ? r1 - r : NB);
        const __amdgpu_buffer_rsrc_t d = rsrc(base + r * 1024 + off, n * 1024);
        v4u x[NB];
#pragma unroll
        for (int k = 0; k < NB; k++)
            x[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(d, k * 1024 + 16 * lane, 0, 2));
#pragma unroll
        for (int k = 0; k < NB; k++)
            acc ^= x[k];
    }
    out[wid * 64 + lane] = acc;
}

int main(int argc, char **argv)
{
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    // ---- 1 + 2: semantics ----
    const uint32_t small = 4096;
    std::vector<uint8_t> h(small);
    for (uint32_t i = 0; i < small; i++)
        h[i] = (uint8_t)(i * 37 + 11);
    uint8_t *d = nullptr;
    v4u *o = nullptr;
    CK(hipMalloc(&d, small));
    CK(hipMalloc(&o, 64 * sizeof(v4u)));
    CK(hipMemcpy(d, h.data(), small, hipMemcpyHostToDevice));
    int bad = 0;
    for (uint32_t off = 0; off < 16; off++) {
        probe_copy<<<1, 64>>>(d, small, off, o);
        CK(hipGetLastError());
        uint8_t got[64 * 16];
        CK(hipMemcpy(got, o, sizeof(got), hipMemcpyDeviceToHost));
        const int ok = !memcmp(got, h.data() + off, sizeof(got));
        bad += !ok;
        printf("{\"probe\":\"unaligned_load\",\"offset\":%u,\"bytes_match\":%s}\n", off, ok ? "true" : "false");
    }
    for (uint32_t past = 1; past < 16; past += (past < 4 ? 1 : 4)) { // load straddling num_records by `past` bytes
        probe_copy<<<1, 64>>>(d, 1024 - past, 0, o);
        CK(hipGetLastError());
        uint8_t got[64 * 16];
        CK(hipMemcpy(got, o, sizeof(got), hipMemcpyDeviceToHost));
        const uint8_t *w = got + 63 * 16; // window [1008, 1024), records end at 1024 - past
        int inb = 0, zeros_past = 1;
        for (uint32_t k = 0; k < 16; k++) {
            if (k < 16 - past)
                inb += w[k] == h[1008 + k];
            else
                zeros_past &= w[k] == 0;
        }
        printf("{\"probe\":\"straddle\",\"bytes_past_end\":%u,\"in_bounds_bytes_returned\":%d,\"of\":%u,"
               "\"past_bytes_zero\":%s}\n",
               past, inb, 16 - past, zeros_past ? "true" : "false");
    }
    CK(hipFree(d));
    CK(hipFree(o));
    // ---- 3: streaming rate ----
    const uint64_t rows = (uint64_t)(gib * (1 << 20)); // 1 KiB rows
    const uint64_t nbytes = rows * 1024 + 64;
    CK(hipMalloc(&d, nbytes));
    CK(hipMemset(d, 0x5A, nbytes));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = ncu;
    CK(hipMalloc(&o, (size_t)grid * 8 * 64 * sizeof(v4u)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t offs[] = {0, 16, 4, 8, 1, 2, 3, 7};
    for (int rep = 0; rep < rounds; rep++)
        for (uint32_t off : offs)
            for (int nb : {8, 16}) {
                auto launch = [&]() {
                    if (nb == 8)
                        probe_stream<8><<<grid, 512>>>(d, rows - 1, off, o);
                    else
                        probe_stream<16><<<grid, 512>>>(d, rows - 1, off, o);
                };
                for (int w = 0; w < 3; w++)
                    launch();
                CK(hipEventRecord(e0));
                const int it = 10;
                for (int i = 0; i < it; i++)
                    launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms /= it;
                printf("{\"probe\":\"stream\",\"round\":%d,\"offset\":%u,\"rows_in_flight\":%d,\"ms\":%.4f,\"TBps\":%.3f}\n",
                       rep, off, nb, ms, (rows - 1) * 1024.0 / (ms * 1e-3) / 1e12);
            }
    CK(hipFree(d));
    CK(hipFree(o));
    return bad ? 1 : 0;
}
