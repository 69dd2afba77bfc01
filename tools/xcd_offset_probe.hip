// xcd_offset_probe.hip -- does a kernel's workgroup 0 always start on XCD 0,
// or does the round-robin dispatch carry over from the previous kernel?
// (tools only; round 5: the context's XCD probe saw a non-b%8 mapping after
// other work in the process).  For each preceding grid size G, launches a
// dummy kernel of G single-wave workgroups, then a probe of 64 workgroups
// that record HW_REG_XCC_ID; prints the XCD of probe workgroups 0..15.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void dummy(int *p) { if (threadIdx.x == 0 && p) p[blockIdx.x] = blockIdx.x; }

__global__ void probe(unsigned *out)
{
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
        out[blockIdx.x] = x;
    }
}

int main()
{
    unsigned *d, h[64];
    int *dd;
    if (hipMalloc(&d, sizeof(h)) || hipMalloc(&dd, 4096 * 4))
        return 2;
    const int grids[] = {0, 1, 2, 3, 5, 7, 8, 9, 13, 256, 257, 1, 1, 3, 3, 0, 0};
    for (int g : grids) {
        if (g)
            hipLaunchKernelGGL(dummy, dim3(g), dim3(64), 0, 0, dd);
        hipLaunchKernelGGL(probe, dim3(64), dim3(64), 0, 0, d);
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost))
            return 3;
        int rr = 1;
        for (int b = 0; b < 64; b++)
            rr &= h[b] == (h[0] + b) % 8;
        printf("{\"preceding_grid\": %d, \"wg0_xcd\": %u, \"round_robin_from_wg0\": %d, \"xcds\": [", g, h[0], rr);
        for (int b = 0; b < 16; b++)
            printf("%u%s", h[b], b < 15 ? ", " : "]}\n");
    }
    // the same probe on several created streams (HIP spreads streams over its
    // hardware queues): does the dispatch start at XCD 0 on every queue?
    hipStream_t st[8];
    for (int i = 0; i < 8; i++)
        if (hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking))
            return 4;
    for (int rep = 0; rep < 2; rep++)
        for (int i = 0; i < 8; i++) {
            hipLaunchKernelGGL(probe, dim3(64), dim3(64), 0, st[i], d);
            if (hipStreamSynchronize(st[i]) || hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost))
                return 5;
            int rr = 1;
            for (int b = 0; b < 64; b++)
                rr &= h[b] == (h[0] + b) % 8;
            printf("{\"stream\": %d, \"wg0_xcd\": %u, \"round_robin_from_wg0\": %d, \"xcds\": [", i, h[0], rr);
            for (int b = 0; b < 16; b++)
                printf("%u%s", h[b], b < 15 ? ", " : "]}\n");
        }
    return 0;
}
