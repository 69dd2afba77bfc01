// xcd_probe.hip -- which XCD runs workgroup b?  (explorer tool, not product)
// Records HW_REG_XCC_ID per workgroup for launches of 256 workgroups, with
// launches of other sizes in between, to see whether round-robin dispatch
// restarts at XCD 0 per launch or continues from the previous dispatch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

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
    unsigned *d;
    hipMalloc(&d, 4096 * 4);
    std::vector<unsigned> h(256);
    const int pre[] = {0, 1, 3, 5, 8, 7, 256, 13};
    for (int t = 0; t < 8; t++) {
        if (pre[t])
            hipLaunchKernelGGL(probe, dim3(pre[t]), dim3(64), 0, 0, d + 1024);
        hipLaunchKernelGGL(probe, dim3(256), dim3(512), 0, 0, d);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, 256 * 4, hipMemcpyDeviceToHost);
        printf("after a %3d-WG launch: xcc of WG 0..15:", pre[t]);
        for (int b = 0; b < 16; b++)
            printf(" %u", h[b]);
        int rr = 1;
        for (int b = 0; b < 256; b++)
            rr &= h[b] == (h[0] + b) % 8;
        printf("   round-robin from xcc %u: %s\n", h[0], rr ? "yes" : "no");
    }
    return 0;
}
