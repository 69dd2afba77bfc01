// Host-side cost of the calls a small segmented call makes: stream-ordered
// alloc/free, event record + stream wait, and an empty kernel launch.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void empty_kernel(int *p) { if (p && threadIdx.x == 1023) p[0] = 0; }

template <class F> double per_call_us(F f, int n)
{
    for (int i = 0; i < 100; i++)
        f();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++)
        f();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main()
{
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess)
        return 1;
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const int n = 20000;
    double a = per_call_us([&] {
        void *p;
        (void)hipMallocAsync(&p, 64 << 10, s);
        (void)hipFreeAsync(p, s);
    }, n);
    (void)hipStreamSynchronize(s);
    double b = per_call_us([&] {
        (void)hipEventRecord(ev, s);
        (void)hipStreamWaitEvent(s, ev, 0);
    }, n);
    (void)hipStreamSynchronize(s);
    double c = per_call_us([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr); }, n);
    (void)hipStreamSynchronize(s);
    double d = per_call_us([&] { hipLaunchKernelGGL(empty_kernel, dim3(512), dim3(512), 0, s, nullptr); }, n);
    (void)hipStreamSynchronize(s);
    double e = per_call_us([&] {
        void *p;
        (void)hipMallocAsync(&p, 64 << 10, s);
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(1024), 0, s, (int *)nullptr);
        hipLaunchKernelGGL(empty_kernel, dim3(512), dim3(512), 0, s, (int *)nullptr);
        hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, (int *)nullptr);
        (void)hipFreeAsync(p, s);
    }, n / 4);
    (void)hipStreamSynchronize(s);
    double f = per_call_us([&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(1024), 0, s, (int *)nullptr);
        hipLaunchKernelGGL(empty_kernel, dim3(512), dim3(512), 0, s, (int *)nullptr);
        hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, (int *)nullptr);
    }, n / 4);
    (void)hipStreamSynchronize(s);
    printf("{\"malloc_free_async_us\": %.2f, \"event_record_wait_us\": %.2f, \"launch_1x64_us\": %.2f, "
           "\"launch_512x512_us\": %.2f, \"seg_call_shape_us\": %.2f, \"seg_call_no_alloc_us\": %.2f}\n",
           a, b, c, d, e, f);
    return 0;
}
