// First-use costs of the HIP runtime in a fresh process: which of a kernel launch, a kernel reading
// page-locked host memory (zero-copy) and a hipMemcpy pays the 90-145 ms one-time set-up.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_read(const float* __restrict__ src, float* __restrict__ dst, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t n = 3u << 20;   // 12 MB
    double t = now_ms();
    if (hipSetDevice(0) != hipSuccess) return 1;
    (void)hipFree(nullptr);
    printf("context                      %8.2f ms\n", now_ms() - t);
    float *h = nullptr, *d = nullptr, *h2 = nullptr;
    t = now_ms();
    if (hipHostMalloc((void**)&h, n * 4, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipHostMalloc((void**)&h2, n * 4, hipHostMallocDefault) != hipSuccess) return 1;
    for (size_t i = 0; i < n; i++) h[i] = (float)i;
    printf("pinned alloc x2 + fill       %8.2f ms\n", now_ms() - t);
    t = now_ms();
    if (hipMalloc((void**)&d, n * 4) != hipSuccess) return 1;
    printf("device alloc                 %8.2f ms\n", now_ms() - t);
    for (int rep = 0; rep < 2; rep++) {
        t = now_ms();
        hipLaunchKernelGGL(k_read, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, h, d, n);
        (void)hipDeviceSynchronize();
        printf("[%d] kernel reading pinned    %8.2f ms\n", rep, now_ms() - t);
        t = now_ms();
        hipLaunchKernelGGL(k_read, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d, h2, n);
        (void)hipDeviceSynchronize();
        printf("[%d] kernel writing pinned    %8.2f ms (h2[7] = %g)\n", rep, now_ms() - t, h2[7]);
        t = now_ms();
        (void)hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
        printf("[%d] hipMemcpy H2D pinned     %8.2f ms\n", rep, now_ms() - t);
    }
    return 0;
}
