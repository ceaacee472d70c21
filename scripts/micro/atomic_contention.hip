// Micro-benchmark: cost of one wave-aggregated atomicAdd per wave on a single counter
// (the pattern k_shade uses for its append queues) vs. a plain store.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_atomic(unsigned* ctr, unsigned* out, int n, int reps) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (int r = 0; r < reps; r++) {
        unsigned long long m = __ballot(i < n);
        int lane = __lane_id();
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(ctr + r, (unsigned)__popcll(m));
        base = __shfl(base, 0);
        acc += base;
    }
    if (i < n) out[i] = acc;
}
__global__ void k_plain(unsigned* out, int n, int reps) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (int r = 0; r < reps; r++) acc += __shfl(i * 3 + r, 0);
    if (i < n) out[i] = acc;
}
int main() {
    int n = 4 << 20, reps = 3;
    unsigned *ctr, *out;
    hipMalloc(&ctr, 64 * sizeof(unsigned));
    hipMalloc(&out, n * sizeof(unsigned));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int it = 0; it < 3; it++) {
        hipMemset(ctr, 0, 64 * sizeof(unsigned));
        hipEventRecord(a);
        hipLaunchKernelGGL(k_atomic, dim3(n / 256), dim3(256), 0, 0, ctr, out, n, reps);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_plain, dim3(n / 256), dim3(256), 0, 0, out, n, reps);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms2; hipEventElapsedTime(&ms2, a, b);
        printf("n=%d waves=%d reps=%d: atomic %.3f ms, plain %.3f ms\n", n, n / 64, reps, ms, ms2);
    }
    return 0;
}
