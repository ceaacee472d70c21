// rtg_tonemap.hip — hw5's global tone-mapping operator on the GPU.
//
// pages/Page5.md:47-53 describes a global operator but src/ has no code for it, so the
// operator is the course's Photographic TMO (Reinhard et al. 2002, global form), specified in
// DESIGN.md §11 and restated on the CPU by oracle/rtg_oracle.c orc_tonemap():
//   Y = (0.2126 R + 0.7152 G) + 0.0722 B, clamped to 0 when not finite / negative
//   Lw = exp(mean(log(1e-5 + Y)))            (double sums: per-256-pixel block partials,
//                                               combined in a fixed tree: deterministic)
//   L = (key / Lw) Y ; Lwhite = L at the (100 - burn)% rank (max when burn = 0)
//   Ld = L (1 + L / Lwhite^2) / (1 + L)
//   out_c = 255 * clamp(Ld * (C / Y)^saturation, 0, 1)^(1 / gamma)
// HBM-bound elementwise work plus one radix sort of the N luminances (for the burn rank).
#include <hipcub/hipcub.hpp>

#include <math.h>
#include <stdint.h>

#include <string>

#include "rtg_internal.h"

namespace rtg {
namespace {

constexpr int kTmBlock = 256;

__device__ __forceinline__ float tm_lum(const float* c) {
    const float y = (0.2126f * c[0] + 0.7152f * c[1]) + 0.0722f * c[2];
    return (__builtin_isfinite(y) && y > 0.0f) ? y : 0.0f;
}

// Y per pixel and one double partial of log(1e-5 + Y) per block (fixed tree order)
__global__ void __launch_bounds__(kTmBlock) k_tm_lum(const float* __restrict__ hdr, int n, float* __restrict__ Y,
                                                    double* __restrict__ part) {
    __shared__ double s[kTmBlock];
    const int i = blockIdx.x * kTmBlock + threadIdx.x;
    double v = 0.0;
    if (i < n) {
        const float y = tm_lum(hdr + 3 * (size_t)i);
        Y[i] = y;
        v = log(1e-5 + (double)y);
    }
    s[threadIdx.x] = v;
    __syncthreads();
    for (int w = kTmBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

// one block: sum of the partials (each thread a strided run, then the same tree) -> scale k
__global__ void __launch_bounds__(kTmBlock) k_tm_scale(const double* __restrict__ part, int nblocks, int n, float key,
                                                      float* __restrict__ kout) {
    __shared__ double s[kTmBlock];
    double v = 0.0;
    for (int b = threadIdx.x; b < nblocks; b += kTmBlock) v += part[b];
    s[threadIdx.x] = v;
    __syncthreads();
    for (int w = kTmBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double lw = exp(s[0] / (double)n);
        kout[0] = (float)((double)key / lw);
    }
}

__global__ void __launch_bounds__(kTmBlock) k_tm_scaled(const float* __restrict__ Y, int n, const float* __restrict__ k,
                                                       float* __restrict__ L) {
    const int i = blockIdx.x * kTmBlock + threadIdx.x;
    if (i < n) L[i] = k[0] * Y[i];
}

__global__ void __launch_bounds__(kTmBlock) k_tm_apply(const float* __restrict__ hdr, const float* __restrict__ Y, int n,
                                                      const float* __restrict__ k, const float* __restrict__ sortedL,
                                                      int white_idx, float saturation, float gamma,
                                                      float* __restrict__ out) {
    const int i = blockIdx.x * kTmBlock + threadIdx.x;
    if (i >= n) return;
    const float y = Y[i];
    const float L = k[0] * y;
    const float lw = sortedL[white_idx];
    const float Ld = lw > 0.0f ? (L * (1.0f + L / (lw * lw))) / (1.0f + L) : L / (1.0f + L);
    const double ig = 1.0 / (double)gamma;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        float v = 0.0f;
        if (y > 0.0f) {
            const float ch = fmaxf(hdr[3 * (size_t)i + c], 0.0f);
            v = Ld * (float)pow((double)(ch / y), (double)saturation);
        }
        v = fminf(fmaxf(v, 0.0f), 1.0f);     // NaN -> 0
        out[3 * (size_t)i + c] = 255.0f * (float)pow((double)v, ig);
    }
}

template <class T>
struct TmBuf {
    T* p = nullptr;
    ~TmBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t n) { return hipMalloc(&p, sizeof(T) * (n ? n : 1)); }
};

}  // namespace

// Burn rank of the (100 - burn)% luminance.
int tonemap_white_index(int n, float burn_percent) {
    if (n <= 0) return 0;
    if (!(burn_percent > 0.0f)) return n - 1;
    double f = 1.0 - (double)burn_percent / 100.0;
    if (f < 0.0) f = 0.0;
    long long idx = (long long)floor((double)(n - 1) * f);
    if (idx < 0) idx = 0;
    if (idx > n - 1) idx = n - 1;
    return (int)idx;
}

int tonemap_device(const float* hdr, int nx, int ny, const rtg_tonemap_desc& tm, float* out, hipStream_t st,
                   std::string& err) {
    const int n = nx * ny;
    if (n <= 0) return 0;
    const int nb = (n + kTmBlock - 1) / kTmBlock;
    TmBuf<float> Y, L, Ls, k;
    TmBuf<double> part;
    TmBuf<unsigned char> tmp;
    hipError_t e;
    if ((e = Y.alloc(n)) != hipSuccess || (e = L.alloc(n)) != hipSuccess || (e = Ls.alloc(n)) != hipSuccess ||
        (e = k.alloc(1)) != hipSuccess || (e = part.alloc(nb)) != hipSuccess) {
        err = std::string("tonemap hipMalloc: ") + hipGetErrorString(e);
        return -1;
    }
    hipLaunchKernelGGL(k_tm_lum, dim3(nb), dim3(kTmBlock), 0, st, hdr, n, Y.p, part.p);
    hipLaunchKernelGGL(k_tm_scale, dim3(1), dim3(kTmBlock), 0, st, part.p, nb, n, tm.key, k.p);
    hipLaunchKernelGGL(k_tm_scaled, dim3(nb), dim3(kTmBlock), 0, st, Y.p, n, k.p, L.p);
    size_t tb = 0;
    if ((e = hipcub::DeviceRadixSort::SortKeys(nullptr, tb, L.p, Ls.p, n, 0, 32, st)) != hipSuccess ||
        (e = tmp.alloc(tb)) != hipSuccess ||
        (e = hipcub::DeviceRadixSort::SortKeys(tmp.p, tb, L.p, Ls.p, n, 0, 32, st)) != hipSuccess) {
        err = std::string("tonemap sort: ") + hipGetErrorString(e);
        return -1;
    }
    hipLaunchKernelGGL(k_tm_apply, dim3(nb), dim3(kTmBlock), 0, st, hdr, Y.p, n, k.p, Ls.p,
                       tonemap_white_index(n, tm.burn_percent), tm.saturation, tm.gamma, out);
    if ((e = hipGetLastError()) != hipSuccess || (e = hipStreamSynchronize(st)) != hipSuccess) {
        err = std::string("tonemap: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

}  // namespace rtg
