// rtg_bvh_gpu.hip — the reference's per-object BVH construction on the GPU.
//
// Reproduces BVH::ConstructionHelper / FindMedian / ComputeBoundingBox (src/BVH.cpp:64-135,
// 268-303) bit for bit -- the same primitive permutation, the same tree, the same node boxes --
// level by level instead of recursively:
//
//   * split: the median of the segment's centres along axis depth % 3 (even count: the mean of
//     the two middle values, computed as (lower + upper) * 0.5f).  One radix sort per level of
//     64-bit keys (segment id << 32 | order-preserving float bits) yields every segment's order
//     statistics at once.
//   * partition: the reference's in-place loop `if (c[i] < split) swap(p[s++], p[i])` (a Lomuto
//     partition) is evaluated in closed form.  With k = #less and lessPrefix(i) = #less in
//     [0, i): the less elements land at lessPrefix(i) in order; the element ending at position
//     j >= k is resolve(j), where resolve(j) = e_j if e_j is not less, else
//     resolve(lessPrefix(j)) (the swap moves the oldest element of the ">= block" to the scan
//     position).  lessPrefix(j) < j, so the chains are resolved by pointer jumping.
//   * boxes: min / max of the primitive boxes over the node's range in the order the reference
//     sees it; ties between equal values (+0 / -0) keep the earliest element, as the reference's
//     `a <= b ? a : b` fold does -- per level, as (value, position) keys reduced with 64-bit atomics
//     over runs of positions (round 5; the one-block-per-node reduction it replaced ran a handful of
//     blocks at the top levels, ~8 ms of a 1 M-triangle build).  Non-finite inputs are rejected (the
//     host builder handles them).
//   * leaves: one primitive, or depth 30 (possibly empty); empty ranges below depth 30 are null.
//
// Node numbering here is breadth-first; the host converts to the reference's pre-order.
#include <float.h>
#include <limits.h>

#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <cstdlib>

#include <string>
#include <vector>

#include "rtg_internal.h"

namespace rtg {
namespace {

constexpr int kMaxDepth = 30;      // src/BVH.cpp:67

__device__ __forceinline__ uint32_t ord_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_bits(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

struct Seg {       // one interior node of the current level
    int start, end, node, off;   // off: position of its keys in the sorted array
};

__global__ void k_segid(int n, const Seg* __restrict__ segs, int S, int* __restrict__ segid) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int lo = 0, hi = S - 1, r = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (segs[mid].start <= i) { r = mid; lo = mid + 1; } else { hi = mid - 1; }
    }
    segid[i] = (r >= 0 && i < segs[r].end) ? r : S;
}

__global__ void k_keys(int n, int axis, const int* __restrict__ segid, int S, const int* __restrict__ perm,
                       const float* __restrict__ c3, unsigned long long* __restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int sid = segid[i];
    unsigned long long k = (unsigned long long)S << 32;
    if (sid < S) k = ((unsigned long long)sid << 32) | ord_bits(c3[3 * perm[i] + axis]);
    keys[i] = k;
}

__global__ void k_split(const Seg* __restrict__ segs, int S, const unsigned long long* __restrict__ sorted,
                        float* __restrict__ split) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const Seg g = segs[s];
    const int len = g.end - g.start, mi = len / 2;
    float v = unord_bits((uint32_t)sorted[g.off + mi]);                 // FindMedian, src/BVH.cpp:117-135
    if (len % 2 == 0) {
        const float lower = unord_bits((uint32_t)sorted[g.off + mi - 1]);
        v = (lower + v) * 0.5f;
    }
    split[s] = v;
}

__global__ void k_less(int n, int axis, const int* __restrict__ segid, int S, const int* __restrict__ perm,
                       const float* __restrict__ c3, const float* __restrict__ split, int* __restrict__ less) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    int l = 0;
    if (i < n) {
        const int sid = segid[i];
        if (sid < S) l = c3[3 * perm[i] + axis] < split[sid];
    }
    less[i] = l;      // less[n] = 0: the exclusive scan then has n + 1 entries
}

__global__ void k_ptr_init(int n, const int* __restrict__ segid, int S, const Seg* __restrict__ segs,
                           const int* __restrict__ G, const int* __restrict__ less, int* __restrict__ ptr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int sid = segid[i];
    int p = i;
    if (sid < S && less[i]) {
        const int st = segs[sid].start;
        p = st + (G[i] - G[st]);           // resolve(i) = resolve(lessPrefix(i))
    }
    ptr[i] = p;
}

// In-place pointer jumping: every write replaces ptr[i] by one of its ancestors, so concurrent
// updates are safe and every chain ends at a non-less element (lessPrefix(j) < j).
__global__ void k_jump(int n, int* ptr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int p = ptr[i];
    while (true) {
        const int q = ptr[p];
        if (q == p) break;
        const int r = ptr[q];
        if (r == q) { p = q; break; }
        p = r;
        ptr[i] = p;
    }
    ptr[i] = p;
}

__global__ void k_scatter(int n, const int* __restrict__ segid, int S, const Seg* __restrict__ segs,
                          const int* __restrict__ G, const int* __restrict__ less, const int* __restrict__ ptr,
                          const int* __restrict__ perm, int* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int sid = segid[i];
    if (sid >= S) { out[i] = perm[i]; return; }
    const Seg g = segs[sid];
    const int k = G[g.end] - G[g.start];
    if (less[i]) out[g.start + (G[i] - G[g.start])] = perm[i];
    if (i >= g.start + k) out[i] = perm[ptr[i]];
}

// Children of every segment: counts of nodes and of interior (next-level) segments.
__device__ __forceinline__ int child_kind(int len, int depth) {   // 0 null, 1 leaf, 2 interior
    if (len == 1 || depth >= kMaxDepth) return 1;                 // src/BVH.cpp:67-76
    if (len == 0) return 0;                                       // BVH.cpp:77
    return 2;
}
__global__ void k_child_count(const Seg* __restrict__ segs, int S, int depth1, const int* __restrict__ G,
                              int* __restrict__ nnodes, int* __restrict__ nint) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > S) return;
    int a = 0, b = 0;
    if (s < S) {
        const Seg g = segs[s];
        const int k = G[g.end] - G[g.start];
        const int kl = child_kind(k, depth1), kr = child_kind(g.end - g.start - k, depth1);
        a = (kl != 0) + (kr != 0);
        b = (kl == 2) + (kr == 2);
    }
    nnodes[s] = a;     // entry S = 0 (exclusive scans of S + 1 entries give the totals)
    nint[s] = b;
}
__global__ void k_child_emit(const Seg* __restrict__ segs, int S, int depth1, const int* __restrict__ G,
                             const int* __restrict__ node_off, const int* __restrict__ int_off, int node_base,
                             int4* __restrict__ nodes, Seg* __restrict__ next) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const Seg g = segs[s];
    const int k = G[g.end] - G[g.start];
    const int r0[2] = {g.start, g.start + k}, r1[2] = {g.start + k, g.end};
    int id = node_base + node_off[s], nx = int_off[s];
    int child[2] = {-1, -1};
    for (int q = 0; q < 2; q++) {
        const int len = r1[q] - r0[q];
        const int kind = child_kind(len, depth1);
        if (kind == 0) continue;
        child[q] = id;
        nodes[id] = make_int4(-1, -1, r0[q], r1[q]);
        if (kind == 2) { Seg c; c.start = r0[q]; c.end = r1[q]; c.node = id; c.off = 0; next[nx++] = c; }
        id++;
    }
    nodes[g.node].x = child[0];
    nodes[g.node].y = child[1];
}

// Segment key offsets: exclusive sum of lengths (written into Seg.off)
__global__ void k_seg_len(const Seg* __restrict__ segs, int S, int* __restrict__ len) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < S) len[s] = segs[s].end - segs[s].start;
}
__global__ void k_seg_off(Seg* __restrict__ segs, int S, const int* __restrict__ off) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < S) segs[s].off = off[s];
}

// ComputeBoundingBox (src/BVH.cpp:268-303): min / max over the node's range in the order the reference
// sees it when it creates the node (after its parent's partition), ties between equal values (+0 / -0)
// to the earliest element (the fold `if (!(m <= v)) m = v`).  Per level, right after the partition:
// every position of a split range adds its box to its child's keys -- 64-bit (value, position) keys
// with -0 folded into +0, so atomicMin picks the least value and, among equal ones, the earliest
// position; the box then takes that element's own value (its sign of zero).  Runs of 16 positions per
// lane, wave-merged when the whole wave feeds one node (the top levels), one atomic per key otherwise.
__device__ __forceinline__ unsigned long long kmin_of(float v, int pos) {
    return ((unsigned long long)ord_bits(v + 0.0f) << 32) | (unsigned)pos;
}
__device__ __forceinline__ unsigned long long kmax_of(float v, int pos) {
    return ((unsigned long long)ord_bits(v + 0.0f) << 32) | (0xFFFFFFFFu - (unsigned)pos);
}
constexpr int kRun = 16;
__global__ void __launch_bounds__(256) k_box_keys(int n, bool root, const int* __restrict__ segid, int S,
                                                  const Seg* __restrict__ segs, const int* __restrict__ G,
                                                  const int4* __restrict__ nodes, const int* __restrict__ perm,
                                                  const float* __restrict__ lo3, const float* __restrict__ hi3,
                                                  unsigned long long* __restrict__ kmin,
                                                  unsigned long long* __restrict__ kmax) {
    const int p0 = (blockIdx.x * blockDim.x + threadIdx.x) * kRun;
    int cur = -1;
    unsigned long long a[3], b[3];
    auto flush = [&]() {
        for (int z = 0; z < 3; z++) {
            atomicMin(&kmin[3 * (size_t)cur + z], a[z]);
            atomicMax(&kmax[3 * (size_t)cur + z], b[z]);
        }
    };
    for (int p = p0; p < min(n, p0 + kRun); p++) {
        int o = 0;
        if (!root) {
            const int sid = segid[p];
            if (sid >= S) continue;
            const Seg g = segs[sid];
            const int k = G[g.end] - G[g.start];
            const int4 pn = nodes[g.node];
            o = p < g.start + k ? pn.x : pn.y;
        }
        if (o != cur) {
            if (cur >= 0) flush();
            cur = o;
            for (int z = 0; z < 3; z++) { a[z] = ~0ull; b[z] = 0ull; }
        }
        const int f = perm[p];
        for (int z = 0; z < 3; z++) {
            a[z] = min(a[z], kmin_of(lo3[3 * f + z], p));
            b[z] = max(b[z], kmax_of(hi3[3 * f + z], p));
        }
    }
    // the last run's partial: merged over the wave when every lane holds one for the same node
    const int c0 = __shfl(cur, 0);
    if (__ballot(cur != c0) == 0ull && c0 >= 0) {
        for (int off = 32; off > 0; off >>= 1)
            for (int z = 0; z < 3; z++) {
                a[z] = min(a[z], (unsigned long long)__shfl_xor((long long)a[z], off));
                b[z] = max(b[z], (unsigned long long)__shfl_xor((long long)b[z], off));
            }
        if ((threadIdx.x & 63) == 0) flush();
    } else if (cur >= 0) {
        flush();
    }
}
__global__ void k_box_final(int first, int count, const int* __restrict__ perm, const float* __restrict__ lo3,
                            const float* __restrict__ hi3, const unsigned long long* __restrict__ kmin,
                            const unsigned long long* __restrict__ kmax, float* __restrict__ box) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const size_t id = (size_t)first + t;
    for (int z = 0; z < 3; z++) {
        const unsigned long long a = kmin[3 * id + z], b = kmax[3 * id + z];
        // an empty leaf (depth 30) keeps the fold's start values
        box[6 * id + z] = a == ~0ull ? FLT_MAX : lo3[3 * perm[(unsigned)a] + z];
        box[6 * id + 3 + z] = b == 0ull ? -FLT_MAX : hi3[3 * perm[0xFFFFFFFFu - (unsigned)b] + z];
    }
}

struct NodeRec40 { int c[4]; float b[6]; };   // = rtg_host.cpp HNode (4-byte aligned: 40 B, no padding)
static_assert(sizeof(NodeRec40) == 40, "40-byte node record");
__global__ void k_node40(const int4* __restrict__ nodes, const float* __restrict__ box, int nn, NodeRec40* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    NodeRec40 r;
    const int4 c = nodes[i];
    r.c[0] = c.x; r.c[1] = c.y; r.c[2] = c.z; r.c[3] = c.w;
    for (int z = 0; z < 6; z++) r.b[z] = box[6 * (size_t)i + z];
    out[i] = r;
}

__global__ void k_iota(int n, int* p) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = i;
}

// Scratch arrays allocated and freed in stream order (hipMallocAsync / hipFreeAsync): hipFree waits for
// the whole device, and the median-tree and traversal-tree builds run side by side on two streams.
template <class T>
struct DevArr {
    T* p = nullptr;
    size_t cap = 0;
    hipStream_t st = nullptr;
    explicit DevArr(hipStream_t s = nullptr) : st(s) {}
    hipError_t grow(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFreeAsync(p, st);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&p), sizeof(T) * (n + 16), st);
        if (e == hipSuccess) cap = n + 16;
        return e;
    }
    ~DevArr() { if (p) (void)hipFreeAsync(p, st); }
};

inline int nb(long long n, int b) { return (int)((n + b - 1) / b); }

}  // namespace

#define BVH_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);           \
            return -1;                                                         \
        }                                                                      \
    } while (0)

// One empty launch: loads this module's code object (the first launch of a module costs ~7 ms).
void gpu_bvh_warm(hipStream_t st) { hipLaunchKernelGGL(k_iota, dim3(1), dim3(64), 0, st, 0, nullptr); }

int gpu_build_bvh(const float* centers, const float* bmin, const float* bmax, int n, GpuBvh& out, std::string& err,
                  hipStream_t st) {
    out.num_nodes = 0;
    out.root = -1;
    if (n <= 0) return 0;
    // RTG_BUILD_TIMING: wall time of the build's stages on stderr (synchronising between them)
    const bool timing = getenv("RTG_BUILD_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!timing) return;
        (void)hipStreamSynchronize(st);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[rtg] gpu bvh %-10s %7.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    DevArr<float> c3(st), lo3(st), hi3(st), box(st);
    DevArr<int> perm(st), perm2(st), segid(st), less(st), G(st), ptr(st), lens(st), offs(st), nn(st), ni(st), nnoff(st), nioff(st);
    DevArr<int4> nodes(st);
    DevArr<unsigned long long> keys(st), sorted(st);
    DevArr<Seg> segs(st), next(st);
    DevArr<float> split(st);
    DevArr<unsigned char> tmp(st);
    BVH_TRY(c3.grow(3 * (size_t)n)); BVH_TRY(lo3.grow(3 * (size_t)n)); BVH_TRY(hi3.grow(3 * (size_t)n));
    BVH_TRY(hipMemcpyAsync(c3.p, centers, sizeof(float) * 3 * n, hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(lo3.p, bmin, sizeof(float) * 3 * n, hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(hi3.p, bmax, sizeof(float) * 3 * n, hipMemcpyHostToDevice, st));
    BVH_TRY(perm.grow(n)); BVH_TRY(perm2.grow(n)); BVH_TRY(segid.grow(n)); BVH_TRY(less.grow(n + 1));
    BVH_TRY(G.grow(n + 1)); BVH_TRY(ptr.grow(n)); BVH_TRY(keys.grow(n)); BVH_TRY(sorted.grow(n));
    // per-segment arrays: a level has at most n / 2 interior segments
    const size_t scap = (size_t)n / 2 + 2;
    BVH_TRY(split.grow(scap)); BVH_TRY(lens.grow(scap)); BVH_TRY(offs.grow(scap)); BVH_TRY(nn.grow(scap));
    BVH_TRY(ni.grow(scap)); BVH_TRY(nnoff.grow(scap)); BVH_TRY(nioff.grow(scap));
    BVH_TRY(segs.grow(scap)); BVH_TRY(next.grow(scap));
    size_t node_cap = 2 * (size_t)n + 64;
    BVH_TRY(nodes.grow(node_cap)); BVH_TRY(box.grow(6 * node_cap));
    lap("alloc+h2d");
    hipLaunchKernelGGL(k_iota, dim3(nb(n, 256)), dim3(256), 0, st, n, perm.p);
    lap("first-kern");

    // root: construct(0, n, 0, 0)
    int num_nodes = 1;
    const int4 root = make_int4(-1, -1, 0, n);
    BVH_TRY(hipMemcpyAsync(nodes.p, &root, sizeof(int4), hipMemcpyHostToDevice, st));
    DevArr<unsigned long long> kmin(st), kmax(st);       // (value, position) box keys per node
    BVH_TRY(kmin.grow(3 * node_cap)); BVH_TRY(kmax.grow(3 * node_cap));
    BVH_TRY(hipMemsetAsync(kmin.p, 0xFF, sizeof(unsigned long long) * 3, st));
    BVH_TRY(hipMemsetAsync(kmax.p, 0, sizeof(unsigned long long) * 3, st));
    hipLaunchKernelGGL(k_box_keys, dim3(nb(nb(n, kRun), 256)), dim3(256), 0, st, n, true, segid.p, 0, segs.p, G.p, nodes.p,
                       perm.p, lo3.p, hi3.p, kmin.p, kmax.p);
    hipLaunchKernelGGL(k_box_final, dim3(1), dim3(64), 0, st, 0, 1, perm.p, lo3.p, hi3.p, kmin.p, kmax.p, box.p);
    int S = 0;
    if (n >= 2) {
        Seg s0; s0.start = 0; s0.end = n; s0.node = 0; s0.off = 0;
        BVH_TRY(hipMemcpyAsync(segs.p, &s0, sizeof(Seg), hipMemcpyHostToDevice, st));
        S = 1;
    }
    size_t tmp_bytes = 0;
    auto ensure_tmp = [&](size_t need) -> hipError_t { if (need > tmp_bytes) { tmp_bytes = need; return tmp.grow(need); } return hipSuccess; };
    for (int depth = 0; S > 0; depth++) {
        const int axis = depth % 3;           // splitType 0,1,2,0,... (src/BVH.cpp:70-72)
        // key offsets of the segments in the sorted array
        hipLaunchKernelGGL(k_seg_len, dim3(nb(S, 256)), dim3(256), 0, st, segs.p, S, lens.p);
        size_t need = 0;
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, lens.p, offs.p, S, st));
        BVH_TRY(ensure_tmp(need));
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, need, lens.p, offs.p, S, st));
        hipLaunchKernelGGL(k_seg_off, dim3(nb(S, 256)), dim3(256), 0, st, segs.p, S, offs.p);
        // order statistics: sort (segment, centre) keys
        hipLaunchKernelGGL(k_segid, dim3(nb(n, 256)), dim3(256), 0, st, n, segs.p, S, segid.p);
        hipLaunchKernelGGL(k_keys, dim3(nb(n, 256)), dim3(256), 0, st, n, axis, segid.p, S, perm.p, c3.p, keys.p);
        const int sbits = 32 - __builtin_clz((unsigned)S);      // S itself (the sentinel) must fit
        need = 0;
        BVH_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, need, keys.p, sorted.p, n, 0, 32 + sbits, st));
        BVH_TRY(ensure_tmp(need));
        BVH_TRY(hipcub::DeviceRadixSort::SortKeys(tmp.p, need, keys.p, sorted.p, n, 0, 32 + sbits, st));
        hipLaunchKernelGGL(k_split, dim3(nb(S, 256)), dim3(256), 0, st, segs.p, S, sorted.p, split.p);
        // partition
        hipLaunchKernelGGL(k_less, dim3(nb(n + 1, 256)), dim3(256), 0, st, n, axis, segid.p, S, perm.p, c3.p, split.p, less.p);
        need = 0;
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, less.p, G.p, n + 1, st));
        BVH_TRY(ensure_tmp(need));
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, need, less.p, G.p, n + 1, st));
        hipLaunchKernelGGL(k_ptr_init, dim3(nb(n, 256)), dim3(256), 0, st, n, segid.p, S, segs.p, G.p, less.p, ptr.p);
        hipLaunchKernelGGL(k_jump, dim3(nb(n, 256)), dim3(256), 0, st, n, ptr.p);
        hipLaunchKernelGGL(k_scatter, dim3(nb(n, 256)), dim3(256), 0, st, n, segid.p, S, segs.p, G.p, less.p, ptr.p,
                           perm.p, perm2.p);
        std::swap(perm.p, perm2.p);
        std::swap(perm.cap, perm2.cap);
        // children
        hipLaunchKernelGGL(k_child_count, dim3(nb(S + 1, 256)), dim3(256), 0, st, segs.p, S, depth + 1, G.p, nn.p, ni.p);
        need = 0;
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, nn.p, nnoff.p, S + 1, st));
        BVH_TRY(ensure_tmp(need));
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, need, nn.p, nnoff.p, S + 1, st));
        BVH_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, need, ni.p, nioff.p, S + 1, st));
        int tot[2] = {0, 0};
        BVH_TRY(hipMemcpyAsync(&tot[0], nnoff.p + S, sizeof(int), hipMemcpyDeviceToHost, st));
        BVH_TRY(hipMemcpyAsync(&tot[1], nioff.p + S, sizeof(int), hipMemcpyDeviceToHost, st));
        BVH_TRY(hipStreamSynchronize(st));
        const int new_nodes = tot[0], S_next = tot[1];
        if ((size_t)(num_nodes + new_nodes) > node_cap) {       // grow the node arrays, keeping contents
            size_t cap2 = std::max(node_cap * 2, (size_t)(num_nodes + new_nodes) + 64);
            int4* n2 = nullptr; float* b2 = nullptr;
            BVH_TRY(hipMallocAsync(reinterpret_cast<void**>(&n2), sizeof(int4) * cap2, st));
            BVH_TRY(hipMallocAsync(reinterpret_cast<void**>(&b2), sizeof(float) * 6 * cap2, st));
            BVH_TRY(hipMemcpyAsync(n2, nodes.p, sizeof(int4) * num_nodes, hipMemcpyDeviceToDevice, st));
            BVH_TRY(hipMemcpyAsync(b2, box.p, sizeof(float) * 6 * num_nodes, hipMemcpyDeviceToDevice, st));
            (void)hipFreeAsync(nodes.p, st); (void)hipFreeAsync(box.p, st);
            nodes.p = n2; nodes.cap = cap2; box.p = b2; box.cap = 6 * cap2;
            node_cap = cap2;
        }
        hipLaunchKernelGGL(k_child_emit, dim3(nb(S, 256)), dim3(256), 0, st, segs.p, S, depth + 1, G.p, nnoff.p, nioff.p,
                           num_nodes, nodes.p, next.p);
        // the new nodes' boxes over their ranges in the order just formed
        if (new_nodes > 0) {
            BVH_TRY(kmin.grow(3 * node_cap)); BVH_TRY(kmax.grow(3 * node_cap));
            BVH_TRY(hipMemsetAsync(kmin.p + 3 * (size_t)num_nodes, 0xFF, sizeof(unsigned long long) * 3 * new_nodes, st));
            BVH_TRY(hipMemsetAsync(kmax.p + 3 * (size_t)num_nodes, 0, sizeof(unsigned long long) * 3 * new_nodes, st));
            hipLaunchKernelGGL(k_box_keys, dim3(nb(nb(n, kRun), 256)), dim3(256), 0, st, n, false, segid.p, S, segs.p, G.p,
                               nodes.p, perm.p, lo3.p, hi3.p, kmin.p, kmax.p);
            hipLaunchKernelGGL(k_box_final, dim3(nb(new_nodes, 256)), dim3(256), 0, st, num_nodes, new_nodes, perm.p,
                               lo3.p, hi3.p, kmin.p, kmax.p, box.p);
        }
        BVH_TRY(hipGetLastError());
        num_nodes += new_nodes;
        std::swap(segs.p, next.p);
        std::swap(segs.cap, next.cap);
        S = S_next;
    }
    lap("levels");
    // the host's node layout on the device (one 40-byte record per node), then both arrays into pooled
    // page-locked staging
    DevArr<NodeRec40> rec(st);
    BVH_TRY(rec.grow(num_nodes));
    hipLaunchKernelGGL(k_node40, dim3(nb(num_nodes, 256)), dim3(256), 0, st, nodes.p, box.p, num_nodes, rec.p);
    if (!out.perm.get(sizeof(int) * (size_t)n) || !out.nodes.get(sizeof(NodeRec40) * (size_t)num_nodes)) {
        err = "page-locked staging allocation failed";
        return -1;
    }
    BVH_TRY(hipMemcpyAsync(out.perm.p, perm.p, sizeof(int) * n, hipMemcpyDeviceToHost, st));
    BVH_TRY(hipMemcpyAsync(out.nodes.p, rec.p, sizeof(NodeRec40) * num_nodes, hipMemcpyDeviceToHost, st));
    BVH_TRY(hipStreamSynchronize(st));
    out.num_nodes = num_nodes;
    lap("d2h");
    out.root = 0;
    return 0;
}

// Process-wide pool of page-locked staging buffers (best fit).  Each buffer keeps its real capacity
// (a reused larger buffer is returned at that capacity, not at the size last asked of it), and the
// pool holds at most kPoolBytes: buffers beyond that are freed (a long-lived process
// creating scenes of varying size must not grow its page-locked memory without bound).
namespace {
std::mutex g_pool_mu;
std::vector<std::pair<void*, size_t>> g_pool;     // (buffer, capacity)
size_t g_pool_bytes = 0;
constexpr size_t kPoolBytes = size_t(1) << 30;
}
void* pinned_pool_get(size_t bytes, size_t* cap) {
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        size_t best = g_pool.size();
        for (size_t k = 0; k < g_pool.size(); k++)
            if (g_pool[k].second >= bytes && (best == g_pool.size() || g_pool[k].second < g_pool[best].second)) best = k;
        if (best < g_pool.size()) {
            void* p = g_pool[best].first;
            *cap = g_pool[best].second;
            g_pool_bytes -= g_pool[best].second;
            g_pool.erase(g_pool.begin() + best);
            return p;
        }
    }
    void* p = nullptr;
    const size_t want = std::max<size_t>(bytes, 1);
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return nullptr;
    *cap = want;
    return p;
}
void pinned_pool_put(void* p, size_t cap) {
    if (!p) return;
    std::vector<void*> drop;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        g_pool.emplace_back(p, cap);
        g_pool_bytes += cap;
        // over the cap: free the smallest buffers first (the large ones are the expensive ones to remake)
        while (g_pool_bytes > kPoolBytes && !g_pool.empty()) {
            size_t k = 0;
            for (size_t j = 1; j < g_pool.size(); j++)
                if (g_pool[j].second < g_pool[k].second) k = j;
            g_pool_bytes -= g_pool[k].second;
            drop.push_back(g_pool[k].first);
            g_pool.erase(g_pool.begin() + k);
        }
    }
    for (void* q : drop) (void)hipHostFree(q);
}

}  // namespace rtg
