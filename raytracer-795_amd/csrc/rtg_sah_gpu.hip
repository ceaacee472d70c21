// rtg_sah_gpu.hip — the traversal tree's binned-SAH BVH2 built on the GPU.
//
// The host builder (rtg_host.cpp sah_split / sah_rec) and this one apply the same rule to a range of
// triangle records: box and centroid bounds; split axis = the widest centroid extent (ties: lowest
// axis); 16 bins over it, bin = min(15, max(0, (int)((centre - c0) * (16 / extent)))); SAH cost in
// double over the bins' boxes (area x count); a range of <= 4 records stays a leaf when splitting does
// not pay; a range with a zero centroid extent is halved by count.  Bins, bounds and the chosen split
// are functions of the range's *set* of records (counts and min / max are order-independent), so both
// builders produce the same tree -- the same node boxes over the same triangle sets -- except where a
// range is halved by count (all centroids equal), where the members of each half depend on the order
// inside the range (host: std::partition's order below 2^18 records, here: a stable partition).  Any
// tree gives the same render results (the traversal tree only orders the candidates; the
// reference tree decides reachability), so that difference is harmless; tests/test_gpu_sah.py compares
// the two trees' order-independent hash on meshes without such ranges.
//
// Two phases:
//   * ranges of more than kSmall records, level by level: bounds and bins per 4096-record chunk in
//     LDS, combined with global atomics (ordered-uint min / max), the decision per range, a stable
//     partition by a global prefix sum of the left flags; the host keeps the (few hundred) ranges;
//   * every range of at most kSmall records: one wave builds its whole subtree depth first (bounds by
//     wave reduction, bins by LDS atomics, the decision on lane 0, a stable ballot partition),
//     nodes from a block reserved for the subtree (2m - 1 for m records).
// Nodes are SahNode2 records, breadth-first for the level phase; the host collapses them to Node4.
#include <float.h>
#include <limits.h>

#include <hipcub/hipcub.hpp>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <functional>
#include <string>
#include <vector>

#include "rtg_internal.h"

namespace rtg {
namespace {

constexpr int kBins = kSahBins;
constexpr int kLeaf = kSahMaxLeaf;
constexpr int kSmall = 512;        // ranges of at most this many records: one wave per subtree
constexpr int kChunk = 4096;       // records per workgroup in the level passes
constexpr int kStack = 24;         // subtree stack (the larger child is pushed: depth <= log2(kSmall) + 1)

__device__ __forceinline__ unsigned ordu(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unordu(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ __forceinline__ float ctr(const SahRec& r, int z) { return 0.5f * (r.lo[z] + r.hi[z]); }
__device__ __forceinline__ double area(const float lo[3], const float hi[3]) {   // sah_area
    const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

// Bounds of a range: box and centroid box (12 ordered uints: lo xyz, hi xyz, clo xyz, chi xyz).
struct Acc { unsigned v[12]; };
__device__ __forceinline__ void acc_init(unsigned* v) {
    for (int z = 0; z < 3; z++) {
        v[z] = 0xFFFFFFFFu; v[3 + z] = 0u; v[6 + z] = 0xFFFFFFFFu; v[9 + z] = 0u;
    }
}
__device__ __forceinline__ void acc_add(unsigned* v, const SahRec& r) {
    for (int z = 0; z < 3; z++) {
        const unsigned c = ordu(ctr(r, z));
        v[z] = min(v[z], ordu(r.lo[z]));
        v[3 + z] = max(v[3 + z], ordu(r.hi[z]));
        v[6 + z] = min(v[6 + z], c);
        v[9 + z] = max(v[9 + z], c);
    }
}

// The split rule (sah_split) on a range's bounds and bins: kind 0 leaf, 1 split at bin best_b (nl
// records left), 2 halve by count.
struct Decision { int kind, best_b, nl, axis; float c0, sc; };
__device__ Decision decide(const float lo[3], const float hi[3], const float clo[3], const float chi[3], int n,
                           const unsigned* cnt, const unsigned* blo, const unsigned* bhi, bool binned) {
    Decision D;
    D.kind = 0; D.best_b = -1; D.nl = 0; D.axis = 0; D.c0 = 0.0f; D.sc = 0.0f;
    if (n <= 1) return D;
    int axis = 0;
    for (int z = 1; z < 3; z++)
        if (chi[z] - clo[z] > chi[axis] - clo[axis]) axis = z;
    const float ext = chi[axis] - clo[axis];
    D.axis = axis;
    if (!(ext > 0.0f)) {
        if (n <= kLeaf) return D;
        D.kind = 2; D.nl = n / 2;
        return D;
    }
    D.sc = (float)kBins / ext;
    D.c0 = clo[axis];
    if (!binned) return D;   // (the caller bins next)
    double rcost[kBins];
    float l3[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, h3[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    int rc = 0;
    for (int b = kBins - 1; b >= 1; b--) {
        rc += (int)cnt[b];
        if (cnt[b])
            for (int z = 0; z < 3; z++) {
                l3[z] = fminf(l3[z], unordu(blo[3 * b + z]));
                h3[z] = fmaxf(h3[z], unordu(bhi[3 * b + z]));
            }
        rcost[b] = rc ? area(l3, h3) * rc : 0.0;
    }
    for (int z = 0; z < 3; z++) { l3[z] = FLT_MAX; h3[z] = -FLT_MAX; }
    int lc = 0, best_b = -1, best_nl = 0;
    double best = 1e300;
    for (int b = 0; b < kBins - 1; b++) {
        lc += (int)cnt[b];
        if (cnt[b])
            for (int z = 0; z < 3; z++) {
                l3[z] = fminf(l3[z], unordu(blo[3 * b + z]));
                h3[z] = fmaxf(h3[z], unordu(bhi[3 * b + z]));
            }
        if (lc == 0 || lc == n) continue;
        const double cost = area(l3, h3) * lc + rcost[b + 1];
        if (cost < best) { best = cost; best_b = b; best_nl = lc; }
    }
    const double leaf_cost = area(lo, hi) * n;
    if (n <= kLeaf && (best_b < 0 || leaf_cost <= area(lo, hi) + best)) return D;
    if (best_b >= 0) { D.kind = 1; D.best_b = best_b; D.nl = best_nl; return D; }
    D.kind = 2; D.nl = n / 2;
    return D;
}
__device__ __forceinline__ int bin_of(const SahRec& r, const Decision& D) {
    return min(kBins - 1, max(0, (int)((ctr(r, D.axis) - D.c0) * D.sc)));
}

// ---------------------------------------------------------------- level phase (large ranges)
struct LSeg { int start, end, node, chunk0; };   // chunk0: first chunk of the range in this level's grid

__device__ __forceinline__ int seg_of_chunk(const LSeg* segs, int S, int chunk) {
    int lo = 0, hi = S - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].chunk0 <= chunk) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__global__ void k_acc_init(unsigned* acc, unsigned* bins, int S) {
    const int s = blockIdx.x;
    if (s >= S) return;
    if (threadIdx.x < 12) {
        unsigned v[12];
        acc_init(v);
        acc[12 * s + threadIdx.x] = v[threadIdx.x];
    }
    for (int k = threadIdx.x; k < kBins * 7; k += blockDim.x) {
        // per bin: cnt, lo xyz (min), hi xyz (max)
        const int f = k % 7;
        bins[(size_t)kBins * 7 * s + k] = f == 0 ? 0u : (f <= 3 ? 0xFFFFFFFFu : 0u);
    }
}

// block reduce of 12 bounds values, then one atomic each
__global__ void __launch_bounds__(256) k_bounds(const SahRec* __restrict__ recs, const LSeg* __restrict__ segs, int S,
                                                unsigned* __restrict__ acc) {
    __shared__ unsigned sh[12];
    const int s = seg_of_chunk(segs, S, blockIdx.x);
    const LSeg g = segs[s];
    const int a = g.start + (blockIdx.x - g.chunk0) * kChunk, b = min(g.end, a + kChunk);
    if (threadIdx.x < 12) { unsigned v[12]; acc_init(v); sh[threadIdx.x] = v[threadIdx.x]; }
    __syncthreads();
    unsigned v[12];
    acc_init(v);
    for (int i = a + threadIdx.x; i < b; i += blockDim.x) acc_add(v, recs[i]);
    for (int off = 32; off > 0; off >>= 1)
        for (int k = 0; k < 12; k++) {
            const unsigned o = __shfl_xor(v[k], off);
            v[k] = ((k % 6) < 3) ? min(v[k], o) : max(v[k], o);
        }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 12; k++) {
            if ((k % 6) < 3) atomicMin(&sh[k], v[k]); else atomicMax(&sh[k], v[k]);
        }
    __syncthreads();
    if (threadIdx.x < 12) {
        const int k = threadIdx.x;
        if ((k % 6) < 3) atomicMin(&acc[12 * s + k], sh[k]); else atomicMax(&acc[12 * s + k], sh[k]);
    }
}

__device__ __forceinline__ void acc_floats(const unsigned* a, float lo[3], float hi[3], float clo[3], float chi[3]) {
    for (int z = 0; z < 3; z++) {
        lo[z] = unordu(a[z]); hi[z] = unordu(a[3 + z]); clo[z] = unordu(a[6 + z]); chi[z] = unordu(a[9 + z]);
    }
}

__global__ void __launch_bounds__(256) k_bins(const SahRec* __restrict__ recs, const LSeg* __restrict__ segs, int S,
                                              const unsigned* __restrict__ acc, unsigned* __restrict__ bins) {
    __shared__ unsigned sb[kBins * 7];
    const int s = seg_of_chunk(segs, S, blockIdx.x);
    const LSeg g = segs[s];
    float lo[3], hi[3], clo[3], chi[3];
    acc_floats(acc + 12 * s, lo, hi, clo, chi);
    const Decision D = decide(lo, hi, clo, chi, g.end - g.start, nullptr, nullptr, nullptr, false);
    if (!(D.sc > 0.0f)) return;                  // no binning (leaf / halve)
    for (int k = threadIdx.x; k < kBins * 7; k += blockDim.x) {
        const int f = k % 7;
        sb[k] = f == 0 ? 0u : (f <= 3 ? 0xFFFFFFFFu : 0u);
    }
    __syncthreads();
    const int a = g.start + (blockIdx.x - g.chunk0) * kChunk, b = min(g.end, a + kChunk);
    for (int i = a + threadIdx.x; i < b; i += blockDim.x) {
        const SahRec r = recs[i];
        unsigned* q = sb + 7 * bin_of(r, D);
        atomicAdd(q, 1u);
        for (int z = 0; z < 3; z++) {
            atomicMin(q + 1 + z, ordu(r.lo[z]));
            atomicMax(q + 4 + z, ordu(r.hi[z]));
        }
    }
    __syncthreads();
    unsigned* gb = bins + (size_t)kBins * 7 * s;
    for (int k = threadIdx.x; k < kBins * 7; k += blockDim.x) {
        const int f = k % 7;
        if (f == 0) { if (sb[k]) atomicAdd(gb + k, sb[k]); }
        else if (f <= 3) { if (sb[k] != 0xFFFFFFFFu) atomicMin(gb + k, sb[k]); }
        else if (sb[k]) atomicMax(gb + k, sb[k]);
    }
}

// one thread per range: the node record and the decision
__global__ void k_decide(const LSeg* __restrict__ segs, int S, const unsigned* __restrict__ acc,
                         const unsigned* __restrict__ bins, SahNode2* __restrict__ nodes, Decision* __restrict__ dec) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const LSeg g = segs[s];
    float lo[3], hi[3], clo[3], chi[3];
    acc_floats(acc + 12 * s, lo, hi, clo, chi);
    const unsigned* gb = bins + (size_t)kBins * 7 * s;
    unsigned cnt[kBins], blo[3 * kBins], bhi[3 * kBins];
    for (int b = 0; b < kBins; b++) {
        cnt[b] = gb[7 * b];
        for (int z = 0; z < 3; z++) { blo[3 * b + z] = gb[7 * b + 1 + z]; bhi[3 * b + z] = gb[7 * b + 4 + z]; }
    }
    const Decision D = decide(lo, hi, clo, chi, g.end - g.start, cnt, blo, bhi, true);
    SahNode2 nd;
    for (int z = 0; z < 3; z++) { nd.lo[z] = lo[z]; nd.hi[z] = hi[z]; }
    nd.left = nd.right = -1;
    nd.start = g.start;
    nd.count = g.end - g.start;
    nodes[g.node] = nd;
    dec[s] = D;
}

__global__ void k_links(const int2* __restrict__ links, int L, SahNode2* __restrict__ nodes) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= L) return;
    nodes[links[k].x].left = links[k].y;
    nodes[links[k].x].right = links[k].y + 1;
}

// left flags of the split ranges' records (0 elsewhere); flags[n] = 0
__global__ void k_flags(const SahRec* __restrict__ recs, const LSeg* __restrict__ segs, int S,
                        const Decision* __restrict__ dec, int* __restrict__ flags) {
    const int s = seg_of_chunk(segs, S, blockIdx.x);
    const LSeg g = segs[s];
    const Decision D = dec[s];
    const int a = g.start + (blockIdx.x - g.chunk0) * kChunk, b = min(g.end, a + kChunk);
    for (int i = a + threadIdx.x; i < b; i += blockDim.x) {
        int f = 0;
        if (D.kind == 1) f = bin_of(recs[i], D) <= D.best_b;
        else if (D.kind == 2) f = (i - g.start) < D.nl;
        flags[i] = f;
    }
}
__global__ void k_scatter(const SahRec* __restrict__ recs, const LSeg* __restrict__ segs, int S,
                          const Decision* __restrict__ dec, const int* __restrict__ G, SahRec* __restrict__ out) {
    const int s = seg_of_chunk(segs, S, blockIdx.x);
    const LSeg g = segs[s];
    const Decision D = dec[s];
    const int a = g.start + (blockIdx.x - g.chunk0) * kChunk, b = min(g.end, a + kChunk);
    const int g0 = G[g.start];
    for (int i = a + threadIdx.x; i < b; i += blockDim.x) {
        int p = i;
        if (D.kind != 0) {
            const int lb = G[i] - g0;                 // left records before i in the range
            const int left = G[i + 1] - G[i];
            p = left ? g.start + lb : g.start + D.nl + ((i - g.start) - lb);
        }
        out[p] = recs[i];
    }
}
__global__ void k_copy_back(const SahRec* __restrict__ from, const LSeg* __restrict__ segs, int S,
                            SahRec* __restrict__ to) {
    const int s = seg_of_chunk(segs, S, blockIdx.x);
    const LSeg g = segs[s];
    const int a = g.start + (blockIdx.x - g.chunk0) * kChunk, b = min(g.end, a + kChunk);
    for (int i = a + threadIdx.x; i < b; i += blockDim.x) to[i] = from[i];
}

// ---------------------------------------------------------------- subtree phase (small ranges)
struct SSeg { int start, end, node, pad; };

// wave-wide min / max of 12 bounds values
__device__ __forceinline__ void wave_bounds(const SahRec* __restrict__ recs, int a, int b, int lane, unsigned* v) {
    acc_init(v);
    for (int i = a + lane; i < b; i += 64) acc_add(v, recs[i]);
    for (int off = 32; off > 0; off >>= 1)
        for (int k = 0; k < 12; k++) {
            const unsigned o = __shfl_xor(v[k], off);
            v[k] = ((k % 6) < 3) ? min(v[k], o) : max(v[k], o);
        }
}

__global__ void __launch_bounds__(64) k_subtrees(SahRec* __restrict__ recs, SahRec* __restrict__ tmp,
                                                 const SSeg* __restrict__ segs, int S, SahNode2* __restrict__ nodes,
                                                 int* __restrict__ node_count) {
    __shared__ unsigned sb[kBins * 7];
    __shared__ int st_s[kStack], st_e[kStack], st_n[kStack];
    __shared__ int s_base;
    const int lane = threadIdx.x;
    const SSeg root = segs[blockIdx.x];
    const int m = root.end - root.start;
    if (lane == 0) s_base = m > 1 ? atomicAdd(node_count, 2 * m - 2) : 0;
    __syncthreads();
    int next_node = s_base;
    int sp = 0;
    int cs = root.start, ce = root.end, cn = root.node;
    while (true) {
        const int n = ce - cs;
        unsigned v[12];
        wave_bounds(recs, cs, ce, lane, v);
        float lo[3], hi[3], clo[3], chi[3];
        acc_floats(v, lo, hi, clo, chi);
        Decision D = decide(lo, hi, clo, chi, n, nullptr, nullptr, nullptr, false);
        if (D.sc > 0.0f) {
            for (int k = lane; k < kBins * 7; k += 64) {
                const int f = k % 7;
                sb[k] = f == 0 ? 0u : (f <= 3 ? 0xFFFFFFFFu : 0u);
            }
            __syncthreads();
            for (int i = cs + lane; i < ce; i += 64) {
                const SahRec r = recs[i];
                unsigned* q = sb + 7 * bin_of(r, D);
                atomicAdd(q, 1u);
                for (int z = 0; z < 3; z++) {
                    atomicMin(q + 1 + z, ordu(r.lo[z]));
                    atomicMax(q + 4 + z, ordu(r.hi[z]));
                }
            }
            __syncthreads();
            unsigned cnt[kBins], blo[3 * kBins], bhi[3 * kBins];
            for (int b = 0; b < kBins; b++) {
                cnt[b] = sb[7 * b];
                for (int z = 0; z < 3; z++) { blo[3 * b + z] = sb[7 * b + 1 + z]; bhi[3 * b + z] = sb[7 * b + 4 + z]; }
            }
            D = decide(lo, hi, clo, chi, n, cnt, blo, bhi, true);
            __syncthreads();                          // sb is re-initialised by the next range
        }
        if (lane == 0) {
            SahNode2 nd;
            for (int z = 0; z < 3; z++) { nd.lo[z] = lo[z]; nd.hi[z] = hi[z]; }
            nd.left = nd.right = -1;
            nd.start = cs;
            nd.count = n;
            if (D.kind != 0) { nd.left = next_node; nd.right = next_node + 1; }
            nodes[cn] = nd;
        }
        if (D.kind == 0) {
            if (sp == 0) break;
            sp--;
            cs = st_s[sp]; ce = st_e[sp]; cn = st_n[sp];
            continue;
        }
        if (D.kind == 1) {
            // stable partition through tmp, then back
            int lb = 0, rb = 0;
            for (int i0 = cs; i0 < ce; i0 += 64) {
                const int i = i0 + lane;
                const bool in = i < ce;
                SahRec r;
                bool left = false;
                if (in) { r = recs[i]; left = bin_of(r, D) <= D.best_b; }
                const unsigned long long ml = __ballot(in && left), mr = __ballot(in && !left);
                const unsigned long long below = (1ull << lane) - 1ull;
                if (in) {
                    const int p = left ? cs + lb + __popcll(ml & below) : cs + D.nl + rb + __popcll(mr & below);
                    tmp[p] = r;
                }
                lb += __popcll(ml);
                rb += __popcll(mr);
            }
            __threadfence_block();
            __syncthreads();
            for (int i = cs + lane; i < ce; i += 64) recs[i] = tmp[i];
            __threadfence_block();
            __syncthreads();
        }
        // (kind 2: halving by count keeps the order)
        const int mid = cs + D.nl;
        const int ln = next_node, rn = next_node + 1;
        next_node += 2;
        // continue with the smaller half, push the larger (stack depth <= log2(m) + 1)
        const bool left_small = (mid - cs) <= (ce - mid);
        const int ps = left_small ? mid : cs, pe = left_small ? ce : mid, pn = left_small ? rn : ln;
        if (lane == 0) { st_s[sp] = ps; st_e[sp] = pe; st_n[sp] = pn; }
        __syncthreads();
        sp++;
        if (left_small) { ce = mid; cn = ln; } else { cs = mid; cn = rn; }
    }
}

__global__ void k_order(const SahRec* __restrict__ recs, int n, int* __restrict__ order) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) order[i] = recs[i].idx;
}

// ---------------------------------------------------------------- collapse to Node4 (rtg_host.cpp collapse_node)
// The 4-wide node over BVH2 node q: its children, the interior slot of largest area expanded while
// slots are free (first of equal areas).
struct Slots { int slot[4], used; };
__device__ Slots slots_of(const SahNode2* __restrict__ bn, int q) {
    Slots S;
    S.slot[0] = bn[q].left; S.slot[1] = bn[q].right; S.slot[2] = S.slot[3] = -1;
    S.used = 2;
    while (S.used < 4) {
        int pick = -1;
        double pa = -1.0;
        for (int j = 0; j < S.used; j++)
            if (bn[S.slot[j]].left >= 0) {
                const double a = area(bn[S.slot[j]].lo, bn[S.slot[j]].hi);
                if (a > pa) { pa = a; pick = j; }
            }
        if (pick < 0) break;
        const int c = S.slot[pick];
        S.slot[pick] = bn[c].left;
        S.slot[S.used++] = bn[c].right;
    }
    return S;
}
__global__ void k_c4_count(const int* __restrict__ Q, int nq, const SahNode2* __restrict__ bn, int* __restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nq) return;
    int c = 0;
    if (i < nq) {
        const Slots S = slots_of(bn, Q[i]);
        for (int j = 0; j < S.used; j++) c += bn[S.slot[j]].left >= 0;
    }
    cnt[i] = c;                 // cnt[nq] = 0: the exclusive scan's last entry is the total
}
// Node4 base_this + i for Q[i]; its k-th interior slot becomes Node4 base_next + off[i] + k
__global__ void k_c4_emit(const int* __restrict__ Q, int nq, const SahNode2* __restrict__ bn, const int* __restrict__ off,
                          int base_this, int base_next, int tri_base, float pad, Node4* __restrict__ out,
                          int* __restrict__ Qn) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const Slots S = slots_of(bn, Q[i]);
    float lo[3][4], hi[3][4];
    int ref[4], info[4];
    int k = off[i];
    for (int j = 0; j < 4; j++) {
        if (j >= S.used) {
            for (int z = 0; z < 3; z++) { lo[z][j] = 0.0f; hi[z][j] = 0.0f; }
            ref[j] = 0; info[j] = -1;
            continue;
        }
        const SahNode2 c = bn[S.slot[j]];
        for (int z = 0; z < 3; z++) {
            lo[z][j] = nextafterf((float)((double)c.lo[z] - pad), -FLT_MAX);
            hi[z][j] = nextafterf((float)((double)c.hi[z] + pad), FLT_MAX);
        }
        if (c.left < 0) { ref[j] = tri_base + c.start; info[j] = c.count; }
        else { ref[j] = base_next + k; info[j] = 0; Qn[k] = S.slot[j]; k++; }
    }
    Node4 nd;
    nd.lox = make_float4(lo[0][0], lo[0][1], lo[0][2], lo[0][3]);
    nd.loy = make_float4(lo[1][0], lo[1][1], lo[1][2], lo[1][3]);
    nd.loz = make_float4(lo[2][0], lo[2][1], lo[2][2], lo[2][3]);
    nd.hix = make_float4(hi[0][0], hi[0][1], hi[0][2], hi[0][3]);
    nd.hiy = make_float4(hi[1][0], hi[1][1], hi[1][2], hi[1][3]);
    nd.hiz = make_float4(hi[2][0], hi[2][1], hi[2][2], hi[2][3]);
    nd.ref = make_int4(ref[0], ref[1], ref[2], ref[3]);
    nd.info = make_int4(info[0], info[1], info[2], info[3]);
    out[base_this + i] = nd;
}

// the order-independent hash of rtg_host.cpp sah_tree_stats over the written nodes (count >= 0; the
// array starts as all ones, so unused reserved slots have count -1)
__device__ __forceinline__ unsigned long long mix64d(unsigned long long x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
__global__ void k_hash(const SahNode2* __restrict__ bn, int nn, unsigned long long* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long h = 0, c = 0;
    if (i < nn && bn[i].count >= 0) {
        const SahNode2 nd = bn[i];
        h = (unsigned long long)(unsigned)nd.count * 0x9E3779B97F4A7C15ULL;
        for (int z = 0; z < 3; z++) {
            const unsigned ua = __float_as_uint(nd.lo[z] + 0.0f), ub = __float_as_uint(nd.hi[z] + 0.0f);
            h = mix64d(h ^ ((unsigned long long)ua << 32 | ub) ^ (unsigned long long)(z + 1));
        }
        c = 1;
    }
    for (int off = 32; off > 0; off >>= 1) {
        h += __shfl_down(h, off);
        c += __shfl_down(c, off);
    }
    if ((threadIdx.x & 63) == 0 && c) { atomicAdd(out, h); atomicAdd(out + 1, c); }
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

}  // namespace

#define SAH_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);           \
            return -1;                                                         \
        }                                                                      \
    } while (0)

int gpu_build_sah(const SahRec* recs_host, int n, int tri_base, float pad, const std::function<Node4*(size_t)>& alloc4,
                  int* order_host, uint64_t& bvh2_nodes, uint64_t& hash, std::string& err) {
    bvh2_nodes = 0;
    hash = 0;
    if (n <= 0) return 0;
    if (n > (1 << 29)) { err = "too many triangles for the GPU SAH build"; return -1; }
    const bool timing = getenv("RTG_BUILD_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    hipStream_t st = nullptr;
    SAH_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct StreamGuard { hipStream_t s; ~StreamGuard() { if (s) { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); } } } sg{st};
    auto lap = [&](const char* what) {
        if (!timing) return;
        (void)hipStreamSynchronize(st);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[rtg] gpu sah %-10s %7.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    DevArr<SahRec> A(st), B(st);
    DevArr<SahNode2> nodes(st);
    DevArr<int> flags(st), G(st), order(st), ncount(st);
    DevArr<unsigned> acc(st), bins(st);
    DevArr<LSeg> dsegs(st);
    DevArr<Decision> ddec(st);
    DevArr<SSeg> dsmall(st);
    DevArr<int2> dlinks(st);
    DevArr<unsigned char> tmp(st);
    const size_t node_cap = 2 * (size_t)n + 2;
    SAH_TRY(A.grow(n)); SAH_TRY(B.grow(n)); SAH_TRY(nodes.grow(node_cap));
    SAH_TRY(hipMemsetAsync(nodes.p, 0xFF, sizeof(SahNode2) * node_cap, st));   // count -1: never written
    SAH_TRY(flags.grow((size_t)n + 1)); SAH_TRY(G.grow((size_t)n + 1)); SAH_TRY(order.grow(n)); SAH_TRY(ncount.grow(1));
    SAH_TRY(hipMemcpyAsync(A.p, recs_host, sizeof(SahRec) * (size_t)n, hipMemcpyHostToDevice, st));
    SAH_TRY(hipMemsetAsync(flags.p, 0, sizeof(int) * ((size_t)n + 1), st));
    lap("h2d");
    // the level phase: ranges > kSmall (the host keeps them: at most n / kSmall per level)
    std::vector<LSeg> segs;
    std::vector<SSeg> small;
    int num_nodes = 1;
    if (n > kSmall) segs.push_back(LSeg{0, n, 0, 0});
    else small.push_back(SSeg{0, n, 0, 0});
    size_t tmp_bytes = 0;
    std::vector<Decision> hdec;
    while (!segs.empty()) {
        const int S = (int)segs.size();
        int chunks = 0;
        for (LSeg& g : segs) { g.chunk0 = chunks; chunks += (g.end - g.start + kChunk - 1) / kChunk; }
        SAH_TRY(dsegs.grow(S)); SAH_TRY(ddec.grow(S)); SAH_TRY(acc.grow(12 * (size_t)S)); SAH_TRY(bins.grow((size_t)kBins * 7 * S));
        SAH_TRY(hipMemcpyAsync(dsegs.p, segs.data(), sizeof(LSeg) * S, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_acc_init, dim3(S), dim3(128), 0, st, acc.p, bins.p, S);
        hipLaunchKernelGGL(k_bounds, dim3(chunks), dim3(256), 0, st, A.p, dsegs.p, S, acc.p);
        hipLaunchKernelGGL(k_bins, dim3(chunks), dim3(256), 0, st, A.p, dsegs.p, S, acc.p, bins.p);
        hipLaunchKernelGGL(k_decide, dim3((S + 63) / 64), dim3(64), 0, st, dsegs.p, S, acc.p, bins.p, nodes.p, ddec.p);
        hipLaunchKernelGGL(k_flags, dim3(chunks), dim3(256), 0, st, A.p, dsegs.p, S, ddec.p, flags.p);
        // ranges' flags are exclusive-scanned over the whole array: positions outside the ranges
        // hold stale flags, but every range only reads G inside itself (differences)
        size_t need = 0;
        SAH_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, flags.p, G.p, n + 1, st));
        if (need > tmp_bytes) { SAH_TRY(tmp.grow(need)); tmp_bytes = need; }
        SAH_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, need, flags.p, G.p, n + 1, st));
        hipLaunchKernelGGL(k_scatter, dim3(chunks), dim3(256), 0, st, A.p, dsegs.p, S, ddec.p, G.p, B.p);
        hipLaunchKernelGGL(k_copy_back, dim3(chunks), dim3(256), 0, st, B.p, dsegs.p, S, A.p);
        SAH_TRY(hipGetLastError());
        hdec.resize(S);
        SAH_TRY(hipMemcpyAsync(hdec.data(), ddec.p, sizeof(Decision) * S, hipMemcpyDeviceToHost, st));
        SAH_TRY(hipStreamSynchronize(st));
        std::vector<LSeg> next;
        std::vector<int2> links;               // (node, first child) of this level's split ranges
        for (int s = 0; s < S; s++) {
            const LSeg g = segs[s];
            const Decision& D = hdec[s];
            if (D.kind == 0) continue;
            const int mid = g.start + D.nl;
            const int ln = num_nodes, rn = num_nodes + 1;
            num_nodes += 2;
            links.push_back(make_int2(g.node, ln));
            const int r0[2] = {g.start, mid}, r1[2] = {mid, g.end}, id[2] = {ln, rn};
            for (int q = 0; q < 2; q++) {
                if (r1[q] - r0[q] > kSmall) next.push_back(LSeg{r0[q], r1[q], id[q], 0});
                else small.push_back(SSeg{r0[q], r1[q], id[q], 0});
            }
        }
        // child links of the split ranges (their node records were written by k_decide)
        if (!links.empty()) {
            SAH_TRY(dlinks.grow(links.size()));
            SAH_TRY(hipMemcpyAsync(dlinks.p, links.data(), sizeof(int2) * links.size(), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(k_links, dim3((unsigned)(links.size() + 63) / 64), dim3(64), 0, st, dlinks.p,
                               (int)links.size(), nodes.p);
            SAH_TRY(hipStreamSynchronize(st));    // (links is a host vector of this iteration)
        }
        segs.swap(next);
    }
    lap("levels");
    // the subtree phase: every small range, one wave each
    if (!small.empty()) {
        SAH_TRY(dsmall.grow(small.size()));
        SAH_TRY(hipMemcpyAsync(dsmall.p, small.data(), sizeof(SSeg) * small.size(), hipMemcpyHostToDevice, st));
        SAH_TRY(hipMemcpyAsync(ncount.p, &num_nodes, sizeof(int), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_subtrees, dim3((unsigned)small.size()), dim3(64), 0, st, A.p, B.p, dsmall.p,
                           (int)small.size(), nodes.p, ncount.p);
        SAH_TRY(hipGetLastError());
        SAH_TRY(hipMemcpyAsync(&num_nodes, ncount.p, sizeof(int), hipMemcpyDeviceToHost, st));
        SAH_TRY(hipStreamSynchronize(st));
    }
    lap("subtrees");
    if ((size_t)num_nodes > node_cap) { err = "GPU SAH build: node overflow"; return -1; }
    hipLaunchKernelGGL(k_order, dim3((n + 255) / 256), dim3(256), 0, st, A.p, n, order.p);
    SAH_TRY(hipMemcpyAsync(order_host, order.p, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost, st));
    // hash + count of the binary nodes
    DevArr<unsigned long long> hc(st);
    SAH_TRY(hc.grow(2));
    SAH_TRY(hipMemsetAsync(hc.p, 0, 2 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_hash, dim3((num_nodes + 255) / 256), dim3(256), 0, st, nodes.p, num_nodes, hc.p);
    unsigned long long hch[2] = {0, 0};
    SAH_TRY(hipMemcpyAsync(hch, hc.p, sizeof hch, hipMemcpyDeviceToHost, st));
    // collapse to 4-wide nodes, breadth first (root interior only: a root leaf has no Node4)
    SahNode2 root;
    SAH_TRY(hipMemcpyAsync(&root, nodes.p, sizeof root, hipMemcpyDeviceToHost, st));
    SAH_TRY(hipStreamSynchronize(st));
    hash = hch[0];
    bvh2_nodes = hch[1];
    lap("order+hash");
    if (root.left < 0) { alloc4(0); return 0; }
    DevArr<Node4> n4(st);
    DevArr<int> Q(st), Qn(st), cnt(st), off(st);
    const size_t cap4 = (size_t)num_nodes;        // at most one Node4 per binary node
    SAH_TRY(n4.grow(cap4)); SAH_TRY(Q.grow(cap4)); SAH_TRY(Qn.grow(cap4)); SAH_TRY(cnt.grow(cap4 + 1)); SAH_TRY(off.grow(cap4 + 1));
    const int zero = 0;
    SAH_TRY(hipMemcpyAsync(Q.p, &zero, sizeof(int), hipMemcpyHostToDevice, st));
    int nq = 1, base = 0;
    while (nq > 0) {
        hipLaunchKernelGGL(k_c4_count, dim3((nq + 256) / 256), dim3(256), 0, st, Q.p, nq, nodes.p, cnt.p);
        size_t need = 0;
        SAH_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, cnt.p, off.p, nq + 1, st));
        if (need > tmp_bytes) { SAH_TRY(tmp.grow(need)); tmp_bytes = need; }
        SAH_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, need, cnt.p, off.p, nq + 1, st));
        hipLaunchKernelGGL(k_c4_emit, dim3((nq + 255) / 256), dim3(256), 0, st, Q.p, nq, nodes.p, off.p, base, base + nq,
                           tri_base, pad, n4.p, Qn.p);
        SAH_TRY(hipGetLastError());
        int next = 0;
        SAH_TRY(hipMemcpyAsync(&next, off.p + nq, sizeof(int), hipMemcpyDeviceToHost, st));
        SAH_TRY(hipStreamSynchronize(st));
        base += nq;
        if ((size_t)base + next > cap4) { err = "GPU SAH collapse: node overflow"; return -1; }
        std::swap(Q.p, Qn.p);
        std::swap(Q.cap, Qn.cap);
        nq = next;
    }
    Node4* dst = alloc4((size_t)base);
    SAH_TRY(hipMemcpyAsync(dst, n4.p, sizeof(Node4) * (size_t)base, hipMemcpyDeviceToHost, st));
    SAH_TRY(hipStreamSynchronize(st));
    lap("collapse+d2h");
    return 0;
}

}  // namespace rtg
