// rtg_host.cpp — C ABI of librtg: scene flattening for gfx950 and the wavefront driver.
//
// rtg_scene_create() performs what Scene::renderScene() does before its pixel loop
// (src/Scene.cpp:296-323): transformation matrices with glm's arithmetic
// (src/Helper.cpp:135-226), smooth vertex normals (src/Shape.cpp:262-290) and one
// median-split BVH per object (src/BVH.cpp:53-135) — reproduced bit-for-bit, then
// linearised into 64-byte child-box nodes and pre-gathered triangles in BVH order.
// rtg_render() drives the per-level kernels of rtg_device.hip.
#include <float.h>
#include <math.h>
#include <cmath>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>
#include <string>
#include <deque>
#include <exception>
#include <thread>
#include <type_traits>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/rtg.h"
#include "rtg_internal.h"

using namespace rtg;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(RTG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------ host vector / glm math
struct V3 { float x, y, z; };
inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline V3 operator/(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
inline float sqn(V3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }   // Eigen redux order
inline float vnorm(V3 a) { return sqrtf(sqn(a)); }
inline V3 normalized(V3 a) {
    float z = sqn(a);
    return z > 0.0f ? a / sqrtf(z) : a;
}
inline V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

struct Mat4 { float c[4][4]; };   // glm column-major
inline V3 xform_point(const Mat4& m, V3 v, float w) {   // glm mat4 * vec4: (c0x + c1y) + (c2z + c3w)
    float r[3];
    for (int i = 0; i < 3; i++) r[i] = (m.c[0][i] * v.x + m.c[1][i] * v.y) + (m.c[2][i] * v.z + m.c[3][i] * w);
    return v3(r[0], r[1], r[2]);
}
Mat4 identity() {
    Mat4 m;
    memset(&m, 0, sizeof m);
    m.c[0][0] = m.c[1][1] = m.c[2][2] = m.c[3][3] = 1.0f;
    return m;
}
Mat4 mul(const Mat4& A, const Mat4& B) {             // glm mat4*mat4, columns summed left to right
    Mat4 R;
    for (int i = 0; i < 4; i++)
        for (int r = 0; r < 4; r++)
            R.c[i][r] = ((A.c[0][r] * B.c[i][0] + A.c[1][r] * B.c[i][1]) + A.c[2][r] * B.c[i][2]) + A.c[3][r] * B.c[i][3];
    return R;
}
Mat4 translate(const Mat4& m, V3 v) {                // glm::translate
    Mat4 R = m;
    for (int r = 0; r < 4; r++) R.c[3][r] = ((m.c[0][r] * v.x + m.c[1][r] * v.y) + m.c[2][r] * v.z) + m.c[3][r];
    return R;
}
Mat4 scale(const Mat4& m, V3 v) {                    // glm::scale
    Mat4 R = m;
    for (int r = 0; r < 4; r++) {
        R.c[0][r] = m.c[0][r] * v.x;
        R.c[1][r] = m.c[1][r] * v.y;
        R.c[2][r] = m.c[2][r] * v.z;
    }
    return R;
}
Mat4 rotate(const Mat4& m, float angle, V3 v) {      // glm::rotate
    float c = (float)cos((double)angle), s = (float)sin((double)angle);
    float inv = 1.0f / sqrtf((v.x * v.x + v.y * v.y) + v.z * v.z);
    V3 ax = v3(v.x * inv, v.y * inv, v.z * inv);
    float omc = 1.0f - c;
    V3 tp = v3(omc * ax.x, omc * ax.y, omc * ax.z);
    float r00 = c + tp.x * ax.x, r01 = tp.x * ax.y + s * ax.z, r02 = tp.x * ax.z - s * ax.y;
    float r10 = tp.y * ax.x - s * ax.z, r11 = c + tp.y * ax.y, r12 = tp.y * ax.z + s * ax.x;
    float r20 = tp.z * ax.x + s * ax.y, r21 = tp.z * ax.y - s * ax.x, r22 = c + tp.z * ax.z;
    Mat4 R;
    for (int r = 0; r < 4; r++) {
        R.c[0][r] = (m.c[0][r] * r00 + m.c[1][r] * r01) + m.c[2][r] * r02;
        R.c[1][r] = (m.c[0][r] * r10 + m.c[1][r] * r11) + m.c[2][r] * r12;
        R.c[2][r] = (m.c[0][r] * r20 + m.c[1][r] * r21) + m.c[2][r] * r22;
        R.c[3][r] = m.c[3][r];
    }
    return R;
}
Mat4 inverse(const Mat4& M) {                        // glm compute_inverse<4,4>
    const float(*m)[4] = M.c;
    float C00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], C02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float C03 = m[1][2] * m[2][3] - m[2][2] * m[1][3], C04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float C06 = m[1][1] * m[3][3] - m[3][1] * m[1][3], C07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float C08 = m[2][1] * m[3][2] - m[3][1] * m[2][2], C10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float C11 = m[1][1] * m[2][2] - m[2][1] * m[1][2], C12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float C14 = m[1][0] * m[3][3] - m[3][0] * m[1][3], C15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float C16 = m[2][0] * m[3][2] - m[3][0] * m[2][2], C18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float C19 = m[1][0] * m[2][2] - m[2][0] * m[1][2], C20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float C22 = m[1][0] * m[3][1] - m[3][0] * m[1][1], C23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    const float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
    const float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
    const float V0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]}, V1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    const float V2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]}, V3a[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    Mat4 I;
    for (int i = 0; i < 4; i++) {
        I.c[0][i] = ((V1[i] * F0[i] - V2[i] * F1[i]) + V3a[i] * F2[i]) * SA[i];
        I.c[1][i] = ((V0[i] * F0[i] - V2[i] * F3[i]) + V3a[i] * F4[i]) * SB[i];
        I.c[2][i] = ((V0[i] * F1[i] - V1[i] * F3[i]) + V3a[i] * F5[i]) * SA[i];
        I.c[3][i] = ((V0[i] * F2[i] - V1[i] * F4[i]) + V2[i] * F5[i]) * SB[i];
    }
    float d0 = m[0][0] * I.c[0][0], d1 = m[0][1] * I.c[1][0], d2 = m[0][2] * I.c[2][0], d3 = m[0][3] * I.c[3][0];
    float ood = 1.0f / ((d0 + d1) + (d2 + d3));
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) I.c[c][r] = I.c[c][r] * ood;
    return I;
}
Mat4 inverse_transpose(const Mat4& M) {              // glm::inverseTranspose (gtc/matrix_inverse)
    const float(*m)[4] = M.c;
    float S00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], S01 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float S02 = m[2][1] * m[3][2] - m[3][1] * m[2][2], S03 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float S04 = m[2][0] * m[3][2] - m[3][0] * m[2][2], S05 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float S06 = m[1][2] * m[3][3] - m[3][2] * m[1][3], S07 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S08 = m[1][1] * m[3][2] - m[3][1] * m[1][2], S09 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float S10 = m[1][0] * m[3][2] - m[3][0] * m[1][2], S11 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S12 = m[1][0] * m[3][1] - m[3][0] * m[1][1], S13 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float S14 = m[1][1] * m[2][3] - m[2][1] * m[1][3], S15 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float S16 = m[1][0] * m[2][3] - m[2][0] * m[1][3], S17 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float S18 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    Mat4 I;
    I.c[0][0] = +((m[1][1] * S00 - m[1][2] * S01) + m[1][3] * S02);
    I.c[0][1] = -((m[1][0] * S00 - m[1][2] * S03) + m[1][3] * S04);
    I.c[0][2] = +((m[1][0] * S01 - m[1][1] * S03) + m[1][3] * S05);
    I.c[0][3] = -((m[1][0] * S02 - m[1][1] * S04) + m[1][2] * S05);
    I.c[1][0] = -((m[0][1] * S00 - m[0][2] * S01) + m[0][3] * S02);
    I.c[1][1] = +((m[0][0] * S00 - m[0][2] * S03) + m[0][3] * S04);
    I.c[1][2] = -((m[0][0] * S01 - m[0][1] * S03) + m[0][3] * S05);
    I.c[1][3] = +((m[0][0] * S02 - m[0][1] * S04) + m[0][2] * S05);
    I.c[2][0] = +((m[0][1] * S06 - m[0][2] * S07) + m[0][3] * S08);
    I.c[2][1] = -((m[0][0] * S06 - m[0][2] * S09) + m[0][3] * S10);
    I.c[2][2] = +((m[0][0] * S11 - m[0][1] * S09) + m[0][3] * S12);
    I.c[2][3] = -((m[0][0] * S08 - m[0][1] * S10) + m[0][2] * S12);
    I.c[3][0] = -((m[0][1] * S13 - m[0][2] * S14) + m[0][3] * S15);
    I.c[3][1] = +((m[0][0] * S13 - m[0][2] * S16) + m[0][3] * S17);
    I.c[3][2] = -((m[0][0] * S14 - m[0][1] * S16) + m[0][3] * S18);
    I.c[3][3] = +((m[0][0] * S15 - m[0][1] * S17) + m[0][2] * S18);
    float det = ((m[0][0] * I.c[0][0] + m[0][1] * I.c[0][1]) + m[0][2] * I.c[0][2]) + m[0][3] * I.c[0][3];
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) I.c[c][r] = I.c[c][r] / det;
    return I;
}
// ComputeObjectTransformations composition (src/Helper.cpp:135-176): reverse list order,
// a Composite replaces the accumulated model.
Mat4 compose(const rtg_scene_desc* d, int first, int count) {
    Mat4 M = identity();
    for (int j = count - 1; j >= 0; j--) {
        const rtg_xform_ref& x = d->xform_refs[first + j];
        int k = x.index - 1;
        switch (x.type) {
        case RTG_XF_TRANSLATION:
            M = translate(M, v3(d->translations[3 * k], d->translations[3 * k + 1], d->translations[3 * k + 2]));
            break;
        case RTG_XF_SCALING:
            M = scale(M, v3(d->scalings[3 * k], d->scalings[3 * k + 1], d->scalings[3 * k + 2]));
            break;
        case RTG_XF_ROTATION: {
            const float* rr = d->rotations + 4 * k;
            M = rotate(M, rr[0] * (float)0.01745329251994329576923690768489, v3(rr[1], rr[2], rr[3]));
            break;
        }
        case RTG_XF_COMPOSITE:
            memcpy(M.c, d->composites + 16 * k, sizeof(float) * 16);
            break;
        default:
            break;
        }
    }
    return M;
}

// ------------------------------------------------------------------ BVH construction
inline float min2(float a, float b) { return a <= b ? a : b; }
inline float max2(float a, float b) { return a >= b ? a : b; }
inline float minOf3(float a, float b, float c) {
    if (a <= b && a <= c) return a;
    else if (b <= a && b <= c) return b;
    return c;
}
inline float maxOf3(float a, float b, float c) {
    if (a >= b && a >= c) return a;
    else if (b >= a && b >= c) return b;
    return c;
}

// Allocator whose value-less construct() leaves the element uninitialised: the scene build's large
// record arrays are written in full by parallel loops, so resize() need not zero hundreds of MB on
// one thread first (the pages are touched first by the threads that fill them).
template <class T>
struct NoInit : std::allocator<T> {
    template <class U> struct rebind { using other = NoInit<U>; };
    NoInit() = default;
    template <class U> NoInit(const NoInit<U>&) noexcept {}
    template <class U, class... A>
    void construct(U* q, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new ((void*)q) U;
        else ::new ((void*)q) U(std::forward<A>(a)...);
    }
};
template <class T> using hvec = std::vector<T, NoInit<T>>;

// Host worker threads of the scene build: up to 16 (the GPU box's CPU share per GPU), chunks of
// at least `grain` items.  f(chunk, begin, end) runs once per chunk; chunks are numbered in order,
// so per-chunk partial results combine deterministically.  Exceptions reach the caller.
inline int build_threads() {
    static const int n = [] {
        const int t = (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(16, t));
    }();
    return n;
}
template <class F>
int parallel_chunks(size_t n, size_t grain, F&& f) {
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)build_threads(), (n + grain - 1) / std::max<size_t>(grain, 1)));
    if (T <= 1) { if (n) f(0, (size_t)0, n); return 1; }
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(T);
    for (int c = 1; c < T; c++)
        th.emplace_back([&, c] {
            try { f(c, n * c / T, n * (c + 1) / T); } catch (...) { err[c] = std::current_exception(); }
        });
    try { f(0, (size_t)0, n / T); } catch (...) { err[0] = std::current_exception(); }
    for (std::thread& t : th) t.join();
    for (auto& e : err) if (e) std::rethrow_exception(e);
    return T;
}

struct HNode {            // pre-order node of the reference tree
    int left, right;      // node numbers, -1 null
    int start, end;
    float mn[3], mx[3];
};

struct ObjBVH {
    hvec<int> perm;               // BVH position -> original prim index
    hvec<HNode> nodes;            // pre-order (host build) or breadth-first (GPU build, bfs)
    int root = -1;
    bool bfs = false;             // nodes in the GPU build's breadth-first order (root 0, children after
                                  // their parent); rtg_scene_object_bvh reports the pre-order
};

struct BuildCtx {
    const V3* centers;            // per original prim
    const V3* bmin;               // per original prim
    const V3* bmax;
    hvec<int>* prims;             // current permutation
    hvec<HNode>* nodes;
    std::vector<float> scratch;
    bool finite = true;           // every primitive box coordinate is finite (construct_par's chunked boxes)
};

void range_box(BuildCtx& B, int start, int end, float mn[3], float mx[3]) {   // ComputeBoundingBox BVH.cpp:268-283
    float a0 = FLT_MAX, a1 = FLT_MAX, a2 = FLT_MAX, b0 = -FLT_MAX, b1 = -FLT_MAX, b2 = -FLT_MAX;
    const int* p = B.prims->data();
    for (int i = start; i < end; i++) {
        const V3 lo = B.bmin[p[i]], hi = B.bmax[p[i]];
        a0 = min2(a0, lo.x); a1 = min2(a1, lo.y); a2 = min2(a2, lo.z);
        b0 = max2(b0, hi.x); b1 = max2(b1, hi.y); b2 = max2(b2, hi.z);
    }
    mn[0] = a0; mn[1] = a1; mn[2] = a2; mx[0] = b0; mx[1] = b1; mx[2] = b2;
}

// BVH::ConstructionHelper (src/BVH.cpp:64-110).  FindMedian's sort (BVH.cpp:117-135) is replaced by
// nth_element selection, which yields the same order statistics.
int construct(BuildCtx& B, int start, int end, int splitType, int depth) {
    if (start == end - 1 || depth >= 30) {
        int n = (int)B.nodes->size();
        HNode h;
        h.left = h.right = -1; h.start = start; h.end = end;
        range_box(B, start, end, h.mn, h.mx);
        B.nodes->push_back(h);
        return n;
    }
    if (start == end) return -1;
    if (splitType > 2) splitType = 0;
    int n = (int)B.nodes->size();
    {
        HNode h;
        h.left = h.right = -1; h.start = start; h.end = end;
        range_box(B, start, end, h.mn, h.mx);
        B.nodes->push_back(h);
    }
    int* p = B.prims->data();
    int len = end - start;
    B.scratch.resize(len);
    for (int i = 0; i < len; i++) B.scratch[i] = comp(B.centers[p[start + i]], splitType);
    int mi = len / 2;
    std::nth_element(B.scratch.begin(), B.scratch.begin() + mi, B.scratch.end());
    float split = B.scratch[mi];
    if (len % 2 == 0) {
        float lower = *std::max_element(B.scratch.begin(), B.scratch.begin() + mi);
        split = (lower + split) * 0.5f;
    }
    int swapIndex = start;
    for (int i = start; i < end; i++) {
        if (comp(B.centers[p[i]], splitType) < split) {
            std::swap(p[swapIndex], p[i]);
            swapIndex++;
        }
    }
    int l = construct(B, start, swapIndex, splitType + 1, depth + 1);
    int r = construct(B, swapIndex, end, splitType + 1, depth + 1);
    (*B.nodes)[n].left = l;
    (*B.nodes)[n].right = r;
    return n;
}

// construct() with the subtrees of the top `pdepth` levels (>= 64K primitives) built on their own
// threads, each into its own pre-order node array (its own BuildCtx), appended left then right with
// their child numbers shifted: the same permutation and the same pre-order nodes as the recursion
// (the two halves partition disjoint ranges of the permutation).  The top node's box is reduced in
// parallel when every coordinate is finite (min / max of finite floats are exact in any order, and
// min2 / max2 keep the first of equal values in both forms); otherwise sequentially, since the
// reference's fold (ComputeBoundingBox, BVH.cpp:268-283, `a <= b ? a : b`) drops everything before the
// last NaN, which a merge of per-chunk results does not reproduce.  The median selection and the
// reference's swap partition stay sequential -- they define the permutation.
int construct_par(BuildCtx& B, int start, int end, int splitType, int depth, int pdepth) {
    if (pdepth <= 0 || end - start < (1 << 16) || start == end - 1 || depth >= 30) return construct(B, start, end, splitType, depth);
    if (splitType > 2) splitType = 0;
    const int n = (int)B.nodes->size();
    {
        HNode h;
        h.left = h.right = -1; h.start = start; h.end = end;
        const int len = end - start;
        if (!B.finite) {
            range_box(B, start, end, h.mn, h.mx);
        } else {
            std::vector<std::array<float, 6>> part(build_threads());
            const int T = parallel_chunks((size_t)len, 1 << 15, [&](int ch, size_t k0, size_t k1) {
                float mn[3], mx[3];
                range_box(B, start + (int)k0, start + (int)k1, mn, mx);
                part[ch] = {mn[0], mn[1], mn[2], mx[0], mx[1], mx[2]};
            });
            for (int z = 0; z < 3; z++) { h.mn[z] = part[0][z]; h.mx[z] = part[0][3 + z]; }
            for (int c = 1; c < T; c++)
                for (int z = 0; z < 3; z++) { h.mn[z] = min2(h.mn[z], part[c][z]); h.mx[z] = max2(h.mx[z], part[c][3 + z]); }
        }
        B.nodes->push_back(h);
    }
    int* p = B.prims->data();
    const int len = end - start;
    B.scratch.resize(len);
    parallel_chunks((size_t)len, 1 << 15, [&](int, size_t k0, size_t k1) {
        for (size_t i = k0; i < k1; i++) B.scratch[i] = comp(B.centers[p[start + i]], splitType);
    });
    const int mi = len / 2;
    std::nth_element(B.scratch.begin(), B.scratch.begin() + mi, B.scratch.end());
    float split = B.scratch[mi];
    if (len % 2 == 0) {
        const float lower = *std::max_element(B.scratch.begin(), B.scratch.begin() + mi);
        split = (lower + split) * 0.5f;
    }
    int swapIndex = start;
    for (int i = start; i < end; i++) {
        if (comp(B.centers[p[i]], splitType) < split) {
            std::swap(p[swapIndex], p[i]);
            swapIndex++;
        }
    }
    hvec<HNode> L, R;
    BuildCtx BL{B.centers, B.bmin, B.bmax, B.prims, &L, {}, B.finite}, BR{B.centers, B.bmin, B.bmax, B.prims, &R, {}, B.finite};
    int l = -1, r = -1;
    std::exception_ptr err;
    std::thread t([&] {
        try { l = construct_par(BL, start, swapIndex, splitType + 1, depth + 1, pdepth - 1); } catch (...) { err = std::current_exception(); }
    });
    try {
        r = construct_par(BR, swapIndex, end, splitType + 1, depth + 1, pdepth - 1);
    } catch (...) {
        t.join();
        throw;
    }
    t.join();
    if (err) std::rethrow_exception(err);
    auto append = [&](const hvec<HNode>& sub, int root) {
        if (root < 0) return -1;
        const int off = (int)B.nodes->size();
        for (HNode x : sub) {
            if (x.left >= 0) x.left += off;
            if (x.right >= 0) x.right += off;
            B.nodes->push_back(x);
        }
        return off + root;
    };
    const int lo = append(L, l);
    const int ro = append(R, r);
    (*B.nodes)[n].left = lo;
    (*B.nodes)[n].right = ro;
    return n;
}

// ------------------------------------------------------------------ traversal tree (SAH, 4-wide)
// The reference's median-split tree (one primitive per leaf, axis = depth % 3) decides *which*
// candidates exist -- a primitive counts only if every interior box above its leaf is hit
// (src/BVH.cpp:137-210) -- but not how fast they are found.  Fast rays walk a second tree per
// mesh: binned SAH over the triangle boxes, leaves of <= 4 triangles, collapsed to 4-wide nodes.
// Its boxes only prune (padded by the eps overhang, like the reference tree's); reachability in
// the reference tree is checked per winning candidate against its reference leaf's parent box
// (the exact slab predicate is monotone under box containment for nonzero finite directions,
// so that one box decides the whole ancestor chain), and ties keep the reference's order
// (distance, rightmost reference leaf, lowest position).
struct SahBox { float lo[3], hi[3]; };
// (SahNode2, SahRec, kSahBins, kSahMaxLeaf: rtg_internal.h, shared with the GPU build)
constexpr int kWinMinPrims = 1;    // Geometry::win threshold (64: dragon 34.7 -> 35.2 ms, r3_ab_window.jsonl)
constexpr int kSahGpuMin = 1 << 16;  // RTG_BVH_AUTO: traversal trees of meshes from this size on the GPU
constexpr int kFlatMaxPrims = 8;   // Geometry::flat_count: meshes tested without a node (incl. a reference
                                   // root over two leaves)

inline double sah_area(const float lo[3], const float hi[3]) {
    const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

// One triangle of the binned-SAH build (SahRec): its box and face index, partitioned in place (32 B,
// so the passes over a range stream through memory instead of gathering through an index array).
// The centroid is the box centre.
inline float sah_ctr(const SahRec& r, int z) { return 0.5f * (r.lo[z] + r.hi[z]); }

// Node box and split of the SAH-ordered range [s, e) (partitions r[s, e)); returns the split
// position, or -1 for a leaf.  Ranges of >= kSahParMin triangles run their passes on the build's
// worker threads (per-chunk bounds and bins combined in chunk order; a stable partition through
// `tmp`), smaller ones on the calling thread (std::partition).
constexpr int kSahParMin = 1 << 18;
// Box and centroid bounds of a range of records (min / max: exact in any order).
struct SahBounds {
    float lo[3], hi[3], clo[3], chi[3];
    void clear() { for (int z = 0; z < 3; z++) { lo[z] = clo[z] = FLT_MAX; hi[z] = chi[z] = -FLT_MAX; } }
    void add(const SahRec& q) {
        for (int z = 0; z < 3; z++) {
            const float c = sah_ctr(q, z);
            lo[z] = std::min(lo[z], q.lo[z]);
            hi[z] = std::max(hi[z], q.hi[z]);
            clo[z] = std::min(clo[z], c);
            chi[z] = std::max(chi[z], c);
        }
    }
    void add(const SahBounds& b) {
        for (int z = 0; z < 3; z++) {
            lo[z] = std::min(lo[z], b.lo[z]); hi[z] = std::max(hi[z], b.hi[z]);
            clo[z] = std::min(clo[z], b.clo[z]); chi[z] = std::max(chi[z], b.chi[z]);
        }
    }
};
// `pre`: the range's bounds when the parent's partition formed them (nullptr: computed here, one
// more pass over the range); `outl` / `outr` receive the two halves' bounds, formed while
// partitioning (*kids_ok = false when the split fell back to halving by count).
int sah_split(SahRec* r, SahRec* tmp, int s, int e, SahNode2& nd, const SahBounds* pre = nullptr,
              SahBounds* outl = nullptr, SahBounds* outr = nullptr, bool* kids_ok = nullptr) {
    const int n = e - s;
    const bool par = n >= kSahParMin;
    if (kids_ok) *kids_ok = false;
    using Bounds = SahBounds;
    auto bounds_of = [&](size_t k0, size_t k1) {
        Bounds B;
        B.clear();
        for (size_t k = k0; k < k1; k++) B.add(r[k]);
        return B;
    };
    Bounds B;
    if (pre) {
        B = *pre;
    } else if (par) {
        std::vector<Bounds> part(build_threads());
        const int T = parallel_chunks((size_t)n, 1 << 15, [&](int ch, size_t k0, size_t k1) { part[ch] = bounds_of(s + k0, s + k1); });
        B = part[0];
        for (int c = 1; c < T; c++)
            for (int z = 0; z < 3; z++) {
                B.lo[z] = std::min(B.lo[z], part[c].lo[z]); B.hi[z] = std::max(B.hi[z], part[c].hi[z]);
                B.clo[z] = std::min(B.clo[z], part[c].clo[z]); B.chi[z] = std::max(B.chi[z], part[c].chi[z]);
            }
    } else {
        B = bounds_of(s, e);
    }
    for (int z = 0; z < 3; z++) { nd.lo[z] = B.lo[z]; nd.hi[z] = B.hi[z]; }
    nd.left = nd.right = -1;
    nd.start = s;
    nd.count = n;
    if (n <= 1) return -1;
    int axis = 0;
    for (int z = 1; z < 3; z++)
        if (B.chi[z] - B.clo[z] > B.chi[axis] - B.clo[axis]) axis = z;
    const float ext = B.chi[axis] - B.clo[axis];
    int mid = -1;
    if (ext > 0.0f) {
        const float sc = (float)kSahBins / ext;
        const float c0 = B.clo[axis];
        auto bin_of = [&](const SahRec& q) {
            return std::min(kSahBins - 1, std::max(0, (int)((sah_ctr(q, axis) - c0) * sc)));
        };
        struct Bins { int cnt[kSahBins]; float lo[kSahBins][3], hi[kSahBins][3]; };
        auto bins_of = [&](size_t k0, size_t k1, Bins& Q) {
            for (int b = 0; b < kSahBins; b++) {
                Q.cnt[b] = 0;
                for (int z = 0; z < 3; z++) { Q.lo[b][z] = FLT_MAX; Q.hi[b][z] = -FLT_MAX; }
            }
            for (size_t k = k0; k < k1; k++) {
                const int b = bin_of(r[k]);
                Q.cnt[b]++;
                for (int z = 0; z < 3; z++) {
                    Q.lo[b][z] = std::min(Q.lo[b][z], r[k].lo[z]);
                    Q.hi[b][z] = std::max(Q.hi[b][z], r[k].hi[z]);
                }
            }
        };
        Bins Q;
        if (par) {
            std::vector<Bins> part(build_threads());
            const int T = parallel_chunks((size_t)n, 1 << 15, [&](int ch, size_t k0, size_t k1) { bins_of(s + k0, s + k1, part[ch]); });
            Q = part[0];
            for (int c = 1; c < T; c++)
                for (int b = 0; b < kSahBins; b++) {
                    Q.cnt[b] += part[c].cnt[b];
                    for (int z = 0; z < 3; z++) {
                        Q.lo[b][z] = std::min(Q.lo[b][z], part[c].lo[b][z]);
                        Q.hi[b][z] = std::max(Q.hi[b][z], part[c].hi[b][z]);
                    }
                }
        } else {
            bins_of(s, e, Q);
        }
        double rcost[kSahBins];
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        int rc = 0;
        for (int b = kSahBins - 1; b >= 1; b--) {
            rc += Q.cnt[b];
            for (int z = 0; z < 3; z++) { lo[z] = std::min(lo[z], Q.lo[b][z]); hi[z] = std::max(hi[z], Q.hi[b][z]); }
            rcost[b] = rc ? sah_area(lo, hi) * rc : 0.0;
        }
        for (int z = 0; z < 3; z++) { lo[z] = FLT_MAX; hi[z] = -FLT_MAX; }
        int lc = 0, best_b = -1;
        double best = 1e300;
        for (int b = 0; b < kSahBins - 1; b++) {
            lc += Q.cnt[b];
            for (int z = 0; z < 3; z++) { lo[z] = std::min(lo[z], Q.lo[b][z]); hi[z] = std::max(hi[z], Q.hi[b][z]); }
            if (lc == 0 || lc == n) continue;
            const double cost = sah_area(lo, hi) * lc + rcost[b + 1];
            if (cost < best) { best = cost; best_b = b; }
        }
        // leaf when splitting does not pay (traversal step ~ one triangle test)
        const double leaf_cost = sah_area(nd.lo, nd.hi) * n;
        if (n <= kSahMaxLeaf && (best_b < 0 || leaf_cost <= sah_area(nd.lo, nd.hi) + best)) return -1;
        if (best_b >= 0) {
            auto left = [&](const SahRec& q) { return bin_of(q) <= best_b; };
            Bounds BL, BR;
            BL.clear(); BR.clear();
            if (par) {
                // stable: per-chunk left counts, then every chunk scatters its records to their
                // places in tmp (forming each side's bounds), then back
                std::vector<Bounds> pl(build_threads() + 1), pr(build_threads() + 1);
                std::vector<int> nl(build_threads() + 1, 0), nr(build_threads() + 1, 0);
                const int T = parallel_chunks((size_t)n, 1 << 15, [&](int ch, size_t k0, size_t k1) {
                    int c = 0;
                    for (size_t k = k0; k < k1; k++) c += left(r[s + k]);
                    nl[ch] = c;
                    nr[ch] = (int)(k1 - k0) - c;
                });
                std::vector<int> lo_at(T), hi_at(T);
                int acc = 0;
                for (int c = 0; c < T; c++) { lo_at[c] = acc; acc += nl[c]; }
                mid = s + acc;
                for (int c = 0; c < T; c++) { hi_at[c] = acc; acc += nr[c]; }
                parallel_chunks((size_t)n, 1 << 15, [&](int ch, size_t k0, size_t k1) {
                    int a = lo_at[ch], b2 = hi_at[ch];
                    Bounds L, R;
                    L.clear(); R.clear();
                    for (size_t k = k0; k < k1; k++) {
                        const SahRec& q = r[s + k];
                        if (left(q)) { tmp[s + a++] = q; L.add(q); } else { tmp[s + b2++] = q; R.add(q); }
                    }
                    pl[ch] = L; pr[ch] = R;
                });
                for (int c = 0; c < T; c++) { BL.add(pl[c]); BR.add(pr[c]); }
                parallel_chunks((size_t)n, 1 << 16, [&](int, size_t k0, size_t k1) {
                    std::copy(tmp + s + k0, tmp + s + k1, r + s + k0);
                });
            } else {
                // std::partition's bidirectional scheme (same resulting order), each record added
                // to its side's bounds once
                SahRec* f = r + s;
                SahRec* l = r + e;
                for (;;) {
                    for (;;) {
                        if (f == l) goto parted;
                        if (!left(*f)) break;
                        BL.add(*f);
                        ++f;
                    }
                    --l;
                    for (;;) {
                        if (f == l) { BR.add(*f); goto parted; }   // *f: the right record the scan above stopped at
                        if (left(*l)) break;
                        BR.add(*l);
                        --l;
                    }
                    std::iter_swap(f, l);
                    BL.add(*f);
                    BR.add(*l);
                    ++f;
                }
            parted:
                mid = (int)(f - r);
            }
            if (outl && outr && mid > s && mid < e) {
                *outl = BL;
                *outr = BR;
                if (kids_ok) *kids_ok = true;
            }
        }
    } else if (n <= kSahMaxLeaf) {
        return -1;
    }
    if (mid <= s || mid >= e) mid = s + n / 2;    // no useful split: halve by count
    return mid;
}

// Pass-schedule levels whose shadow queries all walk wave-uniformly (level 0: camera samples; levels
// 0-1 / 0-2 measured slower on the dragon, k_shadow 10.6 -> 11.3 / 12.4 ms: profiles/history/r5s_*)
constexpr int kUniShadowLevels = 1;

// Levels of the SAH recursion whose subtrees get threads of their own (4 / 5 / 6: second creation
// 136-147 / 121-153 / 120-128 ms on one box).
static int sah_depth() { return 6; }

// Binned SAH BVH2 over [s, e), nodes appended depth first (node, left subtree, right subtree).
int sah_rec(SahRec* r, SahRec* tmp, int s, int e, std::vector<SahNode2>& out, const SahBounds* pre = nullptr) {
    SahNode2 nd;
    SahBounds bl, br;
    bool kids = false;
    const int mid = sah_split(r, tmp, s, e, nd, pre, &bl, &br, &kids);
    const int me = (int)out.size();
    out.push_back(nd);
    if (mid < 0) return me;
    const int l = sah_rec(r, tmp, s, mid, out, kids ? &bl : nullptr);
    const int rr = sah_rec(r, tmp, mid, e, out, kids ? &br : nullptr);
    out[me].left = l;
    out[me].right = rr;
    return me;
}

// Same tree, the subtrees of the top `depth` levels (>= 64K triangles) built on their own threads
// into their own node arrays and appended in sah_rec's depth-first order: the result is identical
// to sah_rec's, node numbering included (1 M-triangle dragon on the GPU box's host: 247 -> 78 ms).
// The two halves partition disjoint ranges of r (and of tmp).
int sah_rec_par(SahRec* r, SahRec* tmp, int s, int e, std::vector<SahNode2>& out, int depth,
                const SahBounds* pre = nullptr) {
    if (depth <= 0 || e - s < (1 << 16)) return sah_rec(r, tmp, s, e, out, pre);
    SahNode2 nd;
    SahBounds bl, br;
    bool kids = false;
    const int mid = sah_split(r, tmp, s, e, nd, pre, &bl, &br, &kids);
    const int me = (int)out.size();
    out.push_back(nd);
    if (mid < 0) return me;
    std::vector<SahNode2> L, R;
    std::exception_ptr err;
    std::thread t([&] {
        try {
            sah_rec_par(r, tmp, s, mid, L, depth - 1, kids ? &bl : nullptr);
        } catch (...) {
            err = std::current_exception();
        }
    });
    try {
        sah_rec_par(r, tmp, mid, e, R, depth - 1, kids ? &br : nullptr);
    } catch (...) {
        t.join();
        throw;
    }
    t.join();
    if (err) std::rethrow_exception(err);
    auto append = [&](const std::vector<SahNode2>& sub) {
        const int off = (int)out.size();
        for (SahNode2 x : sub) {
            if (x.left >= 0) { x.left += off; x.right += off; }
            out.push_back(x);
        }
        return off;                      // the subtree's root (its index 0)
    };
    out[me].left = append(L);
    out[me].right = append(R);
    return me;
}

// Node count and an order-independent hash of a BVH2 (reachable nodes from `root`: the GPU build's
// array may hold unused reserved slots): the sum over nodes of a mix of the box (-0 as +0) and the
// triangle count, so two builds that chose the same splits hash alike whatever their node order.
inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
void sah_tree_stats(const SahNode2* bn, int root, uint64_t& count, uint64_t& hash) {
    count = 0; hash = 0;
    std::vector<int> stack{root};
    while (!stack.empty()) {
        const SahNode2& nd = bn[stack.back()];
        stack.pop_back();
        uint64_t h = (uint64_t)(uint32_t)nd.count * 0x9E3779B97F4A7C15ULL;
        for (int z = 0; z < 3; z++) {
            const float a = nd.lo[z] + 0.0f, b = nd.hi[z] + 0.0f;
            uint32_t ua, ub;
            memcpy(&ua, &a, 4); memcpy(&ub, &b, 4);
            h = mix64(h ^ ((uint64_t)ua << 32 | ub) ^ (uint64_t)(z + 1));
        }
        hash += h;
        count++;
        if (nd.left >= 0) { stack.push_back(nd.left); stack.push_back(nd.right); }
    }
}

// Renumber a 4-wide tree (root 0, interior refs 0-based) into depth-first pre-order, children in slot
// order -- the order sah_collapse produces.  The GPU build emits its nodes breadth first; walks then
// touch more distinct cache lines near the leaves (r6_ab_ident0_ksmall.jsonl: a layout with more
// breadth-first levels cost dragon 30.36 -> 30.74-30.86 ms, cornell_pt 300.9 -> 303.6-304.2 ms).
template <class V>
void node4_preorder(V& nodes) {
    const size_t m = nodes.size();
    std::vector<int> nid(m, -1), order;
    order.reserve(m);
    std::vector<int> stack{0};
    while (!stack.empty()) {
        const int q = stack.back();
        stack.pop_back();
        nid[q] = (int)order.size();
        order.push_back(q);
        const Node4& nd = nodes[q];
        const int rf[4] = {nd.ref.x, nd.ref.y, nd.ref.z, nd.ref.w}, inf[4] = {nd.info.x, nd.info.y, nd.info.z, nd.info.w};
        for (int j = 3; j >= 0; j--)
            if (inf[j] == 0) stack.push_back(rf[j]);
    }
    V out(order.size());
    parallel_chunks(order.size(), 1 << 14, [&](int, size_t k0, size_t k1) {
        for (size_t k = k0; k < k1; k++) {
            Node4 x = nodes[order[k]];
            if (x.info.x == 0) x.ref.x = nid[x.ref.x];
            if (x.info.y == 0) x.ref.y = nid[x.ref.y];
            if (x.info.z == 0) x.ref.z = nid[x.ref.z];
            if (x.info.w == 0) x.ref.w = nid[x.ref.w];
            out[k] = x;
        }
    });
    nodes.swap(out);
}

// Collapse the SAH BVH2 into 4-wide nodes: each node's slots are its children, the interior
// slot with the largest surface area replaced by its own two children while slots are free.
// Slot info: < 0 empty, 0 interior (ref = Node4 index), > 0 leaf of `info` triangles at ref
// (absolute index into the SAH-ordered triangles).  Slot boxes are widened by `pad` (the eps
// overhang of a candidate beyond its triangle, rounded outwards), so the device walk needs no
// parameter-space padding: a t-space pad of pad/|d_a| on every axis would stop pruning rays
// with one small direction component.
// The slots of the 4-wide node over BVH2 node n (children expanded largest-area first) and their
// widened boxes / leaf refs; interior slots get their ref from the caller.
struct Collapsed {
    int slot[4], used;
    float lo[3][4], hi[3][4];
    int ref[4], info[4];
};
Collapsed collapse_node(const SahNode2* bn, int n, int tri_base, float pad) {
    Collapsed C;
    int* slot = C.slot;
    slot[0] = bn[n].left; slot[1] = bn[n].right; slot[2] = slot[3] = -1;
    int used = 2;
    while (used < 4) {
        int pick = -1;
        double pa = -1.0;
        for (int j = 0; j < used; j++)
            if (bn[slot[j]].left >= 0) {
                const double a = sah_area(bn[slot[j]].lo, bn[slot[j]].hi);
                if (a > pa) { pa = a; pick = j; }
            }
        if (pick < 0) break;
        const int c = slot[pick];
        slot[pick] = bn[c].left;
        slot[used++] = bn[c].right;
    }
    C.used = used;
    auto& lo = C.lo;
    auto& hi = C.hi;
    int* ref = C.ref;
    int* info = C.info;
    for (int j = 0; j < 4; j++) {
        if (j >= used) {
            for (int z = 0; z < 3; z++) { lo[z][j] = 0.0f; hi[z][j] = 0.0f; }
            ref[j] = 0; info[j] = -1;
            continue;
        }
        const SahNode2& c = bn[slot[j]];
        for (int z = 0; z < 3; z++) {
            lo[z][j] = std::nextafter((float)((double)c.lo[z] - pad), -FLT_MAX);
            hi[z][j] = std::nextafter((float)((double)c.hi[z] + pad), FLT_MAX);
        }
        if (c.left < 0) { ref[j] = tri_base + c.start; info[j] = c.count; }
        else { ref[j] = 0; info[j] = 0; }
    }
    return C;
}
Node4 node4_of(const Collapsed& C) {
    const auto& lo = C.lo;
    const auto& hi = C.hi;
    const int* ref = C.ref;
    const int* info = C.info;
    Node4 nd;
    nd.lox = make_float4(lo[0][0], lo[0][1], lo[0][2], lo[0][3]);
    nd.loy = make_float4(lo[1][0], lo[1][1], lo[1][2], lo[1][3]);
    nd.loz = make_float4(lo[2][0], lo[2][1], lo[2][2], lo[2][3]);
    nd.hix = make_float4(hi[0][0], hi[0][1], hi[0][2], hi[0][3]);
    nd.hiy = make_float4(hi[1][0], hi[1][1], hi[1][2], hi[1][3]);
    nd.hiz = make_float4(hi[2][0], hi[2][1], hi[2][2], hi[2][3]);
    nd.ref = make_int4(ref[0], ref[1], ref[2], ref[3]);
    nd.info = make_int4(info[0], info[1], info[2], info[3]);
    return nd;
}
template <class V>
int sah_collapse(const SahNode2* bn, int n, int tri_base, float pad, V& out) {
    const int me = (int)out.size();
    out.emplace_back();
    Collapsed C = collapse_node(bn, n, tri_base, pad);
    for (int j = 0; j < C.used; j++)
        if (bn[C.slot[j]].left >= 0) C.ref[j] = sah_collapse(bn, C.slot[j], tri_base, pad, out);
    out[me] = node4_of(C);
    return me;
}
// Same nodes in the same (depth-first) order, the subtrees of the top `depth` levels (>= 64K
// triangles) collapsed on their own threads into their own arrays and appended with their interior
// refs shifted.
template <class V>
int sah_collapse_par(const SahNode2* bn, int n, int tri_base, float pad, V& out, int depth) {
    if (depth <= 0 || bn[n].count < (1 << 16)) return sah_collapse(bn, n, tri_base, pad, out);
    const int me = (int)out.size();
    out.emplace_back();
    Collapsed C = collapse_node(bn, n, tri_base, pad);
    V sub[4];
    std::thread th[4];
    std::exception_ptr err[4];
    for (int j = 0; j < C.used; j++)
        if (bn[C.slot[j]].left >= 0)
            th[j] = std::thread([&, j] {
                try { sah_collapse_par(bn, C.slot[j], tri_base, pad, sub[j], depth - 1); } catch (...) { err[j] = std::current_exception(); }
            });
    for (int j = 0; j < 4; j++) if (th[j].joinable()) th[j].join();
    for (int j = 0; j < 4; j++) if (err[j]) std::rethrow_exception(err[j]);
    for (int j = 0; j < C.used; j++) {
        if (bn[C.slot[j]].left < 0) continue;
        const int off = (int)out.size();
        for (Node4 x : sub[j]) {
            if (x.info.x == 0) x.ref.x += off;
            if (x.info.y == 0) x.ref.y += off;
            if (x.info.z == 0) x.ref.z += off;
            if (x.info.w == 0) x.ref.w += off;
            out.push_back(x);
        }
        C.ref[j] = off;                  // the subtree's root (its index 0)
    }
    out[me] = node4_of(C);
    return me;
}


// ------------------------------------------------------------------ top-level BVH (TLAS)
// World box of one top-level entry: its geometry's root range box expanded by the eps overhang
// of its candidates (prune_pad: an accepted triangle point may lie outside its triangle), mapped
// through the model matrix (8 corners in double), swept by the motion-blur translation (the ray
// origin moves by -blur * time, time in [0, 1): src/Helper.cpp:110-133), then widened by a
// rounding margin far above the float error of the ray transform.  Non-finite -> false.
struct TBox { double lo[3], hi[3]; };

bool entry_world_box(const Mat4& M, const float mn[3], const float mx[3], float pad, const float blur[3], TBox& out) {
    for (int z = 0; z < 3; z++) { out.lo[z] = 1e300; out.hi[z] = -1e300; }
    double scale = 0.0;
    for (int c = 0; c < 8; c++) {
        const double p[3] = {(c & 1) ? (double)mx[0] + pad : (double)mn[0] - pad, (c & 2) ? (double)mx[1] + pad : (double)mn[1] - pad,
                             (c & 4) ? (double)mx[2] + pad : (double)mn[2] - pad};
        for (int r = 0; r < 3; r++) {
            const double w = (double)M.c[0][r] * p[0] + (double)M.c[1][r] * p[1] + (double)M.c[2][r] * p[2] + (double)M.c[3][r];
            if (!std::isfinite(w)) return false;
            out.lo[r] = std::min(out.lo[r], w);
            out.hi[r] = std::max(out.hi[r], w);
            scale = std::max(scale, std::fabs(w));
        }
    }
    for (int z = 0; z < 3; z++) {
        if (!std::isfinite((double)blur[z])) return false;
        out.lo[z] += std::min(0.0, (double)blur[z]);
        out.hi[z] += std::max(0.0, (double)blur[z]);
        scale = std::max(scale, std::fabs((double)blur[z]));
    }
    double ext = 0.0;
    for (int z = 0; z < 3; z++) ext = std::max(ext, out.hi[z] - out.lo[z]);
    const double margin = 1e-4 * (scale + ext) + 1e-6;
    for (int z = 0; z < 3; z++) { out.lo[z] -= margin; out.hi[z] += margin; }
    return true;
}

struct TlasRef {
    int ref, count;          // count 0: interior node `ref`; > 0: leaf, entries tlas_idx[ref .. ref+count)
    double lo[3], hi[3];
};

double half_area(const double lo[3], const double hi[3]) {
    const double dx = std::max(0.0, hi[0] - lo[0]), dy = std::max(0.0, hi[1] - lo[1]), dz = std::max(0.0, hi[2] - lo[2]);
    return dx * dy + dy * dz + dz * dx;
}

// Top-down SAH over the entries' box centres (sorted along the widest centre axis), BVH2 nodes
// with both child boxes (the `Node` layout of the object trees); a leaf holds one entry, or every
// remaining entry at depth kTlasMaxDepth so the GPU's TLAS stack (kTlasStack entries) never
// overflows.  Child boxes are rounded outward to float.
TlasRef tlas_rec(const std::vector<TBox>& box, std::vector<int>& idx, int s, int e, int depth, std::vector<Node>& nodes,
                 std::vector<int>& leaves) {
    TlasRef R;
    for (int z = 0; z < 3; z++) { R.lo[z] = 1e300; R.hi[z] = -1e300; }
    double clo[3] = {1e300, 1e300, 1e300}, chi[3] = {-1e300, -1e300, -1e300};
    for (int k = s; k < e; k++)
        for (int z = 0; z < 3; z++) {
            const TBox& b = box[idx[k]];
            R.lo[z] = std::min(R.lo[z], b.lo[z]);
            R.hi[z] = std::max(R.hi[z], b.hi[z]);
            const double c = 0.5 * (b.lo[z] + b.hi[z]);
            clo[z] = std::min(clo[z], c);
            chi[z] = std::max(chi[z], c);
        }
    if (e - s == 1 || depth >= kTlasMaxDepth) {
        R.ref = (int)leaves.size();
        R.count = e - s;
        for (int k = s; k < e; k++) leaves.push_back(idx[k]);
        return R;
    }
    int axis = 0;
    for (int z = 1; z < 3; z++)
        if (chi[z] - clo[z] > chi[axis] - clo[axis]) axis = z;
    std::stable_sort(idx.begin() + s, idx.begin() + e, [&](int a, int b) {
        return box[a].lo[axis] + box[a].hi[axis] < box[b].lo[axis] + box[b].hi[axis];
    });
    int split = (s + e) / 2;
    if (chi[axis] > clo[axis]) {       // SAH sweep (equal centres everywhere: split by count)
        const int n = e - s;
        std::vector<double> right(n + 1, 0.0);
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (int k = n - 1; k >= 1; k--) {
            const TBox& b = box[idx[s + k]];
            for (int z = 0; z < 3; z++) { lo[z] = std::min(lo[z], b.lo[z]); hi[z] = std::max(hi[z], b.hi[z]); }
            right[k] = half_area(lo, hi) * (n - k);
        }
        for (int z = 0; z < 3; z++) { lo[z] = 1e300; hi[z] = -1e300; }
        double best = 1e308;
        for (int k = 1; k < n; k++) {
            const TBox& b = box[idx[s + k - 1]];
            for (int z = 0; z < 3; z++) { lo[z] = std::min(lo[z], b.lo[z]); hi[z] = std::max(hi[z], b.hi[z]); }
            const double cost = half_area(lo, hi) * k + right[k];
            if (cost < best) { best = cost; split = s + k; }
        }
    }
    const TlasRef L = tlas_rec(box, idx, s, split, depth + 1, nodes, leaves);
    const TlasRef Rr = tlas_rec(box, idx, split, e, depth + 1, nodes, leaves);
    const int me = (int)nodes.size();
    nodes.emplace_back();
    float b[2][6];
    const TlasRef* ch[2] = {&L, &Rr};
    for (int q = 0; q < 2; q++)
        for (int z = 0; z < 3; z++) {
            b[q][z] = std::nextafter((float)ch[q]->lo[z], -INFINITY);
            b[q][3 + z] = std::nextafter((float)ch[q]->hi[z], INFINITY);
        }
    Node& nd = nodes[me];
    nd.a = make_float4(b[0][0], b[0][1], b[0][2], b[0][3]);
    nd.b = make_float4(b[0][4], b[0][5], b[1][0], b[1][1]);
    nd.c = make_float4(b[1][2], b[1][3], b[1][4], b[1][5]);
    nd.d = make_int4(L.ref, Rr.ref, L.count, Rr.count);
    R.ref = me;
    R.count = 0;
    return R;
}

// Mark every child reference of the subtree under node `n` "no distance pruning".
void tlas_mark_noprune(std::vector<Node>& nodes, int n) {
    Node& nd = nodes[n];
    const int l = nd.d.x, r = nd.d.y, lc = nd.d.z, rc = nd.d.w;
    if (lc == 0) tlas_mark_noprune(nodes, l);
    if (rc == 0) tlas_mark_noprune(nodes, r);
    nd.d.x = l | kTlasNoPrune;
    nd.d.y = r | kTlasNoPrune;
}

// Returns the TLAS root node, or -1 (a single entry: no TLAS).  Entries whose transform is
// axis-aligned (aligned[i]) and the others go to separate subtrees under the root; the others'
// child references carry kTlasNoPrune (their gett() error has no world-space bound, so only
// boxes the ray line misses are skipped there).
int build_tlas(const std::vector<TBox>& box, const std::vector<char>& aligned, std::vector<Node>& nodes,
               std::vector<int>& leaves) {
    const int n = (int)box.size();
    if (n < 2) return -1;
    std::vector<int> A, B;
    for (int i = 0; i < n; i++) (aligned[i] ? A : B).push_back(i);
    nodes.clear();
    leaves.clear();
    auto sub = [&](std::vector<int>& idx, int depth) { return tlas_rec(box, idx, 0, (int)idx.size(), depth, nodes, leaves); };
    if (B.empty() || A.empty()) {
        std::vector<int>& all = B.empty() ? A : B;
        const TlasRef root = sub(all, 0);
        if (root.count != 0) return -1;
        if (A.empty()) tlas_mark_noprune(nodes, root.ref);
        return root.ref;
    }
    const TlasRef ra = sub(A, 1), rb = sub(B, 1);
    if (rb.count == 0) tlas_mark_noprune(nodes, rb.ref);
    const int me = (int)nodes.size();
    nodes.emplace_back();
    float b[2][6];
    const TlasRef* ch[2] = {&ra, &rb};
    for (int q = 0; q < 2; q++)
        for (int z = 0; z < 3; z++) {
            b[q][z] = std::nextafter((float)ch[q]->lo[z], -INFINITY);
            b[q][3 + z] = std::nextafter((float)ch[q]->hi[z], INFINITY);
        }
    Node& nd = nodes[me];
    nd.a = make_float4(b[0][0], b[0][1], b[0][2], b[0][3]);
    nd.b = make_float4(b[0][4], b[0][5], b[1][0], b[1][1]);
    nd.c = make_float4(b[1][2], b[1][3], b[1][4], b[1][5]);
    nd.d = make_int4(ra.ref, rb.ref | kTlasNoPrune, ra.count, rb.count);
    return me;
}

// ------------------------------------------------------------------ device buffer helper
struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    size_t used = 0;         // bytes holding data (upload); replicas copy this many
    int grow(size_t need) {
        if (need <= bytes) return RTG_OK;
        if (p) (void)hipFree(p);
        p = nullptr; bytes = 0;
        size_t want = need + need / 4 + 256;
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            return fail(RTG_ERR_OOM, "hipMalloc failed (" + std::to_string(want) + " bytes)");
        }
        bytes = want;
        return RTG_OK;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
    void release() { if (p) (void)hipFree(p); p = nullptr; bytes = 0; used = 0; }
};


template <class V>
int upload(DBuf& b, const V& v) {
    using T = typename V::value_type;
    size_t n = std::max<size_t>(v.size(), 1) * sizeof(T);
    int rc = b.grow(n);
    if (rc) return rc;
    if (!v.empty()) HIP_TRY(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    b.used = v.size() * sizeof(T);
    return RTG_OK;
}

struct Level {
    DBuf rays, meta, hits, nodes, shadows, slist, paths;
    DBuf carry;                // path tracer: each queued ray's running radiance (16 B; k_pt_shade reads it)
    DBuf lv;                   // stream schedule: the queued rays' levels (1 byte each)
    long long rcap = 0;        // plane stride of `rays` (RayQ) as the previous level wrote them
    void release() {
        rays.release(); meta.release(); hits.release(); nodes.release(); shadows.release(); slist.release();
        paths.release(); carry.release(); lv.release();
    }
};

// One in-flight pass: its own stream, level buffers and queue counters, so that while the
// host waits for one pass's level count the GPU runs the other passes' kernels (the tails of
// the per-level launches overlap instead of draining the device).
struct Lane {
    hipStream_t st = nullptr;
    hipEvent_t ev_count = nullptr;          // recorded after the level count copy
    hipEvent_t ev_join = nullptr;           // stream schedule: the lane's work of a segment is done
    hipEvent_t ev_t[6] = {};                // trace start, trace end, shade end, shadow start, shadow end,
                                            // path-tracer gather end
    unsigned long long* h_count = nullptr;  // pinned host slot
    DBuf qcnt;                              // 128 x u64 per pass: [level] next rays | shadow entries << 32
    DBuf lcnt;                              // path tracer: per-light shadow-list counts per level / step
    DBuf prad;                              // path tracer, pass schedule: the pass's sample radiance (16 B)
    std::vector<Level> levels;
    // current pass
    std::vector<int> passes;                // indices into the frame's pass list (this lane's, in order)
    size_t next_pass = 0;
    bool busy = false;
    int pass = -1, level = 0;
    std::vector<int> counts;
    // stream schedule: the current step's queued (survivor) and total ray counts, and the steps run
    // since the lane last took new samples
    int sq = 0, sn = 0, sdrain = 0;
    std::vector<DBuf> snodes;                // reference integrator: node records of each step of a segment
    std::vector<int> step_m, step_g, step_gb;   // ... and each step's survivors, new samples, first new slot
    int create() {
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&ev_count, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
        for (hipEvent_t& e : ev_t) HIP_TRY(hipEventCreate(&e));
        HIP_TRY(hipHostMalloc((void**)&h_count, sizeof(unsigned long long), hipHostMallocDefault));
        return RTG_OK;
    }
    void destroy() {
        for (Level& l : levels) l.release();
        for (DBuf& b : snodes) b.release();
        snodes.clear();
        qcnt.release(); lcnt.release(); prad.release();
        if (h_count) (void)hipHostFree(h_count);
        for (hipEvent_t e : ev_t) if (e) (void)hipEventDestroy(e);
        if (ev_count) (void)hipEventDestroy(ev_count);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (st) (void)hipStreamDestroy(st);
        h_count = nullptr; ev_count = nullptr; ev_join = nullptr; st = nullptr;
        for (hipEvent_t& e : ev_t) e = nullptr;
    }
};

}  // namespace

struct rtg_scene {
    int device = 0;
    int num_objects = 0, num_instances = 0, num_vertices = 0;
    std::vector<ObjBVH> bvh;                 // per object
    std::vector<Mat4> inv, invT;             // per top-level entry
    std::vector<float> vnormals;
    std::vector<int> orig_prim;              // absolute BVH position -> original prim index
    SceneView sv{};
    DBuf d_tops, d_geoms, d_nodes, d_nodes4, d_tris, d_primidx, d_vertices, d_vnormals, d_texcoords, d_materials, d_textures,
        d_texels, d_lights, d_origprim, d_topemit, d_etris, d_ecdf, d_tlas, d_tlasidx, d_stris, d_gates, d_gtris,
        d_gents, d_gtop, d_tsph;
    int num_gtris = 0, num_gents = 0;
    int blas_mode = 0;                       // rtg_build_opts.traversal_tree
    int tlas_mode = 0;                       // rtg_build_opts.tlas
    int tlas_root = -1;                      // top-level BVH root node (-1: linear object loop)
    int tlas_count = 0;                      // its nodes
    float tlas_k[3] = {0, 0, 0};             // per axis: bound of |object-space coordinate x scale| over aligned entries
    int num_emit = 0;                        // hw7 object lights
    // render workspace
    std::vector<Lane> lanes;
    DBuf d_acc, d_counters, d_stats;
    DBuf d_rad;                              // stream schedule: per-sample radiance of a segment
    rtg_render_stats stats{};
    int num_lanes = 8;                       // default passes in flight (rtg_render_opts.streams overrides)
    int stream_lanes = 4;                    // stream schedule's lanes (rtg_render_opts.streams overrides)
    int stream_div = 3;                      // about this many new-sample steps per lane
    int uni_walk = 1;                        // rtg_build_opts.uniform_walk == 0
    int bvh_builder = RTG_BVH_AUTO;
    double bvh_build_ms = 0.0;               // last scene build: BVH construction time (all objects)
    rtg_build_stats bst{};                   // last scene build: per-phase wall times
    std::chrono::steady_clock::time_point build_end{};   // build_scene's last statement (RTG_BUILD_TIMING)
    int bvh_gpu_objects = 0;                 // objects whose BVH the GPU built
    bool replica = false;                    // device copy made by scene_replicate (no host-side structures)
    rtg::MultiState* multi = nullptr;        // num_devices fan-out: replicas, RCCL communicators (rtg_multi.cpp)
};

// Exceptions (std::bad_alloc from host containers, ...) never cross the C ABI.
template <class F>
static int32_t guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return fail(RTG_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(RTG_ERR_INVALID, std::string("internal error: ") + e.what());
    }
}

extern "C" {

int32_t rtg_abi_version(void) { return RTG_ABI_VERSION; }
const char* rtg_last_error(void) { return g_err.c_str(); }

int32_t rtg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static int validate(const rtg_scene_desc* d) {
    if (!d) return fail(RTG_ERR_INVALID, "null scene descriptor");
    if (d->abi_version != RTG_ABI_VERSION) return fail(RTG_ERR_INVALID, "abi_version mismatch");
    if (d->num_vertices < 0 || (d->num_vertices && !d->vertices)) return fail(RTG_ERR_INVALID, "bad vertices");
    if (d->num_objects < 0 || (d->num_objects && !d->objects)) return fail(RTG_ERR_INVALID, "bad objects");
    if (d->num_lights > kMaxLights) return fail(RTG_ERR_UNSUPPORTED, "more than 64 lights");
    auto vok = [&](int v) { return v >= 1 && v <= d->num_vertices; };
    auto xok = [&](int first, int count) {
        if (count < 0 || first < 0 || first + count > d->num_xform_refs) return false;
        for (int j = 0; j < count; j++) {
            const rtg_xform_ref& x = d->xform_refs[first + j];
            int lim = x.type == RTG_XF_TRANSLATION ? d->num_translations
                      : x.type == RTG_XF_SCALING   ? d->num_scalings
                      : x.type == RTG_XF_ROTATION  ? d->num_rotations
                      : x.type == RTG_XF_COMPOSITE ? d->num_composites : -1;
            if (lim < 0 || x.index < 1 || x.index > lim) return false;
        }
        return true;
    };
    for (int i = 0; i < d->num_objects; i++) {
        const rtg_object_desc& o = d->objects[i];
        if (o.material < 1 || o.material > d->num_materials)
            return fail(RTG_ERR_INVALID, "object " + std::to_string(i) + ": material out of range");
        if (o.num_textures < 0 || o.num_textures > 2) return fail(RTG_ERR_INVALID, "object textures");
        for (int t = 0; t < o.num_textures; t++)
            if (o.textures[t] < 1 || o.textures[t] > d->num_textures) return fail(RTG_ERR_INVALID, "object texture index");
        if (!xok(o.xform_first, o.xform_count)) return fail(RTG_ERR_INVALID, "object transformation reference");
        if (o.type == RTG_OBJ_SPHERE) {
            if (!vok(o.center)) return fail(RTG_ERR_INVALID, "sphere center index");
        } else if (o.type == RTG_OBJ_TRIANGLE) {
            if (!vok(o.v[0]) || !vok(o.v[1]) || !vok(o.v[2])) return fail(RTG_ERR_INVALID, "triangle index");
        } else if (o.type == RTG_OBJ_MESH) {
            if (o.face_first < 0 || o.face_count < 0 || o.face_first + o.face_count > d->num_faces)
                return fail(RTG_ERR_INVALID, "mesh face range");
            for (int f = 0; f < o.face_count; f++)
                for (int q = 0; q < 3; q++)
                    if (!vok(d->faces[3 * (o.face_first + f) + q])) return fail(RTG_ERR_INVALID, "mesh face index");
        } else {
            return fail(RTG_ERR_INVALID, "object type");
        }
    }
    for (int i = 0; i < d->num_instances; i++) {
        const rtg_instance_desc& in = d->instances[i];
        if (in.base_object < 0 || in.base_object >= d->num_objects) return fail(RTG_ERR_INVALID, "instance base");
        if (in.material < 1 || in.material > d->num_materials) return fail(RTG_ERR_INVALID, "instance material");
        if (!xok(in.xform_first, in.xform_count)) return fail(RTG_ERR_INVALID, "instance transformation reference");
    }
    for (int i = 0; i < d->num_textures; i++) {
        const rtg_texture_desc& t = d->textures[i];
        if (t.kind == RTG_TEX_IMAGE && (t.width < 1 || t.height < 1 || !t.texels))
            return fail(RTG_ERR_INVALID, "image texture without texels");
    }
    for (int i = 0; i < d->num_lights; i++)
        if (d->lights[i].type == RTG_LIGHT_ENVIRONMENT &&
            (d->lights[i].texture < 0 || d->lights[i].texture >= d->num_textures))
            return fail(RTG_ERR_INVALID, "environment light texture");
    if (d->background_texture >= d->num_textures) return fail(RTG_ERR_INVALID, "background texture");
    if (d->environment_light >= d->num_lights) return fail(RTG_ERR_INVALID, "environment light index");
    return RTG_OK;
}

// The scene's device buffers, in one list (release, replication).
static std::vector<DBuf*> scene_buffers(rtg_scene* s) {
    return {&s->d_tops, &s->d_geoms, &s->d_nodes, &s->d_nodes4, &s->d_tris, &s->d_primidx, &s->d_vertices,
            &s->d_vnormals, &s->d_texcoords, &s->d_materials, &s->d_textures, &s->d_texels, &s->d_lights,
            &s->d_origprim, &s->d_topemit, &s->d_etris, &s->d_ecdf, &s->d_tlas, &s->d_tlasidx, &s->d_stris, &s->d_gtris,
            &s->d_gents, &s->d_gtop, &s->d_tsph,
            &s->d_gates};
}

// Point the kernels' SceneView at this scene's device buffers.
static void bind_view(rtg_scene* s) {
    SceneView& sv = s->sv;
    sv.tops = s->d_tops.as<TopObject>();
    sv.geoms = s->d_geoms.as<Geometry>();
    sv.nodes = s->d_nodes.as<Node>();
    sv.snodes = s->d_nodes4.as<Node4>();
    sv.stris = s->d_stris.as<TriGeom>();
    sv.gates = s->d_gates.as<float>();
    sv.tris = s->d_tris.as<TriGeom>();
    sv.prim_idx = s->d_primidx.as<int4>();
    sv.vertices = s->d_vertices.as<float>();
    sv.vnormals = s->d_vnormals.as<float>();
    sv.texcoords = s->d_texcoords.as<float>();
    sv.materials = s->d_materials.as<MaterialDev>();
    sv.textures = s->d_textures.as<TextureDev>();
    sv.texels = s->d_texels.as<float>();
    sv.lights = s->d_lights.as<LightDev>();
    sv.top_emit = s->d_topemit.as<int>();
    sv.emit_tris = s->d_etris.as<float>();
    sv.emit_cdf = s->d_ecdf.as<float>();
    sv.tlas = s->d_tlas.as<Node>();
    sv.tlas_idx = s->d_tlasidx.as<int>();
    sv.gtris = s->d_gtris.as<TriGeom>();
    sv.gents = s->d_gents.as<GroupEnt>();
    sv.gtop = s->d_gtop.as<TopObject>();
    sv.tsph = s->d_tsph.as<SphereEnt>();
}

static void scene_free(rtg_scene* s) {
    multi_free(s->multi);
    s->multi = nullptr;
    for (DBuf* b : scene_buffers(s)) b->release();
    s->d_acc.release(); s->d_counters.release(); s->d_stats.release(); s->d_rad.release();
    for (Lane& l : s->lanes) l.destroy();
    s->lanes.clear();
}

// Frees a scene build's host record arrays off the caller's thread (unmapping ~300 MB for a 1 M-triangle
// mesh took 18-25 ms of rtg_scene_create).  One worker owned by the library: rtg_scene_destroy waits
// until everything handed to it is freed, and the library's teardown (this object's destructor, at
// process exit or dlclose) drains the queue and joins the worker -- no thread outlives the library.
class Reaper {
public:
    // run del(p) on the worker (or here, if the worker cannot be started)
    void submit(void* p, void (*del)(void*)) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!th_.joinable()) {
                try {
                    th_ = std::thread([this] { run(); });
                } catch (...) {
                    th_ = std::thread();
                }
            }
            if (th_.joinable()) {
                q_.emplace_back(p, del);
                cv_.notify_one();
                return;
            }
        }
        del(p);
    }
    // wait until every submitted free has run
    void drain() {
        std::unique_lock<std::mutex> lk(mu_);
        idle_.wait(lk, [&] { return q_.empty() && !busy_; });
    }
    ~Reaper() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        if (th_.joinable()) th_.join();
    }

private:
    void run() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;                  // stop requested and nothing left
            const auto job = q_.front();
            q_.pop_front();
            busy_ = true;
            lk.unlock();
            job.second(job.first);
            lk.lock();
            busy_ = false;
            if (q_.empty()) idle_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, idle_;
    std::deque<std::pair<void*, void (*)(void*)>> q_;
    bool stop_ = false, busy_ = false;
    std::thread th_;
};
static Reaper g_reaper;

int32_t rtg_scene_destroy(rtg_scene* s) {
    if (!s) return RTG_OK;
    g_reaper.drain();
    if (s->device >= 0) (void)hipSetDevice(s->device);
    scene_free(s);
    delete s;
    return RTG_OK;
}

// Wall-clock laps of the scene build (rtg_build_stats phases).
struct PhaseClock {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    double lap(const char* what = nullptr) {
        const auto n = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
        if (what && getenv("RTG_BUILD_TIMING")) fprintf(stderr, "[rtg] phase %-16s %7.2f ms\n", what, ms);
        return ms;
    }
};

// Triangle record of face f (1-based vertex indices pv[3f..3f+2]): a, a - b, a - c (the Cramer
// operands of Triangle::bvhIntersect, src/Shape.cpp:297-316) and c - b.  With a - b, c - b gives
// the flat normal (c - b) x (a - b) (src/Shape.cpp:327), so the shading of a flat triangle reads
// this record only; the device formed cc - b itself before, and the two agree bit for bit only
// because this is one IEEE f32 subtraction (no contraction can apply to a lone subtraction) on f32
// components, which the static_assert pins.  Covered at run time by the flat, non-Triangle floor
// mesh of the dragon scenes in the simple shading variant (test_gpu_fullsize.py band,
// test_gpu_parity.py images).  p2.yzw is free for the caller (the traversal copy's reference
// position, leaf start and gate flag).
static TriGeom tri_geom(const std::vector<V3>& verts, const std::vector<int>& pv, size_t f) {
    const V3 a = verts[pv[3 * f] - 1], b = verts[pv[3 * f + 1] - 1], c = verts[pv[3 * f + 2] - 1];
    const V3 amb = a - b, amc = a - c, cmb = c - b;
    static_assert(std::is_same<decltype(cmb.x), float>::value, "flat-normal c - b must be f32");
    TriGeom tg;
    tg.p0 = make_float4(a.x, a.y, a.z, amb.x);
    tg.p1 = make_float4(amb.y, amb.z, amc.x, amc.y);
    tg.p2 = make_float4(amc.z, cmb.x, cmb.y, cmb.z);
    return tg;
}

static int build_scene(rtg_scene* s, const rtg_scene_desc* d) {
    PhaseClock pc;
    rtg_build_stats& bs = s->bst;
    const int nv = d->num_vertices;
    std::vector<V3> verts(nv);
    for (int i = 0; i < nv; i++) verts[i] = v3(d->vertices[3 * i], d->vertices[3 * i + 1], d->vertices[3 * i + 2]);
    s->num_objects = d->num_objects;
    s->num_instances = d->num_instances;
    s->num_vertices = nv;

    // per-object primitive lists in parse order
    struct ObjPrims { std::vector<int> v; };   // 3 per prim (sphere: center,0,0)
    std::vector<ObjPrims> op(d->num_objects);
    for (int i = 0; i < d->num_objects; i++) {
        const rtg_object_desc& o = d->objects[i];
        if (o.type == RTG_OBJ_MESH) op[i].v.assign(d->faces + 3 * o.face_first, d->faces + 3 * (o.face_first + o.face_count));
        else if (o.type == RTG_OBJ_TRIANGLE) op[i].v = {o.v[0], o.v[1], o.v[2]};
        else op[i].v = {o.center, 0, 0};
    }

    // matrices (objects, then instances)
    std::vector<Mat4> model(d->num_objects);
    std::vector<Mat4> top_model;             // per top-level entry (objects, then instances)
    s->inv.clear(); s->invT.clear();
    for (int i = 0; i < d->num_objects; i++) {
        model[i] = compose(d, d->objects[i].xform_first, d->objects[i].xform_count);
        s->inv.push_back(inverse(model[i]));
        s->invT.push_back(inverse_transpose(model[i]));
        top_model.push_back(model[i]);
    }
    for (int i = 0; i < d->num_instances; i++) {
        const rtg_instance_desc& in = d->instances[i];
        Mat4 m = compose(d, in.xform_first, in.xform_count);
        if (!in.reset_transform) m = mul(m, model[in.base_object]);
        s->inv.push_back(inverse(m));
        s->invT.push_back(inverse_transpose(m));
        top_model.push_back(m);
    }

    // smooth vertex normals (src/Scene.cpp:302-318)
    std::vector<V3> vn(nv, v3(0, 0, 0));
    for (int i = 0; i < d->num_objects; i++) {
        const rtg_object_desc& o = d->objects[i];
        if (!(o.type == RTG_OBJ_TRIANGLE || (o.type == RTG_OBJ_MESH && o.smooth))) continue;
        const std::vector<int>& pv = op[i].v;
        for (size_t k = 0; k + 2 < pv.size(); k += 3) {
            V3 a = verts[pv[k] - 1], b = verts[pv[k + 1] - 1], c = verts[pv[k + 2] - 1];
            V3 n = normalized(cross(c - b, a - b));
            for (int q = 0; q < 3; q++) vn[pv[k + q] - 1] = vn[pv[k + q] - 1] + n;
        }
    }
    s->vnormals.resize(3 * (size_t)nv);
    for (int i = 0; i < nv; i++) {
        V3 n = normalized(vn[i]);
        s->vnormals[3 * i] = n.x; s->vnormals[3 * i + 1] = n.y; s->vnormals[3 * i + 2] = n.z;
    }
    bs.prep_ms += pc.lap("prep");

    // BVHs and device geometry
    std::vector<Geometry> geoms(d->num_objects);
    hvec<Node> dnodes;
    hvec<Node4> snodes;                      // traversal trees (SAH, 4-wide)
    hvec<TriGeom> stris;                     // their triangles, SAH leaf order (p2 = ref position / leaf / gated)
    hvec<float> gates;                       // per reference position: its leaf's parent box
    hvec<TriGeom> tris;
    std::vector<int> pos_leaf;               // per reference position: first position of its leaf ...
    std::vector<char> pos_gated;             // ... and whether its leaf's parent (gates[]) is not the root
    std::vector<char> geom_finite(d->num_objects, 0);   // every primitive box coordinate finite
    hvec<int4> primidx;
    bool early_upload = false;               // dnodes / gates / tris / primidx / orig_prim / vnormals uploaded by early_thread
    std::thread early_thread;
    int early_rc = RTG_OK;
    std::string early_err;                   // early_thread's rtg_last_error() (thread-local there)
    struct EarlyJoin {                       // joined on every return path (the thread reads this frame's arrays)
        std::thread& t;
        ~EarlyJoin() { if (t.joinable()) t.join(); }
    } early_join{early_thread};
    s->orig_prim.clear();
    s->bvh.assign(d->num_objects, ObjBVH());
    const float ieps = d->intersection_test_eps;
    for (int i = 0; i < d->num_objects; i++) {
        const rtg_object_desc& o = d->objects[i];
        const std::vector<int>& pv = op[i].v;
        int np = (int)(pv.size() / 3);
        hvec<V3> centers(np), bmin(np), bmax(np);
        std::vector<char> fin_chunk(std::max(build_threads(), 1), 1);
        parallel_chunks((size_t)np, 1 << 14, [&](int ch, size_t k0, size_t k1) {
            bool fin = true;
            for (size_t k = k0; k < k1; k++) {
                if (o.type == RTG_OBJ_SPHERE) {                            // Shape.cpp:55-67
                    V3 c = verts[o.center - 1];
                    float R = o.radius;
                    centers[k] = c;
                    bmin[k] = v3(c.x - R, c.y - R, c.z - R);
                    bmax[k] = v3(c.x + R, c.y + R, c.z + R);
                } else {                                                  // Shape.cpp:162-190
                    V3 a = verts[pv[3 * k] - 1], b = verts[pv[3 * k + 1] - 1], c = verts[pv[3 * k + 2] - 1];
                    centers[k] = v3(((a.x + b.x) + c.x) / 3.0f, ((a.y + b.y) + c.y) / 3.0f, ((a.z + b.z) + c.z) / 3.0f);
                    bmin[k] = v3(minOf3(a.x, b.x, c.x), minOf3(a.y, b.y, c.y), minOf3(a.z, b.z, c.z));
                    bmax[k] = v3(maxOf3(a.x, b.x, c.x), maxOf3(a.y, b.y, c.y), maxOf3(a.z, b.z, c.z));
                }
                fin = fin && std::isfinite(centers[k].x) && std::isfinite(centers[k].y) && std::isfinite(centers[k].z) &&
                      std::isfinite(bmin[k].x) && std::isfinite(bmin[k].y) && std::isfinite(bmin[k].z) &&
                      std::isfinite(bmax[k].x) && std::isfinite(bmax[k].y) && std::isfinite(bmax[k].z);
            }
            fin_chunk[ch] = fin;
        });
        bool all_finite = true;
        for (char f : fin_chunk) all_finite = all_finite && f;
        geom_finite[i] = all_finite;
        // traversal tree (SAH, 4-wide; below) of a triangle object with finite primitives: its
        // binned-SAH recursion runs on its own threads, over the triangles in parse order, while the
        // reference's median tree is built (on the GPU for large meshes); its leaves are mapped to
        // reference positions afterwards.  Any tree shape gives the same results (the total order
        // of candidates and the reachability gates), so it needs no reference order.
        const bool sah_try = o.type != RTG_OBJ_SPHERE && np >= 2 && all_finite && s->blas_mode != 1;
        // the eps overhang of a candidate beyond its triangle (Triangle::bvhIntersect's t >= -eps):
        // the traversal tree's boxes and the root window are widened by it (a max over the faces,
        // so the evaluation order does not matter)
        float obj_pad = 0.0f;
        if (o.type != RTG_OBJ_SPHERE) {
            std::vector<float> pad_chunk(build_threads(), 0.0f);
            parallel_chunks((size_t)np, 1 << 14, [&](int ch, size_t k0, size_t k1) {
                float padc = 0.0f;
                for (size_t k = k0; k < k1; k++) {
                    const V3 a = verts[pv[3 * k] - 1], b = verts[pv[3 * k + 1] - 1], c = verts[pv[3 * k + 2] - 1];
                    const double e = (double)(ieps > 0 ? ieps : 0.0f);
                    const double ext = e * ((double)vnorm(b - a) + (double)vnorm(c - a));
                    padc = std::max(padc, (float)(ext * 1.02 + 1e-7));
                }
                pad_chunk[ch] = padc;
            });
            for (float x : pad_chunk) obj_pad = std::max(obj_pad, x);
        }
        hvec<SahRec> sah_rec_buf, sah_tmp;
        hvec<int> sah_idx;
        std::vector<SahNode2> sah_bn;            // host build (the GPU build collapses on the device)
        bool sah_root_interior = false;
        uint64_t sah_hash = 0, sah_bnodes = 0;
        // the traversal tree on the GPU: large meshes of a device scene (the host recursion was the
        // long pole of scene creation, ~75-85 ms for the dragon on its thread)
        const bool sah_gpu = s->device >= 0 && (s->bvh_builder == RTG_BVH_GPU ||
                                                (s->bvh_builder == RTG_BVH_AUTO && np >= kSahGpuMin));
        // the SAH thread also collapses its tree to 4-wide nodes (leaf refs from tri_base0, the
        // object's first traversal-order triangle) and forms the triangles' records in that order
        // (p2.yzw, which need the reference tree, are filled after the join)
        const int tri_base0 = (int)stris.size();
        hvec<Node4> sah_nodes;
        hvec<TriGeom> sah_tris;
        std::thread sah_thread;
        std::exception_ptr sah_err;
        struct Joiner {                    // the SAH thread never outlives this iteration
            std::thread& t;
            ~Joiner() { if (t.joinable()) t.join(); }
        } sah_join{sah_thread};
        if (sah_try) {
            sah_rec_buf.resize(np);
            if (!sah_gpu) sah_tmp.resize(np);
            sah_idx.resize(np);
            parallel_chunks((size_t)np, 1 << 14, [&](int, size_t k0, size_t k1) {
                for (size_t f = k0; f < k1; f++) {
                    SahRec& q = sah_rec_buf[f];
                    for (int z = 0; z < 3; z++) { q.lo[z] = comp(bmin[f], z); q.hi[z] = comp(bmax[f], z); }
                    q.idx = (int)f;
                    q.pad_ = 0;
                }
            });
            if (!sah_gpu) sah_bn.reserve(2 * (size_t)np / kSahMaxLeaf + 16);
            sah_thread = std::thread([&] {
                try {
                    PhaseClock tc;
                    if (sah_gpu) {                   // tree, collapse and hash on the device
                        std::string e;
                        if (hipSetDevice(s->device) != hipSuccess)
                            throw std::runtime_error("GPU SAH build: hipSetDevice failed");
                        auto alloc4 = [&](size_t c) { sah_nodes.resize(c); return sah_nodes.data(); };
                        if (gpu_build_sah(sah_rec_buf.data(), np, tri_base0, obj_pad, alloc4, sah_idx.data(), sah_bnodes,
                                          sah_hash, e))
                            throw std::runtime_error("GPU SAH build: " + e);
                        sah_root_interior = !sah_nodes.empty();
                        tc.lap(" sah_tree+collapse gpu (thread)");
                        if (sah_root_interior) {
                            node4_preorder(sah_nodes);
                            tc.lap(" node4 preorder (thread)");
                        }
                    } else {
                        sah_rec_par(sah_rec_buf.data(), sah_tmp.data(), 0, np, sah_bn, sah_depth());
                        parallel_chunks((size_t)np, 1 << 16, [&](int, size_t k0, size_t k1) {
                            for (size_t k = k0; k < k1; k++) sah_idx[k] = sah_rec_buf[k].idx;
                        });
                        tc.lap(" sah_tree (thread)");
                        sah_tree_stats(sah_bn.data(), 0, sah_bnodes, sah_hash);
                        sah_root_interior = sah_bn[0].left >= 0;
                        if (sah_root_interior) {
                            sah_nodes.reserve((size_t)np / 2 + 16);
                            sah_collapse_par(sah_bn.data(), 0, tri_base0, obj_pad, sah_nodes, 3);
                            tc.lap(" sah_collapse (thread)");
                        }
                    }
                    if (sah_root_interior) {
                        sah_tris.resize(np);
                        parallel_chunks((size_t)np, 1 << 14, [&](int, size_t k0, size_t k1) {
                            for (size_t k = k0; k < k1; k++) sah_tris[k] = tri_geom(verts, pv, (size_t)sah_idx[k]);
                        });
                        tc.lap(" sah_tris (thread)");
                    }
                } catch (...) {
                    sah_err = std::current_exception();
                }
            });
        }
        ObjBVH& ob = s->bvh[i];
        ob.perm.resize(np);
        for (int k = 0; k < np; k++) ob.perm[k] = k;
        BuildCtx B{centers.data(), bmin.data(), bmax.data(), &ob.perm, &ob.nodes, {}};
        bs.prep_ms += pc.lap("prep");
        auto tb0 = std::chrono::steady_clock::now();
        // non-finite centres / boxes: the GPU build does not model NaN folds
        const bool use_gpu = s->device >= 0 && o.type != RTG_OBJ_SPHERE && all_finite &&
                             (s->bvh_builder == RTG_BVH_GPU || (s->bvh_builder == RTG_BVH_AUTO && np >= 4096));
        if (use_gpu) {
            GpuBvh gb;
            std::string err;
            PhaseClock sub;
            if (gpu_build_bvh(&centers[0].x, &bmin[0].x, &bmax[0].x, np, gb, err, nullptr))
                return fail(RTG_ERR_HIP, "GPU BVH build: " + err);
            sub.lap(" gpu_build");
            ob.perm.resize(np);
            parallel_chunks((size_t)np, 1 << 16, [&](int, size_t k0, size_t k1) {
                memcpy(ob.perm.data() + k0, gb.perm.as<int>() + k0, sizeof(int) * (k1 - k0));
            });
            // the nodes stay in the build's breadth-first order: the device records below number
            // the interior nodes in any order (they follow child links), and only the introspection
            // call needs the reference's pre-order (rtg_scene_object_bvh converts).  The build hands
            // them over in HNode's layout.
            static_assert(sizeof(HNode) == 40, "HNode = the GPU build's 40-byte node record");
            const int nn = gb.num_nodes;
            ob.nodes.resize(nn);
            parallel_chunks((size_t)nn, 1 << 15, [&](int, size_t k0, size_t k1) {
                memcpy(ob.nodes.data() + k0, gb.nodes.as<HNode>() + k0, sizeof(HNode) * (k1 - k0));
            });
            ob.bfs = true;
            ob.root = nn > 0 ? 0 : -1;
            s->bvh_gpu_objects++;
            sub.lap(" nodes");
        } else {
            ob.nodes.reserve(2 * (size_t)np + 1);
            B.finite = all_finite;
            ob.root = construct_par(B, 0, np, 0, 0, 4);
        }
        const double bms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count();
        s->bvh_build_ms += bms;
        bs.median_tree_ms += pc.lap("median_tree");
        if (getenv("RTG_BUILD_TIMING"))
            fprintf(stderr, "[rtg] object %d: %d prims, BVH %s %.1f ms\n", i, np, use_gpu ? "gpu" : "host", bms);

        Geometry& g = geoms[i];
        memset(&g, 0, sizeof g);
        g.flat_split = -1;
        g.type = o.type;
        g.prim_base = (int)tris.size();
        g.nprims = np;
        g.num_textures = o.num_textures;
        g.textures[0] = o.textures[0];
        g.textures[1] = o.textures[1];
        g.texture_offset = (o.type == RTG_OBJ_MESH) ? o.texture_offset : 0;
        g.smooth = o.smooth;
        if (o.type == RTG_OBJ_SPHERE) {
            V3 c = verts[o.center - 1];
            g.center[0] = c.x; g.center[1] = c.y; g.center[2] = c.z;
            g.radius = o.radius;
            g.center_index = o.center;
        }
        // primitives in BVH order (chunks of positions in parallel)
        const size_t pbase = tris.size();
        tris.resize(pbase + np);
        primidx.resize(pbase + np);
        s->orig_prim.resize(pbase + np);
        parallel_chunks((size_t)np, 1 << 14, [&](int, size_t k0, size_t k1) {
          for (size_t k = k0; k < k1; k++) {
            const int f = ob.perm[k];
            TriGeom tg;
            int4 pi;
            if (o.type == RTG_OBJ_SPHERE) {
                memset(&tg, 0, sizeof tg);
                pi = make_int4(o.center, 0, 0, 0);
            } else {
                tg = tri_geom(verts, pv, (size_t)f);
                const int smooth = (o.type == RTG_OBJ_TRIANGLE) ? 1 : o.smooth;   // Shape.cpp:262-276 quirk
                pi = make_int4(pv[3 * f], pv[3 * f + 1], pv[3 * f + 2], smooth);
            }
            tris[pbase + k] = tg;
            primidx[pbase + k] = pi;
            s->orig_prim[pbase + k] = f;
          }
        });
        const float pad = obj_pad;
        g.prune_pad = pad;
        // linearise interior nodes (in the tree's node order) into child-box nodes: per-chunk
        // interior counts, then every chunk numbers its own interior nodes from its offset
        const hvec<HNode>& hn = ob.nodes;
        hvec<int> dev_index(hn.size());
        const int node_base = (int)dnodes.size();
        std::vector<int> chunk_cnt(build_threads() + 1, 0);
        const int TN = parallel_chunks(hn.size(), 1 << 15, [&](int ch, size_t k0, size_t k1) {
            int c = 0;
            for (size_t k = k0; k < k1; k++) c += (hn[k].left >= 0 || hn[k].right >= 0);
            chunk_cnt[ch] = c;
        });
        std::vector<int> chunk_off(TN + 1, node_base);
        for (int c = 0; c < TN; c++) chunk_off[c + 1] = chunk_off[c] + chunk_cnt[c];
        const int cnt = chunk_off[TN] - node_base;
        parallel_chunks(hn.size(), 1 << 15, [&](int ch, size_t k0, size_t k1) {
            int at = chunk_off[ch];
            for (size_t k = k0; k < k1; k++) dev_index[k] = (hn[k].left >= 0 || hn[k].right >= 0) ? at++ : -1;
        });
        dnodes.resize(node_base + cnt);
        parallel_chunks(hn.size(), 1 << 15, [&](int, size_t k0, size_t k1) {
          for (size_t k = k0; k < k1; k++) {
            if (dev_index[k] < 0) continue;
            Node nd;
            float box[2][6];
            int ref[2], count[2];
            int ch[2] = {hn[k].left, hn[k].right};
            for (int q = 0; q < 2; q++) {
                int c = ch[q];
                for (int z = 0; z < 6; z++) box[q][z] = 0.0f;
                if (c < 0) { ref[q] = 0; count[q] = -1; continue; }
                const HNode& cn = hn[c];
                for (int z = 0; z < 3; z++) { box[q][z] = cn.mn[z]; box[q][3 + z] = cn.mx[z]; }
                if (cn.left < 0 && cn.right < 0) {
                    int len = cn.end - cn.start;
                    ref[q] = g.prim_base + cn.start;
                    count[q] = len > 0 ? len : -1;
                } else {
                    ref[q] = dev_index[c];
                    count[q] = 0;
                }
            }
            nd.a = make_float4(box[0][0], box[0][1], box[0][2], box[0][3]);
            nd.b = make_float4(box[0][4], box[0][5], box[1][0], box[1][1]);
            nd.c = make_float4(box[1][2], box[1][3], box[1][4], box[1][5]);
            nd.d = make_int4(ref[0], ref[1], count[0], count[1]);
            dnodes[dev_index[k]] = nd;
          }
        });
        // reference leaf of every position: its first position (tie order) and the box of the
        // interior node above it, which gates it (none under the root: closest_hit tests the root)
        gates.resize(6 * (size_t)(g.prim_base + np));
        parallel_chunks(6 * (size_t)np, 1 << 16, [&](int, size_t k0, size_t k1) {
            std::fill(gates.begin() + 6 * (size_t)g.prim_base + k0, gates.begin() + 6 * (size_t)g.prim_base + k1, 0.0f);
        });
        std::vector<int> leaf_start(np, 0);
        std::vector<char> gated(np, 0);
        if (ob.root >= 0 && hn[ob.root].left < 0 && hn[ob.root].right < 0)
            for (int k = hn[ob.root].start; k < hn[ob.root].end; k++) leaf_start[k] = g.prim_base + hn[ob.root].start;
        parallel_chunks(hn.size(), 1 << 15, [&](int, size_t n0, size_t n1) {   // a leaf has one parent
          for (size_t n2 = n0; n2 < n1; n2++) {
            const int ch[2] = {hn[n2].left, hn[n2].right};
            for (int c : ch) {
                if (c < 0 || hn[c].left >= 0 || hn[c].right >= 0) continue;
                for (int k = hn[c].start; k < hn[c].end; k++) {
                    leaf_start[k] = g.prim_base + hn[c].start;
                    gated[k] = (int)n2 != ob.root;
                    for (int z = 0; z < 3; z++) {
                        gates[6 * (size_t)(g.prim_base + k) + z] = hn[n2].mn[z];
                        gates[6 * (size_t)(g.prim_base + k) + 3 + z] = hn[n2].mx[z];
                    }
                }
            }
          }
        });
        if (np <= kFlatMaxPrims) {                  // small meshes: kept for the flat group
            pos_leaf.resize(std::max(pos_leaf.size(), (size_t)(g.prim_base + np)), 0);
            pos_gated.resize(std::max(pos_gated.size(), (size_t)(g.prim_base + np)), 0);
            for (int k = 0; k < np; k++) { pos_leaf[g.prim_base + k] = leaf_start[k]; pos_gated[g.prim_base + k] = gated[k]; }
        }
        // traversal tree (SAH, 4-wide) of a triangle object with an interior reference root and
        // finite primitives (its boxes must bound every candidate; NaN / inf objects keep the
        // reference-tree walk)
        g.sah_base = -1;
        const bool sah_ok = sah_try && ob.root >= 0 && (hn[ob.root].left >= 0 || hn[ob.root].right >= 0);
        bs.records_ms += pc.lap("records");
        PhaseClock sub;
        // The last object's reference-tree records are final now: a helper thread uploads them while
        // this one finishes the traversal tree and the top level (joined before the remaining uploads;
        // nothing below writes these arrays).  Dragon1m: ~7-10 ms of host-to-device copies.
        if (s->device >= 0 && i == d->num_objects - 1 && sah_thread.joinable()) {
            early_thread = std::thread([&, dev = s->device] {
                if (hipSetDevice(dev) != hipSuccess) { early_rc = RTG_ERR_HIP; early_err = "hipSetDevice"; return; }
                int rc2;
                if ((rc2 = upload(s->d_nodes, dnodes)) || (rc2 = upload(s->d_gates, gates)) || (rc2 = upload(s->d_tris, tris)) ||
                    (rc2 = upload(s->d_primidx, primidx)) || (rc2 = upload(s->d_origprim, s->orig_prim)) ||
                    (rc2 = upload(s->d_vnormals, s->vnormals))) {
                    early_rc = rc2;
                    early_err = rtg_last_error();
                }
            });
            early_upload = true;
            sub.lap(" early_upload start");
        }
        if (sah_thread.joinable()) sah_thread.join();
        if (sah_err) std::rethrow_exception(sah_err);
        sub.lap(" sah_join_wait");
        if (sah_ok) {
            bs.traversal_nodes += sah_bnodes;
            bs.traversal_hash += sah_hash;
            if (sah_gpu) bs.sah_gpu_objects++;
            if (sah_root_interior) {
                // SAH leaf order: face index -> reference position (inverse of the median tree's
                // perm); the thread's records get their reference position, leaf and gate flag
                std::vector<int> pos_of(np);
                parallel_chunks((size_t)np, 1 << 16, [&](int, size_t k0, size_t k1) {
                    for (size_t k = k0; k < k1; k++) pos_of[ob.perm[k]] = (int)k;
                });
                const int tri_base = (int)stris.size();
                if (tri_base != tri_base0) return fail(RTG_ERR_UNSUPPORTED, "internal: traversal-tree triangle base");
                parallel_chunks((size_t)np, 1 << 14, [&](int, size_t k0, size_t k1) {
                    for (size_t k = k0; k < k1; k++) {
                        const int r = pos_of[sah_idx[k]];
                        TriGeom& t = sah_tris[k];
                        const int pos = g.prim_base + r, gt = gated[r];
                        memcpy(&t.p2.y, &pos, 4);
                        memcpy(&t.p2.z, &leaf_start[r], 4);
                        memcpy(&t.p2.w, &gt, 4);
                    }
                });
                if (stris.empty()) stris = std::move(sah_tris);
                else stris.insert(stris.end(), sah_tris.begin(), sah_tris.end());
                sub.lap(" stris");
                // the thread's nodes, interior refs shifted to this mesh's first node
                const size_t first = snodes.size();
                const size_t nsub = sah_nodes.size();
                const int off = (int)first;
                if (first == 0) {
                    snodes = std::move(sah_nodes);
                } else {
                    snodes.resize(first + sah_nodes.size());
                    parallel_chunks(sah_nodes.size(), 1 << 15, [&](int, size_t k0, size_t k1) {
                        for (size_t k = k0; k < k1; k++) {
                            Node4 x = sah_nodes[k];
                            if (x.info.x == 0) x.ref.x += off;
                            if (x.info.y == 0) x.ref.y += off;
                            if (x.info.z == 0) x.ref.z += off;
                            if (x.info.w == 0) x.ref.w += off;
                            snodes[first + k] = x;
                        }
                    });
                }
                g.sah_base = off;
                sub.lap(" nodes");
                if (nsub == 1 && np <= kFlatMaxPrims) { g.flat_first = tri_base; g.flat_count = np; }
            }
        }
        bs.traversal_tree_ms += pc.lap("traversal_tree");
        if (ob.root < 0) {
            g.node_base = -1; g.root_leaf_start = g.prim_base; g.root_leaf_count = -1;
        } else if (hn[ob.root].left < 0 && hn[ob.root].right < 0) {
            int len = hn[ob.root].end - hn[ob.root].start;
            g.node_base = -1;
            g.root_leaf_start = g.prim_base + hn[ob.root].start;
            g.root_leaf_count = len > 0 ? len : -1;
        } else {
            g.node_base = dev_index[ob.root];
            g.root_leaf_start = 0; g.root_leaf_count = -1;
            for (int z = 0; z < 3; z++) {
                g.root_min[z] = hn[ob.root].mn[z]; g.root_max[z] = hn[ob.root].mx[z];
                g.win_min[z] = std::nextafter((float)((double)g.root_min[z] - g.prune_pad), -FLT_MAX);
                g.win_max[z] = std::nextafter((float)((double)g.root_max[z] + g.prune_pad), FLT_MAX);
            }
            // every mesh by default: on the dragon the 2-triangle floor is skipped by every ray going
            // up (frame 35.9 -> 35.5 ms against meshes of >= 64 triangles only), cornell / cornell_pt
            // lose about 1 % (profiles/history/r3_ab_flat.jsonl)
            g.win = g.nprims >= kWinMinPrims;
            // a reference root over two leaves (the walk always visits both: leaves carry no tested box)
            const HNode& rn = hn[ob.root];
            auto leaf_of = [&](int c) { return c >= 0 && hn[c].left < 0 && hn[c].right < 0 && hn[c].end > hn[c].start; };
            if (g.sah_base < 0 && np <= kFlatMaxPrims && leaf_of(rn.left) && leaf_of(rn.right) &&
                hn[rn.right].start == hn[rn.left].end) {
                g.flat_first = g.prim_base + hn[rn.left].start;
                g.flat_split = g.prim_base + hn[rn.right].start;
                g.flat_count = hn[rn.right].end - hn[rn.left].start;
            }
        }
    }

    // top-level entries
    std::vector<TopObject> tops(d->num_objects + d->num_instances);
    for (int i = 0; i < d->num_objects + d->num_instances; i++) {
        TopObject& T = tops[i];
        memset(&T, 0, sizeof T);
        memcpy(T.inv, s->inv[i].c, 64);
        memcpy(T.invT, s->invT[i].c, 64);
        if (i < d->num_objects) {
            const rtg_object_desc& o = d->objects[i];
            T.blur[0] = o.blur[0]; T.blur[1] = o.blur[1]; T.blur[2] = o.blur[2];
            T.kind = o.type == RTG_OBJ_SPHERE ? 0 : 1;
            T.material = o.material;
            T.geom = i;
        } else {
            const rtg_instance_desc& in = d->instances[i - d->num_objects];
            T.blur[0] = in.blur[0]; T.blur[1] = in.blur[1]; T.blur[2] = in.blur[2];
            T.kind = d->objects[in.base_object].type == RTG_OBJ_SPHERE ? 0 : 1;
            T.material = in.material;
            T.geom = in.base_object;
            T.is_instance = 1;
        }
        // identity fast path of transform_ray: rows 0-2 of inv exactly the identity with +0
        // off-diagonal entries, and +0 blur
        bool ident = true;
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 3; r++) {
                float want = (c == r) ? 1.0f : 0.0f;
                ident = ident && memcmp(&T.inv[c * 4 + r], &want, 4) == 0;
            }
        for (int k = 0; k < 3; k++) {
            float z = 0.0f;
            ident = ident && memcmp(&T.blur[k], &z, 4) == 0;
        }
        // A sphere whose inverse is the identity up to the signs of its zeros (compared by value) and
        // whose blur is zero -- an untransformed sphere: glm's inverse leaves -0 entries -- takes the
        // same fast path: for a finite ray the transformed ray equals o + 0, d + 0 in value, and the
        // sphere test, its point and gett() give the same values (signed zeros aside, on which no
        // outcome depends: the test compares, t > 0 is required), so the hit record is the same.
        if (!ident && T.kind == 0) {
            bool unit = true;
            for (int c = 0; c < 4; c++)
                for (int r = 0; r < 3; r++) unit = unit && T.inv[c * 4 + r] == (c == r ? 1.0f : 0.0f);
            for (int k = 0; k < 3; k++) unit = unit && T.blur[k] == 0.0f;
            T.ident = unit ? 2 : 0;    // (hit_record keeps the product: transform_ray's strict)
        } else {
            T.ident = ident ? 1 : 0;
        }
    }

    std::vector<SphereEnt> tsph(tops.size());
    for (size_t i = 0; i < tops.size(); i++) {
        SphereEnt& S = tsph[i];
        memset(&S, 0, sizeof S);
        S.prim = -1;
        if (tops[i].kind == 0) {
            const Geometry& g = geoms[tops[i].geom];
            S.c = make_float4(g.center[0], g.center[1], g.center[2], g.radius);
            S.prim = g.nprims > 0 ? g.prim_base : -1;
        }
    }
    // world boxes of the transformed entries: the object loop skips such an entry, before its ray
    // transform, for a lane whose ray line misses the box (closest_hit).  (Round 5 measured every entry
    // with a world box and, for axis-aligned ones, the top-level BVH's distance pruning -- behind the
    // origin / beyond the winner so far -- in the object loop: dragon 30.1 -> 31.5, cornell_pt 300 ->
    // 311 ms per frame; not kept.)
    for (int i = 0; i < d->num_objects + d->num_instances; i++) {
        TopObject& T = tops[i];
        T.wbox = 0;
        const ObjBVH& ob = s->bvh[T.geom];
        if ((T.ident && T.kind != 0) || ob.root < 0) continue;   // (a sphere has no root-box test)
        TBox b;
        const HNode& r = ob.nodes[ob.root];
        if (!entry_world_box(top_model[i], r.mn, r.mx, geoms[T.geom].prune_pad, T.blur, b)) continue;
        bool fin = true;
        for (int z = 0; z < 3; z++) {
            T.wlo[z] = std::nextafter((float)b.lo[z], -FLT_MAX);
            T.whi[z] = std::nextafter((float)b.hi[z], FLT_MAX);
            fin = fin && std::isfinite(T.wlo[z]) && std::isfinite(T.whi[z]);
        }
        T.wbox = fin ? 1 : 0;
        // the bounding sphere (TopObject::bsph): centre c0 = M (root box middle), radius the largest
        // distance of a triangle corner through the model matrix (double; one parallel pass, no storage),
        // then the blur sweep (centre + blur / 2, radius + |blur| / 2), the eps overhang through the
        // matrix (Frobenius norm) and the world box's margin.  The device test adds 3e-5 |oc|^2
        // (squared) for its own rounding and the object-space line's (far origins: a skipped line has
        // |oc| > r, so that slack is >= 1e-5 |oc|, above the transform's ~2e-7 cond |o|); taken only for a
        // well-conditioned matrix and a sphere of at most 60 % of the box's volume.
        T.bsph = 0;
        const Geometry& gg = geoms[T.geom];
        if (T.wbox && T.kind == 1 && gg.nprims > 0 && gg.prim_base + gg.nprims <= (int)tris.size()) {
            const Mat4& M = top_model[i];
            double fro = 0.0, fri = 0.0;
            for (int c = 0; c < 3; c++)
                for (int r = 0; r < 3; r++) {
                    fro += (double)M.c[c][r] * M.c[c][r];
                    fri += (double)T.inv[c * 4 + r] * T.inv[c * 4 + r];
                }
            fro = std::sqrt(fro); fri = std::sqrt(fri);
            if (std::isfinite(fro) && std::isfinite(fri) && fro * fri <= 6.0) {     // 3 for a similarity
                double c0[3];
                const HNode& rt = ob.nodes[ob.root];
                const double m[3] = {0.5 * ((double)rt.mn[0] + rt.mx[0]), 0.5 * ((double)rt.mn[1] + rt.mx[1]),
                                     0.5 * ((double)rt.mn[2] + rt.mx[2])};
                for (int r = 0; r < 3; r++) {
                    c0[r] = (double)M.c[0][r] * m[0] + (double)M.c[1][r] * m[1] + (double)M.c[2][r] * m[2] + (double)M.c[3][r];
                }
                std::vector<double> part(build_threads(), 0.0);
                parallel_chunks((size_t)gg.nprims, 65536, [&](int ch, size_t b0, size_t b1) {
                    double mx2 = 0.0;
                    for (size_t k = (size_t)gg.prim_base + b0; k < (size_t)gg.prim_base + b1; k++) {
                        const TriGeom& tg = tris[k];
                        const double a[3] = {tg.p0.x, tg.p0.y, tg.p0.z};
                        const double e[2][3] = {{tg.p0.w, tg.p1.x, tg.p1.y}, {tg.p1.z, tg.p1.w, tg.p2.x}};
                        for (int q = 0; q < 3; q++) {
                            double v[3], d2 = 0.0;
                            for (int z = 0; z < 3; z++) v[z] = q == 0 ? a[z] : a[z] - e[q - 1][z];
                            for (int r = 0; r < 3; r++) {
                                const double w = (double)M.c[0][r] * v[0] + (double)M.c[1][r] * v[1] +
                                                 (double)M.c[2][r] * v[2] + (double)M.c[3][r] - c0[r];
                                d2 += w * w;
                            }
                            mx2 = d2 > mx2 || d2 != d2 ? d2 : mx2;    // NaN propagates (no sphere)
                        }
                    }
                    part[ch] = mx2;
                });
                double r2 = 0.0, bl = 0.0, scale = 0.0, ext = 0.0, vol = 1.0;
                for (double v : part) r2 = v > r2 || v != v ? v : r2;
                for (int z = 0; z < 3; z++) {
                    bl += (double)T.blur[z] * T.blur[z];
                    scale = std::max(scale, std::max(std::fabs((double)T.wlo[z]), std::fabs((double)T.whi[z])));
                    ext = std::max(ext, (double)T.whi[z] - (double)T.wlo[z]);
                    vol *= (double)T.whi[z] - (double)T.wlo[z];
                }
                const double rad = std::sqrt(r2) + 0.5 * std::sqrt(bl) + (double)gg.prune_pad * fro +
                                   1e-4 * (scale + ext) + 1e-6;
                const double svol = 4.18879020478639 * rad * rad * rad;
                if (std::isfinite(rad) && svol <= 0.6 * vol) {
                    T.bsph = 1;
                    for (int z = 0; z < 3; z++) T.bs[z] = (float)(c0[z] + 0.5 * (double)T.blur[z]);
                    T.bs[3] = std::nextafter((float)(rad * rad * (1.0 + 1e-6)), FLT_MAX);
                }
            }
        }
    }

    // top-level BVH over the entries (objects, then instances): replaces the reference's linear
    // object loop (src/Helper.cpp:32-73) for scenes with many objects
    std::vector<Node> tlas_nodes;
    std::vector<int> tlas_idx;
    s->tlas_root = -1;
    const int ntops = d->num_objects + d->num_instances;
    const bool want_tlas = s->tlas_mode == 2 ? ntops >= 2 : (s->tlas_mode == 0 && ntops >= kTlasMinEntries);
    for (int z = 0; z < 3; z++) s->tlas_k[z] = 0.0f;
    if (want_tlas) {
        std::vector<TBox> boxes(ntops);
        std::vector<char> aligned(ntops, 0);
        bool ok = true;
        for (int i = 0; i < ntops && ok; i++) {
            const int gi = tops[i].geom;
            const ObjBVH& ob = s->bvh[gi];
            if (ob.root < 0) {            // no primitives: never hit; an empty box far away
                for (int z = 0; z < 3; z++) { boxes[i].lo[z] = 1e300; boxes[i].hi[z] = -1e300; }
                continue;
            }
            const HNode& r = ob.nodes[ob.root];
            ok = entry_world_box(top_model[i], r.mn, r.mx, geoms[gi].prune_pad, tops[i].blur, boxes[i]);
            // axis-aligned: the inverse's 3x3 part is diagonal (scaling / translation / blur only),
            // so the object-space direction has the world direction's zero pattern and gett()'s
            // error is bounded in world terms (closest_hit, TLAS pruning)
            const Mat4& iv = s->inv[i];
            bool al = true;
            for (int c = 0; c < 3; c++)
                for (int r2 = 0; r2 < 3; r2++)
                    al = al && (c == r2 ? (std::isfinite(iv.c[c][r2]) && iv.c[c][r2] != 0.0f) : iv.c[c][r2] == 0.0f);
            aligned[i] = al;
            if (al && ok)
                for (int z = 0; z < 3; z++) {
                    const double k = std::max(std::fabs(boxes[i].lo[z]), std::fabs(boxes[i].hi[z])) +
                                     std::fabs((double)tops[i].blur[z]) + std::fabs((double)top_model[i].c[3][z]);
                    s->tlas_k[z] = std::max(s->tlas_k[z], (float)(k * 1.01));
                }
        }
        if (ok) s->tlas_root = build_tlas(boxes, aligned, tlas_nodes, tlas_idx);
        s->tlas_count = s->tlas_root >= 0 ? (int)tlas_nodes.size() : 0;
    }

    // the flat group (GroupEnt, closest_hit), linear-loop scenes only.  (An untransformed object's glm
    // inverse is the identity with signed zeros, so TopObject::ident -- +0 entries only -- is rarely set;
    // the group asks only that its members share one transform.)
    std::vector<TriGeom> gtris;
    std::vector<GroupEnt> gents;
    for (int i = 0; i < ntops && s->tlas_root < 0; i++) {
        TopObject& T = tops[i];
        const Geometry& g = geoms[T.geom];
        if (g.type == RTG_OBJ_SPHERE) continue;
        // one transform for the whole group: the first member's inverse and blur, bit for bit
        if (!gents.empty() && (memcmp(T.inv, tops[gents[0].entry].inv, sizeof T.inv) != 0 ||
                               memcmp(T.blur, tops[gents[0].entry].blur, sizeof T.blur) != 0))
            continue;
        GroupEnt G;
        memset(&G, 0, sizeof G);
        G.entry = i;
        G.first = (int)gtris.size();
        // a small mesh (<= kFlatMaxPrims triangles, any reference-tree shape): its triangles in
        // reference order, each with its leaf (tie order) and gate -- the reference walk reaches a
        // candidate iff the root box and its leaf's parent box pass the exact slab test (visit_object)
        const ObjBVH& ob = s->bvh[T.geom];
        // (finite only: the gate argument needs every reference box to contain its descendants')
        if (ob.root < 0 || !geom_finite[T.geom] || g.nprims > kFlatMaxPrims ||
            g.prim_base + g.nprims > (int)pos_leaf.size())
            continue;
        std::vector<TriGeom> recs;
        for (int k = g.prim_base; k < g.prim_base + g.nprims; k++) {
            TriGeom r = tris[k];
            const int w[3] = {k, pos_leaf[k], (int)pos_gated[k]};
            memcpy(&r.p2.y, &w[0], 4); memcpy(&r.p2.z, &w[1], 4); memcpy(&r.p2.w, &w[2], 4);
            recs.push_back(r);
        }
        G.root_box = g.node_base >= 0;              // an interior root: its box is tested (a root leaf: none)
        if ((int)(gtris.size() + recs.size()) > kGroupMaxTris || (int)gents.size() >= kGroupMaxEnts) continue;
        for (int z = 0; z < 3; z++) {
            G.root_min[z] = g.root_min[z]; G.root_max[z] = g.root_max[z];
            G.win_min[z] = g.win_min[z]; G.win_max[z] = g.win_max[z];
        }
        G.win = g.node_base >= 0 && g.win;
        G.count = (int)recs.size();
        gtris.insert(gtris.end(), recs.begin(), recs.end());
        gents.push_back(G);
        T.grouped = 1;
    }
    s->num_gtris = (int)gtris.size();
    s->num_gents = (int)gents.size();
    std::vector<TopObject> gtop;
    if (!gents.empty()) {
        gtop.push_back(tops[gents[0].entry]);
        // The group's transform the identity up to the signs of its zeros, zero blur (untransformed
        // meshes): flat_group takes transform_ray's identity path (o + 0, d + 0).  The group runs only
        // for finite rays whose direction components are all nonzero (fast), so d2 is d bit for bit
        // and o2 equals o in value; every division the group's tests do is by a direction component or
        // by a determinant of edges and direction, neither of which involves o2, and the rest compares
        // values -- the hit record is the same (t > 0 is required, so its bits are too).
        TopObject& G0 = gtop[0];
        bool unit = true;
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 3; r++) unit = unit && G0.inv[c * 4 + r] == (c == r ? 1.0f : 0.0f);
        for (int k = 0; k < 3; k++) unit = unit && G0.blur[k] == 0.0f;
        if (unit && !G0.ident) G0.ident = 2;
    }
    bs.flat_group_entries = s->num_gents;

    // materials, textures, lights
    std::vector<MaterialDev> mats(d->num_materials);
    for (int i = 0; i < d->num_materials; i++) {
        const rtg_material_desc& m = d->materials[i];
        MaterialDev& M = mats[i];
        M.type = m.type; M.brdf = m.brdf; M.phong_exp = m.phong_exp; M.is_rough = m.is_rough; M.roughness = m.roughness;
        memcpy(M.ambient, m.ambient, 12); memcpy(M.diffuse, m.diffuse, 12); memcpy(M.specular, m.specular, 12);
        memcpy(M.mirror, m.mirror, 12);
        M.refraction_index = m.refraction_index; M.absorption_index = m.absorption_index;
        memcpy(M.absorption, m.absorption_coeff, 12);
    }
    std::vector<TextureDev> texs(d->num_textures);
    std::vector<float> texels;
    for (int i = 0; i < d->num_textures; i++) {
        const rtg_texture_desc& t = d->textures[i];
        TextureDev& T = texs[i];
        T.kind = t.kind; T.decal = t.decal; T.interp = t.interp; T.nc = t.noise_conv; T.normalizer = t.normalizer;
        T.noise_scale = t.noise_scale; T.bump = t.bump_factor; T.w = t.width; T.h = t.height;
        T.texel_offset = (long long)texels.size();
        if (t.kind == RTG_TEX_IMAGE && t.texels) texels.insert(texels.end(), t.texels, t.texels + (size_t)t.width * t.height * 3);
    }
    std::vector<LightDev> lights(d->num_lights);
    for (int i = 0; i < d->num_lights; i++) {
        const rtg_light_desc& l = d->lights[i];
        LightDev& L = lights[i];
        memset(&L, 0, sizeof L);
        L.type = l.type;
        memcpy(L.pos, l.position, 12); memcpy(L.inten, l.intensity, 12);
        L.size = l.size; L.tex = l.texture;
        V3 dir = v3(l.direction[0], l.direction[1], l.direction[2]);
        if (l.type == RTG_LIGHT_DIRECTIONAL || l.type == RTG_LIGHT_SPOT) {   // Light.cpp:256-260, 327-336
            V3 n = normalized(dir);
            L.dir[0] = n.x; L.dir[1] = n.y; L.dir[2] = n.z;
        }
        if (l.type == RTG_LIGHT_SPOT) {
            L.coverage = (float)((double)(l.coverage_deg * 0.5f) * (3.14159265358979323846 / 180.0f));
            L.fall = (float)((double)(l.falloff_deg * 0.5f) * (3.14159265358979323846 / 180.0f));
            L.cos_fall = (float)cos((double)L.fall);
            L.cos_cov = (float)cos((double)L.coverage);
        }
        if (l.type == RTG_LIGHT_AREA) {                                      // Light.cpp:442-455
            V3 n = normalized(dir);
            float a0 = fabsf(n.x), a1 = fabsf(n.y), a2 = fabsf(n.z);
            V3 nl = n;
            if (a0 <= a1 && a0 <= a2) nl.x = 1.0f;
            else if (a1 <= a0 && a1 <= a2) nl.y = 1.0f;
            else nl.z = 1.0f;
            V3 u = normalized(cross(n, nl));
            V3 v = cross(n, u);
            L.normal[0] = n.x; L.normal[1] = n.y; L.normal[2] = n.z;
            L.u[0] = u.x; L.u[1] = u.y; L.u[2] = u.z;
            L.v[0] = v.x; L.v[1] = v.y; L.v[2] = v.z;
        }
    }

    // hw7 object lights (path tracer NEE): appended after the scene's lights, in object order.
    // World-space geometry sampled at time 0, exactly as oracle/rtg_oracle.c builds it.
    std::vector<int> top_emit(d->num_objects + d->num_instances, -1);
    std::vector<float> etris, ecdf;
    s->num_emit = 0;
    for (int i = 0; i < d->num_objects; i++) {
        const rtg_object_desc& o = d->objects[i];
        if (!o.is_light) continue;
        if (d->num_lights + s->num_emit + 1 > kMaxLights) return fail(RTG_ERR_UNSUPPORTED, "more than 64 lights + object lights");
        LightDev L;
        memset(&L, 0, sizeof L);
        memcpy(L.inten, o.radiance, 12);
        const Mat4& M = model[i];
        if (o.type == RTG_OBJ_SPHERE) {
            L.type = kLightEmitSphere;
            V3 c = xform_point(M, verts[o.center - 1], 1.0f);
            L.pos[0] = c.x; L.pos[1] = c.y; L.pos[2] = c.z;
            L.size = o.radius * vnorm(v3(M.c[0][0], M.c[0][1], M.c[0][2]));
        } else {
            L.type = kLightEmitMesh;
            const std::vector<int>& pv = op[i].v;
            L.tri_first = (int)ecdf.size();
            L.tri_count = (int)(pv.size() / 3);
            float acc = 0.0f;
            for (size_t k = 0; k + 2 < pv.size(); k += 3) {       // parse order
                V3 a = xform_point(M, verts[pv[k] - 1], 1.0f), b = xform_point(M, verts[pv[k + 1] - 1], 1.0f),
                   c = xform_point(M, verts[pv[k + 2] - 1], 1.0f);
                const float t9[9] = {a.x, a.y, a.z, b.x, b.y, b.z, c.x, c.y, c.z};
                etris.insert(etris.end(), t9, t9 + 9);
                acc = acc + 0.5f * vnorm(cross(b - a, c - a));
                ecdf.push_back(acc);
            }
            L.coverage = acc;
        }
        top_emit[i] = d->num_lights + s->num_emit;
        lights.push_back(L);
        s->num_emit++;
    }

    bs.top_level_ms += pc.lap("top_level");
    if (s->device < 0) {                // host-only build (introspection / CPU tests)
        s->build_end = std::chrono::steady_clock::now();
        return RTG_OK;
    }
    std::vector<float> vflat(d->vertices, d->vertices + 3 * (size_t)nv);
    std::vector<float> tcflat;
    if (d->num_texcoords > 0) tcflat.assign(d->texcoords, d->texcoords + 2 * (size_t)d->num_texcoords);
    int rc;
    if (early_thread.joinable()) early_thread.join();
    if (early_rc != RTG_OK) return fail(early_rc, "scene upload (reference-tree records): " + early_err);
    if (!early_upload &&
        ((rc = upload(s->d_nodes, dnodes)) || (rc = upload(s->d_gates, gates)) || (rc = upload(s->d_tris, tris)) ||
         (rc = upload(s->d_primidx, primidx)) || (rc = upload(s->d_origprim, s->orig_prim)) ||
         (rc = upload(s->d_vnormals, s->vnormals))))
        return rc;
    if ((rc = upload(s->d_tops, tops)) || (rc = upload(s->d_geoms, geoms)) ||
        (rc = upload(s->d_nodes4, snodes)) || (rc = upload(s->d_stris, stris)) ||
        (rc = upload(s->d_vertices, vflat)) || (rc = upload(s->d_texcoords, tcflat)) ||
        (rc = upload(s->d_materials, mats)) || (rc = upload(s->d_textures, texs)) || (rc = upload(s->d_texels, texels)) ||
        (rc = upload(s->d_lights, lights)) ||
        (rc = upload(s->d_topemit, top_emit)) || (rc = upload(s->d_etris, etris)) || (rc = upload(s->d_ecdf, ecdf)) ||
        (rc = upload(s->d_tlas, tlas_nodes)) || (rc = upload(s->d_tlasidx, tlas_idx)) ||
        (rc = upload(s->d_gtris, gtris)) || (rc = upload(s->d_gents, gents)) || (rc = upload(s->d_gtop, gtop)) ||
        (rc = upload(s->d_tsph, tsph)))
        return rc;
    bs.upload_bytes = 0;
    for (DBuf* b : scene_buffers(s)) bs.upload_bytes += b->used;
    bs.upload_ms += pc.lap("upload");

    SceneView& sv = s->sv;
    bind_view(s);
    sv.num_tops = (int)tops.size(); sv.num_objects = d->num_objects;
    sv.num_texcoords = d->num_texcoords;
    sv.num_materials = d->num_materials;
    sv.num_textures = d->num_textures;
    sv.num_lights = d->num_lights;
    sv.num_emit = s->num_emit;
    sv.tlas_root = s->tlas_root;
    sv.num_gtris = s->num_gtris;
    sv.num_gents = s->num_gents;
    for (int z = 0; z < 3; z++) sv.tlas_k[z] = s->tlas_k[z];
    sv.pt_flags = 0;
    sv.max_depth = d->max_recursion_depth;
    sv.shadow_eps = d->shadow_ray_eps;
    sv.int_eps = d->intersection_test_eps;
    memcpy(sv.background, d->background, 12);
    memcpy(sv.ambient, d->ambient_light, 12);
    sv.bg_texture = d->background_texture;
    sv.env_light = d->environment_light;
    // The simple shading variant compiles out texturing, BRDFs and area/environment lights.
    sv.full = d->num_textures > 0 || d->background_texture != -1 || d->environment_light != -1;
    for (int i = 0; i < d->num_lights; i++)
        sv.full |= d->lights[i].type == RTG_LIGHT_AREA || d->lights[i].type == RTG_LIGHT_ENVIRONMENT;
    int any_brdf = 0;
    for (int i = 0; i < d->num_materials; i++) any_brdf |= d->materials[i].brdf != RTG_BRDF_NONE;
    sv.brdf_only = !sv.full && any_brdf;
    sv.brdf_ts = 0;
    for (int i = 0; i < d->num_materials; i++)
        sv.brdf_ts |= d->materials[i].brdf == RTG_BRDF_TS || d->materials[i].brdf == RTG_BRDF_TSF;
    sv.tex = any_brdf;
    for (int i = 0; i < d->num_objects; i++) sv.tex |= d->objects[i].num_textures > 0;
    sv.full |= any_brdf;
    sv.spot = 0;
    for (int i = 0; i < d->num_lights; i++) sv.spot |= d->lights[i].type == RTG_LIGHT_SPOT;
    sv.heavy = sv.spot || d->environment_light != -1;
    for (int i = 0; i < d->num_lights; i++) sv.heavy |= d->lights[i].type == RTG_LIGHT_ENVIRONMENT;
    int any_rough = 0;
    for (int i = 0; i < d->num_materials; i++) any_rough |= d->materials[i].is_rough != 0;
    sv.meta_free = !sv.full && !any_rough;
    sv.has_blur = 0;
    for (int i = 0; i < d->num_objects; i++)
        for (int k = 0; k < 3; k++) sv.has_blur |= !(d->objects[i].blur[k] == 0.0f);
    for (int i = 0; i < d->num_instances; i++)
        for (int k = 0; k < 3; k++) sv.has_blur |= !(d->instances[i].blur[k] == 0.0f);
    sv.bary = 0;
    for (int i = 0; i < d->num_objects; i++) {
        const rtg_object_desc& o = d->objects[i];
        if (o.type == RTG_OBJ_TRIANGLE || (o.type == RTG_OBJ_MESH && (o.smooth || o.num_textures > 0))) sv.bary = 1;
    }
    sv.uni_walk = s->uni_walk;
    sv.lean_shadow = d->num_lights == 1 && d->num_materials < kNodeMatMax &&
                     (d->lights[0].type == RTG_LIGHT_POINT || d->lights[0].type == RTG_LIGHT_SPOT ||
                      d->lights[0].type == RTG_LIGHT_DIRECTIONAL);
    sv.lit_nodes = d->num_lights == 1 && d->num_materials < kNodeMatMax;
    sv.pnt_all = !(d->shadow_ray_eps < 1e17f);
    for (int i = 0; i < d->num_materials; i++) {
        const rtg_material_desc& m = d->materials[i];
        if (m.type == RTG_MAT_DIELECTRIC &&
            !(m.absorption_coeff[0] == 0.0f && m.absorption_coeff[1] == 0.0f && m.absorption_coeff[2] == 0.0f))
            sv.pnt_all = 1;
    }
    pc.lap("view");
    // The host copies of the uploaded records (~300 MB for a 1 M-triangle mesh) are freed by the
    // library's reaper thread (Reaper, above): unmapping them took 18-25 ms of rtg_scene_create on the
    // GPU box's host (RTG_BUILD_TIMING "release").  Only memory owned by this call goes there.
    {
        struct Grave {
            hvec<Node> dnodes; hvec<Node4> snodes; hvec<TriGeom> stris, tris; hvec<float> gates; hvec<int4> primidx;
            std::vector<V3> verts, vn; std::vector<ObjPrims> op; std::vector<float> vflat;
        };
        Grave* g = new (std::nothrow) Grave;
        if (g) {
            g->dnodes.swap(dnodes); g->snodes.swap(snodes); g->stris.swap(stris); g->tris.swap(tris);
            g->gates.swap(gates); g->primidx.swap(primidx); g->verts.swap(verts); g->vn.swap(vn); g->op.swap(op);
            g->vflat.swap(vflat);
            g_reaper.submit(g, [](void* p) { delete static_cast<Grave*>(p); });
        }
    }
    s->build_end = std::chrono::steady_clock::now();
    return RTG_OK;
}

int32_t rtg_scene_create(const rtg_scene_desc* desc, int32_t device, rtg_scene** out) {
    return rtg_scene_create_ex(desc, device, nullptr, out);
}

int32_t rtg_scene_create_ex(const rtg_scene_desc* desc, int32_t device, const rtg_build_opts* opts, rtg_scene** out) {
    return guarded([&]() -> int32_t {
        if (!out) return fail(RTG_ERR_INVALID, "null out pointer");
        if (opts && (opts->bvh_builder < RTG_BVH_AUTO || opts->bvh_builder > RTG_BVH_GPU))
            return fail(RTG_ERR_INVALID, "bvh_builder");
        if (opts && (opts->tlas < 0 || opts->tlas > 2)) return fail(RTG_ERR_INVALID, "tlas");
        if (opts && (opts->traversal_tree < 0 || opts->traversal_tree > 1)) return fail(RTG_ERR_INVALID, "traversal_tree");
        if (opts && (opts->uniform_walk < 0 || opts->uniform_walk > 1)) return fail(RTG_ERR_INVALID, "uniform_walk");
        *out = nullptr;
        PhaseClock whole;
        int rc = validate(desc);
        if (rc) return rc;
        const double validate_ms = whole.lap();
        if (device >= 0) {
            int n = 0;
            if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RTG_ERR_NO_DEVICE, "no HIP device");
            if (device >= n) return fail(RTG_ERR_NO_DEVICE, "device index out of range");
            HIP_TRY(hipSetDevice(device));
        } else if (device != RTG_DEVICE_HOST_ONLY) {
            return fail(RTG_ERR_INVALID, "device index");
        }
        rtg_scene* s = new (std::nothrow) rtg_scene();
        if (!s) return fail(RTG_ERR_OOM, "host allocation");
        s->device = device;
        s->bvh_builder = opts ? opts->bvh_builder : RTG_BVH_AUTO;
        s->tlas_mode = opts ? opts->tlas : 0;
        s->blas_mode = opts ? opts->traversal_tree : 0;
        s->uni_walk = opts ? opts->uniform_walk == 0 : 1;
        s->bst.validate_ms = validate_ms;
        // The HIP runtime's first host-to-device copy in a process costs 90-145 ms (its copy path is
        // set up then: scripts/hip_init_probe.py on MI355X), even after the device context exists,
        // and the first launch from a code object a few ms more.  Start both now on their own
        // thread (a 256-byte pinned copy, one empty launch), so that they overlap the
        // host part of the build (descriptor checks, primitive boxes, the traversal tree's SAH build)
        // instead of stalling the first upload.  Errors are left to the build's own calls.
        std::thread warm;
        struct WarmJoin {
            std::thread& t;
            ~WarmJoin() { if (t.joinable()) t.join(); }
        } warm_join{warm};
        if (device >= 0)
            warm = std::thread([device] {
                if (hipSetDevice(device) != hipSuccess) return;
                void* h = nullptr;
                void* dptr = nullptr;
                if (hipHostMalloc(&h, 256, hipHostMallocDefault) != hipSuccess) return;
                memset(h, 0, 256);
                if (hipMalloc(&dptr, 256) == hipSuccess) {
                    (void)hipMemcpy(dptr, h, 256, hipMemcpyHostToDevice);
                    (void)hipFree(dptr);
                }
                (void)hipHostFree(h);
                // and the GPU build's code object (loading the render kernels' here as well delayed
                // the build without shortening the first frame)
                gpu_bvh_warm(nullptr);
                (void)hipStreamSynchronize(nullptr);
            });
        rc = build_scene(s, desc);
        if (getenv("RTG_BUILD_TIMING") && rc == RTG_OK)
            fprintf(stderr, "[rtg] phase %-16s %7.2f ms\n", "release",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - s->build_end).count());
        if (warm.joinable()) {
            PhaseClock wc;
            warm.join();
            wc.lap("warm_join");
        }
        if (rc) {
            scene_free(s);
            delete s;
            return rc;
        }
        s->bst.total_ms = validate_ms + whole.lap();
        *out = s;
        return RTG_OK;
    });
}

// Camera::Camera (src/Camera.cpp:7-61)
// Pixel-order band height in owned rows (tile_pixel): the default tile_band is kBandRows / tile height.
constexpr int kBandRows = 64;

static CameraDev make_camera(const rtg_camera_desc* c) {
    CameraDev k;
    memset(&k, 0, sizeof k);
    int i = 1;
    k.sample_count = 1;
    while (i < 1000) {
        if (i * i >= c->num_samples) { k.sample_count = i; break; }
        i++;
    }
    V3 gz = v3(c->gaze[0], c->gaze[1], c->gaze[2]), up = v3(c->up[0], c->up[1], c->up[2]);
    V3 g = normalized(gz);
    V3 w = c->left_handed ? normalized(gz) : normalized(v3(-gz.x, -gz.y, -gz.z));
    V3 right = normalized(cross(up, w));
    V3 u2 = cross(w, right);
    memcpy(k.pos, c->position, 12);
    k.gaze[0] = g.x; k.gaze[1] = g.y; k.gaze[2] = g.z;
    k.up[0] = u2.x; k.up[1] = u2.y; k.up[2] = u2.z;
    k.right[0] = right.x; k.right[1] = right.y; k.right[2] = right.z;
    k.l = c->left; k.r = c->right; k.b = c->bottom; k.t = c->top; k.dist = c->near_distance;
    k.nx = c->nx; k.ny = c->ny;
    k.nxDA = 1.0f / (float)c->nx;
    k.nyDA = 1.0f / (float)c->ny;
    k.pw = (k.r - k.l) * k.nxDA;
    k.ph = (k.t - k.b) * k.nyDA;
    k.sw = k.pw / (float)k.sample_count;
    k.sh = k.ph / (float)k.sample_count;
    k.total = c->num_samples;
    k.dof = c->is_dof;
    k.focus = c->focus_distance;
    k.aperture = c->aperture_size;
    return k;
}

static int render_impl(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* opts, float* out_dev,
                       hipStream_t st) {
    if (cam->nx < 1 || cam->ny < 1 || cam->num_samples < 1) return fail(RTG_ERR_INVALID, "bad camera");
    rtg_render_opts o{};
    if (opts) o = *opts;
    if (o.num_devices > 1 || o.devices) return fail(RTG_ERR_INVALID, "num_devices / devices need rtg_render / rtg_render_device");
    int stride = o.row_stride > 1 ? o.row_stride : 1;
    int off = o.row_offset;
    if (off < 0 || off >= stride) return fail(RTG_ERR_INVALID, "row_offset out of range");
    const int block = o.row_block > 1 ? o.row_block : 1;
    CameraDev cd = make_camera(cam);
    const int rows_owned = rtg_shard_rows(cam->ny, off, stride, block);
    long long npix_ll = (long long)rows_owned * cam->nx;
    if (npix_ll > (1LL << 30)) return fail(RTG_ERR_UNSUPPORTED, "image too large");
    int npix = (int)npix_ll;
    int total = cam->num_samples;
    if (cam->integrator != RTG_INTEGRATOR_REFERENCE && cam->integrator != RTG_INTEGRATOR_PATH)
        return fail(RTG_ERR_INVALID, "unknown integrator");
    const bool pt = cam->integrator == RTG_INTEGRATOR_PATH;
    SceneView sv = s->sv;                    // per-render view: the path tracer's light loop
    if (pt) {
        sv.pt_flags = cam->pt_flags;
        if (cam->pt_flags & RTG_PT_NEE) sv.num_lights += s->num_emit;
    }
    const int nL = sv.num_lights;
    // auto batch: a whole multiple of the lanes in flight, as few passes as the ray cap allows,
    // at least 2M rays each -- every lane gets the same number of equal passes, so the lanes'
    // level tails end together and overlap each other's work (1080p64 dragon, passes x lanes:
    // 1 GPU 16x3 -> 8x8 58.2 -> 58.1 ms; a 1/4 row shard 4x3 -> 8x8 16.0 -> 15.2 ms; a 1/8 shard
    // 3x3 -> 8x8 9.15 -> 8.1 ms).  The cap is 24M rays, lowered so that every lane's level buffers
    // fit half the device memory (rtg_pass_rays: many lights cost 68 B per ray and light).
    const int lanes_req = o.streams > 0 ? std::min(o.streams, 8) : s->num_lanes;
    const long long frame_rays = (long long)npix * total;
    int ns_chunk, np_pass;
    size_t dev_total_b = 0;
    {
        size_t free_b = 0;
        if (hipMemGetInfo(&free_b, &dev_total_b) != hipSuccess) dev_total_b = 0;
    }
    if (o.max_batch_rays > 0) {
        const long long max_batch = o.max_batch_rays;
        // passes: all samples of a pixel range (chunks of samples only when spp exceeds the batch)
        ns_chunk = (int)std::max<long long>(1, std::min<long long>(total, max_batch));
        np_pass = (int)std::max<long long>(1, std::min<long long>(npix, max_batch / ns_chunk));
    } else {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) total_b = 0;
        const long long kMax = rtg_pass_rays(nL, pt ? 1 : 0, lanes_req, (uint64_t)total_b);
        const long long kMin = std::min<long long>(2LL << 20, kMax);
        const long long lanes_eff = std::max(1LL, std::min<long long>(lanes_req, (frame_rays + kMin - 1) / kMin));
        // (an empty shard -- fewer row blocks than ranks -- has no rays: one empty pass, not a division by 0)
        const long long passes = std::max(1LL, lanes_eff * ((frame_rays + lanes_eff * kMax - 1) / (lanes_eff * kMax)));
        if (total > kMax) {                 // absurd spp: sample chunks of one pixel
            ns_chunk = (int)kMax;
            np_pass = 1;
        } else {
            ns_chunk = total;
            np_pass = (int)std::max<long long>(1, (npix + passes - 1) / passes);   // `passes` pixel ranges
        }
    }
    int exhaustive = o.traversal == 1;

    int rc;
    if ((rc = s->d_acc.grow(sizeof(float) * 3 * std::max<size_t>(npix, 1)))) return rc;
    // d_cnt[0]: NaN shadow queries (all passes)
    if ((rc = s->d_counters.grow(sizeof(unsigned) * 64))) return rc;
    if ((rc = s->d_stats.grow(sizeof(Counters)))) return rc;
    unsigned* d_cnt = s->d_counters.as<unsigned>();
    Counters* d_stats = s->d_stats.as<Counters>();
    HIP_TRY(hipMemsetAsync(s->d_counters.p, 0, sizeof(unsigned) * 64, st));
    HIP_TRY(hipMemsetAsync(s->d_stats.p, 0, sizeof(Counters), st));
    uint64_t shadow_listed = 0;

    struct Events {                     // RAII: released on every return path
        hipEvent_t e[3] = {};
        ~Events() { for (hipEvent_t x : e) if (x) (void)hipEventDestroy(x); }
    } ev;
    for (hipEvent_t& x : ev.e) HIP_TRY(hipEventCreate(&x));
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1], ejoin = ev.e[2];
    HIP_TRY(hipEventRecord(e0, st));
    const bool timing = o.collect_timing != 0;
    Counters* sctr = o.collect_stats ? d_stats : nullptr;

    // the frame's passes: pixel ranges (outer) x sample chunks (inner); all chunks of one pixel
    // range go to the same lane, in order (the in-order sum of MultiSample, src/Scene.cpp:386-409)
    // pixel order (tile_pixel): bands 16 tiles high, walked in columns of tiles.  1080p64 dragon,
    // one-tile-high bands -> 16: k_trace 14.7 -> 13.3 ms, k_shadow 13.1 -> 12.3 ms per frame, frame
    // 36.9 -> 36.0 ms; a 1/8 row shard 5.6 -> 5.1 ms (its passes become blocks of columns instead of
    // row strips, so each holds a mix of sky, floor and glass).  4 / 8 / 32 / 64 tiles: in between.
    if (o.tile_band < 0 || o.segment_pixels < 0 || o.segment_nodes < 0)
        return fail(RTG_ERR_INVALID, "tile_band / segment_pixels / segment_nodes");
    // Band height (round 6): kBandRows owned rows, whatever the tile height -- bands of
    // 8 tiles for the full frame's 8-row tiles and 16 for a row shard's 4-row tiles, which are the optima
    // round 5 found by sweeping each case separately (`profiles/history/r6_ab_schedule_sweep.jsonl`,
    // `r6_shard_band.txt`: 1/8 dragon shard 5.39 ms with 32-row bands, 4.40 with 64); one rule instead of
    // a special case for shards (its measurements per N: profiles/r7/shard_probe*.txt).
    const int tile_h = stride > 1 && block < 8 ? (block >= 4 ? 4 : block >= 2 ? 2 : 1) : 8;
    int tile_s = o.tile_band > 0 ? std::min(o.tile_band, 1 << 12) : std::max(1, kBandRows / tile_h);
    // tile_pixel (device) forms band * (tile_h * tile_s * nx) in 32-bit ints: keep one band of the
    // widest tiles (tile_h <= 8) below 2^31 pixels
    if ((long long)8 * cam->nx >= (1LL << 31)) return fail(RTG_ERR_UNSUPPORTED, "image wider than 2^28 pixels");
    tile_s = (int)std::min<long long>(tile_s, ((1LL << 31) - 1) / (8LL * cam->nx));
    std::vector<PassDev> plist;
    for (int p0 = 0; p0 < npix; p0 += np_pass)
        for (int s0 = 0; s0 < total; s0 += ns_chunk) {
            PassDev ps;
            ps.s0 = s0; ps.ns = std::min(ns_chunk, total - s0);
            ps.p0 = p0; ps.npass = std::min(np_pass, npix - p0);
            ps.row_offset = off; ps.row_stride = stride; ps.rows_owned = rows_owned; ps.row_block = block;
            ps.tile_h = tile_h;
            ps.tile_s = tile_s;
            plist.push_back(ps);
        }
    const int nranges = npix > 0 ? (npix + np_pass - 1) / np_pass : 1;
    const int want_lanes = std::max(1, std::min(o.streams > 0 ? std::min(o.streams, 8) : s->num_lanes, nranges));
    while ((int)s->lanes.size() < want_lanes) {
        s->lanes.emplace_back();
        if ((rc = s->lanes.back().create())) { s->lanes.back().destroy(); s->lanes.pop_back(); return rc; }
    }
    const int L = want_lanes;
    for (int k = 0; k < L; k++) {
        Lane& ln = s->lanes[k];
        ln.passes.clear(); ln.next_pass = 0; ln.busy = false;
        HIP_TRY(hipStreamWaitEvent(ln.st, e0, 0));
    }
    for (size_t k = 0; k < plist.size(); k++) {
        const int prange = plist[k].p0 / np_pass;
        s->lanes[prange % L].passes.push_back((int)k);
    }

    rtg_render_stats stt{};
    const int max_levels = (pt && (cam->pt_flags & RTG_PT_RUSSIAN_ROULETTE)) ? RTG_PT_MAX_BOUNCES
                                                                             : std::max(0, s->sv.max_depth) + 1;
    // enqueue trace / shade / shadow of the lane's current level and the count read-back
    auto enqueue_level = [&](Lane& ln) -> int {
        const PassDev& ps = plist[ln.pass];
        const int level = ln.level;
        const int n = ln.counts[level];
        if ((int)ln.levels.size() < level + 2) ln.levels.resize(level + 2);
        Level& Lc = ln.levels[level];
        Level& Ln = ln.levels[level + 1];
        int rc2;
        if ((rc2 = Lc.hits.grow(std::max(sizeof(HitRec), kHitBytes) * (size_t)n)) || (rc2 = Lc.nodes.grow(sizeof(NodeRec) * (size_t)n)) ||
            (rc2 = Lc.shadows.grow(sizeof(ShadowRec) * (size_t)n * std::max(nL, 1))) ||
            (rc2 = Lc.slist.grow(sizeof(int) * (size_t)n * std::max(nL, 1))))
            return rc2;
        const bool may_spawn = level + 1 < max_levels;
        const size_t cap = may_spawn ? 2 * (size_t)n : 1;
        if ((rc2 = Ln.rays.grow(kRayBytes * cap)) || (rc2 = Ln.meta.grow(sizeof(RayMeta) * cap))) return rc2;
        Ln.rcap = (long long)cap;
        const RayQ cur_q = level == 0 ? RayQ{} : ray_planes(Lc.rays.p, Lc.rcap, sv.has_blur);
        const RayQ next_q = ray_planes(Ln.rays.p, Ln.rcap, sv.has_blur);
        if (pt && ((rc2 = Lc.paths.grow(sizeof(PathRec) * (size_t)n)) || (rc2 = Ln.paths.grow(sizeof(PathRec) * cap)) ||
                   (rc2 = Lc.carry.grow(kCarryBytes * (size_t)n)) || (rc2 = Ln.carry.grow(kCarryBytes * cap))))
            return rc2;
        unsigned long long* qc = ln.qcnt.as<unsigned long long>() + level;
        const PtRad pr = pt ? PtRad{Lc.carry.as<float4>(), Ln.carry.as<float4>(), ln.prad.as<float4>(),
                                    ln.lcnt.as<unsigned>() + (size_t)level * std::max(nL, 1)}
                            : PtRad{};
        if (timing) HIP_TRY(hipEventRecord(ln.ev_t[0], ln.st));
        // level 0: k_trace / k_shade / k_pt_shade regenerate the primary rays (no level-0 ray buffer)
        const bool gen = level == 0;
        launch_trace(sv, cur_q, Lc.hits.as<HitRec>(), n, exhaustive, sctr, ln.st,
                     gen ? &cd : nullptr, gen ? &ps : nullptr, o.seed, /*compact=*/true);
        if (timing) HIP_TRY(hipEventRecord(ln.ev_t[1], ln.st));
        if (pt)
            launch_pt_shade(sv, cd, level, ps, o.seed, cur_q,
                            gen ? nullptr : Lc.meta.as<RayMeta>(), Lc.hits.as<HitRec>(),
                            Lc.paths.as<PathRec>(), Lc.nodes.as<NodeRec>(), Lc.shadows.as<ShadowRec>(), Lc.slist.as<int>(),
                            next_q, Ln.meta.as<RayMeta>(), Ln.paths.as<PathRec>(), qc, n, ln.st,
                            gen, gen ? 0 : n, 0, nullptr, nullptr, pr, sctr);
        else
            launch_shade(sv, cd, level, ps, o.seed, cur_q,
                         gen ? nullptr : Lc.meta.as<RayMeta>(), Lc.hits.as<HitRec>(),
                         Lc.nodes.as<NodeRec>(), Lc.shadows.as<ShadowRec>(), Lc.slist.as<int>(), next_q,
                         Ln.meta.as<RayMeta>(), qc, n, ln.st);
        if (timing) HIP_TRY(hipEventRecord(ln.ev_t[2], ln.st));
        // the next level's size is known once shade is done: read it back now, so the host can
        // enqueue that level while this level's shadow queries still run (no host round trip
        // between the levels on the stream)
        HIP_TRY(hipMemcpyAsync(ln.h_count, qc, sizeof(unsigned long long), hipMemcpyDeviceToHost, ln.st));
        HIP_TRY(hipEventRecord(ln.ev_count, ln.st));
        if (timing) HIP_TRY(hipEventRecord(ln.ev_t[3], ln.st));
        // (the path tracer: one launch per light, in light order, adding each vertex's T (x) v to its
        // sample's running radiance -- PtRad; no gather kernel)
        if (pt)
            launch_pt_shadow(sv, Lc.shadows.as<ShadowRec>(), Lc.slist.as<int>(), Lc.nodes.as<NodeRec>(), n, exhaustive,
                             sctr, d_cnt, ln.st, /*uni_from=*/level < kUniShadowLevels ? 0 : INT_MAX, pr);
        else
            launch_shadow(sv, Lc.shadows.as<ShadowRec>(), Lc.slist.as<int>(),
                          reinterpret_cast<const unsigned*>(qc) + 1,   // high word (little endian)
                          Lc.nodes.as<NodeRec>(), n, exhaustive, sctr, d_cnt, ln.st, /*light_sum=*/true,
                          /*uni_from=*/level < kUniShadowLevels ? 0 : INT_MAX);
        if (timing) HIP_TRY(hipEventRecord(ln.ev_t[4], ln.st));
        HIP_TRY(hipGetLastError());
        return RTG_OK;
    };
    auto start_pass = [&](Lane& ln) -> int {
        ln.pass = ln.passes[ln.next_pass++];
        const PassDev& ps = plist[ln.pass];
        const int n0 = ps.ns * ps.npass;
        int rc2;
        if ((rc2 = ln.qcnt.grow(sizeof(unsigned long long) * 128))) return rc2;
        HIP_TRY(hipMemsetAsync(ln.qcnt.p, 0, sizeof(unsigned long long) * 128, ln.st));
        if (pt) {
            const size_t nlc = (size_t)(max_levels + 1) * std::max(nL, 1);
            if ((rc2 = ln.prad.grow((size_t)16 * std::max(n0, 1))) || (rc2 = ln.lcnt.grow(sizeof(unsigned) * nlc))) return rc2;
            HIP_TRY(hipMemsetAsync(ln.lcnt.p, 0, sizeof(unsigned) * nlc, ln.st));
        }
        ln.counts.assign(1, n0);
        ln.level = 0;
        if ((int)ln.levels.size() < 1) ln.levels.resize(1);
        // both integrators generate their primary rays inside level 0's kernels (primary_ray)
        stt.primary_rays += (uint64_t)n0;
        ln.busy = true;
        return enqueue_level(ln);
    };
    // collect_timing: one launch between two events, waited for (roofline frames only)
    auto timed_launch = [&](Lane& ln, auto&& launch, double& ms, int& launches) -> int {
        if (timing) HIP_TRY(hipEventRecord(ln.ev_t[0], ln.st));
        launch();
        if (timing) {
            float a = 0.0f;
            HIP_TRY(hipEventRecord(ln.ev_t[1], ln.st));
            HIP_TRY(hipEventSynchronize(ln.ev_t[1]));
            HIP_TRY(hipEventElapsedTime(&a, ln.ev_t[0], ln.ev_t[1]));
            ms += a;
            launches++;
        }
        return RTG_OK;
    };
    auto finish_pass = [&](Lane& ln) -> int {
        const PassDev& ps = plist[ln.pass];
        const int level = ln.level;
        stt.max_level = std::max(stt.max_level, level);
        int rc2;
        // bottom-up (round 5): levels level-1 .. 2 two at a time (k_resolve2: a level and, inline, its
        // children, which no one else reads), the odd one alone, and levels 1 and 0 inside the
        // accumulation -- every resolved level is stored only where its parents are not resolved
        // in the same launch.  The nodes of `level` itself are final.
        auto N = [&](int l) { return ln.levels[l].nodes.as<NodeRec>(); };
        int l = level - 1;
        for (; l >= 3 && !pt; l -= 2)
            if ((rc2 = timed_launch(ln, [&] {
                     launch_resolve2(sv, N(l - 1), N(l), N(l + 1), ln.counts[l - 1], ln.counts[l], ln.counts[l + 1], ln.st);
                 }, stt.resolve_ms, stt.resolve_launches)))
                return rc2;
        if (l == 2 && !pt &&
            (rc2 = timed_launch(ln, [&] { launch_resolve(sv, N(2), N(3), ln.counts[2], ln.counts[3], ln.st); },
                                stt.resolve_ms, stt.resolve_launches)))
            return rc2;
        const int mode = (total == 1) ? 2 : (ps.s0 == 0 ? 1 : 0);
        const NodeRec* level1 = level >= 1 ? N(1) : nullptr;
        const NodeRec* level2 = level >= 2 ? N(2) : nullptr;
        if ((rc2 = timed_launch(ln, [&] {
                 // (the path tracer: the pass's sample radiance, PtRad)
                 launch_accumulate(sv, pt ? ln.prad.as<NodeRec>() : N(0), level1, !pt && level >= 1, s->d_acc.as<float>(), ps,
                                   cam->nx, mode, ln.st, !pt,
                                   ln.counts[0], level >= 1 ? ln.counts[1] : 0, pt ? nullptr : level2,
                                   level >= 2 ? ln.counts[2] : 0);
             }, stt.accumulate_ms, stt.accumulate_launches)))
            return rc2;
        stt.passes++;
        ln.busy = false;
        return RTG_OK;
    };
    std::deque<int> waiting;           // lanes with a level in flight, in enqueue order
    // next lane to service: the first (in enqueue order) whose count read-back has landed, so a
    // lane with a long level does not hold up the others (head-of-line blocking)
    auto next_ready = [&](int& pick) -> int {
        for (;;) {
            for (size_t i = 0; i < waiting.size(); i++) {
                const hipError_t q = hipEventQuery(s->lanes[waiting[i]].ev_count);
                if (q == hipSuccess) { pick = (int)i; return RTG_OK; }
                if (q != hipErrorNotReady) HIP_TRY(q);
            }
            if (waiting.size() == 1) { pick = 0; return RTG_OK; }
            std::this_thread::yield();
        }
    };
    // ------------------------------------------------------------ stream schedule
    // (round 4).  On the pass schedule every level of every pass is its own launch
    // (C5: ~22 passes x ~31 levels, the deep levels a few thousand rays each, each behind a host
    // count read-back; an N=8 dragon shard: the passes holding the glass sphere run their seven
    // levels alone at the end).  Here each lane runs steps of at most R rays: the survivors of its
    // previous step -- children of any level, each carrying its slot and level (the path tracer: its
    // path record too) -- followed by new camera samples from the frame's slot cursor.  A lane runs
    // a sample's ray tree in consecutive steps of one stream, so every per-sample sum keeps its
    // order and the frame is bit-identical to the pass schedule (and to the oracle):
    //  * path tracer: each queued ray carries its sample's running radiance (PtRad); k_pt_shade
    //    and the per-light k_shadow launches add each vertex's terms in level order, and the
    //    radiance of a segment of pixels lives in one buffer (16 B per slot, segments sized to an
    //    eighth of the device memory) and is summed per pixel in sample order (MultiSample,
    //    src/Scene.cpp:386-411) once the segment's paths have ended;
    //  * reference integrator: a step's node records [survivors | new samples] stay in HBM; a node's
    //    children are survivors of the lane's next step (their queue index is their node index
    //    there).  When a segment's trees have all ended, each lane evaluates RecursiveShading
    //    bottom-up (src/Scene.cpp:148-219), last step first, and sums the new samples of each step
    //    per pixel (their level-0 nodes resolved inside the sum).  New samples come in whole pixels;
    //    a segment closes (no new samples until its trees end) when its node records reach a quarter
    //    of the device memory.
    if (o.schedule < RTG_SCHEDULE_AUTO || o.schedule > RTG_SCHEDULE_STREAM) return fail(RTG_ERR_INVALID, "schedule");
    const bool want_stream = o.schedule == RTG_SCHEDULE_STREAM ||
                             (o.schedule == RTG_SCHEDULE_AUTO && pt);
    const bool stream = want_stream && npix > 0 && (long long)npix * total < (1LL << 31) &&
                        true;
    if (stream) {
        const int SL = o.streams > 0 ? std::min(o.streams, 8) : s->stream_lanes;
        while ((int)s->lanes.size() < SL) {
            s->lanes.emplace_back();
            if ((rc = s->lanes.back().create())) { s->lanes.back().destroy(); s->lanes.pop_back(); return rc; }
        }
        // rays per step: an even share of the frame, about s->stream_div new-sample steps per lane,
        // within the memory cap of a pass
        const long long kR = rtg_pass_rays(nL, pt ? 1 : 0, SL, (uint64_t)dev_total_b);
        const long long share = (frame_rays + (long long)SL * s->stream_div - 1) / ((long long)SL * s->stream_div);
        const long long R = o.max_batch_rays > 0 ? std::max<long long>(64, o.max_batch_rays)
                                                 : std::max<long long>(std::min<long long>(kR, 1LL << 16),
                                                                       std::min(kR, share));
        const long long rad_slots = std::max<long long>(total, (long long)(dev_total_b ? dev_total_b / 8 / 16 : 1LL << 28));
        int seg_np = pt ? (int)std::max<long long>(1, std::min<long long>(npix, rad_slots / total)) : npix;
        if (pt && o.segment_pixels > 0) seg_np = std::min(seg_np, o.segment_pixels);
        if (pt && (rc = s->d_rad.grow((size_t)16 * (size_t)seg_np * total))) return rc;
        const double node_budget = o.segment_nodes > 0 ? (double)sizeof(NodeRec) * o.segment_nodes
                                                       : (dev_total_b ? 0.25 * (double)dev_total_b : 16e9);
        const int nLb = std::max(nL, 1);
        for (int k = 0; k < SL; k++) {
            Lane& ln = s->lanes[k];
            if ((int)ln.levels.size() < 3) ln.levels.resize(3);
            if (pt)
                for (int b2 = 0; b2 < 2; b2++) {
                    Level& Q = ln.levels[b2];
                    if ((rc = Q.rays.grow(kRayBytes * (size_t)R)) || (rc = Q.meta.grow(sizeof(int) * (size_t)R)) ||
                        (rc = Q.lv.grow((size_t)R)) || (rc = Q.paths.grow(sizeof(PathRec) * (size_t)R)) ||
                        (rc = Q.carry.grow(kCarryBytes * (size_t)R)))
                        return rc;
                    Q.rcap = R;
                }
            if ((rc = ln.qcnt.grow(sizeof(unsigned long long) * 128))) return rc;
            if (pt && (rc = ln.lcnt.grow(sizeof(unsigned) * 2 * (size_t)nLb))) return rc;
            HIP_TRY(hipStreamWaitEvent(ln.st, e0, 0));
        }
        PassDev F;
        F.s0 = 0; F.ns = total; F.p0 = 0; F.npass = npix;
        F.row_offset = off; F.row_stride = stride; F.rows_owned = rows_owned; F.row_block = block;
        F.tile_h = tile_h;
        F.tile_s = tile_s;
        long long cursor = 0, seg_end = 0, seg_slots = 0;
        double seg_node_bytes = 0.0;
        bool seg_closed = false;
        // one step of lane ln: its m survivors (queued by its previous step) + g new samples
        auto enqueue_step = [&](Lane& ln, int m, int g) -> int {
            const int n = m + g;
            const int gbase = (int)cursor;
            cursor += g;
            if (g > 0) ln.sdrain = 0; else ln.sdrain++;
            stt.max_level = std::max(stt.max_level, ln.sdrain);
            stt.primary_rays += (uint64_t)g;
            ln.sq = m; ln.sn = n;
            const int step = ln.level;
            Level& A = ln.levels[step & 1];          // this step's queue (survivors)
            Level& B = ln.levels[(step + 1) & 1];    // the next step's
            Level& W = pt ? A : ln.levels[2];        // hits / shadow records / lists of the step
            int rc2;
            if ((rc2 = W.hits.grow(std::max(sizeof(HitRec), kHitBytes) * (size_t)n)) ||
                (rc2 = W.shadows.grow(sizeof(ShadowRec) * (size_t)n * nLb)) ||
                (rc2 = W.slist.grow(sizeof(int) * (size_t)n * nLb)))
                return rc2;
            DBuf* nodes = &A.nodes;
            if (!pt) {                               // the step's node records stay until the resolve
                if ((int)ln.snodes.size() <= step) ln.snodes.resize(step + 1);
                if ((int)ln.step_m.size() <= step) { ln.step_m.resize(step + 1); ln.step_g.resize(step + 1); ln.step_gb.resize(step + 1); }
                nodes = &ln.snodes[step];
                ln.step_m[step] = m; ln.step_g[step] = g; ln.step_gb[step] = gbase;
                // children: at most two per ray (DielectricRefraction, src/Scene.cpp:166-209)
                // (B is free: its rays were the previous step's queue, consumed earlier on this stream)
                const long long cap = 2LL * std::max(n, 1);
                if (B.rcap < cap) B.rcap = cap + cap / 4;        // the planes' stride
                if ((rc2 = B.rays.grow(kRayBytes * (size_t)B.rcap)) || (rc2 = B.lv.grow((size_t)B.rcap)) ||
                    (!sv.meta_free && (rc2 = B.meta.grow(sizeof(RayMeta) * (size_t)B.rcap))))
                    return rc2;
                seg_node_bytes += (double)sizeof(NodeRec) * n;
                if (seg_node_bytes > node_budget) seg_closed = true;
            } else {
                if ((rc2 = A.nodes.grow(sizeof(NodeRec) * (size_t)n))) return rc2;
            }
            if ((rc2 = nodes->grow(sizeof(NodeRec) * (size_t)n))) return rc2;
            const RayQ cur_q = ray_planes(A.rays.p, A.rcap, sv.has_blur);
            const RayQ next_q = ray_planes(B.rays.p, B.rcap, sv.has_blur);
            unsigned long long* qc = ln.qcnt.as<unsigned long long>() + (step & 1);
            HIP_TRY(hipMemsetAsync(qc, 0, sizeof(unsigned long long), ln.st));
            // the path tracer's radiance (PtRad): survivors' sums in A, their children's in B, a
            // sample's last vertex writes the segment's rad; per-light list counts of the step
            PtRad pr{};
            if (pt) {
                pr = PtRad{A.carry.as<float4>(), B.carry.as<float4>(), s->d_rad.as<float4>(),
                           ln.lcnt.as<unsigned>() + (size_t)(step & 1) * nLb};
                HIP_TRY(hipMemsetAsync(pr.lcnt, 0, sizeof(unsigned) * nLb, ln.st));
            }
            if (timing) HIP_TRY(hipEventRecord(ln.ev_t[0], ln.st));
            launch_trace(sv, cur_q, W.hits.as<HitRec>(), n, exhaustive, sctr, ln.st, g > 0 ? &cd : nullptr, &F, o.seed,
                         /*compact=*/true, m, gbase);
            if (timing) HIP_TRY(hipEventRecord(ln.ev_t[1], ln.st));
            if (pt)
                launch_pt_shade(sv, cd, 0, F, o.seed, cur_q, A.meta.as<RayMeta>(), W.hits.as<HitRec>(), A.paths.as<PathRec>(),
                                nodes->as<NodeRec>(), W.shadows.as<ShadowRec>(), W.slist.as<int>(), next_q,
                                B.meta.as<RayMeta>(), B.paths.as<PathRec>(), qc, n, ln.st, g > 0, m, gbase,
                                A.lv.as<unsigned char>(), B.lv.as<unsigned char>(), pr, sctr);
            else
                launch_shade(sv, cd, 0, F, o.seed, cur_q, A.meta.as<RayMeta>(), W.hits.as<HitRec>(), nodes->as<NodeRec>(),
                             W.shadows.as<ShadowRec>(), W.slist.as<int>(), next_q, B.meta.as<RayMeta>(), qc, n, ln.st, g > 0 ? 1 : 0, m, gbase, A.lv.as<unsigned char>(), B.lv.as<unsigned char>());
            if (timing) HIP_TRY(hipEventRecord(ln.ev_t[2], ln.st));
            HIP_TRY(hipMemcpyAsync(ln.h_count, qc, sizeof(unsigned long long), hipMemcpyDeviceToHost, ln.st));
            HIP_TRY(hipEventRecord(ln.ev_count, ln.st));
            if (timing) HIP_TRY(hipEventRecord(ln.ev_t[3], ln.st));
            // the step's new camera samples: nodes [m, n) (uni_from); the path tracer: one launch per
            // light, in light order, adding each vertex's T (x) v to its sample's radiance (PtRad)
            if (pt)
                launch_pt_shadow(sv, W.shadows.as<ShadowRec>(), W.slist.as<int>(), nodes->as<NodeRec>(), n, exhaustive,
                                 sctr, d_cnt, ln.st, /*uni_from=*/g > 0 ? m : INT_MAX, pr);
            else
                launch_shadow(sv, W.shadows.as<ShadowRec>(), W.slist.as<int>(), reinterpret_cast<const unsigned*>(qc) + 1,
                              nodes->as<NodeRec>(), n, exhaustive, sctr, d_cnt, ln.st, /*whitted=*/true,
                              /*uni_from=*/g > 0 ? m : INT_MAX);
            if (timing) HIP_TRY(hipEventRecord(ln.ev_t[4], ln.st));
            HIP_TRY(hipGetLastError());
            ln.level++;
            ln.busy = true;
            return RTG_OK;
        };
        // new samples for a lane's next step: up to R rays with its survivors, whole pixels on the
        // reference integrator (a pixel's samples are summed from one step's nodes)
        auto new_samples = [&](long long m) -> int {
            const long long left = seg_end - cursor;
            if (left <= 0 || seg_closed) return 0;
            long long g = std::min(left, std::max(0LL, R - m));
            if (!pt) {
                g = (g / total) * total;
                if (g == 0 && m == 0) g = std::min<long long>(left, total);
            }
            return (int)g;
        };
        const long long all_slots = (long long)npix * total;
        while (cursor < all_slots) {
            // one segment: [cursor, seg_end) of the slots (the path tracer: a radiance buffer's worth)
            const long long seg_begin = cursor;
            if (pt) {
                F.p0 = (int)(cursor / total);
                F.npass = std::min(seg_np, npix - F.p0);
                seg_slots = (long long)F.npass * total;
                seg_end = cursor + seg_slots;
                cursor = 0;                          // path tracer slots are segment-relative
                seg_end = seg_slots;
            } else {
                seg_end = all_slots;
            }
            seg_node_bytes = 0.0;
            seg_closed = false;
            for (int k = 0; k < SL; k++) {
                Lane& ln = s->lanes[k];
                ln.level = 0; ln.sdrain = 0; ln.busy = false;
                const int g = new_samples(0);
                if (g <= 0) continue;
                if ((rc = enqueue_step(ln, 0, g))) return rc;
                waiting.push_back(k);
            }
            while (!waiting.empty()) {
                int pick = 0;
                if ((rc = next_ready(pick))) return rc;
                const int k = waiting[pick];
                waiting.erase(waiting.begin() + pick);
                Lane& ln = s->lanes[k];
                HIP_TRY(hipEventSynchronize(ln.ev_count));
                const unsigned long long q = *ln.h_count;
                const unsigned next = (unsigned)q;
                shadow_listed += q >> 32;
                if (timing) {
                    float a = 0.0f, b = 0.0f, c = 0.0f;
                    HIP_TRY(hipEventElapsedTime(&a, ln.ev_t[0], ln.ev_t[1]));
                    HIP_TRY(hipEventElapsedTime(&c, ln.ev_t[1], ln.ev_t[2]));
                    HIP_TRY(hipEventSynchronize(ln.ev_t[4]));
                    HIP_TRY(hipEventElapsedTime(&b, ln.ev_t[3], ln.ev_t[4]));
                    stt.trace_ms += a; stt.trace_launches++;
                    stt.shade_ms += c; stt.shade_launches++;
                    if (nL > 0) { stt.shadow_ms += b; stt.shadow_launches++; }
                }
                if ((long long)next > (pt ? 1LL : 2LL) * ln.sn) return fail(RTG_ERR_HIP, "stream queue overflow");
                if (!pt && next > 0 && ln.level >= (1 << 20)) return fail(RTG_ERR_UNSUPPORTED, "stream: too many steps");
                stt.secondary_rays += next;
                const int g = new_samples(next);
                if ((long long)next + g > 0) {
                    if ((rc = enqueue_step(ln, (int)next, g))) return rc;
                    waiting.push_back(k);
                } else {
                    ln.busy = false;
                }
            }
            const int mode = total == 1 ? 2 : 1;
            if (pt) {
                // the segment's paths have ended: sum every pixel's samples in order, on lane 0 once
                // every lane's last gather is done; the next segment's gathers wait for that sum
                Lane& l0 = s->lanes[0];
                for (int k = 1; k < SL; k++) {
                    HIP_TRY(hipEventRecord(s->lanes[k].ev_join, s->lanes[k].st));
                    HIP_TRY(hipStreamWaitEvent(l0.st, s->lanes[k].ev_join, 0));
                }
                if ((rc = timed_launch(l0, [&] {
                         launch_accumulate(sv, s->d_rad.as<NodeRec>(), nullptr, false, s->d_acc.as<float>(), F, cam->nx,
                                           mode, l0.st, /*whitted=*/false, (int)seg_slots, 0);
                     }, stt.accumulate_ms, stt.accumulate_launches)))
                    return rc;
                HIP_TRY(hipEventRecord(l0.ev_join, l0.st));
                for (int k = 1; k < SL; k++) HIP_TRY(hipStreamWaitEvent(s->lanes[k].st, l0.ev_join, 0));
                cursor = (long long)(F.p0 + F.npass) * total;       // back to frame slots
            } else {
                // every tree of the segment has ended: bottom-up, last step first, per lane
                for (int k = 0; k < SL; k++) {
                    Lane& ln = s->lanes[k];
                    const int K = ln.level;
                    for (int j = K - 1; j >= 0; j--) {
                        const int n = ln.step_m[j] + ln.step_g[j];
                        const NodePlanes self = node_planes(ln.snodes[j].as<NodeRec>(), n);
                        const NodePlanes child = j + 1 < K ? node_planes(ln.snodes[j + 1].as<NodeRec>(),
                                                                         ln.step_m[j + 1] + ln.step_g[j + 1])
                                                           : self;     // no children: every link is -1
                        if (ln.step_m[j] > 0 &&
                            (rc = timed_launch(ln, [&] { launch_resolve_planes(sv, self, child, ln.step_m[j], ln.st); },
                                               stt.resolve_ms, stt.resolve_launches)))
                            return rc;
                        if (ln.step_g[j] > 0) {
                            const int mj = ln.step_m[j];
                            const NodePlanes l0 = {self.col + mj, self.pnt + mj, self.link + mj};
                            PassDev P = F;
                            P.p0 = ln.step_gb[j] / total;
                            P.npass = ln.step_g[j] / total;
                            if ((rc = timed_launch(ln, [&] {
                                     launch_accumulate_planes(sv, l0, child, true, s->d_acc.as<float>(), P, cam->nx, mode,
                                                              ln.st);
                                 }, stt.accumulate_ms, stt.accumulate_launches)))
                                return rc;
                        }
                    }
                    HIP_TRY(hipGetLastError());
                }
                if (cursor == seg_begin) return fail(RTG_ERR_OOM, "stream: a segment made no progress");
            }
            stt.passes++;
        }
    }
    for (int k = 0; k < L && !stream; k++)
        if (!s->lanes[k].passes.empty() && npix > 0) {
            if ((rc = start_pass(s->lanes[k]))) return rc;
            waiting.push_back(k);
        }
    while (!waiting.empty()) {
        int pick = 0;
        if ((rc = next_ready(pick))) return rc;
        const int k = waiting[pick];
        waiting.erase(waiting.begin() + pick);
        Lane& ln = s->lanes[k];
        HIP_TRY(hipEventSynchronize(ln.ev_count));
        const unsigned long long q = *ln.h_count;
        const unsigned next = (unsigned)q;
        shadow_listed += q >> 32;
        if (timing) {
            float a = 0.0f, b = 0.0f, c = 0.0f;
            HIP_TRY(hipEventElapsedTime(&a, ln.ev_t[0], ln.ev_t[1]));
            HIP_TRY(hipEventElapsedTime(&c, ln.ev_t[1], ln.ev_t[2]));
            stt.trace_ms += a;
            stt.trace_launches++;
            stt.shade_ms += c;
            stt.shade_launches++;
            if (nL > 0) {
                HIP_TRY(hipEventSynchronize(ln.ev_t[4]));   // the count arrives before the shadow pass ends
                HIP_TRY(hipEventElapsedTime(&b, ln.ev_t[3], ln.ev_t[4]));
                stt.shadow_ms += b;
                stt.shadow_launches++;
            }
        }
        const int n = ln.counts[ln.level];
        const bool may_spawn = ln.level + 1 < max_levels;
        const size_t cap = may_spawn ? 2 * (size_t)n : 1;
        if (next > cap) return fail(RTG_ERR_HIP, "secondary queue overflow");
        if (next > 0 && may_spawn) {
            if (ln.level + 1 >= 62) return fail(RTG_ERR_UNSUPPORTED, "recursion deeper than 62 levels");
            ln.counts.push_back((int)next);
            stt.secondary_rays += next;
            ln.level++;
            if ((rc = enqueue_level(ln))) return rc;
            waiting.push_back(k);
            continue;
        }
        if ((rc = finish_pass(ln))) return rc;
        if (ln.next_pass < ln.passes.size()) {
            if ((rc = start_pass(ln))) return rc;
            waiting.push_back(k);
        }
    }
    for (int k = 0; k < (int)s->lanes.size(); k++) {
        HIP_TRY(hipEventRecord(ejoin, s->lanes[k].st));
        HIP_TRY(hipStreamWaitEvent(st, ejoin, 0));
    }
    if (o.compact_rows)
        launch_finalize(s->d_acc.as<float>(), out_dev, cam->nx, rows_owned, 0, 1, 1, total, st);
    else
        launch_finalize(s->d_acc.as<float>(), out_dev, cam->nx, cam->ny, off, stride, block, total, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e1, st));
    HIP_TRY(hipEventSynchronize(e1));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    unsigned nan_queries = 0;
    Counters ctr{};
    HIP_TRY(hipMemcpy(&nan_queries, d_cnt, sizeof(unsigned), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&ctr, d_stats, sizeof(Counters), hipMemcpyDeviceToHost));
    stt.shadow_rays = shadow_listed - nan_queries;
    stt.total_rays = stt.primary_rays + stt.secondary_rays + stt.shadow_rays;
    stt.render_ms = ms;
    stt.node_visits = ctr.node_visits;
    stt.tri_tests = ctr.tri_tests;
    stt.shadow_node_visits = ctr.shadow_node_visits;
    stt.shadow_tri_tests = ctr.shadow_tri_tests;
    stt.trace_steps = ctr.trace_steps;
    stt.shadow_steps = ctr.shadow_steps;
    stt.trace_lane_slots = ctr.trace_lane_slots;
    stt.shadow_lane_slots = ctr.shadow_lane_slots;
    stt.shadow_blocked = ctr.shadow_blocked;
    stt.shadow_blocked_steps = ctr.shadow_blocked_steps;
    stt.shadow_blocked_tris = ctr.shadow_blocked_tris;
    stt.trace_entry_visits = ctr.trace_entry_visits;
    stt.trace_entry_slots = ctr.trace_entry_slots;
    stt.shadow_entry_visits = ctr.shadow_entry_visits;
    stt.shadow_entry_slots = ctr.shadow_entry_slots;
    for (int b = 0; b < 8; b++) {
        stt.shadow_hist_before[b] = ctr.shadow_hist_before[b];
        stt.shadow_hist_after[b] = ctr.shadow_hist_after[b];
    }
    stt.shadow_blocked_steps_before = ctr.shadow_blocked_steps_before;
    stt.shadow_blocked_steps_before_wavemin = ctr.shadow_blocked_steps_before_wavemin;
    for (int b = 0; b < 4; b++) stt.pt_shade_cycles[b] = ctr.pt_shade_cycles[b];
    stt.trace_group_work = ctr.trace_group_work;
    stt.trace_group_slots = ctr.trace_group_slots;
    stt.shadow_group_work = ctr.shadow_group_work;
    stt.shadow_group_slots = ctr.shadow_group_slots;
    for (int b = 0; b < 2; b++) {
        stt.trace_group_cycles[b] = ctr.trace_group_cycles[b];
        stt.shadow_group_cycles[b] = ctr.shadow_group_cycles[b];
    }
    for (int b = 0; b < 16; b++) {
        stt.trace_entry_cycles[b] = ctr.trace_entry_cycles[b];
        stt.shadow_entry_cycles[b] = ctr.shadow_entry_cycles[b];
    }
    stt.devices = 1;
    s->stats = stt;
    return RTG_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ hooks for rtg_multi.cpp
namespace rtg {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
int scene_device(const rtg_scene* s) { return s->device; }
int scene_render(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* o, float* out_dev, hipStream_t st) {
    return render_impl(s, cam, o, out_dev, st);
}
rtg_render_stats scene_stats(const rtg_scene* s) { return s->stats; }
void scene_set_stats(rtg_scene* s, const rtg_render_stats& st) { s->stats = st; }
MultiState*& scene_multi(rtg_scene* s) { return s->multi; }

// A render-only copy of `src` on `device`: every device buffer copied device to device
// (hipMemcpyPeer), the kernels' view re-pointed.  No host-side structures (introspection) and
// its own render workspace, so one host thread per replica can render concurrently.
int scene_replicate(rtg_scene* src, int device, rtg_scene** out) {
    *out = nullptr;
    rtg_scene* r = new (std::nothrow) rtg_scene();
    if (!r) return fail(RTG_ERR_OOM, "host allocation");
    r->device = device;
    r->replica = true;
    r->num_objects = src->num_objects; r->num_instances = src->num_instances; r->num_vertices = src->num_vertices;
    r->num_emit = src->num_emit;
    r->num_lanes = src->num_lanes;
    r->sv = src->sv;
    const std::vector<DBuf*> from = scene_buffers(src), to = scene_buffers(r);
    int rc = RTG_OK;
    if (hipSetDevice(device) != hipSuccess) rc = fail(RTG_ERR_NO_DEVICE, "replica device");
    for (size_t i = 0; i < from.size() && rc == RTG_OK; i++) {
        const size_t n = from[i]->used;
        rc = to[i]->grow(std::max<size_t>(n, 1));
        if (rc == RTG_OK && n) {
            const hipError_t e = hipMemcpyPeer(to[i]->p, device, from[i]->p, src->device, n);
            if (e != hipSuccess) rc = fail(RTG_ERR_HIP, std::string("scene replica copy: ") + hipGetErrorString(e));
        }
        to[i]->used = n;
    }
    if (rc != RTG_OK) {
        scene_free(r);
        delete r;
        return rc;
    }
    bind_view(r);
    *out = r;
    return RTG_OK;
}
}  // namespace rtg

extern "C" {

int32_t rtg_render_device(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* opts, float* rgb_out_device,
                          void* stream) {
    return guarded([&]() -> int32_t {
        if (!s || !cam || !rgb_out_device) return fail(RTG_ERR_INVALID, "null argument");
        if (s->device < 0) return fail(RTG_ERR_NO_DEVICE, "host-only scene cannot render");
        HIP_TRY(hipSetDevice(s->device));
        if (opts && (opts->num_devices > 1 || opts->devices)) return render_multi(s, cam, opts, rgb_out_device, (hipStream_t)stream);
        return render_impl(s, cam, opts, rgb_out_device, (hipStream_t)stream);
    });
}

int64_t rtg_pass_rays(int32_t num_lights, int32_t path_tracer, int32_t lanes, uint64_t device_bytes) {
    // device bytes per ray of a pass, per level in flight: hit 16 + node records 48 + shadow
    // records 64 and list entry 4 per light + room for two child rays (32 + 16 each) [+ path
    // records 16 for the ray and 32 for its children]; x2 for the level that spawned it
    const double per_ray = 2.0 * (16.0 + 48.0 + 68.0 * std::max(num_lights, 1) + 96.0 + (path_tracer ? 48.0 : 0.0));
    const long long kCap = 24LL << 20, kFloor = 1LL << 16;
    if (device_bytes == 0) return kCap;
    const double budget = 0.5 * (double)device_bytes / (double)std::max(lanes, 1);
    return std::max(kFloor, std::min(kCap, (long long)(budget / per_ray)));
}

int32_t rtg_shard_rows(int32_t ny, int32_t row_offset, int32_t row_stride, int32_t row_block) {
    const int stride = row_stride > 1 ? row_stride : 1, block = row_block > 1 ? row_block : 1;
    if (ny <= 0 || row_offset < 0 || row_offset >= stride) return 0;
    int rows = 0;
    for (long long b = row_offset; b * block < ny; b += stride) rows += (int)std::min<long long>(block, ny - b * block);
    return rows;
}

int32_t rtg_render(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_opts* opts, float* rgb_out) {
    return guarded([&]() -> int32_t {
        if (!s || !cam || !rgb_out) return fail(RTG_ERR_INVALID, "null argument");
        if (cam->nx < 1 || cam->ny < 1) return fail(RTG_ERR_INVALID, "bad camera");
        if (s->device < 0) return fail(RTG_ERR_NO_DEVICE, "host-only scene cannot render");
        HIP_TRY(hipSetDevice(s->device));
        const int out_rows = opts && opts->compact_rows ? rtg_shard_rows(cam->ny, opts->row_offset, opts->row_stride,
                                                                         opts->row_block) : cam->ny;
        size_t bytes = sizeof(float) * 3 * (size_t)cam->nx * std::max(out_rows, 1);
        float* d_out = nullptr;
        HIP_TRY(hipMalloc(&d_out, bytes));
        int rc = (opts && (opts->num_devices > 1 || opts->devices)) ? render_multi(s, cam, opts, d_out, nullptr)
                                                 : render_impl(s, cam, opts, d_out, nullptr);
        if (rc == RTG_OK) {
            hipError_t e = hipMemcpy(rgb_out, d_out, bytes, hipMemcpyDeviceToHost);
            if (e != hipSuccess) rc = fail(RTG_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
        }
        (void)hipFree(d_out);
        return rc;
    });
}

static int check_tonemap(int32_t device, int32_t nx, int32_t ny, const rtg_tonemap_desc* tm) {
    if (!tm) return fail(RTG_ERR_INVALID, "null tonemap descriptor");
    if (tm->tmo != RTG_TMO_PHOTOGRAPHIC) return fail(RTG_ERR_UNSUPPORTED, "tone-mapping operator");
    if (!(tm->gamma > 0.0f) || !(tm->key > 0.0f) || !(tm->burn_percent >= 0.0f) || !(tm->burn_percent <= 100.0f))
        return fail(RTG_ERR_INVALID, "tonemap parameters");
    if (nx < 1 || ny < 1 || (long long)nx * ny > (1LL << 30)) return fail(RTG_ERR_INVALID, "tonemap image size");
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return fail(RTG_ERR_NO_DEVICE, "no such device");
    return RTG_OK;
}

int32_t rtg_tonemap_device(int32_t device, const float* hdr, int32_t nx, int32_t ny, const rtg_tonemap_desc* tm,
                           float* out, void* stream) {
    return guarded([&]() -> int32_t {
        if (!hdr || !out) return fail(RTG_ERR_INVALID, "null argument");
        int rc = check_tonemap(device, nx, ny, tm);
        if (rc) return rc;
        HIP_TRY(hipSetDevice(device));
        std::string err;
        if (tonemap_device(hdr, nx, ny, *tm, out, (hipStream_t)stream, err)) return fail(RTG_ERR_HIP, err);
        return RTG_OK;
    });
}

int32_t rtg_tonemap(int32_t device, const float* hdr, int32_t nx, int32_t ny, const rtg_tonemap_desc* tm, float* out) {
    return guarded([&]() -> int32_t {
        if (!hdr || !out) return fail(RTG_ERR_INVALID, "null argument");
        int rc = check_tonemap(device, nx, ny, tm);
        if (rc) return rc;
        HIP_TRY(hipSetDevice(device));
        const size_t bytes = sizeof(float) * 3 * (size_t)nx * ny;
        float *dh = nullptr, *dl = nullptr;
        if (hipMalloc(&dh, bytes) != hipSuccess || hipMalloc(&dl, bytes) != hipSuccess) {
            if (dh) (void)hipFree(dh);
            return fail(RTG_ERR_OOM, "tonemap buffers");
        }
        std::string err;
        rc = RTG_OK;
        if (hipMemcpy(dh, hdr, bytes, hipMemcpyHostToDevice) != hipSuccess) rc = fail(RTG_ERR_HIP, "tonemap upload");
        else if (tonemap_device(dh, nx, ny, *tm, dl, nullptr, err)) rc = fail(RTG_ERR_HIP, err);
        else if (hipMemcpy(out, dl, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(RTG_ERR_HIP, "tonemap download");
        (void)hipFree(dh);
        (void)hipFree(dl);
        return rc;
    });
}

int32_t rtg_scene_build_stats(const rtg_scene* s, rtg_build_stats* out) {
    if (!s || !out) return fail(RTG_ERR_INVALID, "null argument");
    *out = s->bst;
    out->bvh_build_ms = s->bvh_build_ms;
    out->bvh_gpu_objects = s->bvh_gpu_objects;
    out->num_objects = s->num_objects;
    out->tlas_nodes = s->tlas_count;
    return RTG_OK;
}

int32_t rtg_last_render_stats(const rtg_scene* s, rtg_render_stats* out) {
    if (!s || !out) return fail(RTG_ERR_INVALID, "null argument");
    *out = s->stats;
    return RTG_OK;
}

int32_t rtg_trace_closest(rtg_scene* s, const rtg_ray* rays, int32_t n, rtg_hit* hits, int32_t traversal) {
    return guarded([&]() -> int32_t {
        if (!s || n < 0 || (n && (!rays || !hits))) return fail(RTG_ERR_INVALID, "bad arguments");
        if (n == 0) return RTG_OK;
        if (s->device < 0) return fail(RTG_ERR_NO_DEVICE, "host-only scene cannot trace");
        HIP_TRY(hipSetDevice(s->device));
        // the rays as RayQ planes (with times: API rays may carry any time)
        std::vector<float> rr((size_t)7 * n);
        for (int i = 0; i < n; i++) {
            const rtg_ray& r = rays[i];
            float* a = &rr[(size_t)4 * i];
            float* b = &rr[(size_t)4 * n + 2 * (size_t)i];
            a[0] = r.origin[0]; a[1] = r.origin[1]; a[2] = r.origin[2]; a[3] = r.direction[0];
            b[0] = r.direction[1]; b[1] = r.direction[2];
            rr[(size_t)6 * n + i] = r.time;
        }
        DBuf dr, dh, dout;
        int rc;
        if ((rc = upload(dr, rr)) || (rc = dh.grow(sizeof(HitRec) * (size_t)n)) || (rc = dout.grow(sizeof(rtg_hit) * (size_t)n))) {
            dr.release(); dh.release(); dout.release();
            return rc;
        }
        const RayQ q = ray_planes(dr.p, n, true);
        launch_trace(s->sv, q, dh.as<HitRec>(), n, traversal == 1, nullptr, nullptr);
        launch_hit_details(s->sv, q, dh.as<HitRec>(), dout.as<rtg_hit>(), s->d_origprim.as<int>(), n, nullptr);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpy(hits, dout.p, sizeof(rtg_hit) * (size_t)n, hipMemcpyDeviceToHost);
        dr.release(); dh.release(); dout.release();
        if (e != hipSuccess) return fail(RTG_ERR_HIP, std::string("trace: ") + hipGetErrorString(e));
        return RTG_OK;
    });
}

int32_t rtg_scene_object_bvh(const rtg_scene* s, int32_t object, int32_t* num_prims, int32_t* num_nodes, int32_t* perm,
                             int32_t* nodes, float* boxes) {
    return guarded([&]() -> int32_t {
        if (!s || object < 0 || object >= s->num_objects) return fail(RTG_ERR_INVALID, "object index");
        const ObjBVH& b = s->bvh[object];
        if (num_prims) *num_prims = (int)b.perm.size();
        if (num_nodes) *num_nodes = (int)b.nodes.size();
        if (perm) memcpy(perm, b.perm.data(), sizeof(int) * b.perm.size());
        // pre-order (node, left subtree, right subtree): a GPU-built tree is stored breadth-first
        std::vector<int> order, pre;
        if (b.bfs && !b.nodes.empty()) {
            pre.assign(b.nodes.size(), -1);
            std::vector<int> stk{b.root};
            while (!stk.empty()) {
                const int id = stk.back();
                stk.pop_back();
                pre[id] = (int)order.size();
                order.push_back(id);
                if (b.nodes[id].right >= 0) stk.push_back(b.nodes[id].right);
                if (b.nodes[id].left >= 0) stk.push_back(b.nodes[id].left);
            }
        }
        for (size_t k = 0; k < b.nodes.size(); k++) {
            HNode h = b.nodes[b.bfs ? order[k] : k];
            if (b.bfs) {
                if (h.left >= 0) h.left = pre[h.left];
                if (h.right >= 0) h.right = pre[h.right];
            }
            if (nodes) { nodes[4 * k] = h.left; nodes[4 * k + 1] = h.right; nodes[4 * k + 2] = h.start; nodes[4 * k + 3] = h.end; }
            if (boxes) for (int z = 0; z < 3; z++) { boxes[6 * k + z] = h.mn[z]; boxes[6 * k + 3 + z] = h.mx[z]; }
        }
        return RTG_OK;
    });
}

int32_t rtg_scene_object_matrices(const rtg_scene* s, int32_t top, float* inv16, float* invT16) {
    if (!s || top < 0 || top >= (int)s->inv.size()) return fail(RTG_ERR_INVALID, "object index");
    if (inv16) memcpy(inv16, s->inv[top].c, 64);
    if (invT16) memcpy(invT16, s->invT[top].c, 64);
    return RTG_OK;
}

int32_t rtg_scene_vertex_normals(const rtg_scene* s, float* normals) {
    if (!s || !normals) return fail(RTG_ERR_INVALID, "null argument");
    memcpy(normals, s->vnormals.data(), sizeof(float) * s->vnormals.size());
    return RTG_OK;
}

}  // extern "C"
