// rtg_device.hip — gfx950 kernels of the wavefront render loop.
//
// The reference's recursive per-pixel loop (src/Scene.cpp:148-219, 269-292, 365-411) is
// flattened into levels: raygen -> [trace -> shade -> shadow] per ray-tree level ->
// bottom-up resolve -> in-order sample accumulation.  Every floating-point expression
// follows the reference's evaluation order (compiled with -ffp-contract=off and correctly
// rounded f32 div/sqrt), so hit indices are bit-identical to the oracle and colours agree
// to the transcendental convention documented in oracle/rtg_oracle.c.
#include <float.h>
#include <math.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "rtg_internal.h"

namespace rtg {

#define DEV __device__ __forceinline__
// Traversal occupancy.  Round 1: k_shadow 135 -> 128 VGPRs (3 -> 4 waves/SIMD): 32.6 -> 30.9 ms per
// dragon frame.  Round 3: k_trace / k_shadow at 6 waves per SIMD (80 VGPRs, 16-96 B of spill besides
// the stack's scratch part), possible since the LDS stack holds 16 entries (rtg_internal.h kLdsStack):
// dragon 33.0 -> 31.6 ms, cornell_pt 392.8 -> 364.3 ms (profiles/history/r3_ab_ldsstack.jsonl).
#ifndef RTG_TRAVERSAL_WAVES
#define RTG_TRAVERSAL_WAVES 6
#endif
// the top-level-BVH instantiations (many-entry scenes, LDS also holds their 16-entry top-level
// stack) keep the previous target: spheres 1080p64 37.3 -> 32.3 ms against 6 waves
// (profiles/history/r3_ab_tlaswaves.jsonl)
#ifndef RTG_TLAS_WAVES
#define RTG_TLAS_WAVES 4
#endif
#define RTG_SHADOW_ATTR __attribute__((amdgpu_waves_per_eu(TLAS ? RTG_TLAS_WAVES : RTG_TRAVERSAL_WAVES)))
#define RTG_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(TLAS ? RTG_TLAS_WAVES : RTG_TRAVERSAL_WAVES)))
// Kept traversal / shading shortcuts (each measured and kept): the wave-uniform walk of
// camera-sample waves and their shadow queries, uniform-entry record reads in shading, flat-triangle
// normals from the TriGeom record, entry world boxes, root-box windows, windowed triangle tests and the
// object-light shadow bound.  Experiments measured and not kept were removed in round 5.
// k_shade: the full variant (textures / BRDFs / area & environment lights) needs > 256 registers;
// capped at 2 waves per SIMD it spills 236 B/lane and is still faster (cornell_dynamic 1080p64:
// 34.0 -> 29.7 ms).
// The simple variant (point / directional lights, no textures or BRDFs) at 6 waves per SIMD: 90 -> 80
// VGPRs with an 8-byte spill, dragon k_shade 8.80 -> 7.87 ms per frame (7 waves: 8.6 ms;
// profiles/history/r3_ab_shadewaves.jsonl); the spot variant (182 VGPRs) keeps the minimum of 2.
#ifndef RTG_SHADE_WAVES
#define RTG_SHADE_WAVES 6
#endif
#ifndef RTG_SHADE_FULL_WAVES
#define RTG_SHADE_FULL_WAVES 2
#endif
// Round 4: the full variant without textures / BRDFs and without spot / environment lights
// (SPOT = false, light_sample) needs 105 VGPRs instead of 255; capped at 5 waves per SIMD it fits
// 94 with no spill (cornell_dynamic 1080p64: 16.4 ms/frame at 5 waves, 16.8 at 4 or 3)
#ifndef RTG_SHADE_LIGHT_WAVES
#define RTG_SHADE_LIGHT_WAVES 5
#endif
// Its block size: 512 threads like the simple variant (256 dated from the 2-wave days).  C4
// cornell_dynamic 1080p64, streams=1 frame: k_shade 6.04 -> 5.2 ms (three A/B pairs, same box,
// profiles/history/r5e_ab_light_block.txt); the 8-lane frame is unchanged (16.5 ms), where its shading
// overlaps other lanes' traversals.
constexpr int kShadeLightBlock = 512;
#define RTG_SHADE_ATTR __attribute__((amdgpu_waves_per_eu(FULL ? (!SPOT && !TEX ? RTG_SHADE_LIGHT_WAVES : RTG_SHADE_FULL_WAVES) \
                                                            : SPOT ? 2 : RTG_SHADE_WAVES)))
// k_pt_shade: the simple / BRDF-only variants at 3 waves per SIMD (192 -> 168 VGPRs, 64 B/lane
// spill): cornell_pt 1080p256 585 -> 576 ms; 4 waves (236 B spill) is slower (594 ms); round 3, with
// one BRDF call site (167 VGPRs, no spill at 3 waves): 4 waves spill 140-164 B and lose, 398 -> 404
// ms (profiles/history/r3_ab_ptwaves.jsonl); the full variants keep the default
#ifndef RTG_PT_WAVES
#define RTG_PT_WAVES 3
#endif
// BRDF-only variants without Torrance-Sparrow models (round 4): 143 VGPRs uncapped
#ifndef RTG_PT_WAVES_NOTS
#define RTG_PT_WAVES_NOTS 3
#endif
#define RTG_PT_SHADE_ATTR __attribute__((amdgpu_waves_per_eu((!FULL && !SPOT) ? (BRDF == 1 ? RTG_PT_WAVES_NOTS : RTG_PT_WAVES) : 1)))
constexpr int kPtBlock = 256;      // k_pt_shade threads per block (128 / 64: slower, r3_ab_ptblock.jsonl)
constexpr double PI_D = 3.14159265358979323846;

// ------------------------------------------------------------------ vectors (Eigen order)
struct f3 { float x, y, z; };
DEV f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
DEV f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
DEV f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
DEV f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
DEV f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
DEV f3 operator/(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
DEV f3 cw(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
DEV float dot(f3 a, f3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
DEV float sqn(f3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
DEV float norm(f3 a) { return sqrtf(sqn(a)); }
DEV f3 normalized(f3 a) {
    float z = sqn(a);
    if (z > 0.0f) return a / sqrtf(z);
    return a;
}
DEV f3 cross(f3 a, f3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DEV bool isnan3(f3 a) { return a.x != a.x || a.y != a.y || a.z != a.z; }
DEV f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
DEV float fmax0(float x) { return (0.0f < x) ? x : 0.0f; }
DEV float stdmin(float a, float b) { return (b < a) ? b : a; }
DEV float vget(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// transcendental convention: (float) of the double-precision function
DEV float f_acos(float x) { return (float)acos((double)x); }
DEV float f_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
DEV float f_cos(float x) { return (float)cos((double)x); }
DEV float f_sin(float x) { return (float)sin((double)x); }
// (float)cos((double)x) and (float)sin((double)x) with one argument reduction (ocml's sin, cos and
// sincos share it; the path tracer's two uniform-angle samples per vertex)
DEV void f_sincos(float x, float& s, float& c) {
    double sd, cd;
    sincos((double)x, &sd, &cd);
    s = (float)sd;
    c = (float)cd;
}
DEV float f_exp(float x) { return (float)exp((double)x); }
// std::pow(float, int) == (float)pow(double, double).  Integer exponent by binary powering in
// double: within ~log2(n) double ulps of the exact power, so the float result is the
// correctly rounded one except within ~1e-15 of a float rounding boundary.
DEV float f_powi(float x, int n) {
    if (n == 0) return 1.0f;
    double b = (double)x, r = 1.0;
    unsigned e = n < 0 ? 0u - (unsigned)n : (unsigned)n;
    while (e) {
        if (e & 1u) r *= b;
        e >>= 1;
        if (e) b *= b;
    }
    return (float)(n < 0 ? 1.0 / r : r);
}
// pow(double(f), 2.0): the square of a float is exact in double
DEV double sq_d(float x) { const double d = (double)x; return d * d; }

// glm mat4 (column-major) * (v, w): (c0*x + c1*y) + (c2*z + c3*w)
DEV f3 xform(const float* m, f3 v, float w) {
    float r[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float add0 = m[0 * 4 + i] * v.x + m[1 * 4 + i] * v.y;
        float add1 = m[2 * 4 + i] * v.z + m[3 * 4 + i] * w;
        r[i] = add0 + add1;
    }
    return mk(r[0], r[1], r[2]);
}

// ------------------------------------------------------------------ Philox4x32-10
enum { RNG_CAMERA = 1, RNG_ROUGH = 2, RNG_AREA = 3, RNG_ENV = 4, RNG_PT_BOUNCE = 5, RNG_PT_EMIT = 6 };
DEV void rng4(uint64_t seed, uint32_t pixel, uint32_t sample, uint64_t path, uint32_t purpose, uint32_t light,
              uint32_t iter, float out[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ (uint32_t)(path >> 32);
    uint32_t c0 = pixel, c1 = sample, c2 = (uint32_t)path;
    uint32_t c3 = (purpose << 28) | ((light & 0xFFFu) << 16) | (iter & 0xFFFFu);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    uint32_t c[4] = {c0, c1, c2, c3};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float f = (float)c[i] / 4294967296.0f;
        out[i] = (f >= 1.0f) ? 0x1.fffffep-1f : f;
    }
}

// ------------------------------------------------------------------ BVH helpers (src/BVH.cpp)
DEV float min3(float a, float b, float c) {
    if (a <= b && a <= c) return a;
    else if (b <= a && b <= c) return b;
    return c;
}
DEV float max3(float a, float b, float c) {
    if (a >= b && a >= c) return a;
    else if (b >= a && b >= c) return b;
    return c;
}
// BVH::RayBBoxIntersection, src/BVH.cpp:212-266 (exact divisions: it decides reachability)
DEV bool box_test(f3 o, f3 d, float mnx, float mny, float mnz, float mxx, float mxy, float mxz) {
    float txe, txl, tye, tyl, tze, tzl;
    if (d.x > 0) { txe = (mnx - o.x) / d.x; txl = (mxx - o.x) / d.x; }
    else { txe = (mxx - o.x) / d.x; txl = (mnx - o.x) / d.x; }
    if (d.y > 0) { tye = (mny - o.y) / d.y; tyl = (mxy - o.y) / d.y; }
    else { tye = (mxy - o.y) / d.y; tyl = (mny - o.y) / d.y; }
    if (d.z > 0) { tze = (mnz - o.z) / d.z; tzl = (mxz - o.z) / d.z; }
    else { tze = (mxz - o.z) / d.z; tzl = (mnz - o.z) / d.z; }
    float sl = min3(txl, tyl, tzl);
    float le = max3(txe, tye, tze);
    return !(sl < le);
}
// Same predicate, decided with reciprocal multiplies when that is provably safe.
// q = fl(fl(b-o) * fl(1/d)) is within 3 ulp of the exact t = fl(fl(b-o)/d), so the min3/max3
// of either set differ by < 2^-21 (|sl|+|le|); outside that band the fast answer equals the
// exact one, inside it (and whenever 1/d is not finite: d = +-0, denormal d) the exact
// division test decides.  NaN cannot arise on the fast path (all operands finite).
DEV bool box_hit(f3 o, f3 d, f3 inv, bool fast_ok, float mnx, float mny, float mnz, float mxx, float mxy, float mxz) {
    if (fast_ok) {
        float ax = (mnx - o.x) * inv.x, bx = (mxx - o.x) * inv.x;
        float ay = (mny - o.y) * inv.y, by = (mxy - o.y) * inv.y;
        float az = (mnz - o.z) * inv.z, bz = (mxz - o.z) * inv.z;
        float sl = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
        float le = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
        float e = (fabsf(sl) + fabsf(le)) * 9.5367431640625e-7f;   // 2^-20
        if (sl < le - e) return false;
        if (sl >= le + e) return true;
    }
    return box_test(o, d, mnx, mny, mnz, mxx, mxy, mxz);
}
// Window pruning of one (already padded) box, the traversal's slot test without the reachability
// part: false when the box meets the line only outside [tlo, thi].  Reciprocal slabs with
// the 2^-20 band of box_hit; a NaN from overflowing terms compares false (box kept).
DEV bool window_meets(f3 o, f3 inv, float mnx, float mny, float mnz, float mxx, float mxy, float mxz, float tlo,
                      float thi) {
    const float ax = (mnx - o.x) * inv.x, bx = (mxx - o.x) * inv.x;
    const float ay = (mny - o.y) * inv.y, by = (mxy - o.y) * inv.y;
    const float az = (mnz - o.z) * inv.z, bz = (mxz - o.z) * inv.z;
    const float sl = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    const float le = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float e = (fabsf(sl) + fabsf(le)) * 9.5367431640625e-7f;   // 2^-20
    const float lo = le - e, hi = sl + e;
    return !(hi < lo || hi < tlo || lo > thi);
}
// Squared Euclidean distance from o to the box (pruning / ordering only).
DEV float box_dist2(f3 o, float mnx, float mny, float mnz, float mxx, float mxy, float mxz) {
    float dx = fmaxf(fmaxf(mnx - o.x, o.x - mxx), 0.0f);
    float dy = fmaxf(fmaxf(mny - o.y, o.y - mxy), 0.0f);
    float dz = fmaxf(fmaxf(mnz - o.z, o.z - mxz), 0.0f);
    return dx * dx + dy * dy + dz * dz;
}
// Subtrees whose squared box distance exceeds this can hold no candidate at distance <= bound:
// candidates lie within `pad` of their primitive's box; margins cover rounding of p = o+d*t,
// of |p-o| and of the squared distance itself.
DEV float prune_threshold2(float bound, float pad, float oabs) {
    if (!(bound < FLT_MAX)) return INFINITY;
    float r = (bound + pad) * (1.0f + 1e-5f) + 1e-6f * (oabs + bound) + 1e-30f;
    return r * r * (1.0f + 1e-5f);
}
// Eigen 3x3 determinant (row-0 expansion) of the matrix with columns c0, c1, c2
DEV float det3(f3 c0, f3 c1, f3 c2) {
    float h0 = c0.x * (c1.y * c2.z - c1.z * c2.y);
    float h1 = c1.x * (c0.y * c2.z - c0.z * c2.y);
    float h2 = c2.x * (c0.y * c1.z - c0.z * c1.y);
    return (h0 - h1) + h2;
}

struct Cand {           // Triangle::bvhIntersect acceptance + point (src/Shape.cpp:297-345)
    bool ok;
    float beta, gamma, t;
    f3 p;
};
// Fast rejection of Triangle::bvhIntersect's acceptance (src/Shape.cpp:297-345): quotients formed with
// v_rcp_f32 (1 ulp) lie within 2^-21 (relative) of the correctly rounded ones, so a quotient that misses
// the acceptance bounds by more than 2^-20 of its magnitude is rejected by the exact test too.  Only
// for fastq (det within [1e-30, 1e30]); a non-finite operand compares false (not rejected).
// thi (the caller's parameter window, round 4's windowed test): a candidate whose t lies beyond it cannot
// become the object's winner that matters -- the same bound the traversal's slot boxes are pruned
// with (visit_object) -- so it may be rejected as well; INFINITY keeps every candidate.
DEV bool tri_reject_t(float nt, float r, float eps, float thi) {
    const float m = 9.5367431640625e-7f;   // 2^-20
    const float tq = nt * r;
    return tq < (-eps - fabsf(tq) * m) - 1e-37f || tq > (thi + fabsf(tq) * m) + 1e-37f;
}
DEV bool tri_reject_bary(float nb, float ng, float r, float eps) {
    const float m = 9.5367431640625e-7f;
    const float bq = nb * r, gq = ng * r;
    return bq < (-eps - fabsf(bq) * m) - 1e-37f || gq < (-eps - fabsf(gq) * m) - 1e-37f ||
           bq + gq > (1.0f + (fabsf(bq) + fabsf(gq)) * (2.0f * m)) + m;
}
DEV Cand tri_test(const TriGeom& g, f3 o, f3 d, float eps, float thi = INFINITY) {
    f3 a = mk(g.p0.x, g.p0.y, g.p0.z);
    f3 amb = mk(g.p0.w, g.p1.x, g.p1.y);
    f3 amc = mk(g.p1.z, g.p1.w, g.p2.x);
    f3 amo = a - o;
    Cand c;
    float det = det3(amb, amc, d);
    float nt = det3(amb, amc, amo);
    // The fast rejection (above) where det allows it, the exact divisions otherwise.  The ray
    // parameter is tested first, against [-eps, thi]: a candidate behind the origin or beyond the
    // window costs two determinants, not four (round 4).
    const float ad = fabsf(det);
    const bool fastq = ad >= 1e-30f && ad <= 1e30f;
    const float r = __builtin_amdgcn_rcpf(det);
    if (fastq && tri_reject_t(nt, r, eps, thi)) {
        c.ok = false;
        c.beta = c.gamma = c.t = 0.0f;
        c.p = o;
        return c;
    }
    float nb = det3(amo, amc, d), ng = det3(amb, amo, d);
    if (fastq && tri_reject_bary(nb, ng, r, eps)) {
        c.ok = false;
        c.beta = c.gamma = c.t = 0.0f;
        c.p = o;
        return c;
    }
    c.beta = nb / det;
    c.gamma = ng / det;
    c.t = nt / det;
    c.ok = (c.t >= -eps && (c.beta + c.gamma <= 1) && c.beta >= -eps && c.gamma >= -eps);
    c.p = o + d * c.t;
    return c;
}
// tri_test's fast rejection alone: false only when tri_test(g, o, d, eps, thi) would reject.
DEV bool tri_maybe(const TriGeom& g, f3 o, f3 d, float eps, float thi) {
    const f3 a = mk(g.p0.x, g.p0.y, g.p0.z);
    const f3 amb = mk(g.p0.w, g.p1.x, g.p1.y);
    const f3 amc = mk(g.p1.z, g.p1.w, g.p2.x);
    const f3 amo = a - o;
    const float det = det3(amb, amc, d);
    const float ad = fabsf(det);
    if (!(ad >= 1e-30f && ad <= 1e30f)) return true;
    const float r = __builtin_amdgcn_rcpf(det);
    if (tri_reject_t(det3(amb, amc, amo), r, eps, thi)) return false;
    return !tri_reject_bary(det3(amo, amc, d), det3(amb, amo, d), r, eps);
}
// Sphere::bvhIntersect root selection (src/Shape.cpp:347-391)
DEV bool sphere_test(f3 o, f3 d, f3 c, float R, float eps, f3& ip) {
    f3 oc = o - c;
    float dd = dot(d, oc);
    float disc = dd * dd - dot(d, d) * (dot(oc, oc) - R * R);
    if (disc < eps) return false;
    float sq = sqrtf(disc);
    float t1 = (-dd + sq) / dot(d, d);
    float t2 = (-dd - sq) / dot(d, d);
    if (t1 >= 0 && t2 < 0) ip = o + d * t1;
    else if (t2 >= 0 && t1 < 0) ip = o + d * t2;
    else if (t1 < 0 && t2 < 0) return false;
    else ip = (t1 < t2) ? (o + d * t1) : (o + d * t2);
    return true;
}
// Ray::gett (src/Ray.cpp:21-36)
DEV float gett(f3 o, f3 d, f3 p) {
    float t = (p.x - o.x) / d.x;
    if (t == t) return t;
    t = (p.y - o.y) / d.y;
    if (t == t) return t;
    t = (p.z - o.z) / d.z;
    return t;
}
// Transforming::TransformRay (src/Helper.cpp:110-133)
// fin: every component of o, d and time is finite (ray_finite), computed once per ray -- as seven
// separate tests the compiler hoisted them out of the object loop as seven lane masks, and the
// SGPRs they held were spilled in k_shadow / k_trace.
DEV bool ray_finite(f3 o, f3 d, float time) {
    const float s = (((o.x * 0.0f + o.y * 0.0f) + (o.z * 0.0f + d.x * 0.0f)) + (d.y * 0.0f + d.z * 0.0f)) + time * 0.0f;
    return s == 0.0f;       // x * 0 is NaN exactly for x = +-inf or NaN
}
// strict: only the +0 identity (ident == 1) returns the ray -- hit_record, whose sphere texture
// coordinates (atan2) and normals see the signs of zeros; the traversal also takes ident == 2 (the
// identity up to zero signs, rtg_host.cpp), whose outcomes depend on values only.
DEV void transform_ray(const TopObject& T, f3 o, f3 d, float time, f3& o2, f3& d2, bool fin, bool strict = false) {
    if ((strict ? T.ident == 1 : T.ident != 0) && fin) {
        // identity inverse, +0 blur: (x*1 + y*0) + (z*0 + w*0) == x + 0 for finite inputs
        // (the only effect is -0 -> +0)
        o2 = mk(o.x + 0.0f, o.y + 0.0f, o.z + 0.0f);
        d2 = mk(d.x + 0.0f, d.y + 0.0f, d.z + 0.0f);
        return;
    }
    f3 b = mk(T.blur[0] * time, T.blur[1] * time, T.blur[2] * time);
    f3 oo = o;
    oo.x -= b.x; oo.y -= b.y; oo.z -= b.z;
    o2 = xform(T.inv, oo, 1.0f);
    d2 = xform(T.inv, d, 0.0f);
}

// steps: node steps of this lane (the wave runs the max over its lanes)
// entries: top-level entries this lane visited (entry-start code: ray transform, root test, ...);
// considered: entries the lane's loop went through (the wave runs each for all its lanes)
// cand_step: node steps taken when the current object's best candidate was accepted; win_step: the
// same for the query's final winner (the steps after it only prove that it is the nearest)
// gwork: the flat group's triangle tests this lane ran (fast rejections + its own exact tests); gslot:
// the group triangle tests its wave ran while the lane was in the group (the wave runs the max)
struct Stats { unsigned nodes, tris, steps, entries, considered, cand_step, win_step, gwork, gslot; };

// ------------------------------------------------------------------ closest hit
// BVHMethods::FindIntersection (src/Helper.cpp:18-80) with the per-object nearest
// candidate of BVH::FindIntersectionWithBVH (src/BVH.cpp:137-210).  The reference visits
// both children of every node whose box the infinite line crosses; its result is the
// candidate of minimal Euclidean distance, ties -> rightmost leaf, then lowest index in
// the leaf.  This ordered traversal computes the same total order and prunes subtrees
// whose distance lower bound exceeds the current best (EXHAUSTIVE disables pruning).
// `tmax`: hits with gett() >= tmax are irrelevant to the caller (shadow queries).
// TLAS: the entries are enumerated by the top-level BVH (near first, world boxes that cannot hold
// an accepted hit at t <= nearest skipped) instead of the reference's linear loop; an entry
// replaces the winner iff t < nearest, or t == nearest and it comes earlier in the loop order
// (objects before instances, lower index first), which is the loop's first-wins rule.

// One top-level entry of BVHMethods::FindIntersection's loop (src/Helper.cpp:32-73): the object's
// winner (closest_hit's comments) and the top-level acceptance against `nearest` / `out`.
// Traversal stack entry sp of a lane: LDS for the first kLdsStack entries, the lane's scratch array
// beyond (kLdsStack < kStackDepth builds only: a smaller LDS stack for more waves per CU).
DEV void stk_put(int* stack, int sstride, int* spill, int sp, int v) {
    if (kLdsStack >= kStackDepth || sp < kLdsStack) stack[sp * sstride] = v;
    else spill[sp - kLdsStack] = v;
}
DEV int stk_get(const int* stack, int sstride, const int* spill, int sp) {
    return (kLdsStack >= kStackDepth || sp < kLdsStack) ? stack[sp * sstride] : spill[sp - kLdsStack];
}

template <bool EXHAUSTIVE, bool STATS, bool UNI = false>
DEV void visit_object(const SceneView& sv, const int i, const f3 o, const f3 d, const float time, const bool fin,
                      float& nearest, HitRec& out, int* stack, int sstride, Stats& st, int* spill, const bool uni = false) {
    const float eps = sv.int_eps;
    const TopObject& T = sv.tops[i];
    const Geometry& g = sv.geoms[T.geom];
    f3 o2, d2;
    transform_ray(T, o, d, time, o2, d2, fin);
    bool found = false;
    int bprim = -1;
    f3 bp = mk(0, 0, 0);
    if (T.kind == 0) {            // a sphere: its test data by entry index (SphereEnt)
        const SphereEnt& S = sv.tsph[i];
        if (S.prim >= 0) {
            f3 ip;
            if (sphere_test(o2, d2, mk(S.c.x, S.c.y, S.c.z), S.c.w, eps, ip)) {
                float dist = norm(ip - o2);
                if (dist < FLT_MAX) { found = true; bprim = S.prim; bp = ip; if (STATS) st.cand_step = st.steps; }
            }
        }
    } else {
        // Reciprocal direction for the fast slab test (v_rcp_f32, 1 ulp: the 2^-20 margin of
        // child() covers it).  Components outside [1e-30, 1e30] (zero, denormal, huge, NaN)
        // send every box to the exact division test instead.
        const float adx = fabsf(d2.x), ady = fabsf(d2.y), adz = fabsf(d2.z);
        const bool fast = adx >= 1e-30f && adx <= 1e30f && ady >= 1e-30f && ady <= 1e30f && adz >= 1e-30f &&
                          adz <= 1e30f;
        const f3 inv = mk(__builtin_amdgcn_rcpf(d2.x), __builtin_amdgcn_rcpf(d2.y), __builtin_amdgcn_rcpf(d2.z));
        // the root box first: an object whose root the line misses costs no further setup
        // (small scenes are dominated by the reference's linear loop over objects)
        const bool root_ok = g.node_base < 0 ? g.root_leaf_count > 0
                           : box_hit(o2, d2, inv, fast, g.root_min[0], g.root_min[1], g.root_min[2], g.root_max[0],
                                     g.root_max[1], g.root_max[2]);
        if (!root_ok) return;
        // distance bound from the best hit so far (see DESIGN.md "pruning")
        float boundD = FLT_MAX;
        const float da = d2.x != 0.0f ? d2.x : (d2.y != 0.0f ? d2.y : d2.z);
        const float oa = d2.x != 0.0f ? o2.x : (d2.y != 0.0f ? o2.y : o2.z);
        // (bounds only: 1-ulp v_sqrt / v_rcp, inside the 1e-5 / 2e-5 margins)
        const float dnorm = __builtin_amdgcn_sqrtf(d2.x * d2.x + d2.y * d2.y + d2.z * d2.z);
        if (!EXHAUSTIVE && nearest < FLT_MAX) {
            const float dl = dnorm;
            if (da != 0.0f) {
                float tm = (nearest + 4.0f * 5.96e-8f * fabsf(oa) * __builtin_amdgcn_rcpf(fabsf(da))) * (1.0f + 1e-5f);
                boundD = tm * dl * (1.0f + 2e-5f) + 1e-30f;
                if (!(boundD == boundD)) boundD = FLT_MAX;
            }
        }
        const float pad = g.prune_pad;
        float best_d = FLT_MAX;
        int best_leaf = -1;
        // Parameter window that can hold a useful candidate: t >= -eps (Triangle::bvhIntersect
        // acceptance) and t <= min(tm, best_d/|d'|) (farther hits cannot win).  A subtree is
        // skipped when its box, expanded by `pad`, meets the line only outside that window.
        const float padt = fast ? (pad * fmaxf(fmaxf(fabsf(inv.x), fabsf(inv.y)), fabsf(inv.z))) * 1.0001f : 0.0f;
        const float tlo = -(fabsf(eps) + 1e-6f);
        const float inv_dn = __builtin_amdgcn_rcpf(dnorm);   // 1 ulp: inside the 2e-5 margins of thi
        float thi = INFINITY;
        if (!EXHAUSTIVE && boundD < FLT_MAX) thi = boundD * inv_dn * (1.0f + 2e-5f) + 1e-30f;
        const float thi0 = thi;     // thi never exceeds the window of the best hit so far
        // The root box, widened by the eps overhang (win_*), meets the line only outside the window:
        // no candidate of this object can matter (behind the origin, or beyond the winner so far /
        // the shadow query's bound), so the walk would prune every slot of its first node.
        if (!EXHAUSTIVE && fast && g.win &&
            !window_meets(o2, inv, g.win_min[0], g.win_min[1], g.win_min[2], g.win_max[0], g.win_max[1], g.win_max[2],
                          tlo, thi))
            return;
        // all primitives of one leaf, ties -> rightmost leaf (larger start), then lower index
        auto test_prim = [&](const TriGeom& tg, int k, int start) {
            if (STATS) st.tris++;
            Cand c = tri_test(tg, o2, d2, eps, thi);
            if (c.ok) {
                float dist = norm(c.p - o2);
                if (dist < FLT_MAX &&
                    (dist < best_d || (dist == best_d && (start > best_leaf || (start == best_leaf && k < bprim))))) {
                    best_d = dist; best_leaf = start; bprim = k; found = true; bp = c.p;
                    if (STATS) st.cand_step = st.steps;
                    if (!EXHAUSTIVE) thi = fminf(thi0, best_d * inv_dn * (1.0f + 2e-5f) + 1e-30f);
                }
            }
        };
        // a traversal-tree triangle (stris): its reference position and leaf in p2.y / p2.z; a gated one
        // (p2.w) is accepted as the object's winner only if the reference walk reaches it (§4 "gate")
        auto test_sah = [&](const TriGeom& tg) {
            if (STATS) st.tris++;
            Cand c = tri_test(tg, o2, d2, eps, thi);
            if (!c.ok) return;
            const float dist = norm(c.p - o2);
            const int k = __float_as_int(tg.p2.y), start = __float_as_int(tg.p2.z);
            if (!(dist < FLT_MAX &&
                  (dist < best_d || (dist == best_d && (start > best_leaf || (start == best_leaf && k < bprim))))))
                return;
            if (__float_as_int(tg.p2.w)) {          // src/BVH.cpp:178 on the leaf's parent
                const float* gb = sv.gates + 6 * (size_t)k;
                if (!box_hit(o2, d2, inv, fast, gb[0], gb[1], gb[2], gb[3], gb[4], gb[5])) return;
            }
            best_d = dist; best_leaf = start; bprim = k; found = true; bp = c.p;
            if (STATS) st.cand_step = st.steps;
            if (!EXHAUSTIVE) thi = fminf(thi0, best_d * inv_dn * (1.0f + 2e-5f) + 1e-30f);
        };
        // Flat meshes (<= kFlatMaxPrims triangles tested without a node, round 3): the loop over them is
        // wave-uniform, so a triangle's exact test (three correctly rounded divisions, the distance, the
        // tie rule) ran whenever ANY lane of the wave needed it -- for bounce rays in a room, every
        // triangle of every wall.  Round 5: first the fast rejection of every triangle for every lane
        // (tri_maybe: straight-line, all lanes active), then each lane runs the full test on its own
        // candidates only (usually the one triangle it hits).  The winner is the minimum of a total
        // order, so testing a lane's candidates in index order with the window shrinking between them
        // gives the same result as testing them all.  split < 0: the one-node traversal tree's records
        // (stris); split >= 0: a reference root over two leaves (tris[first, split), [split, end)).
        auto flat_mesh = [&](const TriGeom* recs, const int split) {
            const int first = g.flat_first, count = g.flat_count;
            unsigned cand = 0;
            for (int j = 0; j < count; j++)
                if (tri_maybe(recs[first + j], o2, d2, eps, thi)) cand |= 1u << j;
            while (cand) {
                const int j = __builtin_ctz(cand);
                cand &= cand - 1;
                const int k = first + j;
                if (split < 0) test_sah(recs[k]);
                else test_prim(recs[k], k, k < split ? first : split);
            }
        };
        // one child box: reachability (interior, exact predicate) + window pruning + entry key
        auto child = [&](float mnx, float mny, float mnz, float mxx, float mxy, float mxz, bool interior,
                         float& key) -> bool {
            key = 0.0f;
            if (!EXHAUSTIVE && fast) {
                float ax = (mnx - o2.x) * inv.x, bx = (mxx - o2.x) * inv.x;
                float ay = (mny - o2.y) * inv.y, by = (mxy - o2.y) * inv.y;
                float az = (mnz - o2.z) * inv.z, bz = (mxz - o2.z) * inv.z;
                float sl = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
                float le = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
                float e = (fabsf(sl) + fabsf(le)) * 9.5367431640625e-7f;   // 2^-20
                float lo = le - e - padt, hi = sl + e + padt;
                key = lo;
                if (hi < lo || hi < tlo || lo > thi) return false;
                if (!interior) return true;
                if (sl < le - e) return false;
                if (sl >= le + e) return true;
                return box_test(o2, d2, mnx, mny, mnz, mxx, mxy, mxz);
            }
            if (!interior) return true;
            return box_test(o2, d2, mnx, mny, mnz, mxx, mxy, mxz);
        };
        if (g.node_base < 0) {
            for (int k = g.root_leaf_start; k < g.root_leaf_start + g.root_leaf_count; k++)
                test_prim(sv.tris[k], k, g.root_leaf_start);
        } else {                // root box already hit (root_ok)
            // Leaf children are resolved as soon as they are reached.
            auto leaf = [&](int start, int count) {
                for (int k = start; k < start + count; k++) test_prim(sv.tris[k], k, start);
            };
            // BVH2 walk (ordered, pruned): the reference tree node by node.
            auto walk2 = [&]() {
                int sp = 0;
                int cur = g.node_base;
                while (true) {
                    if (STATS) { st.nodes += 2; st.steps++; }   // one 64-B node = two 32-B child records
                    const Node nd = sv.nodes[cur];
                    const int lref = nd.d.x, rref = nd.d.y, lcnt = nd.d.z, rcnt = nd.d.w;
                    float lk = 0.0f, rk = 0.0f;
                    bool lok = lcnt >= 0 && child(nd.a.x, nd.a.y, nd.a.z, nd.a.w, nd.b.x, nd.b.y, lcnt == 0, lk);
                    bool rok = rcnt >= 0 && child(nd.b.z, nd.b.w, nd.c.x, nd.c.y, nd.c.z, nd.c.w, rcnt == 0, rk);
                    bool lleaf = lok && lcnt > 0, rleaf = rok && rcnt > 0;
                    if (lleaf && rleaf && rk < lk) {
                        leaf(rref, rcnt);
                        if (EXHAUSTIVE || !(lk > thi)) leaf(lref, lcnt);
                        lok = rok = false;
                    } else {
                        if (lleaf) { leaf(lref, lcnt); lok = false; }
                        if (rleaf) {
                            if (EXHAUSTIVE || !(rk > thi)) leaf(rref, rcnt);
                            rok = false;
                        }
                    }
                    if (!EXHAUSTIVE) {
                        lok = lok && !(lk > thi);
                        rok = rok && !(rk > thi);
                    }
                    if (lok && rok) {
                        int nearc = lref, farc = rref;
                        if (rk < lk) { nearc = rref; farc = lref; }
                        stk_put(stack, sstride, spill, sp, farc);
                        sp++;
                        cur = nearc;
                    } else if (lok) {
                        cur = lref;
                    } else if (rok) {
                        cur = rref;
                    } else {
                        if (sp == 0) break;
                        sp--;
                        cur = stk_get(stack, sstride, spill, sp);
                    }
                }
            };
            // Fast rays walk the mesh's traversal tree (SAH, 4-wide; rtg_host.cpp): slots are
            // pruned by the parameter window only (boxes widened by the eps overhang), leaves are
            // tested nearer-first as they are reached, interior slots visited nearest-first.  A
            // candidate that would become the object's winner must be reachable in the
            // reference tree: its reference leaf's parent box (the only ancestor box that can
            // fail when the candidate lies outside its triangle) gets the exact slab test.
            // Exhaustive traversal, rays with a zero / denormal / huge direction component and
            // a stack that would overflow (> kStackDepth entries) use the reference tree's BVH2
            // walk; candidates already accepted stay valid (they are reachable).
            bool use2 = EXHAUSTIVE || !fast || g.sah_base < 0;
            if (!use2) {
                int sp = 0;
                int cur = g.sah_base;
                // a one-node tree of a few triangles: test them all instead of loading the node (the
                // winner is the minimum of a total order, so testing candidates the slot boxes would
                // have skipped changes nothing: they lie outside the window and lose either here or
                // at the object-level t < nearest)
                if (g.flat_count > 0) {             // (flat_split < 0 here: sah_base >= 0)
                    flat_mesh(sv.stris, -1);
                } else if (UNI && uni) {
                    // Wave-uniform walk (coherent waves: a pixel's camera samples).  The wave visits a
                    // node when any of its lanes needs it; node, triangle and stack values are
                    // uniform, so they come through the scalar cache instead of 64 identical vector
                    // gathers.  Each lane still prunes by its own window and accepts by its own test,
                    // so it sees a superset of its own walk's candidates, every one of which is a
                    // valid candidate: the winner, the minimum of a total order, is unchanged.
                    while (true) {
                        cur = __builtin_amdgcn_readfirstlane(cur);
                        if (STATS) { st.nodes += 4; st.steps++; }
                        const Node4 nd = sv.snodes[cur];
                        const float lx[4] = {nd.lox.x, nd.lox.y, nd.lox.z, nd.lox.w};
                        const float ly[4] = {nd.loy.x, nd.loy.y, nd.loy.z, nd.loy.w};
                        const float lz[4] = {nd.loz.x, nd.loz.y, nd.loz.z, nd.loz.w};
                        const float hx[4] = {nd.hix.x, nd.hix.y, nd.hix.z, nd.hix.w};
                        const float hy[4] = {nd.hiy.x, nd.hiy.y, nd.hiy.z, nd.hiy.w};
                        const float hz[4] = {nd.hiz.x, nd.hiz.y, nd.hiz.z, nd.hiz.w};
                        const int rf[4] = {nd.ref.x, nd.ref.y, nd.ref.z, nd.ref.w};
                        const int inf[4] = {nd.info.x, nd.info.y, nd.info.z, nd.info.w};
                        float key[4];
                        int okm = 0;
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const float ax = (lx[j] - o2.x) * inv.x, bx = (hx[j] - o2.x) * inv.x;
                            const float ay = (ly[j] - o2.y) * inv.y, by = (hy[j] - o2.y) * inv.y;
                            const float az = (lz[j] - o2.z) * inv.z, bz = (hz[j] - o2.z) * inv.z;
                            const float sl = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
                            const float le = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
                            const float e = (fabsf(sl) + fabsf(le)) * 9.5367431640625e-7f;   // 2^-20
                            const float lo = le - e, hi = sl + e;
                            key[j] = lo;
                            okm |= (inf[j] >= 0 && !(hi < lo || hi < tlo || lo > thi)) << j;
                        }
                        // leaf slots any lane still needs, each lane testing only its own
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            if (inf[j] <= 0) continue;
                            const bool mine = ((okm >> j) & 1) && !(key[j] > thi);
                            if (__ballot(mine) == 0ull) continue;
                            if (mine)
                                for (int q = rf[j]; q < rf[j] + inf[j]; q++) test_sah(sv.stris[q]);
                        }
                        // interior slots any lane needs, in the first such lane's near-first order
                        float k4[4];
                        int r4[4];
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const bool take = inf[j] == 0 && ((okm >> j) & 1) && !(key[j] > thi);
                            const bool any = __ballot(take) != 0ull;
                            const unsigned long long tm = __ballot(take);
                            const float kf = take ? key[j] : INFINITY;
                            const int lead = any ? (int)__builtin_ctzll(tm) : 0;
                            k4[j] = any ? __shfl(kf, lead) : INFINITY;
                            r4[j] = any ? rf[j] : -1;
                        }
                        auto ce = [&](int a, int b) {
                            const bool sw = k4[b] < k4[a];
                            const float ka = k4[a], kb = k4[b];
                            const int ra = r4[a], rb = r4[b];
                            k4[a] = sw ? kb : ka; k4[b] = sw ? ka : kb;
                            r4[a] = sw ? rb : ra; r4[b] = sw ? ra : rb;
                        };
                        ce(0, 1); ce(2, 3); ce(0, 2); ce(1, 3); ce(1, 2);
                        const int npush = (r4[1] >= 0) + (r4[2] >= 0) + (r4[3] >= 0);
                        if (sp + npush > kStackDepth) { use2 = true; break; }
                        for (int j = 3; j >= 1; j--)
                            if (r4[j] >= 0) { stk_put(stack, sstride, spill, sp, r4[j]); sp++; }
                        if (r4[0] >= 0) {
                            cur = r4[0];
                        } else {
                            if (sp == 0) break;
                            sp--;
                            cur = stk_get(stack, sstride, spill, sp);
                        }
                    }
                } else
                while (true) {
                    if (STATS) { st.nodes += 4; st.steps++; }   // one node = four 32-B child records (the model's unit)
                    const Node4 nd = sv.snodes[cur];
                    const float lx[4] = {nd.lox.x, nd.lox.y, nd.lox.z, nd.lox.w};
                    const float ly[4] = {nd.loy.x, nd.loy.y, nd.loy.z, nd.loy.w};
                    const float lz[4] = {nd.loz.x, nd.loz.y, nd.loz.z, nd.loz.w};
                    const float hx[4] = {nd.hix.x, nd.hix.y, nd.hix.z, nd.hix.w};
                    const float hy[4] = {nd.hiy.x, nd.hiy.y, nd.hiy.z, nd.hiy.w};
                    const float hz[4] = {nd.hiz.x, nd.hiz.y, nd.hiz.z, nd.hiz.w};
                    const int rf[4] = {nd.ref.x, nd.ref.y, nd.ref.z, nd.ref.w};
                    const int inf[4] = {nd.info.x, nd.info.y, nd.info.z, nd.info.w};
                    float key[4];
                    int okm = 0, leafm = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const float ax = (lx[j] - o2.x) * inv.x, bx = (hx[j] - o2.x) * inv.x;
                        const float ay = (ly[j] - o2.y) * inv.y, by = (hy[j] - o2.y) * inv.y;
                        const float az = (lz[j] - o2.z) * inv.z, bz = (hz[j] - o2.z) * inv.z;
                        const float sl = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
                        const float le = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
                        const float e = (fabsf(sl) + fabsf(le)) * 9.5367431640625e-7f;   // 2^-20
                        const float lo = le - e, hi = sl + e;      // boxes carry the pad
                        key[j] = lo;
                        const bool ok = inf[j] >= 0 && !(hi < lo || hi < tlo || lo > thi);
                        okm |= ok << j;
                        leafm |= (inf[j] > 0) << j;
                    }
                    // interior slots first, so the node's boxes are dead during the leaf tests
                    float k4[4];
                    int r4[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const bool take = ((okm >> j) & 1) && !((leafm >> j) & 1);
                        k4[j] = take ? fminf(key[j], FLT_MAX) : INFINITY;
                        r4[j] = take ? rf[j] : -1;
                    }
                    int leaf_mask = okm & leafm;
                    while (leaf_mask) {          // leaves now, one code site (thi may shrink between them)
                        const int j = __builtin_ctz(leaf_mask);
                        leaf_mask &= leaf_mask - 1;
                        const float kj = j == 0 ? key[0] : j == 1 ? key[1] : j == 2 ? key[2] : key[3];
                        if (kj > thi) continue;
                        const int start = j == 0 ? rf[0] : j == 1 ? rf[1] : j == 2 ? rf[2] : rf[3];
                        const int cnt = j == 0 ? inf[0] : j == 1 ? inf[1] : j == 2 ? inf[2] : inf[3];
                        for (int q = start; q < start + cnt; q++) test_sah(sv.stris[q]);
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (k4[j] > thi) { k4[j] = INFINITY; r4[j] = -1; }
                    // interior slots, nearest first: sort (key, ref), push the others farthest first
                    auto ce = [&](int a, int b) {
                        const bool sw = k4[b] < k4[a];
                        const float ka = k4[a], kb = k4[b];
                        const int ra = r4[a], rb = r4[b];
                        k4[a] = sw ? kb : ka; k4[b] = sw ? ka : kb;
                        r4[a] = sw ? rb : ra; r4[b] = sw ? ra : rb;
                    };
                    ce(0, 1); ce(2, 3); ce(0, 2); ce(1, 3); ce(1, 2);
                    const int npush = (r4[1] >= 0) + (r4[2] >= 0) + (r4[3] >= 0);
                    if (sp + npush > kStackDepth) { use2 = true; break; }
                    for (int j = 3; j >= 1; j--)
                        if (r4[j] >= 0) { stk_put(stack, sstride, spill, sp, r4[j]); sp++; }
                    if (r4[0] >= 0) {
                        cur = r4[0];
                    } else {
                        if (sp == 0) break;
                        sp--;
                        cur = stk_get(stack, sstride, spill, sp);
                    }
                }
            }
            if (use2) {
                if (!EXHAUSTIVE && g.flat_split >= 0) {     // root over two leaves: both, no node load
                    flat_mesh(sv.tris, g.flat_split);
                } else {
                    walk2();
                }
            }
        }
    }
    if (found) {
        float t = gett(o2, d2, bp);
        if (t > 0 && (t < nearest || (t == nearest && i < out.obj))) {   // src/Helper.cpp:43, 64
            nearest = t;
            out.obj = i; out.prim = bprim; out.t = t;
            if (STATS) st.win_step = st.cand_step;
        }
    }
}

// The flat group (SceneView::gents, round 5): the entries whose mesh is tested without a node and whose
// transform (inverse matrix and blur) is bit-identical -- in practice the untransformed ones, whose glm
// inverse is the identity with signed zeros -- for a finite ray whose object-space direction is fast,
// all at once.  visit_object spends on every entry a prologue (transform, root
// box, window, the direction's reciprocals and norms) that costs several triangle tests, and the
// wave-uniform loop over a flat mesh's triangles runs a triangle's exact test whenever any lane needs
// it; in a room (C4 / C5: walls, floor, ceiling, light quads) both happened for nearly every wave.
// Here the direction set-up is done once, every group triangle gets tri_test's fast rejection (all
// lanes), and then each entry with candidates runs its reference root test (box_hit, exact) and each
// lane's own candidates through the exact test, in index order with the window shrinking -- the
// object's winner is the minimum of the total order (dist, -leaf_start, prim) over its accepted,
// reachable candidates either way (visit_object) -- followed by the top-level acceptance of
// src/Helper.cpp:39-49, 64.  Visiting these entries before the others is harmless: an entry replaces
// the winner iff t < nearest, or t == nearest and it comes earlier in the loop order.
// Returns false (nothing done) for a ray whose object-space direction is not fast: its lane visits the
// group's entries in the object loop.
// STATS: lane work / slots in st.gwork / st.gslot; wave cycles of the set-up (transform, reciprocals,
// window: up to the first triangle) and of the tests charged to ecyc[16] / ecyc[17].
template <bool STATS = false>
DEV bool flat_group(const SceneView& sv, const f3 o, const f3 d, const float time, float& nearest, HitRec& out,
                    Stats& st, unsigned long long* ecyc) {
    const unsigned long long c0 = STATS ? __builtin_amdgcn_s_memtime() : 0ull;
    auto charge = [&](int slot, unsigned long long t0) {
        if (STATS && ecyc && (__ballot(1) & __lanemask_lt()) == 0ull)
            atomicAdd(ecyc + slot, __builtin_amdgcn_s_memtime() - t0);
    };
    f3 o2, d2;
    transform_ray(*sv.gtop, o, d, time, o2, d2, true);   // the members' common transform
    const float adx = fabsf(d2.x), ady = fabsf(d2.y), adz = fabsf(d2.z);
    if (!(adx >= 1e-30f && adx <= 1e30f && ady >= 1e-30f && ady <= 1e30f && adz >= 1e-30f && adz <= 1e30f)) {
        charge(16, c0);
        return false;
    }
    const float eps = sv.int_eps;
    const f3 inv = mk(__builtin_amdgcn_rcpf(d2.x), __builtin_amdgcn_rcpf(d2.y), __builtin_amdgcn_rcpf(d2.z));
    const float da = d2.x != 0.0f ? d2.x : (d2.y != 0.0f ? d2.y : d2.z);
    const float oa = d2.x != 0.0f ? o2.x : (d2.y != 0.0f ? o2.y : o2.z);
    const float dnorm = __builtin_amdgcn_sqrtf(d2.x * d2.x + d2.y * d2.y + d2.z * d2.z);
    const float inv_dn = __builtin_amdgcn_rcpf(dnorm);
    // visit_object's parameter window for an object visited now (bounds: 1-ulp v_rcp / v_sqrt)
    auto window = [&]() -> float {
        if (!(nearest < FLT_MAX) || da == 0.0f) return INFINITY;
        const float tm = (nearest + 4.0f * 5.96e-8f * fabsf(oa) * __builtin_amdgcn_rcpf(fabsf(da))) * (1.0f + 1e-5f);
        const float boundD = tm * dnorm * (1.0f + 2e-5f) + 1e-30f;
        if (!(boundD < FLT_MAX)) return INFINITY;
        return boundD * inv_dn * (1.0f + 2e-5f) + 1e-30f;
    };
    const float thi1 = window();
    const float tlo = -(fabsf(eps) + 1e-6f);
    charge(16, c0);
    const unsigned long long c1 = STATS ? __builtin_amdgcn_s_memtime() : 0ull;
    unsigned cand = 0;
    for (int e = 0; e < sv.num_gents; e++) {
        const GroupEnt& G = sv.gents[e];
        // the entry's root box widened by the eps overhang against the parameter window (visit_object):
        // a coherent wave (a pixel's samples) skips the walls it does not face.  (Round 6 measured a
        // per-lane loop over each lane's own members here: the triangle records then come as per-lane
        // gathers instead of scalar loads -- cornell_pt k_shadow 99.5 -> 108 ms,
        // profiles/r7/ab_group_perlane.jsonl.)
        const bool need = !G.win || window_meets(o2, inv, G.win_min[0], G.win_min[1], G.win_min[2], G.win_max[0],
                                                 G.win_max[1], G.win_max[2], tlo, thi1);
        if (__ballot(need) == 0ull) continue;
        if (STATS) { st.gslot += G.count; st.gwork += need ? G.count : 0; }
        for (int j = G.first; j < G.first + G.count; j++)
            if (need && tri_maybe(sv.gtris[j], o2, d2, eps, thi1)) cand |= 1u << j;
    }
    // each member with candidates: its reference root test (box_hit, exact), the lane's own candidates
    // through the exact test in index order with the window shrinking, the gate, and the top-level
    // acceptance.  Members are visited in index order per lane, so a lane's sequence of member visits is
    // the same whether the wave walks the members uniformly (every lane the same members: scalar record
    // loads) or each lane its own (round 6: a mixed wave issues the most members one lane needs).
    auto member = [&](const GroupEnt& G, unsigned m) {
        if (G.root_box && !box_hit(o2, d2, inv, true, G.root_min[0], G.root_min[1], G.root_min[2], G.root_max[0],
                                   G.root_max[1], G.root_max[2]))
            return;
        const float thi0 = window();
        float thi = thi0, best_d = FLT_MAX;
        int best_leaf = -1, bprim = -1;
        bool found = false;
        f3 bp = mk(0, 0, 0);
        while (m) {
            const int j = __builtin_ctz(m);
            m &= m - 1u;
            const TriGeom tg = sv.gtris[G.first + j];
            const Cand c = tri_test(tg, o2, d2, eps, thi);
            if (!c.ok) continue;
            const float dist = norm(c.p - o2);
            const int k = __float_as_int(tg.p2.y), start = __float_as_int(tg.p2.z);
            if (!(dist < FLT_MAX &&
                  (dist < best_d || (dist == best_d && (start > best_leaf || (start == best_leaf && k < bprim))))))
                continue;
            if (__float_as_int(tg.p2.w)) {           // src/BVH.cpp:178 on the leaf's parent
                const float* gb = sv.gates + 6 * (size_t)k;
                if (!box_hit(o2, d2, inv, true, gb[0], gb[1], gb[2], gb[3], gb[4], gb[5])) continue;
            }
            best_d = dist; best_leaf = start; bprim = k; found = true; bp = c.p;
            thi = fminf(thi0, best_d * inv_dn * (1.0f + 2e-5f) + 1e-30f);
        }
        if (found) {
            const float t = gett(o2, d2, bp);
            const int i = G.entry;
            if (t > 0 && (t < nearest || (t == nearest && i < out.obj))) {   // src/Helper.cpp:43, 64
                nearest = t;
                out.obj = i; out.prim = bprim; out.t = t;
            }
        }
    };
    unsigned cm = 0;                                  // members holding candidates of this lane
    for (int e = 0; e < sv.num_gents; e++) {
        const GroupEnt& G = sv.gents[e];
        if ((cand >> G.first) & ((1u << G.count) - 1u)) cm |= 1u << e;
    }
    // the wave's union of members (ballots: active lanes only -- the group runs for finite rays) and
    // whether every lane has fewer: only then does the per-lane walk visit fewer members than the union
    // (a one-member group, the dragon's floor, never takes it)
    unsigned un = 0;
    for (int e = 0; e < sv.num_gents; e++)
        if (__ballot((cm >> e) & 1u)) un |= 1u << e;
    const int pu = __popc(un);
    const bool perlane = pu > 1 && __ballot(__popc(cm) >= pu) == 0ull;
    if (STATS) {        // the exact tests: each lane its own candidates, the wave the most any lane has
        // (a max over the active lanes only -- lanes of non-finite rays are not in here -- by ballots)
        const unsigned k = __popc(cand);
        unsigned wm = 0;
        for (int bit = 5; bit >= 0; bit--)
            if (__ballot(k >= (wm | (1u << bit)))) wm |= 1u << bit;
        st.gslot += wm;
        st.gwork += k;
    }
    if (!perlane) {
        unsigned mm = un;                           // every lane skips the members it has no candidate in
        while (mm) {
            const int e = __builtin_ctz(mm);
            mm &= mm - 1u;
            const GroupEnt& G = sv.gents[e];
            const unsigned m = (cand >> G.first) & ((1u << G.count) - 1u);
            if (m) member(G, m);
        }
    } else {
        unsigned mm = cm;
        while (mm) {
            const int e = __builtin_ctz(mm);
            mm &= mm - 1u;
            const GroupEnt& G = sv.gents[e];
            member(G, (cand >> G.first) & ((1u << G.count) - 1u));
        }
    }
    charge(17, c1);
    return true;
}

#ifndef RTG_BSPH
#define RTG_BSPH 1            // the transformed meshes' bounding-sphere skip (A/B: 0)
#endif
// ecyc (STATS): per-entry wave-cycle accumulators in LDS (the kernel flushes them to Counters); the
// flat group's cycles are charged to slot 15
// BDIST (the path tracer's shadow queries): the bounding sphere's parameter test too (below)
template <bool EXHAUSTIVE, bool STATS, bool TLAS = false, bool UNI = false, bool BDIST = false>
DEV HitRec closest_hit(const SceneView& sv, f3 o, f3 d, float time, float tmax, int* stack, int sstride, Stats& st,
                       short* tstack = nullptr, bool uni = false, unsigned long long* ecyc = nullptr) {
    HitRec out;
    out.obj = -1; out.prim = -1; out.t = 0.0f; out.pad = 0;
    if (isnan3(o) || isnan3(d)) return out;
    float nearest = tmax;
    const bool fin = ray_finite(o, d, time);
    int spill[kStackDepth > kLdsStack ? kStackDepth - kLdsStack : 1];
    auto visit = [&](const int i) {
        visit_object<EXHAUSTIVE, STATS, UNI>(sv, i, o, d, time, fin, nearest, out, stack, sstride, st, spill, uni);
    };
    const float adx = fabsf(d.x), ady = fabsf(d.y), adz = fabsf(d.z);
    const bool wfast = adx >= 1e-30f && adx <= 1e30f && ady >= 1e-30f && ady <= 1e30f && adz >= 1e-30f && adz <= 1e30f;
    // the reference's linear loop; a transformed entry whose world box (TopObject::wbox) the ray line
    // misses holds no candidate -- its hit points lie in the box and on the line, up to margins far
    // above the transform's rounding (the top-level BVH's test, below) -- so a lane skips it before
    // the ray transform (times outside [0, 1] leave the blur sweep: no skip)
    const bool tin = time >= 0.0f && time <= 1.0f;
    if (!TLAS || EXHAUSTIVE || sv.tlas_root < 0 || !wfast) {   // wfast is per lane: the others walk on
        // the flat group first (finite rays, fast in object space; the other lanes visit its entries in
        // the loop)
        bool grouped = false;
        if (!EXHAUSTIVE && sv.num_gents > 0 && __ballot(fin) != 0ull) {
            const unsigned long long c0 = STATS ? __builtin_amdgcn_s_memtime() : 0ull;
            if (fin) grouped = flat_group<STATS>(sv, o, d, time, nearest, out, st, ecyc);
            if (STATS && ecyc && (__ballot(1) & __lanemask_lt()) == 0ull)
                atomicAdd(ecyc + 15, __builtin_amdgcn_s_memtime() - c0);
        }
        for (int i = 0; i < sv.num_tops; i++) {
            if (STATS) st.considered++;
            const unsigned long long c0 = STATS ? __builtin_amdgcn_s_memtime() : 0ull;
            bool skip = grouped && sv.tops[i].grouped;
            if (!skip && !EXHAUSTIVE && sv.tops[i].wbox && wfast && tin) {
                const TopObject& T = sv.tops[i];
                const f3 wi = mk(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
                const float ax = (T.wlo[0] - o.x) * wi.x, bx = (T.whi[0] - o.x) * wi.x;
                const float ay = (T.wlo[1] - o.y) * wi.y, by = (T.whi[1] - o.y) * wi.y;
                const float az = (T.wlo[2] - o.z) * wi.z, bz = (T.whi[2] - o.z) * wi.z;
                const float sl = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
                const float le = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
                const float e = (fabsf(sl) + fabsf(le)) * 3.814697265625e-6f + 1e-30f;   // 2^-18
                skip = sl + e < le - e;
                // the bounding sphere (TopObject::bsph): the line's squared distance from its centre,
                // |oc x d|^2 / |d|^2, against r^2 plus 3e-5 |oc|^2 (the rounding here and the object-space
                // line's offset for far origins); NaN / inf compare false (entry kept)
                if (!skip && RTG_BSPH && T.bsph) {
                    const f3 oc = o - mk(T.bs[0], T.bs[1], T.bs[2]);
                    const f3 cr = cross(oc, d);
                    const float dd = dot(d, d);
                    skip = dot(cr, cr) > T.bs[3] * dd + 3e-5f * (dot(oc, oc) * dd);
                    if (BDIST && !skip) {
                        // the sphere's parameter interval t* -+ r/|d| (t* = -oc.d/|d|^2, scaled by |d|^2):
                        // wholly behind the origin (every candidate's gett() <= 0 fails t > 0) or wholly
                        // beyond tmax / the winner so far (t > nearest fails t < nearest; ties need
                        // equality, which the slack excludes).  Slack 1e-5 (|o| + |c| + r) |d| + 1e-5
                        // nearest |d|^2: the object-space t of a matrix with Frobenius product <= 6 (host)
                        // is the world t up to ~1e-6 of those terms.  Measured: the path tracer's shadow
                        // queries gain (C5 k_shadow -1.7 ms), the Whitted ones and camera / bounce rays
                        // lose (profiles/r7/ab_bsph_param_test_dropped.jsonl), so only k_shadow<PT> asks.
                        const float q = dot(oc, d);
                        const float dn = __builtin_amdgcn_sqrtf(dd);
                        const float r = __builtin_amdgcn_sqrtf(T.bs[3]);
                        const float S = 1e-5f * ((((fabsf(o.x) + fabsf(o.y)) + fabsf(o.z)) +
                                                  ((fabsf(T.bs[0]) + fabsf(T.bs[1])) + fabsf(T.bs[2])) + r) * dn);
                        const float rd = r * dn * 1.00001f;
                        skip = q > rd + S || -q - rd > nearest * dd * 1.00001f + S;
                    }
                }
            }
            if (!skip) {
                if (STATS) st.entries++;
                visit(i);
            }
            // STATS: the entry's wave cycles, charged once per wave after the lanes reconverge
            if (STATS && ecyc && (__ballot(1) & __lanemask_lt()) == 0ull)
                atomicAdd(ecyc + (i < 15 ? i : 15), __builtin_amdgcn_s_memtime() - c0);
        }
        return out;
    }
    // top-level walk.  A child box is skipped when the ray line misses it (its entries' hit points
    // lie on the line and in the box: host margins cover the rounding, the reciprocal slab adds
    // 2^-18 of the magnitudes, NaN comparisons keep a box).  Distance pruning -- boxes wholly
    // behind the origin or wholly beyond the winner so far -- needs gett()'s error: gett divides
    // by the first nonzero object-space direction component a (src/Ray.cpp:21-36), so a tiny d_a
    // makes t coarse (two spheres at different depths can get the same t).  For axis-aligned
    // entries that error is at most 2^-22 (|t| + K_a / |d_a|) with K_a the scene's bound on
    // |coordinate| + |translation| + |blur| along a (SceneView::tlas_k); pruning allows 16 times
    // that.  Subtrees of other entries (rotations, shears) carry kTlasNoPrune: line test only.
    const f3 winv = mk(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
    const float ka = d.x != 0.0f ? sv.tlas_k[0] : (d.y != 0.0f ? sv.tlas_k[1] : sv.tlas_k[2]);
    const float da = d.x != 0.0f ? adx : (d.y != 0.0f ? ady : adz);
    const float slack0 = 3.814697265625e-6f * (ka / da) + 1e-30f;        // 2^-18 K_a / |d_a|
    auto beyond = [&](float k) { return k > nearest + (3.814697265625e-6f * nearest + slack0); };
    auto tchild = [&](float mnx, float mny, float mnz, float mxx, float mxy, float mxz, bool prune, float& key) -> bool {
        const float ax = (mnx - o.x) * winv.x, bx = (mxx - o.x) * winv.x;
        const float ay = (mny - o.y) * winv.y, by = (mxy - o.y) * winv.y;
        const float az = (mnz - o.z) * winv.z, bz = (mxz - o.z) * winv.z;
        const float sl = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
        const float le = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
        const float e = (fabsf(sl) + fabsf(le)) * 3.814697265625e-6f + 1e-30f;   // 2^-18
        key = le - e;
        if (sl + e < key) return false;
        if (!prune) return true;
        if (sl + e < -slack0) return false;
        return !beyond(key);
    };
    // The walk is wave-uniform: the lanes of a wave (a pixel's samples, or a compacted run of
    // their children) share one traversal.  A child is entered when any lane needs it, node and
    // entry indices are uniform (scalar loads, one per-object code path per entry), and each lane
    // visits only the entries of leaves its own ray line passes.  That is a superset of what the
    // lane's own near-first walk would visit (pruning depends only on its own `nearest`), and
    // visiting an extra entry is harmless: every entry is a valid visit of the linear loop, and
    // equal t goes to the lower index in any order.
    int tsp = 0;
    int cur = sv.tlas_root;
    while (true) {
        const Node nd = sv.tlas[cur];
        const bool lpr = !(nd.d.x & kTlasNoPrune), rpr = !(nd.d.y & kTlasNoPrune);
        const int lref = nd.d.x & ~kTlasNoPrune, rref = nd.d.y & ~kTlasNoPrune, lcnt = nd.d.z, rcnt = nd.d.w;
        float lk = 0.0f, rk = 0.0f;
        bool lok = lcnt >= 0 && tchild(nd.a.x, nd.a.y, nd.a.z, nd.a.w, nd.b.x, nd.b.y, lpr, lk);
        bool rok = rcnt >= 0 && tchild(nd.b.z, nd.b.w, nd.c.x, nd.c.y, nd.c.z, nd.c.w, rpr, rk);
        auto still = [&](float k, bool prune) { return !prune || !beyond(k); };
        const bool lleaf = lcnt > 0, rleaf = rcnt > 0;
        if (lleaf || rleaf) {
            // leaf children, the nearer (for the wave's first lane) first; a lane takes the second
            // only if the first did not push its winner in front of it.  One visit() call site.
            const bool rfirst = rleaf && (!lleaf || __builtin_amdgcn_readfirstlane((int)(rk < lk)) != 0);
            for (int q = 0; q < 2; q++) {
                const bool take_r = (q == 0) == rfirst;
                if (take_r ? !rleaf : !lleaf) continue;
                const bool need = take_r ? (rok && still(rk, rpr)) : (lok && still(lk, lpr));
                if (__ballot(need) == 0ull) continue;
                const int ref = take_r ? rref : lref, cnt = take_r ? rcnt : lcnt;
                for (int k = ref; k < ref + cnt; k++) {
                    const int e = sv.tlas_idx[k];
                    if (STATS) { st.considered++; st.entries += need ? 1u : 0u; }
                    if (need) visit(e);
                }
            }
            if (lleaf) lok = false;
            if (rleaf) rok = false;
        }
        const bool anyl = __ballot(lok && still(lk, lpr)) != 0ull;
        const bool anyr = __ballot(rok && still(rk, rpr)) != 0ull;
        if (anyl && anyr) {
            const bool rnear = __builtin_amdgcn_readfirstlane((int)(rk < lk)) != 0;
            tstack[tsp * sstride] = (short)(rnear ? lref : rref);
            tsp++;
            cur = rnear ? rref : lref;
        } else if (anyl) {
            cur = lref;
        } else if (anyr) {
            cur = rref;
        } else {
            if (tsp == 0) break;
            tsp--;
            cur = __builtin_amdgcn_readfirstlane((int)tstack[tsp * sstride]);
        }
    }
    return out;
}

// ------------------------------------------------------------------ textures / Perlin
DEV f3 tex_pixel(const SceneView& sv, const TextureDev& t, int i, int j) {   // src/Texture.cpp:41-74
    if (i < 0) i = 0; else if (i >= t.w) i = t.w - 1;
    if (j < 0) j = 0; else if (j >= t.h) j = t.h - 1;
    const float* p = sv.texels + t.texel_offset + ((long long)j * t.w + i) * 3;
    return mk(p[0], p[1], p[2]);
}
DEV f3 tex_color(const SceneView& sv, const TextureDev& t, float u, float v) {   // Texture.cpp:111-131
    u = u - floorf(u);
    v = v - floorf(v);
    float i = u * (float)t.w;
    float j = v * (float)t.h;
    if (t.interp == RTG_INTERP_NN) return tex_pixel(sv, t, (int)i, (int)j);
    int li = (int)floorf(i), lj = (int)floorf(j);
    float a = i - (float)li, b = j - (float)lj;
    f3 c00 = tex_pixel(sv, t, li, lj), c01 = tex_pixel(sv, t, li, lj + 1);
    f3 c10 = tex_pixel(sv, t, li + 1, lj), c11 = tex_pixel(sv, t, li + 1, lj + 1);
    float w00 = (1 - a) * (1 - b), w01 = (1 - a) * b, w10 = a * (1 - b), w11 = a * b;
    return ((c00 * w00 + c01 * w01) + c10 * w10) + c11 * w11;
}
DEV void tex_change(const SceneView& sv, const TextureDev& t, float u, float v, float& du, float& dv) {  // Texture.cpp:76-109
    u = u - floorf(u);
    v = v - floorf(v);
    int i = (int)(u * (float)t.w);
    int j = (int)(v * (float)t.h);
    if (i < 0) i = 0; else if (i >= t.w - 1) i = t.w - 2;
    if (j < 0) j = 0; else if (j >= t.h - 1) j = t.h - 2;
    f3 a = tex_pixel(sv, t, i + 1, j), b = tex_pixel(sv, t, i, j), c = tex_pixel(sv, t, i, j + 1);
    float dede = ((a.x + a.y) + a.z) / 3.0f;
    float nene = ((b.x + b.y) + b.z) / 3.0f;
    f3 dd = c - b;
    du = dede - nene;
    dv = ((dd.x + dd.y) + dd.z) / 3.0f;
}

__constant__ float c_perlin_table[16][3] = {
    {1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1}, {1, 0, -1}, {-1, 0, -1},
    {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1}, {1, 1, 0}, {-1, 1, 0}, {0, -1, 1}, {0, -1, -1}};
__constant__ int c_perlin_shuffled[16] = {12, 7, 15, 6, 11, 0, 4, 9, 13, 3, 14, 8, 2, 5, 1, 10};
DEV int perlin_P(int i) { int idx = i % 16; if (idx < 0) idx += 16; return c_perlin_shuffled[idx]; }
DEV float perlin_weight(float x) {                      // src/Perlin.cpp:27-30 (double pow)
    double xd = (double)fabsf(x);
    return (float)((((-6) * pow(xd, 5.0)) + (15 * pow(xd, 4.0))) - (10 * pow(xd, 3.0)) + 1);
}
DEV float perlin_compute(f3 p, float scale, int nc) {   // src/Perlin.cpp:52-84
    f3 pt = p * scale;
    int ii = (int)floorf(pt.x), jj = (int)floorf(pt.y), kk = (int)floorf(pt.z);
    float value = 0;
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                int lx = ii + i, ly = jj + j, lz = kk + k;
                int idx = perlin_P(lx + perlin_P(ly + perlin_P(lz)));
                f3 g = mk(c_perlin_table[idx][0], c_perlin_table[idx][1], c_perlin_table[idx][2]);
                f3 l = pt - mk((float)lx, (float)ly, (float)lz);
                float w = (perlin_weight(l.x) * perlin_weight(l.y)) * perlin_weight(l.z);
                value += dot(g, l) * w;
            }
    if (nc == RTG_NC_LINEAR) value = (value + 1) * 0.5f;
    else if (nc == RTG_NC_ABSVAL) value = fabsf(value);
    return value;
}
DEV f3 perlin_gradient(f3 p, float scale, int nc) {     // src/Perlin.cpp:36-50
    const float eps = 0.001f;
    f3 xe = p, ye = p, ze = p;
    xe.x += eps; ye.y += eps; ze.z += eps;
    float o = perlin_compute(p, scale, nc);
    return mk((perlin_compute(xe, scale, nc) - o) / eps, (perlin_compute(ye, scale, nc) - o) / eps,
              (perlin_compute(ze, scale, nc) - o) / eps);
}
DEV f3 ortho_u(f3 v) {                                  // src/Helper.cpp:322-342
    float a0 = fabsf(v.x), a1 = fabsf(v.y), a2 = fabsf(v.z);
    f3 nl = v;
    if (a0 <= a1 && a0 <= a2) nl.x = 1.0f;
    else if (a1 <= a0 && a1 <= a2) nl.y = 1.0f;
    else nl.z = 1.0f;
    return normalized(cross(v, nl));
}

// ------------------------------------------------------------------ full hit record
struct Ret {            // ReturnVal (src/defs.h:13-22)
    f3 point, normal;
    int matIndex, dm;
    f3 tc;
    float tn;
};

DEV f3 tbn_apply(f3 T, f3 B, f3 N, f3 r) {   // Matrix3f(T,B,N cols) * r, rows summed x0+(x1+x2)
    return mk(T.x * r.x + (B.x * r.y + N.x * r.z), T.y * r.x + (B.y * r.y + N.y * r.z),
              T.z * r.x + (B.z * r.y + N.z * r.z));
}
DEV void perlin_decal(const TextureDev& t, Ret& ret) {
    if (t.decal == RTG_DECAL_REPLACE_KD) {
        ret.dm = t.decal;
        float p = perlin_compute(ret.point, t.noise_scale, t.nc);
        ret.tc = mk(p, p, p);
        ret.tn = 1;
    } else if (t.decal == RTG_DECAL_BUMP_NORMAL) {
        f3 g = perlin_gradient(ret.point, t.noise_scale, t.nc);
        f3 gpar = ret.normal * dot(g, ret.normal);
        f3 nn = ret.normal - (g - gpar) * t.bump;
        ret.normal = (dot(ret.normal, nn) > 0) ? nn : -nn;
        ret.normal = normalized(ret.normal);
    }
}
// Sphere::TextureComputation, src/Shape.cpp:400-503
DEV void sphere_texture(const SceneView& sv, const Geometry& g, Ret& ret) {
    ret.dm = RTG_DECAL_NONE;
    f3 c = ld3(g.center);
    float R = g.radius;
    for (int i = 0; i < g.num_textures; i++) {
        const TextureDev t = sv.textures[g.textures[i] - 1];
        if (t.kind == RTG_TEX_IMAGE) {
            f3 lc = ret.point - c;
            float theta = f_acos(lc.y / R);
            float phi = f_atan2(lc.z, lc.x);
            float tu = (float)((-(double)phi + PI_D) / (2 * PI_D));
            float tv = (float)((double)theta / PI_D);
            if (t.decal == RTG_DECAL_REPLACE_KD || t.decal == RTG_DECAL_BLEND_KD || t.decal == RTG_DECAL_REPLACE_ALL) {
                ret.dm = t.decal;
                ret.tc = tex_color(sv, t, tu, tv);
                ret.tn = (float)t.normalizer;
            } else if (t.decal == RTG_DECAL_REPLACE_NORMAL || t.decal == RTG_DECAL_BUMP_NORMAL) {
                float pi = (float)PI_D;
                f3 dpdu = mk((lc.z * 2) * pi, 0, (lc.x * (-2)) * pi);
                f3 dpdv = mk((lc.y * f_cos(phi)) * pi, (((-1) * R) * f_sin(theta)) * pi, (lc.y * f_sin(phi)) * pi);
                if (t.decal == RTG_DECAL_REPLACE_NORMAL) {
                    f3 rn = tex_color(sv, t, tu, tv) / 255.0f;
                    rn = normalized(rn - mk(0.5f, 0.5f, 0.5f));
                    ret.normal = tbn_apply(normalized(dpdu), normalized(dpdv), ret.normal, rn);
                } else {
                    float du, dv;
                    tex_change(sv, t, tu, tv, du, dv);
                    du = du * t.bump; dv = dv * t.bump;
                    f3 dpu = dpdu + ret.normal * du;
                    f3 dpv = dpdv + ret.normal * dv;
                    f3 nn = normalized(cross(dpv, dpu));
                    ret.normal = (dot(ret.normal, nn) > 0) ? nn : -nn;
                }
            }
        } else {
            perlin_decal(t, ret);
        }
    }
}
DEV void texcoord(const SceneView& sv, int idx, float& u, float& v) {
    if (idx < 0 || idx >= sv.num_texcoords) { u = 0; v = 0; return; }
    u = sv.texcoords[2 * idx]; v = sv.texcoords[2 * idx + 1];
}
// Triangle::TextureComputation, src/Shape.cpp:505-616
DEV void triangle_texture(const SceneView& sv, const Geometry& g, int4 vi, f3 e1, f3 e2, float beta, float gamma,
                          Ret& ret) {
    ret.dm = RTG_DECAL_NONE;
    if (g.num_textures == 0) return;
    float alpha = (1 - beta) - gamma;
    float u0, v0, u1, v1, u2, v2;
    texcoord(sv, vi.x - 1 + g.texture_offset, u0, v0);
    texcoord(sv, vi.y - 1 + g.texture_offset, u1, v1);
    texcoord(sv, vi.z - 1 + g.texture_offset, u2, v2);
    float uu = (u0 * alpha + u1 * beta) + u2 * gamma;
    float vv = (v0 * alpha + v1 * beta) + v2 * gamma;
    for (int i = 0; i < g.num_textures; i++) {
        const TextureDev t = sv.textures[g.textures[i] - 1];
        if (t.kind == RTG_TEX_IMAGE) {
            if (t.decal == RTG_DECAL_REPLACE_KD || t.decal == RTG_DECAL_BLEND_KD || t.decal == RTG_DECAL_REPLACE_ALL) {
                ret.dm = t.decal;
                ret.tc = tex_color(sv, t, uu, vv);
                ret.tn = (float)t.normalizer;
            } else if (t.decal == RTG_DECAL_REPLACE_NORMAL || t.decal == RTG_DECAL_BUMP_NORMAL) {
                float a00 = u1 - u0, a01 = v1 - v0, a10 = u2 - u0, a11 = v2 - v0;
                float invdet = 1.0f / (a00 * a11 - a10 * a01);
                float i00 = a11 * invdet, i10 = -a10 * invdet, i01 = -a01 * invdet, i11 = a00 * invdet;
                f3 T = mk(i00 * e1.x + i01 * e2.x, i00 * e1.y + i01 * e2.y, i00 * e1.z + i01 * e2.z);
                f3 B = mk(i10 * e1.x + i11 * e2.x, i10 * e1.y + i11 * e2.y, i10 * e1.z + i11 * e2.z);
                if (t.decal == RTG_DECAL_REPLACE_NORMAL) {
                    f3 rn = tex_color(sv, t, uu, vv) / 255.0f;
                    rn = normalized(rn - mk(0.5f, 0.5f, 0.5f));
                    ret.normal = tbn_apply(T, B, ret.normal, rn);
                } else {
                    float du, dv;
                    tex_change(sv, t, uu, vv, du, dv);
                    du = du * t.bump; dv = dv * t.bump;
                    f3 dpu = T + ret.normal * du;
                    f3 dpv = B + ret.normal * dv;
                    f3 nn = normalized(cross(dpv, dpu));
                    ret.normal = (dot(ret.normal, nn) > 0) ? nn : -nn;
                }
            }
        } else {
            perlin_decal(t, ret);
        }
    }
}

// Re-derive the full ReturnVal of a hit found by closest_hit: the winning primitive's
// object-space intersection (identical arithmetic), texturing, then the top-level
// world point and TransformNormal (src/Helper.cpp:39-77).
// FULL = false: the scene has no textures (the host checks), so texturing is compiled out.
template <bool FULL = true>
DEV Ret hit_record(const SceneView& sv, f3 o, f3 d, float time, const HitRec& h) {
    const TopObject& T = sv.tops[h.obj];
    const Geometry& g = sv.geoms[T.geom];
    f3 o2, d2;
    transform_ray(T, o, d, time, o2, d2, ray_finite(o, d, time), /*strict=*/true);
    Ret ret;
    ret.matIndex = T.material;
    ret.dm = RTG_DECAL_NONE;
    ret.tc = mk(0, 0, 0);
    ret.tn = 0;
    if (g.type == RTG_OBJ_SPHERE) {
        f3 ip = mk(0, 0, 0);
        sphere_test(o2, d2, ld3(g.center), g.radius, sv.int_eps, ip);
        ret.point = ip;
        f3 pc = ip - ld3(g.center);
        ret.normal = pc / norm(pc);
        if (FULL) sphere_texture(sv, g, ret);
    } else if (!FULL && !(g.type == RTG_OBJ_TRIANGLE || g.smooth)) {
        // flat triangle, no texturing: the normal from the record's a - b and c - b (prim_idx.w is
        // the object's smooth flag, 1 for Triangle objects: Shape.cpp:262-276), no vertex loads
        const TriGeom tg = sv.tris[h.prim];
        const Cand c = tri_test(tg, o2, d2, sv.int_eps);
        const f3 normal = cross(mk(tg.p2.y, tg.p2.z, tg.p2.w), mk(tg.p0.w, tg.p1.x, tg.p1.y));
        ret.normal = normal / norm(normal);
        ret.point = c.p;
    } else {
        int4 vi = sv.prim_idx[h.prim];
        const TriGeom tg = sv.tris[h.prim];
        const Cand c = tri_test(tg, o2, d2, sv.int_eps);
        const f3 a = mk(tg.p0.x, tg.p0.y, tg.p0.z);
        f3 b = ld3(sv.vertices + 3 * (vi.y - 1)), cc = ld3(sv.vertices + 3 * (vi.z - 1));
        f3 normal;
        if (vi.w) {
            float alpha = (1 - c.beta) - c.gamma;
            f3 n1 = ld3(sv.vnormals + 3 * (vi.x - 1)), n2 = ld3(sv.vnormals + 3 * (vi.y - 1)),
               n3 = ld3(sv.vnormals + 3 * (vi.z - 1));
            normal = (n1 * alpha + n2 * c.beta) + n3 * c.gamma;
        } else {
            normal = cross(cc - b, a - b);
        }
        ret.normal = normal / norm(normal);
        ret.point = c.p;
        if (FULL) triangle_texture(sv, g, vi, b - a, cc - a, c.beta, c.gamma, ret);
    }
    float t = gett(o2, d2, ret.point);
    ret.point = o + d * t;
    ret.normal = normalized(xform(T.invT, ret.normal, 1.0f));
    return ret;
}

// ------------------------------------------------------------------ lights (src/Light.cpp)
DEV float conductor_fresnel(float n_t, float k_t, f3 ray, f3 normal) {   // Light.cpp:18-28, Scene.cpp:135-146
    float cos_t = -dot(ray, normal);
    float twoNtCost = (2 * n_t) * cos_t;
    float cosSquared = (float)sq_d(cos_t);
    float ntk = (float)(sq_d(n_t) + sq_d(k_t));
    float rs = ((ntk - twoNtCost) + cosSquared) / ((ntk + twoNtCost) + cosSquared);
    float rp = ((ntk * cosSquared - twoNtCost) + 1) / ((ntk * cosSquared + twoNtCost) + 1);
    return 0.5f * (rs + rp);
}
DEV float geometry_ts(f3 wi, f3 wo, f3 wh, f3 n) {      // Light.cpp:49-60
    float left = (2.0f * dot(n, wh)) * dot(n, wo);
    left = left / dot(wo, wh);
    float right = (2.0f * dot(n, wh)) * dot(n, wi);
    right = right / dot(wi, wh);
    float x = stdmin(left, right);
    return stdmin(1.0f, x);
}
DEV float distribution_ts(float cosAlpha, int p) {       // Light.cpp:12-16
    float x = (float)((double)((float)p + 2.0f) / (double)(2.0f * PI_D));
    x = (float)((double)x * pow((double)cosAlpha, (double)p));
    return x;
}
// TS: the Torrance-Sparrow models compiled in (their distribution term is a double-precision
// pow(cos, p), whose code alone takes the path tracer's BRDF shading from 143 to 189 VGPRs); a scene
// without TS / TSF materials runs the variants without it (SceneView::brdf_ts).
template <bool TS = true>
DEV f3 term_brdf(f3 wi, f3 wo, f3 n, const MaterialDev& m) {   // Light.cpp:62-155
    f3 kd = ld3(m.diffuse), ks = ld3(m.specular);
    int p = m.phong_exp;
    switch (m.brdf) {
    case RTG_BRDF_MP:
    case RTG_BRDF_OP:
    case RTG_BRDF_MPN: {
        float n_wi = dot(n, wi);
        f3 wr = -wi + (n * 2) * n_wi;
        wr = wr / norm(wr);
        float cosAngle = fmax0(dot(wr, wo));
        if (m.brdf == RTG_BRDF_MP) return kd + ks * f_powi(cosAngle, p);
        if (m.brdf == RTG_BRDF_OP) {
            float cti = fmax0(dot(wi, n));
            if (cti < 0.001f) return mk(0, 0, 0);
            return kd + (ks * f_powi(cosAngle, p)) / cti;
        }
        return kd / (float)PI_D + (ks * (float)((p + 2) / (2 * PI_D))) * f_powi(cosAngle, p);
    }
    case RTG_BRDF_MBP:
    case RTG_BRDF_OBP:
    case RTG_BRDF_MBPN: {
        f3 h = normalized(wo + wi);
        float cosAngle = fmax0(dot(n, h));
        if (m.brdf == RTG_BRDF_MBP) return kd + ks * f_powi(cosAngle, p);
        if (m.brdf == RTG_BRDF_OBP) {
            float cti = fmax0(dot(wi, n));
            if (cti < 0.001f) return mk(0, 0, 0);
            return kd + (ks * f_powi(cosAngle, p)) / cti;
        }
        return kd / (float)PI_D + (ks * (float)((p + 8) / (8 * PI_D))) * f_powi(cosAngle, p);
    }
    case RTG_BRDF_TS:
    case RTG_BRDF_TSF: if constexpr (TS) {
        f3 wh = normalized(wo + wi);
        float f = 0;
        f3 dp = kd / (float)PI_D;
        if (m.brdf == RTG_BRDF_TSF) {
            f = conductor_fresnel(m.refraction_index, m.absorption_index, -wo, n);
            dp = dp * (1 - f);
        }
        float cosAlpha = dot(wh, n), cosTheta = dot(wi, n), cosPhi = dot(wo, n);
        float gg = geometry_ts(wi, wo, wh, n);
        float dd = distribution_ts(cosAlpha, p);
        f3 sp = (ks * gg) * dd;
        sp = sp / ((4.0f * cosPhi) * cosTheta);
        if (m.brdf == RTG_BRDF_TSF) sp = sp * f;
        return dp + sp;
    }
    default:
        return mk(0, 0, 0);
    }
}
template <bool TS = true>
DEV f3 brdf(f3 wi, f3 wo, f3 n, f3 radiance, const MaterialDev& m) {   // Light.cpp:157-162
    f3 t = term_brdf<TS>(wi, wo, n, m);
    float cosAngle = fmax0(dot(wi, n));
    return cw(radiance, t) * cosAngle;
}
DEV f3 diffuse_term(f3 LC, const Ret& ret, const MaterialDev& m, float alpha) {
    if (ret.dm == RTG_DECAL_REPLACE_KD) return cw(LC, (ret.tc / ret.tn) * alpha);
    if (ret.dm == RTG_DECAL_BLEND_KD) return cw(LC, ((ld3(m.diffuse) + ret.tc / ret.tn) * 0.5f) * alpha);
    return cw(LC, ld3(m.diffuse) * alpha);
}
DEV f3 specular_term(f3 LC, f3 wo, f3 wi, const Ret& ret, const MaterialDev& m) {
    f3 s = wo + wi;
    f3 h = s / norm(s);
    float alpha = fmax0(dot(ret.normal, h));
    return cw(LC, ld3(m.specular) * f_powi(alpha, m.phong_exp));
}
// BRDF: 0 the reference's Blinn-Phong terms only, 1 the BRDF models without Torrance-Sparrow, 2 all
template <int BRDF = 2>
DEV f3 phong_or_brdf(f3 LC, f3 wo, f3 wi, const Ret& ret, const MaterialDev& m) {
    if (BRDF != 0 && m.brdf != RTG_BRDF_NONE) return brdf<BRDF == 2>(wi, wo, ret.normal, LC, m);
    float alpha = fmax0(dot(ret.normal, wi));
    return diffuse_term(LC, ret, m, alpha) + specular_term(LC, wo, wi, ret, m);
}
DEV f3 env_radiance(const SceneView& sv, const LightDev& L, f3 dir) {   // Light.cpp:563-575
    float theta = f_acos(dir.y);
    float phi = f_atan2(dir.z, dir.x);
    float tu = (float)((-(double)phi + PI_D) / (2 * PI_D));
    float tv = (float)((double)theta / PI_D);
    f3 rad = tex_color(sv, sv.textures[L.tex], tu, tv);
    return (rad * 2) * (float)PI_D;
}

// Unshadowed contribution of light li plus the shadow query it needs.
// Shadow-ray direction toward a light point and the query's t bound: shared by light_sample
// and the lean k_shadow, which rebuilds them from the stored origin / hit point (bit-identical).
DEV f3 toward(f3 lpos, f3 p) {
    f3 dv = lpos - p;
    return dv / norm(dv);
}
// The query's t bound from dl = |p - L| (light_sample stores dl; k_shadow rebuilds the bound).
DEV float shadow_tmax_dl(f3 origin, float dl, float eps) {
    // hits with gett() beyond |p-L| + eps can never satisfy the blocking test
    float oabs = fmaxf(fmaxf(fabsf(origin.x), fabsf(origin.y)), fabsf(origin.z));
    float tmax = (dl + eps) * (1.0f + 1e-4f) + 1e-5f * oabs + 1e-30f;
    if (!(tmax == tmax)) tmax = FLT_MAX;
    return tmax;
}
DEV float shadow_tmax(f3 origin, f3 p, f3 lp, float eps) { return shadow_tmax_dl(origin, norm(p - lp), eps); }
// Object-light (NEE) query bound: k_shadow blocks iff |p - hp| < lim = dl - (eps + 1e-4 dl)
// (Page7.md:143-147 as the oracle states it), hp = o + d t, o = p + w (w = the normal offset).
// With |d| = 1, |p - hp|^2 = t^2 + 2t (d.w) + |w|^2, so every hit with t >= tcut = -(d.w) +
// sqrt((d.w)^2 - |w|^2 + lim^2) leaves the query unblocked.  The light's own surface, at
// t ~ dl - (d.w), lies eps + 1e-4 dl beyond tcut, so the query no longer walks to it.  Margins:
// 1e-5 relative and 1e-5 |o| absolute, far above the rounding of k_shadow's test.
DEV float emit_shadow_tmax(f3 origin, f3 p, float dl, f3 d, float eps) {
    const float lim = dl - (eps + 1e-4f * dl);
    const f3 w = origin - p;
    const float dw = dot(d, w);
    const float tcut = -dw + sqrtf(fmax0(dw * dw - dot(w, w) + lim * lim));
    const float oabs = fmaxf(fmaxf(fabsf(origin.x), fabsf(origin.y)), fabsf(origin.z));
    const float t = (lim > 0.0f ? tcut * (1.0f + 1e-5f) : 0.0f) + 1e-5f * (oabs + dl) + 1e-30f;
    return t == t ? t : FLT_MAX;
}

// EMIT: the hw7 object-light cases (the path tracer's NEE; the Whitted light loop never reaches
// them: the render adds the object lights to the loop only for the path tracer)
// SPOT: the scene has a spot or (full variants) an environment light (SceneView::heavy).  Their
// double-precision libm code (spot fall-off: acos, cos, pow; environment: acos, atan2 and the
// rejection loop) sets the register peak of the shading kernels: inlined into the full k_shade it
// takes the light loop from 79 to 244 VGPRs (cross-compiled resource usage, round 4), so scenes
// without such lights get variants without that code.
template <bool FULL = true, bool SPOT = true, int BRDF = FULL ? 2 : 0, bool EMIT = true>
DEV void light_sample(const SceneView& sv, int li, f3 primeDir, float time, const Ret& ret, const MaterialDev& m,
                      uint64_t seed, uint32_t pixel, uint32_t sample, uint64_t path, ShadowRec& sr) {
    const LightDev& L = sv.lights[li];
    f3 wo = -primeDir;
    f3 origin = ret.point + ret.normal * sv.shadow_eps;
    f3 c = mk(0, 0, 0);
    f3 dir = mk(0, 0, 0), lp = mk(0, 0, 0);
    float mode = 0.0f;
    // every case leaves the light colour and direction of its single BRDF call here; the call
    // follows the switch (one inlined copy of the BRDF code instead of one per light type)
    f3 LCs = mk(0, 0, 0), wis = mk(0, 0, 0);
    bool lit = false;
    float post = 1.0f;              // spot FallOf(angle), applied after the BRDF (Light.cpp:428-431)
    bool use_post = false;
    switch (L.type) {
    case RTG_LIGHT_POINT: {                                     // PointLight::BasicShading Light.cpp:238-250
        f3 pos = ld3(L.pos);
        dir = toward(pos, ret.point);
        lp = pos;
        mode = 1.0f;
        float dist = norm(ret.point - pos);
        LCs = ld3(L.inten) / (dist * dist);
        wis = normalized(pos - ret.point);
        lit = true;
        break;
    }
    case RTG_LIGHT_DIRECTIONAL: {                               // Light.cpp:309-321
        dir = -ld3(L.dir);
        mode = 2.0f;
        LCs = ld3(L.inten);
        wis = dir;
        lit = true;
        break;
    }
    case RTG_LIGHT_SPOT: if constexpr (SPOT) {                  // Light.cpp:409-436
        f3 pos = ld3(L.pos);
        dir = toward(pos, ret.point);
        lp = pos;
        f3 dtp = normalized(ret.point - pos);
        float angle = f_acos(dot(dtp, ld3(L.dir)));
        if (angle < L.fall || angle < L.coverage) {
            mode = 1.0f;
            float dist = norm(ret.point - pos);
            LCs = ld3(L.inten) / (dist * dist);
            wis = normalized(pos - ret.point);
            lit = true;
            if (!(angle < L.fall)) {
                post = (float)pow((cos((double)angle) - (double)L.cos_cov) / (double)(L.cos_fall - L.cos_cov), 4.0);
                use_post = true;
            }
        }
        break;
    }
    case RTG_LIGHT_AREA: if constexpr (FULL) {                 // Light.cpp:522-545
        float xi[4];
        rng4(seed, pixel, sample, path, RNG_AREA, (uint32_t)li, 0, xi);
        float uChi = xi[0] - 0.5f, vChi = xi[1] - 0.5f;
        f3 smp = (ld3(L.pos) + (ld3(L.u) * L.size) * uChi) + (ld3(L.v) * L.size) * vChi;
        f3 dv = smp - ret.point;
        dir = dv / norm(dv);
        lp = smp;
        mode = 1.0f;
        f3 pms = ret.point - smp;
        float cosTheta = fabsf(dot(normalized(pms), ld3(L.normal)));
        float dSq = norm(pms);
        dSq = dSq * dSq;
        LCs = ld3(L.inten) * ((L.size * L.size) * (cosTheta / dSq));
        wis = normalized(smp - ret.point);
        lit = true;
        break;
    }
    case RTG_LIGHT_ENVIRONMENT: if constexpr (FULL && SPOT) {  // Light.cpp:628-660
        f3 n = ret.normal;
        f3 u = ortho_u(n);
        f3 w = cross(n, u);
        f3 direction = n;
        for (uint32_t it = 0; it <= 1000000u; it++) {
            float xi[4];
            rng4(seed, pixel, sample, path, RNG_ENV, (uint32_t)li, it, xi);
            float x = xi[0] * 2 - 1.0f, y = xi[1] * 2 - 1.0f, z = xi[2] * 2 - 1.0f;
            f3 smp = ((ret.point + u * x) + n * y) + w * z;
            f3 dd = smp - ret.point;
            if (dot(dd, n) > 0 && norm(dd) <= 1) { direction = normalized(dd); break; }
        }
        dir = direction;
        mode = 2.0f;
        LCs = env_radiance(sv, L, direction);
        wis = direction;
        lit = true;
        break;
    }
    case kLightEmitMesh:                                        // hw7 object lights: NEE sample
    case kLightEmitSphere: if constexpr (EMIT) {                // (oracle emitter_shading)
        float xi[4];
        rng4(seed, pixel, sample, path, RNG_PT_EMIT, (uint32_t)li, 0, xi);
        const f3 p = ret.point;
        f3 LC;
        if (L.type == kLightEmitSphere) {                       // uniform in the subtended cone
            const f3 C = ld3(L.pos);
            const float Rw = L.size;
            const f3 dv = C - p;
            const float dd = norm(dv);
            const bool inside = !(dd > Rw);                     // inside: all directions
            float cosmax = -1.0f;
            if (!inside) {
                const float sin2 = (Rw * Rw) / (dd * dd);
                cosmax = sqrtf(fmax0(1.0f - sin2));
            }
            const float cosT = 1.0f - xi[0] * (1.0f - cosmax);
            const float sinT = sqrtf(fmax0(1.0f - cosT * cosT));
            const float phi = (float)(2 * PI_D) * xi[1];
            const f3 dn = dd > 0.0f ? dv / dd : mk(0, 1, 0);
            const f3 u = ortho_u(dn), w = cross(dn, u);
            float sp, cp;
            f_sincos(phi, sp, cp);
            dir = normalized((u * (sinT * cp) + w * (sinT * sp)) + dn * cosT);
            const f3 oc = p - C;
            const float b = dot(dir, oc);
            const float disc = b * b - (sqn(oc) - Rw * Rw);
            const float t = inside ? -b + sqrtf(fmax0(disc)) : -b - sqrtf(fmax0(disc));
            lp = p + dir * t;
            LC = ld3(L.inten) * ((float)(2 * PI_D) * (1.0f - cosmax));
        } else {                                                // area-weighted triangle, uniform point
            const float* cdf = sv.emit_cdf + L.tri_first;
            const float target = xi[0] * L.coverage;
            int lo = 0, hi = L.tri_count - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (target < cdf[mid]) hi = mid; else lo = mid + 1;
            }
            const float* T = sv.emit_tris + 9 * (size_t)(L.tri_first + lo);
            const f3 a = ld3(T), b = ld3(T + 3), cc = ld3(T + 6);
            const float sq = sqrtf(xi[1]);
            lp = (a * (1.0f - sq) + b * (sq * (1.0f - xi[2]))) + cc * (sq * xi[2]);
            const f3 nl = normalized(cross(b - a, cc - a));
            const f3 dv = lp - p;
            const float dd = norm(dv);
            dir = dv / dd;
            const float cosl = fabsf(dot(dir, nl));
            LC = ld3(L.inten) * ((cosl * L.coverage) / (dd * dd));
        }
        LCs = LC;
        wis = dir;
        lit = true;
        mode = 3.0f;            // 0 below when the contribution is exactly zero
        break;
    }
    }
    if (lit) {
        c = phong_or_brdf<BRDF>(LCs, wo, wis, ret, m);
        if (use_post) c = c * post;
    }
    // an object-light sample that contributes exactly zero (light behind the surface) needs no
    // shadow ray: blocked or not it adds 0 (oracle emitter_shading does the same)
    if (mode == 3.0f && c.x == 0.0f && c.y == 0.0f && c.z == 0.0f) mode = 0.0f;
    // A query whose unshadowed contribution is exactly +0 in every channel (a light behind
    // the surface with no specular lobe left) need not be traced: blocked, the light adds the
    // reference's Vector3f(0,0,0) (src/Light.cpp:188-204, 270-275), unblocked it adds c = +0;
    // both leave the running sum bit-identical.  -0 / NaN channels keep the query.
    if ((mode == 1.0f || mode == 2.0f) && (__float_as_uint(c.x) | __float_as_uint(c.y) | __float_as_uint(c.z)) == 0u)
        mode = 0.0f;
    // distance tests (modes 1 / 3): only |p - L| is needed, by k_shadow's t bound (shadow_query_tmax)
    // and its blocking test; directional / environment queries have no light point
    const float dl = (mode == 1.0f || mode == 3.0f) ? norm(ret.point - lp) : 0.0f;
    sr.o = make_float4(origin.x, origin.y, origin.z, time);
    sr.d = make_float4(dir.x, dir.y, dir.z, dl);
    sr.c = make_float4(c.x, c.y, c.z, mode);
}

// The traced mode of a query to light li (a query is listed only when light_sample left a nonzero
// mode, which depends on the light type alone): 2 = any hit blocks (directional, environment),
// 3 = object light (hw7), else 1 = distance test against the light point.
DEV float shadow_mode(const SceneView& sv, int li) {
    const int t = sv.lights[li].type;
    return (t == RTG_LIGHT_DIRECTIONAL || t == RTG_LIGHT_ENVIRONMENT) ? 2.0f
         : (t == kLightEmitMesh || t == kLightEmitSphere) ? 3.0f : 1.0f;
}
// k_shadow's t bound of a traced query (what light_sample formed before round 6, bit for bit):
// p = the node's hit point (mode 3 only), dl from the direction plane's w.
// EMIT: object-light queries (mode 3) can occur -- the path tracer's instantiations only.
template <bool EMIT>
DEV float shadow_query_tmax(float mode, f3 origin, f3 p, f3 d, float dl, float eps) {
    if (mode == 2.0f) return FLT_MAX;
    float tmax = shadow_tmax_dl(origin, dl, eps);
    if (EMIT && mode == 3.0f) tmax = fminf(tmax, emit_shadow_tmax(origin, p, dl, d, eps));
    return tmax;
}

// ------------------------------------------------------------------ camera / background
// Pixel order of a pass (t -> x, k = owned-row index): tiles of (64 / th) x th pixels, row-major
// inside a tile; th = the shard's row block (<= 8), so a tile is always image-contiguous.  Bands of
// ts tiles' height over the owned rows, each band in columns of tiles, a column's tiles top to
// bottom (edge columns / tiles narrower or lower).  A kernel's in-flight rays are a window of
// consecutive t; ts > 1 makes that window squarer than a one-tile-high strip.
// (idiv: rtg_internal.h)
DEV void tile_pixel(int t, int nx, int rows_owned, int th, int ts, int& x, int& k) {
    const int tw = 64 >> __builtin_ctz((unsigned)th);   // th is 1, 2, 4 or 8
    const int sh = th * ts;                          // band height (rows)
    const int band = idiv(t, sh * nx);
    const int u = t - band * sh * nx;
    const int hs = min(sh, rows_owned - sh * band);  // rows in this band
    const int c = idiv(u, tw * hs);                  // tile column
    const int u2 = u - c * tw * hs;
    const int wb = min(tw, nx - tw * c);
    const int rt = idiv(u2, wb * th);                // tile in the column
    const int u3 = u2 - rt * wb * th;
    const int r = idiv(u3, wb);
    x = tw * c + (u3 - r * wb);
    k = sh * band + th * rt + r;
}
DEV void slot_pixel(const CameraDev& cam, const PassDev& ps, int slot, uint32_t& pixel, uint32_t& sample, int& x,
                    int& y) {
    const int pl = idiv(slot, ps.ns), sl = slot - pl * ps.ns;
    int k;
    tile_pixel(ps.p0 + pl, cam.nx, ps.rows_owned, ps.tile_h, ps.tile_s, x, k);
    y = shard_row(k, ps.row_offset, ps.row_stride, ps.row_block);
    pixel = (uint32_t)(y * cam.nx + x);
    sample = (uint32_t)(ps.s0 + sl);
}
DEV f3 background(const SceneView& sv, const CameraDev& cam, int row, int col, f3 dir) {   // Scene.cpp:413-435
    if (sv.env_light != -1) {
        const LightDev& L = sv.lights[sv.env_light];
        if (L.type != RTG_LIGHT_ENVIRONMENT) return ld3(sv.background);
        float theta = f_acos(dir.y);
        float phi = f_atan2(dir.z, dir.x);
        float tu = (float)((-(double)phi + PI_D) / (2 * PI_D));
        float tv = (float)((double)theta / PI_D);
        return tex_color(sv, sv.textures[L.tex], tu, tv);
    }
    if (sv.bg_texture == -1) return ld3(sv.background);
    float u = ((float)col) / (float)cam.nx;
    float v = ((float)row) / (float)cam.ny;
    return tex_color(sv, sv.textures[sv.bg_texture], u, v);
}

// ------------------------------------------------------------------ kernels
// Primary ray of sample slot i of the pass (Camera::getPrimaryRay / getSampleRay).  Level 0's
// k_trace / k_shade / k_pt_shade compute it from the slot (same function, so bit-identical)
// instead of storing a queued ray + RayMeta per primary ray and re-reading it twice.
DEV void primary_ray(const CameraDev& cam, const PassDev& ps, uint64_t seed, int i, f3& o_out, f3& d_out,
                     float& time_out) {
    uint32_t pixel, sample;
    int x, y;
    slot_pixel(cam, ps, i, pixel, sample, x, y);
    f3 pos = ld3(cam.pos), gaze = ld3(cam.gaze), right = ld3(cam.right), up = ld3(cam.up);
    f3 o = pos, d;
    float time = 0.0f;
    if (cam.total > 1) {
        // PixelLBCorner (Camera.cpp:84-92) + getSampleRay (Camera.cpp:94-113) + AddDepthOfField (Camera.cpp:119-139)
        float u = cam.l + (float)x * cam.pw;
        float v = cam.t - (float)(y + 1) * cam.ph;
        f3 m = pos + gaze * cam.dist;
        m = m + right * u;
        m = m + up * v;
        float xi[4];
        rng4(seed, pixel, sample, 1, RNG_CAMERA, 0, 0, xi);
        int si = (int)sample;
        const int jj = idiv(si, cam.sample_count), ii = si - jj * cam.sample_count;
        m = m + right * (((float)ii + xi[0]) * cam.sw);
        m = m + up * (((float)jj + xi[1]) * cam.sh);
        f3 dv = m - pos;
        d = dv / norm(dv);
        if (cam.dof) {
            float xa = xi[2] - 0.5f, xb = xi[3] - 0.5f;
            f3 q = pos;
            q = q + right * (cam.aperture * xa);
            q = q + up * (cam.aperture * xb);
            f3 dir = normalized(m - pos);
            float tfd = cam.focus / dot(dir, gaze);
            f3 p = pos + d * tfd;
            o = q;
            d = normalized(p - q);
        } else {
            time = xi[2];
        }
    } else {
        // getPrimaryRay (Camera.cpp:63-72)
        float u = cam.l + ((cam.r - cam.l) * ((float)x + 0.5f)) * cam.nxDA;
        float v = cam.t - ((cam.t - cam.b) * ((float)y + 0.5f)) * cam.nyDA;
        f3 m = pos + gaze * cam.dist;
        m = m + right * u;
        m = m + up * v;
        f3 dv = m - pos;
        d = dv / norm(dv);
    }
    o_out = o; d_out = d; time_out = time;
}

// Render-path hit records: 8 bytes per ray, (object, primitive); k_shade / k_pt_shade rebuild the
// hit by re-running the winning test (hit_record) -- cheaper than storing and gathering its ray
// parameter and barycentrics (DESIGN.md §4 "hit records").
struct HitIn { HitRec h; };
DEV HitIn load_hit_planes(const HitRec* hits, int n, int i) {
    const HitPlanes hp = hit_planes(const_cast<HitRec*>(hits), n);
    const int2 v = hp.id[i];
    HitIn r;
    r.h.obj = v.x; r.h.prim = v.y; r.h.t = 0.0f; r.h.pad = 0;
    return r;
}

// Queued ray i (RayQ planes).
DEV void load_ray(const RayQ& q, int i, f3& o, f3& d, float& time) {
    const float4 a = q.a[i];
    const float2 b = q.b[i];
    o = mk(a.x, a.y, a.z);
    d = mk(a.w, b.x, b.y);
    time = q.t ? q.t[i] : 0.0f;
}
DEV void store_ray(const RayQ& q, int k, f3 o, f3 d, float time) {
    q.a[k] = make_float4(o.x, o.y, o.z, d.x);
    q.b[k] = make_float2(d.y, d.z);
    if (q.t) q.t[k] = time;
}

// GEN: the launch may generate primary rays: rays [0, nq) are queued, ray i >= nq is
// primary_ray(slot gbase + i - nq) (level 0 of a pass: nq = 0, gbase = 0; a regenerating step of
// the path tracer's stream schedule: the survivors of the previous step, then new camera samples).
template <bool EXHAUSTIVE, bool STATS, bool GEN = false, bool TLAS = false>
__global__ void __launch_bounds__(kTraceBlock) RTG_TRACE_ATTR k_trace(const SceneView sv, const RayQ rays,
                                                       HitRec* __restrict__ hits, int n, Counters* ctr,
                                                       const CameraDev cam, const PassDev ps, uint64_t seed,
                                                       bool compact, int nq, int gbase) {
    __shared__ int s_stack[kLdsStack * kTraceBlock];
    __shared__ short s_tstack[TLAS ? kTlasStack * kTraceBlock : 1];
    __shared__ unsigned long long s_ecyc[STATS ? 18 : 1];   // entries 0..15, group set-up / tests
    if (STATS && threadIdx.x < 18) s_ecyc[threadIdx.x] = 0ull;
    if (STATS) __syncthreads();
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    Stats st = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (i < n) {
        f3 o, d;
        float time, tmax;
        if (GEN && i >= nq) {
            primary_ray(cam, ps, seed, gbase + (i - nq), o, d, time);
            tmax = FLT_MAX;
        } else {
            load_ray(rays, i, o, d, time);
            tmax = FLT_MAX;
        }
        // a wave of camera samples only (a pixel's samples, or adjacent pixels'): the wave-uniform walk
        constexpr bool KUNI = GEN && !TLAS && !EXHAUSTIVE;
        const bool uni = KUNI && sv.uni_walk && (int)(blockIdx.x * blockDim.x) >= nq;
        HitRec h = closest_hit<EXHAUSTIVE, STATS, TLAS, KUNI>(sv, o, d, time, tmax, s_stack + threadIdx.x, kTraceBlock, st,
                                                             s_tstack + (TLAS ? threadIdx.x : 0), uni,
                                                             STATS ? s_ecyc : nullptr);
        if (compact) {
            hit_planes(hits, n).id[i] = make_int2(h.obj, h.prim);
        } else {
            hits[i] = h;
        }
    }
    if (STATS) {
        unsigned long long nv = st.nodes, nt = st.tris, ns = st.steps, ne = st.entries, gw = st.gwork;
        unsigned mx = st.steps, mc = st.considered, mg = st.gslot;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_down(nv, off);
            nt += __shfl_down(nt, off);
            ns += __shfl_down(ns, off);
            ne += __shfl_down(ne, off);
            gw += __shfl_down(gw, off);
            mx = max(mx, (unsigned)__shfl_xor((int)mx, off));
            mc = max(mc, (unsigned)__shfl_xor((int)mc, off));
            mg = max(mg, (unsigned)__shfl_xor((int)mg, off));
        }
        __syncthreads();
        if (threadIdx.x < 16 && s_ecyc[threadIdx.x]) atomicAdd(&ctr->trace_entry_cycles[threadIdx.x], s_ecyc[threadIdx.x]);
        if (threadIdx.x >= 16 && threadIdx.x < 18 && s_ecyc[threadIdx.x])
            atomicAdd(&ctr->trace_group_cycles[threadIdx.x - 16], s_ecyc[threadIdx.x]);
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&ctr->trace_group_work, gw);
            atomicAdd(&ctr->trace_group_slots, 64ull * mg);
            atomicAdd(&ctr->node_visits, nv);
            atomicAdd(&ctr->tri_tests, nt);
            atomicAdd(&ctr->trace_lane_slots, 64ull * mx);
            atomicAdd(&ctr->trace_steps, ns);
            atomicAdd(&ctr->trace_entry_visits, ne);
            atomicAdd(&ctr->trace_entry_slots, 64ull * mc);
        }
    }
}

struct QRay { f3 o, d; float time; };      // a child ray on its way to the next level's queue
DEV QRay make_ray(f3 o, f3 d, float time) {
    QRay r;
    r.o = o; r.d = d; r.time = time;
    return r;
}

// Scene::MirrorReflectance (src/Scene.cpp:32-55): reflected ray of node `path`
DEV void mirror_ray(const SceneView& sv, f3 dir, const Ret& ret, const MaterialDev& m, uint64_t seed,
                    uint32_t pixel, uint32_t sample, uint64_t path, f3& ro, f3& rd) {
    f3 wo = -dir;
    float n_wo = dot(ret.normal, wo);
    f3 wr = -wo + (ret.normal * 2) * n_wo;
    wr = wr / norm(wr);
    if (m.is_rough) {
        f3 u = ortho_u(wr);
        f3 v = cross(wr, u);
        float xi[4];
        rng4(seed, pixel, sample, path, RNG_ROUGH, 0, 0, xi);
        float uChi = xi[0] - 0.5f, vChi = xi[1] - 0.5f;
        wr = normalized(wr + (u * uChi + v * vChi) * m.roughness);
    }
    ro = ret.point + ret.normal * sv.shadow_eps;
    rd = wr;
}

// TEX (full variant only): object texturing and BRDFs compiled in; a full scene without them
// (area / environment lights, background texture) runs k_shade<true, *, 256, false>, which has
// far fewer live registers.
// One ray's shading step (Scene::RecursiveShading for the node) plus the level's compaction of
// child rays and shadow queries.  Called by every thread of the block (it synchronises); lanes
// with i >= n only take part in the compaction.  h / o / d / time / mt: the traced ray and its hit.
template <bool FULL, bool SPOT, int BLOCK, bool TEX>
DEV void shade_ray(const SceneView& sv, const CameraDev& cam, int level, const PassDev& ps, uint64_t seed, int i,
                   int n, const HitIn& hin, const f3 o, const f3 d, const float time, const RayMeta& mt,
                   const NodePlanes& nodes, const ShadowPlanes& shadows, int* __restrict__ slist,
                   const RayQ& next_rays, RayMeta* __restrict__ next_meta, unsigned long long* qcount,
                   unsigned char* __restrict__ lv_out) {
    const HitRec& h = hin.h;
    // (the point store below; decided here for the whole wave -- a superset -- so that neither the
    // origin nor a per-lane flag is live across the shading)
    const bool o_far = __ballot(!(fabsf(o.x) < 1e17f && fabsf(o.y) < 1e17f && fabsf(o.z) < 1e17f)) != 0ull;
    int nchild = 0;
    QRay c0r, c1r;
    RayMeta c0m, c1m;
    bool has0 = false, has1 = false;
    bool hit = false;
    NodeRec nd;
    unsigned long long smask = 0;   // lights whose shadow query must be traced
    if (i < n) {
        uint32_t pixel, sample;
        int x, y;
        slot_pixel(cam, ps, mt.slot, pixel, sample, x, y);
        uint64_t path = ((uint64_t)mt.path_hi << 32) | mt.path_lo;
        nd.px = nd.py = nd.pz = 0.0f;
        nd.cr = nd.cg = nd.cb = 0.0f;
        nd.kind = NK_FINAL;
        nd.F = 0.0f;
        nd.child0 = nd.child1 = -1;
        nd.material = 0;
        nd.slot = mt.slot;
        bool basic = false;
        if (h.obj < 0) {
            if (level == 0) {
                // SingleSample passes (row=x, col=y) (Scene.cpp:365-380); MultiSample (row=y, col=x)
                f3 bg = !FULL ? ld3(sv.background)
                      : (cam.total > 1) ? background(sv, cam, y, x, d) : background(sv, cam, x, y, d);
                nd.cr = bg.x; nd.cg = bg.y; nd.cb = bg.z;
            }
        } else {
            hit = true;
            // a wave whose hits are all on one entry (a pixel's samples on the dragon, say) reads that
            // entry's records and material through the scalar cache: the same calls with the entry index
            // made wave-uniform (readfirstlane), instead of 64 identical per-lane gathers
            Ret ret;
            MaterialDev m;
            const int ob0 = __builtin_amdgcn_readfirstlane(h.obj);
            if (__ballot(h.obj != ob0) == 0ull) {
                HitRec hu = h;
                hu.obj = ob0;
                ret = hit_record<FULL && TEX>(sv, o, d, time, hu);
                m = sv.materials[sv.tops[ob0].material - 1];
            } else {
                ret = hit_record<FULL && TEX>(sv, o, d, time, h);
                m = sv.materials[ret.matIndex - 1];
            }
            nd.px = ret.point.x; nd.py = ret.point.y; nd.pz = ret.point.z;
            nd.material = ret.matIndex;
            if (level == 0 && ret.dm == RTG_DECAL_REPLACE_ALL) {          // Scene::Shading Scene.cpp:230-241
                nd.cr = ret.tc.x; nd.cg = ret.tc.y; nd.cb = ret.tc.z;
            } else {
                int depth = mt.depth;
                uint64_t p0 = 2 * path, p1 = 2 * path + 1;
                if (m.type == RTG_MAT_NORMAL || depth <= 0) {            // RecursiveShading Scene.cpp:148-158
                    basic = true;
                } else if (m.type == RTG_MAT_MIRROR) {                   // Scene.cpp:159-165
                    basic = true;
                    nd.kind = NK_MIRROR;
                    f3 ro, rd;
                    mirror_ray(sv, d, ret, m, seed, pixel, sample, path, ro, rd);
                    if (!(isnan3(ro) || isnan3(rd))) {
                        has1 = true; c1r = make_ray(ro, rd, time);
                        c1m.slot = mt.slot; c1m.path_lo = (unsigned)p1; c1m.path_hi = (unsigned)(p1 >> 32); c1m.depth = depth - 1;
                    }
                } else if (m.type == RTG_MAT_DIELECTRIC) {               // Scene.cpp:166-209, DielectricRefraction Scene.cpp:57-118
                    float dp = dot(d, ret.normal);
                    float nt = m.refraction_index;
                    float snell, n_t, n_i;
                    f3 normal;
                    bool entering;
                    if (dp < 0) { snell = 1.0f / nt; normal = ret.normal; n_t = nt; n_i = 1; entering = true; }
                    else { snell = nt; normal = -ret.normal; n_t = 1; n_i = nt; entering = false; }
                    float cosTheta = -dot(d, normal);
                    f3 leftPart = (d + normal * cosTheta) * snell;
                    float srp = (float)(1 - sq_d(snell) * (1 - sq_d(cosTheta)));
                    bool isTir = srp < 0;
                    srp = sqrtf(srp);
                    f3 tdir = normalized(leftPart - normal * srp);
                    f3 torg = ret.point - normal * sv.shadow_eps;
                    float cos_t = -dot(tdir, normal);
                    float cos_i = -dot(d, normal);
                    float rPar = (n_t * cos_i - n_i * cos_t) / (n_t * cos_i + n_i * cos_t);
                    float rPer = (n_i * cos_i - n_t * cos_t) / (n_i * cos_i + n_t * cos_t);
                    nd.F = (float)(0.5f * (sq_d(rPar) + sq_d(rPer)));
                    nd.kind = entering ? NK_DIEL_ENTER : (isTir ? NK_DIEL_TIR : NK_DIEL_EXIT);
                    basic = entering;
                    if (!(isnan3(torg) || isnan3(tdir))) {
                        // the refracted ray is traced in every case (its hit point feeds Beer's law)
                        has0 = true; c0r = make_ray(torg, tdir, time);
                        c0m.slot = mt.slot; c0m.path_lo = (unsigned)p0; c0m.path_hi = (unsigned)(p0 >> 32); c0m.depth = depth - 1;
                    }
                    f3 ro, rd;
                    mirror_ray(sv, d, ret, m, seed, pixel, sample, path, ro, rd);
                    if (!(isnan3(ro) || isnan3(rd))) {
                        has1 = true; c1r = make_ray(ro, rd, time);
                        c1m.slot = mt.slot; c1m.path_lo = (unsigned)p1; c1m.path_hi = (unsigned)(p1 >> 32); c1m.depth = depth - 1;
                    }
                } else {                                                 // conductor Scene.cpp:210-218
                    basic = true;
                    nd.kind = NK_CONDUCTOR;
                    nd.F = conductor_fresnel(m.refraction_index, m.absorption_index, d, ret.normal);
                    f3 ro, rd;
                    mirror_ray(sv, d, ret, m, seed, pixel, sample, path, ro, rd);
                    if (!(isnan3(ro) || isnan3(rd))) {
                        has1 = true; c1r = make_ray(ro, rd, time);
                        c1m.slot = mt.slot; c1m.path_lo = (unsigned)p1; c1m.path_hi = (unsigned)(p1 >> 32); c1m.depth = depth - 1;
                    }
                }
                if (basic) {
                    // Scene::ambient Scene.cpp:22-30 (0 + La*ka); the lights are added in order by
                    // k_shadow (one light) or k_light_sum (several)
                    f3 amb = mk(0, 0, 0) + cw(ld3(sv.ambient), ld3(m.ambient));
                    nd.cr = amb.x; nd.cg = amb.y; nd.cb = amb.z;
                    for (int li = 0; li < sv.num_lights; li++) {
                        ShadowRec sr;
                        light_sample<FULL, SPOT, (FULL && TEX) ? 2 : 0, false>(sv, li, d, time, ret, m, seed, pixel, sample, path, sr);
                        // one light: a query that is not traced is never read (k_light_sum reads
                        // every record when there are several)
                        if (sr.c.w != 0.0f || sv.num_lights > 1) {
                            const size_t k = (size_t)li * shadows.nn + i;     // light-major (ShadowPlanes)
                            if (sv.lean_shadow && !sv.has_blur) {
                                // the 12-byte origin plane only (lit node, below)
                                reinterpret_cast<float3*>(shadows.o)[i] = make_float3(sr.o.x, sr.o.y, sr.o.z);
                            } else {
                                // the origin (+ time) is the node's, whatever the light: one record
                                // per node, at the node's index; the direction (+ light distance) only
                                // for a traced query (k_light_sum reads every contribution; one
                                // light: no contribution plane, k_shadow knows the mode from the light)
                                if (li == 0) shadows.o[i] = sr.o;
                                if (!sv.lit_nodes) shadows.c[k] = sr.c;
                                if (!sv.lean_shadow && sr.c.w != 0.0f) shadows.d[k] = sr.d;
                            }
                            // one light (SceneView::lit_nodes): the node stores its lit colour
                            // (ambient + contribution) and its material, and k_shadow puts the
                            // ambient term back if the light is blocked
                            if (sv.lit_nodes && sr.c.w != 0.0f) {
                                nd.cr = nd.cr + sr.c.x; nd.cg = nd.cg + sr.c.y; nd.cb = nd.cb + sr.c.z;
                                nd.kind |= nd.material << kNodeMatShift;
                            }
                        }
                        if (sr.c.w != 0.0f) smask |= 1ull << li;
                        else if (sv.num_lights == 1) { nd.cr = nd.cr + 0.0f; nd.cg = nd.cg + 0.0f; nd.cb = nd.cb + 0.0f; }
                    }
                }
            }
        }
        if (basic) nd.kind |= 0x100;
        nchild = (has0 ? 1 : 0) + (has1 ? 1 : 0);
    }
    // Compaction of the next level's rays and of the shadow-query list (entries
    // i * nLights + li, light-major within a wave): ballot prefixes inside each wave, wave
    // totals combined in LDS, ONE 64-bit atomic per block on the level's queue counter
    // (low word: rays, high word: shadow entries).  Same-address atomics serialise at the L2
    // (~11 ns each), so they are kept to one per block.
    __shared__ unsigned s_wc[BLOCK / 64], s_ws[BLOCK / 64];
    __shared__ unsigned long long s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = __lanemask_lt();
    const unsigned long long m1 = __ballot(nchild >= 1), m2 = __ballot(nchild >= 2);
    const unsigned coff = __popcll(m1 & lt) + __popcll(m2 & lt);
    unsigned stot = 0;
    for (int li = 0; li < sv.num_lights; li++) stot += __popcll(__ballot((smask >> li) & 1ull));
    if (lane == 0) { s_wc[w] = __popcll(m1) + __popcll(m2); s_ws[w] = stot; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned c = 0, sh = 0;
        for (int k = 0; k < BLOCK / 64; k++) {
            const unsigned a = s_wc[k], b = s_ws[k];
            s_wc[k] = c; s_ws[k] = sh;
            c += a; sh += b;
        }
        s_base = (c | sh) ? atomicAdd(qcount, ((unsigned long long)sh << 32) | c) : 0ull;
    }
    __syncthreads();
    int idx = (int)((unsigned)s_base + s_wc[w] + coff);
    if (i < n) {
        auto put_ray = [&](int k, const QRay& rr, const RayMeta& mm) {
            store_ray(next_rays, k, rr.o, rr.d, rr.time);
            if (!sv.meta_free) next_meta[k] = mm;
            if (lv_out) lv_out[k] = (unsigned char)(level + 1);
        };
        if (has0) { put_ray(idx, c0r, c0m); nd.child0 = idx; idx++; }
        if (has1) { put_ray(idx, c1r, c1m); nd.child1 = idx; }
        // kNodeFar: a hit point whose distance to another could overflow (or is not finite) --
        // k_resolve then reads it even for Beer's law with zero absorption
        const bool far = hit && !(fabsf(nd.px) < 1e18f && fabsf(nd.py) < 1e18f && fabsf(nd.pz) < 1e18f);
        nodes.col[i] = make_float4(nd.cr, nd.cg, nd.cb,
                                   __int_as_float(nd.kind | (hit ? kNodeHit : 0) | (far ? kNodeFar : 0)));
        // the point plane's readers: k_shadow (a node with a query: on the lean path, the material
        // bits of its kind word), this node's own resolve (conductor / dielectric: F and, for Beer's
        // law, p) and a dielectric parent's Beer's law on its refracted child -- read only when the
        // parent's material absorbs (sv.pnt_all) or a point is far: the child's own (kNodeFar) or
        // the parent's, whose refracted ray then starts far from the origin too (|o| >= 1e18 - eps;
        // SceneView::pnt_all also covers eps >= 1e17)
        const int nk = nd.kind & 0xFF;
        if (hit && (!sv.lean_shadow || sv.has_blur || sv.pnt_all || (nd.kind >> kNodeMatShift) != 0 || far ||
                    o_far || (nk != NK_FINAL && nk != NK_MIRROR)))
            nodes.pnt[i] = make_float4(nd.px, nd.py, nd.pz, nd.F);
        if ((nd.kind & 0xFF) != NK_FINAL) nodes.link[i] = make_int4(nd.child0, nd.child1, nd.material, 0);
    }
    unsigned sb = (unsigned)(s_base >> 32) + s_ws[w];
    for (int li = 0; li < sv.num_lights; li++) {
        const bool need = (smask >> li) & 1ull;
        const unsigned long long m = __ballot(need);
        if (need) slist[sb + __popcll(m & lt)] = li * shadows.nn + i;
        sb += __popcll(m);
    }
}

// Level-0 ray of slot i (no ray buffer) or the queued ray i.
DEV void level_ray(const CameraDev& cam, const PassDev& ps, uint64_t seed, const RayQ& rays, int i,
                   f3& o, f3& d, float& time) {
    if (rays.a == nullptr) primary_ray(cam, ps, seed, i, o, d, time);
    else load_ray(rays, i, o, d, time);
}
DEV RayMeta level_meta(const SceneView& sv, int level, const RayQ& rays, const RayMeta* __restrict__ meta, int i) {
    RayMeta mt;
    if (rays.a == nullptr) {          // level 0: the primary ray's meta
        mt.slot = i; mt.path_lo = 1u; mt.path_hi = 0u; mt.depth = sv.max_depth;
    } else if (sv.meta_free && level > 0) {   // nothing below level 0 draws random numbers
        // (depth from the level: the launch's, or the ray's own in a stream step)
        mt.slot = 0; mt.path_lo = 0u; mt.path_hi = 0u; mt.depth = sv.max_depth - level;
    } else {
        mt = meta[i];
    }
    return mt;
}

// GEN: the launch holds generated primary rays at i >= nq (slot gbase + i - nq; a pass's level 0:
// nq = 0), else queued rays only -- separate instantiations, so a queued-only launch carries no
// ray-generation live ranges.  A queued ray's level is lv_in[i] in a stream step (levels mixed in
// one launch), else `level_in`; lv_out (when set) receives the children's levels.
template <bool FULL, bool SPOT, int BLOCK = FULL ? 256 : kShadeBlock, bool TEX = FULL, bool GEN = false>
__global__ void __launch_bounds__(BLOCK) RTG_SHADE_ATTR k_shade(const SceneView sv, const CameraDev cam, int level_in, const PassDev ps,
                                               uint64_t seed,
                                               const RayQ rays, const RayMeta* __restrict__ meta,
                                               const HitRec* __restrict__ hits, const NodePlanes nodes,
                                               const ShadowPlanes shadows, int* __restrict__ slist,
                                               const RayQ next_rays, RayMeta* __restrict__ next_meta,
                                               unsigned long long* qcount, int n, int nq, int gbase,
                                               const unsigned char* __restrict__ lv_in,
                                               unsigned char* __restrict__ lv_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    HitIn h;
    h.h.obj = -1; h.h.prim = -1; h.h.t = 0.0f; h.h.pad = 0;
    f3 o = mk(0, 0, 0), d = mk(0, 0, 0);
    float time = 0.0f;
    RayMeta mt = {};
    int level = level_in;
    if (i < n) {
        h = load_hit_planes(hits, n, i);
        if (GEN && i >= nq) {
            const int slot = gbase + (i - nq);
            primary_ray(cam, ps, seed, slot, o, d, time);
            mt.slot = slot; mt.path_lo = 1u; mt.path_hi = 0u; mt.depth = sv.max_depth;
            level = 0;
        } else {
            if (lv_in) level = lv_in[i];
            load_ray(rays, i, o, d, time);
            mt = level_meta(sv, level, rays, meta, i);
        }
    }
    shade_ray<FULL, SPOT, BLOCK, TEX>(sv, cam, level, ps, seed, i, n, h, o, d, time, mt, nodes, shadows, slist,
                                      next_rays, next_meta, qcount, lv_out);
}

// ------------------------------------------------------------------ hw7 path tracer
// One shading step of oracle/rtg_oracle.c pt_sample() per ray (no reference code exists:
// pages/Page7.md describes the integrator in prose; DESIGN.md §8 fixes it).  Adds the vertex's
// T (x) v to the sample's running radiance (PtRad) when no shadow query is pending, else leaves the
// node record (colour, point + last light, throughput + radiance target) for k_shadow, and queues
// at most one continuation ray.
struct DielSplit {
    bool entering, tir;
    float F;
    f3 tdir, torg;
};
DEV DielSplit dielectric_split(const SceneView& sv, f3 d, const Ret& ret, const MaterialDev& m) {   // Scene.cpp:57-128
    DielSplit r;
    float dp = dot(d, ret.normal);
    float nt = m.refraction_index;
    float snell, n_t, n_i;
    f3 normal;
    if (dp < 0) { snell = 1.0f / nt; normal = ret.normal; n_t = nt; n_i = 1; r.entering = true; }
    else { snell = nt; normal = -ret.normal; n_t = 1; n_i = nt; r.entering = false; }
    float cosTheta = -dot(d, normal);
    f3 leftPart = (d + normal * cosTheta) * snell;
    float srp = (float)(1 - sq_d(snell) * (1 - sq_d(cosTheta)));
    r.tir = srp < 0;
    srp = sqrtf(srp);
    r.tdir = normalized(leftPart - normal * srp);
    r.torg = ret.point - normal * sv.shadow_eps;
    float cos_t = -dot(r.tdir, normal);
    float cos_i = -dot(d, normal);
    float rPar = (n_t * cos_i - n_i * cos_t) / (n_t * cos_i + n_i * cos_t);
    float rPer = (n_i * cos_i - n_t * cos_t) / (n_i * cos_i + n_t * cos_t);
    r.F = (float)(0.5f * (sq_d(rPar) + sq_d(rPer)));
    return r;
}

constexpr int kContrib = 0x200;   // NodeRec.kind: the vertex adds T (x) colour to the sample

// GEN: the launch may hold generated primary rays (level 0) at i >= nq, slot gbase + i - nq (a
// pass's level 0: nq = 0; a stream step: survivors then new samples), else queued rays only
// (separate instantiations, as k_shade).  A queued ray's level is lv_in[i] when the schedule
// mixes levels in one launch (stream steps), else `level_in`; lv_out (when set) receives the
// continuation's level.
template <bool FULL, bool SPOT, int BRDF, bool GEN = false>
__global__ void __launch_bounds__(kPtBlock) RTG_PT_SHADE_ATTR k_pt_shade(const SceneView sv, const CameraDev cam, int level_in, const PassDev ps,
                                                  uint64_t seed, const RayQ rays,
                                                  const RayMeta* __restrict__ meta, const HitRec* __restrict__ hits,
                                                  PathRec* __restrict__ paths, const NodePlanes nodes,
                                                  const ShadowPlanes shadows, int* __restrict__ slist,
                                                  const RayQ next_rays, RayMeta* __restrict__ next_meta,
                                                  PathRec* __restrict__ next_paths, unsigned long long* qcount, int n,
                                                  int nq, int gbase, const unsigned char* __restrict__ lv_in,
                                                  unsigned char* __restrict__ lv_out, const PtRad pr, Counters* ctr) {
    constexpr int BLOCK = kPtBlock;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    // collect_stats (ctr): wave cycles by phase (Counters::pt_shade_cycles), charged by each wave's
    // first active lane at the end of the phase
    __shared__ unsigned long long s_cyc[4];
    if (ctr && threadIdx.x < 4) s_cyc[threadIdx.x] = 0ull;
    if (ctr) __syncthreads();
    const unsigned long long t_start = ctr ? __builtin_amdgcn_s_memtime() : 0ull;
    auto charge = [&](int r, unsigned long long t0) {
        if (ctr && (__ballot(1) & __lanemask_lt()) == 0ull) atomicAdd(&s_cyc[r], __builtin_amdgcn_s_memtime() - t0);
    };
    bool has = false;
    QRay cr;
    RayMeta cm;
    PathRec cp;
    NodeRec nd;
    f3 Tg = mk(0, 0, 0);            // the vertex's Beer-attenuated throughput
    f3 Lrun = mk(0, 0, 0);          // the sample's radiance before this vertex (a new sample: 0)
    unsigned long long smask = 0;
    int level = 0;
    if (i < n) {
        f3 o, d;
        float time;
        RayMeta mt;
        const bool gen = GEN && i >= nq;
        if (gen) {                      // level 0 without a ray queue: generate the primary ray and its meta
            const int slot = gbase + (i - nq);
            primary_ray(cam, ps, seed, slot, o, d, time);
            mt.slot = slot; mt.path_lo = 1u; mt.path_hi = 0u; mt.depth = sv.max_depth;
        } else {
            // a path's queued ray carries only its sample slot (4 bytes in the meta buffer) and,
            // in a stream step, its level (1 byte): the path key is level + 1 and the remaining
            // depth max_depth - level at every level
            level = lv_in ? (int)lv_in[i] : level_in;
            load_ray(rays, i, o, d, time);
            mt.slot = reinterpret_cast<const int*>(meta)[i];
            mt.path_lo = (unsigned)level + 1u; mt.path_hi = 0u; mt.depth = sv.max_depth - level;
        }
        const HitIn hin = load_hit_planes(hits, n, i);
        const HitRec& h = hin.h;
        uint32_t pixel, sample;
        int x, y;
        slot_pixel(cam, ps, mt.slot, pixel, sample, x, y);
        const uint64_t path = (uint64_t)level + 1;
        const int flags = sv.pt_flags;
        f3 T = mk(1, 1, 1);
        int spec = 1, medium = 0;
        if (!gen && level > 0) {
            const PathRec ph = paths[i];
            T = mk(ph.tr, ph.tg, ph.tb);
            spec = ph.flags & 1;
            medium = ph.flags >> 8;
            const float4 z = pr.carry_in[i];        // the sample's radiance so far (PtRad)
            Lrun = mk(z.x, z.y, z.z);
        }
        nd.px = nd.py = nd.pz = 0.0f;
        nd.cr = nd.cg = nd.cb = 0.0f;
        nd.F = 0.0f;
        nd.child0 = nd.child1 = -1;
        nd.material = 0;
        nd.slot = mt.slot;
        int kind = NK_FINAL;
        if (h.obj < 0) {
            if (level == 0) {     // primary miss: the reference's background rules
                f3 bg = !FULL ? ld3(sv.background)
                      : (cam.total > 1) ? background(sv, cam, y, x, d) : background(sv, cam, x, y, d);
                nd.cr = bg.x; nd.cg = bg.y; nd.cb = bg.z;
                kind |= kContrib;
            }
        } else {
            // one entry for the whole wave (camera samples on one surface): its records through the
            // scalar cache (as k_shade)
            Ret ret;
            const int ob0 = __builtin_amdgcn_readfirstlane(h.obj);
            if (__ballot(h.obj != ob0) == 0ull) {
                HitRec hu = h;
                hu.obj = ob0;
                ret = hit_record<FULL>(sv, o, d, time, hu);
            } else {
                ret = hit_record<FULL>(sv, o, d, time, h);
            }
            nd.px = ret.point.x; nd.py = ret.point.y; nd.pz = ret.point.z;
            nd.material = ret.matIndex;
            if (medium) {                                              // Beer's law inside
                const MaterialDev& mm = sv.materials[medium - 1];
                const float bd = norm(ret.point - o);
                T = cw(T, mk(f_exp(-mm.absorption[0] * bd), f_exp(-mm.absorption[1] * bd),
                             f_exp(-mm.absorption[2] * bd)));
            }
            const int em = sv.top_emit[h.obj];
            if (em >= 0) {                                             // object light: emit, stop
                if (level == 0 || !(flags & RTG_PT_NEE) || spec) {
                    const LightDev& L = sv.lights[em];
                    nd.cr = L.inten[0]; nd.cg = L.inten[1]; nd.cb = L.inten[2];
                    kind |= kContrib;
                }
            } else if (level == 0 && ret.dm == RTG_DECAL_REPLACE_ALL) {
                nd.cr = ret.tc.x; nd.cg = ret.tc.y; nd.cb = ret.tc.z;
                kind |= kContrib;
            } else {
                MaterialDev m;
                const int mi0 = __builtin_amdgcn_readfirstlane(ret.matIndex);
                if (__ballot(ret.matIndex != mi0) == 0ull) m = sv.materials[mi0 - 1];
                else m = sv.materials[ret.matIndex - 1];
                DielSplit ds;
                ds.entering = true; ds.tir = false; ds.F = 0.0f;
                if (m.type == RTG_MAT_DIELECTRIC) ds = dielectric_split(sv, d, ret, m);
                charge(0, t_start);
                const unsigned long long t_nee = ctr ? __builtin_amdgcn_s_memtime() : 0ull;
                if (ds.entering) {                                     // BasicShading + NEE
                    kind |= kContrib | 0x100;
                    const f3 amb = mk(0, 0, 0) + cw(ld3(sv.ambient), ld3(m.ambient));
                    nd.cr = amb.x; nd.cg = amb.y; nd.cb = amb.z;
                    for (int li = 0; li < sv.num_lights; li++) {
                        ShadowRec sr;
                        light_sample<FULL, SPOT, BRDF>(sv, li, d, time, ret, m, seed, pixel, sample, path, sr);
                        const size_t k = (size_t)li * shadows.nn + i;   // light-major (ShadowPlanes)
                        // only traced queries' records: k_shadow reads nothing else (no light sum)
                        if (sr.c.w != 0.0f) {
                            shadows.c[k] = sr.c;
                            shadows.d[k] = sr.d;
                            smask |= 1ull << li;
                        } else if (sv.num_lights == 1) {
                            nd.cr = nd.cr + 0.0f; nd.cg = nd.cg + 0.0f; nd.cb = nd.cb + 0.0f;
                        }
                    }
                    // the query origin, per node (k_shade's layout; light_sample's origin is the same
                    // for every light), only when a query is traced
                    if (smask) {
                        const f3 og = ret.point + ret.normal * sv.shadow_eps;
                        shadows.o[i] = make_float4(og.x, og.y, og.z, time);
                    }
                }
                charge(1, t_nee);
                const unsigned long long t_cont = ctr ? __builtin_amdgcn_s_memtime() : 0ull;
                const bool cont = (flags & RTG_PT_RUSSIAN_ROULETTE) ? (level + 1 < RTG_PT_MAX_BOUNCES) : (mt.depth > 0);
                if (cont) {
                    float xi[4];
                    rng4(seed, pixel, sample, path, RNG_PT_BOUNCE, 0, 0, xi);
                    f3 w = mk(1, 1, 1), no, ndir;
                    int nspec = 1, nmedium = medium;
                    if (m.type == RTG_MAT_NORMAL) {                    // hemisphere sample
                        const f3 nn = ret.normal, u = ortho_u(nn), bt = cross(nn, u);
                        const float phi = (float)(2 * PI_D) * xi[0];
                        const float cosT = (flags & RTG_PT_IMPORTANCE) ? sqrtf(1.0f - xi[1]) : xi[1];
                        const float sinT = sqrtf(fmax0(1.0f - cosT * cosT));
                        float sp, cp;
                        f_sincos(phi, sp, cp);
                        const f3 wi = normalized((u * (sinT * cp) + nn * cosT) + bt * (sinT * sp));
                        const f3 fc = phong_or_brdf<BRDF>(mk(1, 1, 1), -d, wi, ret, m);
                        if (flags & RTG_PT_IMPORTANCE) w = cosT > 0.0f ? fc * ((float)PI_D / cosT) : mk(0, 0, 0);
                        else w = fc * (float)(2 * PI_D);
                        no = ret.point + nn * sv.shadow_eps;
                        ndir = wi;
                        nspec = 0;
                    } else if (m.type == RTG_MAT_DIELECTRIC && !ds.tir && !(xi[3] < ds.F)) {   // refract
                        no = ds.torg;
                        ndir = ds.tdir;
                        nmedium = ds.entering ? ret.matIndex : 0;
                    } else {                                           // reflect
                        mirror_ray(sv, d, ret, m, seed, pixel, sample, path, no, ndir);
                        if (m.type == RTG_MAT_MIRROR) w = ld3(m.mirror);
                        else if (m.type == RTG_MAT_CONDUCTOR)
                            w = ld3(m.mirror) * conductor_fresnel(m.refraction_index, m.absorption_index, d, ret.normal);
                    }
                    bool ok = !(isnan3(no) || isnan3(ndir));
                    if (ok && (flags & RTG_PT_RUSSIAN_ROULETTE)) {
                        const float qc = fabsf(dot(ret.normal, ndir));
                        ok = xi[2] < qc;
                        if (ok) w = w / qc;
                    }
                    if (ok) {
                        const f3 Tn = cw(T, w);
                        if (!(Tn.x == 0.0f && Tn.y == 0.0f && Tn.z == 0.0f)) {
                            has = true;
                            cr = make_ray(no, ndir, time);
                            cm.slot = mt.slot; cm.path_lo = (unsigned)(path + 1); cm.path_hi = 0u; cm.depth = mt.depth - 1;
                            cp.tr = Tn.x; cp.tg = Tn.y; cp.tb = Tn.z; cp.flags = nspec | (nmedium << 8);
                        }
                    }
                }
                charge(2, t_cont);
            }
        }
        nd.kind = kind;
        Tg = T;
    }
    const unsigned long long t_store = ctr ? __builtin_amdgcn_s_memtime() : 0ull;
    // compaction: one continuation per lane (one 64-bit atomic per block: continuations | shadow
    // queries << 32, the host's counts), and per light one list (slist + li * n, counted in
    // pr.lcnt[li]: k_shadow runs the lights' lists one launch after the other, in light order).  Wave
    // counts in LDS, then one thread per light forms its waves' offsets and takes the light's base
    // (one atomic per light with queries): two barriers for all of it.
    __shared__ unsigned s_wc[BLOCK / 64];
    __shared__ unsigned s_lw[kMaxLights][BLOCK / 64];   // per light: the waves' query counts ...
    __shared__ unsigned s_lo[kMaxLights][BLOCK / 64];   // ... and their offsets in the light's list
    __shared__ unsigned s_lbase[kMaxLights];
    __shared__ unsigned long long s_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long lt = __lanemask_lt();
    const unsigned long long m1 = __ballot(has);
    const unsigned coff = __popcll(m1 & lt);
    for (int li = 0; li < sv.num_lights; li++) {
        const unsigned c = __popcll(__ballot((smask >> li) & 1ull));
        if (lane == 0) s_lw[li][wv] = c;
    }
    if (lane == 0) s_wc[wv] = __popcll(m1);
    __syncthreads();
    if (threadIdx.x < sv.num_lights) {
        const int li = threadIdx.x;
        unsigned c = 0;
        for (int k = 0; k < BLOCK / 64; k++) {
            s_lo[li][k] = c;
            c += s_lw[li][k];
        }
        s_lbase[li] = c ? atomicAdd(pr.lcnt + li, c) : 0u;
    }
    if (threadIdx.x == 0) {
        unsigned c = 0, sh = 0;
        for (int k = 0; k < BLOCK / 64; k++) {
            const unsigned a = s_wc[k];
            s_wc[k] = c;
            c += a;
            for (int li = 0; li < sv.num_lights; li++) sh += s_lw[li][k];
        }
        s_base = (c | sh) ? atomicAdd(qcount, ((unsigned long long)sh << 32) | c) : 0ull;
    }
    __syncthreads();
    const int idx = (int)((unsigned)s_base + s_wc[wv] + coff);
    if (i < n) {
        if (has) {
            store_ray(next_rays, idx, cr.o, cr.d, cr.time);
            reinterpret_cast<int*>(next_meta)[idx] = cm.slot;
            next_paths[idx] = cp;
            if (lv_out) lv_out[idx] = (unsigned char)(level + 1);
        }
        // the radiance's target: the continuation's queue slot, or the sample's slot of rad
        float4* tgt = has ? pr.carry_out + idx : pr.rad + nd.slot;
        if (smask == 0) {
            // nothing pending: L + T (x) v here (Scene::RecursiveShading's col = ((amb + L0) + L1) + ...
            // with every light term +0 -- v is never -0, so adding +0 leaves it unchanged)
            f3 L = Lrun;
            if (nd.kind & kContrib) L = L + cw(Tg, mk(nd.cr, nd.cg, nd.cb));
            *tgt = make_float4(L.x, L.y, L.z, 0.0f);
        } else {
            // traced queries: k_shadow adds the lit lights to the colour and the last one writes
            // L + T (x) v to the target; L waits in this ray's own queue slot (its carry was read
            // above).  pnt.w: that last light's index.
            pr.carry_in[i] = make_float4(Lrun.x, Lrun.y, Lrun.z, 0.0f);
            nodes.col[i] = make_float4(nd.cr, nd.cg, nd.cb, __int_as_float(nd.kind));
            nodes.pnt[i] = make_float4(nd.px, nd.py, nd.pz, __int_as_float(63 - __clzll((long long)smask)));
            nodes.link[i] = make_int4(__float_as_int(Tg.x), __float_as_int(Tg.y), __float_as_int(Tg.z),
                                      has ? idx : ~nd.slot);
        }
    }
    for (int li = 0; li < sv.num_lights; li++) {
        const bool need = (smask >> li) & 1ull;
        const unsigned long long m = __ballot(need);
        if (need) slist[(size_t)li * n + s_lbase[li] + s_lo[li][wv] + __popcll(m & lt)] = li * shadows.nn + i;
    }
    if (ctr) {
        charge(3, t_store);
        __syncthreads();
        if (threadIdx.x < 4 && s_cyc[threadIdx.x]) atomicAdd(&ctr->pt_shade_cycles[threadIdx.x], s_cyc[threadIdx.x]);
    }
}

// Shadow queries + in-order light sum of Scene::BasicShading (src/Scene.cpp:243-267).
// One thread per traced shadow query (compacted by k_shade).  With one light the result is
// added to the node colour here (col + c or col + 0, as Scene::BasicShading's light loop
// does); with several, the visibility is recorded and k_light_sum adds them in light order.
// Each query is a full closest-hit FindIntersection, as Light::IsShadow does
// (src/Light.cpp:188-204): the distance test below decides blocking.
// PT: the path tracer's queries of one light (one launch per light, in light order; PtRad): a lit
// query adds its light's term to the node colour, and the node's last traced light adds T (x) v to
// the sample's running radiance in its target (the continuation's queue slot or rad[slot]).
template <bool EXHAUSTIVE, bool STATS, bool TLAS = false, bool PT = false>
__global__ void __launch_bounds__(kTraceBlock) RTG_SHADOW_ATTR k_shadow(const SceneView sv,
                                                                       const ShadowPlanes shadows, bool lean,
                                                                       const int* __restrict__ slist,
                                                                       const unsigned* scount, const NodePlanes nodes,
                                                                       unsigned* nan_queries, Counters* ctr,
                                                                       int uni_from, const PtRad pr) {
    __shared__ int s_stack[kLdsStack * kTraceBlock];
    __shared__ short s_tstack[TLAS ? kTlasStack * kTraceBlock : 1];
    __shared__ unsigned long long s_ecyc[STATS ? 18 : 1];   // entries 0..15, group set-up / tests
    if (STATS && threadIdx.x < 18) s_ecyc[threadIdx.x] = 0ull;
    if (STATS) __syncthreads();
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned nanq = 0;
    Stats st = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    bool was_blocked = false;
    if (j < (int)*scount) {
        // list entry li * nn + i (ShadowPlanes: light-major); one light: the node index itself
        // (the path tracer's launches are per light: no division)
        const int idx = slist[j];
        const int li = PT ? pr.light : sv.num_lights == 1 ? 0 : (int)((unsigned)idx / (unsigned)shadows.nn);
        const int i = idx - li * shadows.nn;    // shading node of the query
        // lean3: one point / spot / directional light and no motion blur -- 12-byte origin and
        // lit-colour planes (k_shade), time 0, the mode follows from the light type
        const bool lean3 = lean && !sv.has_blur;
        float4 so;
        if (lean3) {
            const float3 q = reinterpret_cast<const float3*>(shadows.o)[i];
            so = make_float4(q.x, q.y, q.z, 0.0f);
        } else {
            so = shadows.o[i];                  // one origin record per node
        }
        const f3 o = mk(so.x, so.y, so.z);
        f3 d;
        float tmax;
        if (lean) {     // one point / spot / directional light (node idx, light 0): rebuild d, tmax
            const LightDev& L = sv.lights[0];
            if (L.type == RTG_LIGHT_DIRECTIONAL) {
                d = -ld3(L.dir);
                tmax = FLT_MAX;
            } else {
                const float4 pf = nodes.pnt[i];
                const f3 p = mk(pf.x, pf.y, pf.z), lp = ld3(L.pos);
                d = toward(lp, p);
                tmax = shadow_tmax(o, p, lp, sv.shadow_eps);
            }
        } else {
            // direction + light distance; the t bound light_sample used to store, rebuilt (the node's
            // point only for an object light's bound)
            const float4 sd = shadows.d[idx];
            d = mk(sd.x, sd.y, sd.z);
            // (object lights, mode 3, exist only for the path tracer: the Whitted instantiations leave
            // their bound out, which is their register peak's business)
            const float qm = shadow_mode(sv, li);
            f3 p = mk(0, 0, 0);
            if (PT && qm == 3.0f) {
                const float4 pf = nodes.pnt[i];
                p = mk(pf.x, pf.y, pf.z);
            }
            tmax = shadow_query_tmax<PT>(qm, o, p, d, sd.w, sv.shadow_eps);
        }
        if (isnan3(o) || isnan3(d)) nanq++;     // not a traced ray (the host subtracts these)
        auto ld = [&](const float* a) { return __builtin_nontemporal_load(a); };
        // queries of camera-sample nodes (nodes >= uni_from: level 0 of a pass, a stream step's new
        // samples): a wave whose queries all leave such nodes -- neighbouring points of one or two
        // pixels -- walks wave-uniformly (visit_object)
        constexpr bool KUNI = !EXHAUSTIVE && !TLAS;
        const bool uni = KUNI && sv.uni_walk && __ballot(i < uni_from) == 0ull;
        HitRec h = closest_hit<EXHAUSTIVE, STATS, TLAS, KUNI, PT>(sv, o, d, so.w, EXHAUSTIVE ? FLT_MAX : tmax,
                                                             s_stack + threadIdx.x, kTraceBlock, st,
                                                             s_tstack + (TLAS ? threadIdx.x : 0), uni,
                                                             STATS ? s_ecyc : nullptr);
        // PT: the tail's records in one round of loads after the traversal (the node's point + last
        // light, colour, the query's origin / direction / lit colour; in the last light's launch the
        // throughput + target and L too): one memory latency instead of three dependent ones
        const bool pt_last = PT && pr.light == sv.num_lights - 1;
        float4 t_o, t_d, t_pnt, t_col, t_c, t_lr;
        int4 t_lk;
        if constexpr (PT) {
            t_o = shadows.o[i];
            t_d = shadows.d[idx];
            t_pnt = nodes.pnt[i];
            t_col = nodes.col[i];
            t_c = shadows.c[idx];
            if (pt_last) {
                t_lk = nodes.link[i];
                t_lr = pr.carry_in[i];
            }
        }
        // the query's mode from its light's type (shadow_mode), not a stored record
        const float mode = lean3 ? (sv.lights[0].type == RTG_LIGHT_DIRECTIONAL ? 2.0f : 1.0f) : shadow_mode(sv, li);
        bool blocked;
        if (mode == 1.0f || mode == 3.0f) {
            blocked = false;
            if (h.obj >= 0) {
                // re-read (not kept live across the traversal: register pressure)
                f3 o_;
                if (PT) {
                    o_ = mk(t_o.x, t_o.y, t_o.z);
                } else if (lean3) {
                    const float* qo = reinterpret_cast<const float*>(shadows.o) + 3 * (size_t)i;
                    o_ = mk(ld(qo), ld(qo + 1), ld(qo + 2));
                } else {
                    const float* qo = reinterpret_cast<const float*>(shadows.o + i);
                    o_ = mk(ld(qo), ld(qo + 1), ld(qo + 2));
                }
                const float* pp = reinterpret_cast<const float*>(nodes.pnt + i);
                const f3 p_ = PT ? mk(t_pnt.x, t_pnt.y, t_pnt.z) : mk(ld(pp), ld(pp + 1), ld(pp + 2));
                f3 d_;
                float dl;                       // |p - L|
                if (PT) {
                    d_ = mk(t_d.x, t_d.y, t_d.z);
                    dl = t_d.w;
                } else if (lean) {     // mode 1 with one light: a point / spot light
                    const f3 l_ = ld3(sv.lights[0].pos);
                    d_ = toward(l_, p_);
                    dl = norm(p_ - l_);
                } else {
                    const float* qd = reinterpret_cast<const float*>(shadows.d + idx);
                    d_ = mk(ld(qd), ld(qd + 1), ld(qd + 2));
                    dl = ld(qd + 3);
                }
                f3 hp = o_ + d_ * h.t;
                if (!PT || mode == 1.0f) {      // PointLight::IsShadow: |p - L| > |p - hit|
                    blocked = dl > norm(p_ - hp);
                } else {   // object light (hw7, Page7.md:143-147): an occluder nearer than the sample
                    blocked = norm(p_ - hp) < dl - (sv.shadow_eps + 1e-4f * dl);
                }
            }
        } else {
            blocked = h.obj >= 0;               // directional / environment: any hit
        }
        was_blocked = blocked;
        // lit node (one light, Whitted: SceneView::lit_nodes; its kind word carries the material):
        // k_shade stored the lit colour; blocked: the ambient term alone, recomputed as k_shade
        // formed it (Scene.cpp:22-30: 0 + La * ka; the light's term is 0 and col + 0 == col: the
        // ambient term is never -0).  The path tracer's single-light nodes add the contribution.
        auto restore_ambient = [&](int mi) {
            const MaterialDev& m = sv.materials[mi - 1];
            const f3 amb = mk(0, 0, 0) + cw(ld3(sv.ambient), ld3(m.ambient));
            *reinterpret_cast<float3*>(nodes.col + i) = make_float3(amb.x, amb.y, amb.z);
        };
        if constexpr (PT) {
            // lights in order (this launch is light li's): col = ((amb + L0) + L1) + ..., a blocked or
            // untraced light's term is +0 and leaves the colour unchanged (it is never -0: amb = 0 + La ka)
            f3 v = mk(t_col.x, t_col.y, t_col.z);
            if (!blocked) v = v + mk(t_c.x, t_c.y, t_c.z);
            if (!pt_last && li != __float_as_int(t_pnt.w)) {
                if (!blocked) {
                    float* cp = reinterpret_cast<float*>(nodes.col + i);
                    cp[0] = v.x; cp[1] = v.y; cp[2] = v.z;
                }
            } else {            // the node's last traced light: L + T (x) v (pt_sample's running sum)
                if (!pt_last) {
                    t_lk = nodes.link[i];
                    t_lr = pr.carry_in[i];
                }
                float4* tp = t_lk.w >= 0 ? pr.carry_out + t_lk.w : pr.rad + ~t_lk.w;
                const f3 L = mk(t_lr.x, t_lr.y, t_lr.z) +
                             cw(mk(__int_as_float(t_lk.x), __int_as_float(t_lk.y), __int_as_float(t_lk.z)), v);
                *tp = make_float4(L.x, L.y, L.z, 0.0f);
            }
        } else if (lean3) {
            if (blocked) restore_ambient((int)((unsigned)__float_as_int(nodes.col[i].w) >> kNodeMatShift));
        } else if (sv.num_lights == 1) {
            float* cp = reinterpret_cast<float*>(nodes.col + i);
            const int mi = (int)((unsigned)__float_as_int(cp[3]) >> kNodeMatShift);
            if (mi != 0) {
                if (blocked) restore_ambient(mi);
            } else {
                const float* scp = reinterpret_cast<const float*>(shadows.c + idx);
                f3 add = blocked ? mk(0, 0, 0) : mk(ld(scp), ld(scp + 1), ld(scp + 2));
                cp[0] = cp[0] + add.x;
                cp[1] = cp[1] + add.y;
                cp[2] = cp[2] + add.z;
            }
        } else {
            // blocked: the query's mode (c.w) becomes 0, so the light sum reads one plane only
            if (blocked) reinterpret_cast<float*>(shadows.c + idx)[3] = 0.0f;
        }
    }
    // NaN queries are rare: one atomic per wave that has any
    const unsigned long long nm = __ballot(nanq != 0);
    if (nm && (threadIdx.x & 63) == 0) atomicAdd(nan_queries, (unsigned)__popcll(nm));
    if (STATS) {
        if (was_blocked) {        // node steps until the blocker was accepted / after it (proof of nearest)
            const unsigned before = st.win_step, after = st.steps - st.win_step;
            auto bin = [](unsigned x) { return x == 0 ? 0 : x == 1 ? 1 : x == 2 ? 2 : x <= 4 ? 3 : x <= 8 ? 4 : x <= 16 ? 5 : x <= 32 ? 6 : 7; };
            atomicAdd(&ctr->shadow_hist_before[bin(before)], 1ull);
            atomicAdd(&ctr->shadow_hist_after[bin(after)], 1ull);
            atomicAdd(&ctr->shadow_blocked_steps_before, (unsigned long long)before);
        }
        // the fewest steps before its blocker any blocked query of this wave took
        unsigned wmin = was_blocked ? st.win_step : 0xFFFFFFFFu;
        for (int off = 32; off > 0; off >>= 1) wmin = min(wmin, (unsigned)__shfl_xor((int)wmin, off));
        unsigned long long wm = was_blocked ? (unsigned long long)wmin : 0ull;
        unsigned long long nv = st.nodes, nt = st.tris, ns = st.steps, ne = st.entries, gw = st.gwork;
        unsigned long long bq = was_blocked ? 1ull : 0ull, bs = was_blocked ? st.steps : 0ull,
                           bt = was_blocked ? st.tris : 0ull;
        unsigned mx = st.steps, mc = st.considered, mg = st.gslot;
        for (int off = 32; off > 0; off >>= 1) {
            gw += __shfl_down(gw, off);
            mg = max(mg, (unsigned)__shfl_xor((int)mg, off));
            nv += __shfl_down(nv, off);
            nt += __shfl_down(nt, off);
            ns += __shfl_down(ns, off);
            ne += __shfl_down(ne, off);
            mc = max(mc, (unsigned)__shfl_xor((int)mc, off));
            bq += __shfl_down(bq, off);
            bs += __shfl_down(bs, off);
            bt += __shfl_down(bt, off);
            wm += __shfl_down(wm, off);
            mx = max(mx, (unsigned)__shfl_xor((int)mx, off));
        }
        __syncthreads();
        if (threadIdx.x < 16 && s_ecyc[threadIdx.x]) atomicAdd(&ctr->shadow_entry_cycles[threadIdx.x], s_ecyc[threadIdx.x]);
        if (threadIdx.x >= 16 && threadIdx.x < 18 && s_ecyc[threadIdx.x])
            atomicAdd(&ctr->shadow_group_cycles[threadIdx.x - 16], s_ecyc[threadIdx.x]);
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&ctr->shadow_group_work, gw);
            atomicAdd(&ctr->shadow_group_slots, 64ull * mg);
            atomicAdd(&ctr->shadow_node_visits, nv);
            atomicAdd(&ctr->shadow_tri_tests, nt);
            atomicAdd(&ctr->shadow_lane_slots, 64ull * mx);
            atomicAdd(&ctr->shadow_steps, ns);
            atomicAdd(&ctr->shadow_blocked, bq);
            atomicAdd(&ctr->shadow_blocked_steps, bs);
            atomicAdd(&ctr->shadow_blocked_tris, bt);
            atomicAdd(&ctr->shadow_blocked_steps_before_wavemin, wm);
            atomicAdd(&ctr->shadow_entry_visits, ne);
            atomicAdd(&ctr->shadow_entry_slots, 64ull * mc);
        }
    }
}

// Several lights: Scene::RecursiveShading's in-order sum col = ((amb + L0) + L1) + ...
__global__ void __launch_bounds__(256) k_light_sum(const SceneView sv, const ShadowPlanes shadows,
                                                   const NodePlanes nodes, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 nc = nodes.col[i];
    if (!(__float_as_int(nc.w) & 0x100)) return;
    f3 col = mk(nc.x, nc.y, nc.z);
    for (int li = 0; li < sv.num_lights; li++) {
        const float4 sc = shadows.c[(size_t)li * shadows.nn + i];
        const bool lit = sc.w != 0.0f;      // a traced query k_shadow found blocked has mode 0
        col = col + (lit ? mk(sc.x, sc.y, sc.z) : mk(0, 0, 0));
    }
    nodes.col[i] = make_float4(col.x, col.y, col.z, nc.w);
}

DEV f3 nan_check(f3 c) { return isnan3(c) ? mk(0, 0, 0) : c; }   // Scene::NanCheck Scene.cpp:221-228

// Bottom-up combination of RecursiveShading (src/Scene.cpp:148-219): the colour of one node
// from its basic shading and its children's (already resolved) colours.
// Node i of `self` (colour record nc); child_col(c) / child_pnt(c): child c's resolved colour (w: its
// kind bits) and its point.  A missed refracted child's point is (0,0,0) (src/Helper.cpp:21): the
// child's point plane is read only for hits.
template <class CC, class CP>
DEV f3 resolve_with(const SceneView& sv, float4 nc, int i, const NodePlanes& self, CC&& child_col, CP&& child_pnt) {
    const int kind = __float_as_int(nc.w) & 0xFF;
    f3 basic = mk(nc.x, nc.y, nc.z);
    if (kind == NK_FINAL) return basic;
    const int4 lk = self.link[i];
    // a mirror node needs neither its point nor F (k_shade may not have stored them)
    const float4 pf = kind == NK_MIRROR ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : self.pnt[i];
    const MaterialDev& m = sv.materials[lk.z - 1];
    f3 p = mk(pf.x, pf.y, pf.z);
    // Beer's law with zero absorption is exp(-0 * bd) = 1 for every finite distance bd, so the
    // refracted child's hit point is read only when the material absorbs or a point is far enough
    // (kNodeFar, or this node's own) for |q0 - p| to overflow
    const bool absorbs = !(m.absorption[0] == 0.0f && m.absorption[1] == 0.0f && m.absorption[2] == 0.0f);
    const bool p_far = !(fabsf(p.x) < 1e18f && fabsf(p.y) < 1e18f && fabsf(p.z) < 1e18f);
    f3 c0 = mk(0, 0, 0), c1 = mk(0, 0, 0), q0 = mk(0, 0, 0);
    if (lk.x >= 0) {
        const float4 a = child_col(lk.x);
        c0 = mk(a.x, a.y, a.z);
        const int ck = __float_as_int(a.w);
        if ((ck & kNodeHit) && (absorbs || p_far || (ck & kNodeFar))) {
            const float4 ap = child_pnt(lk.x);
            q0 = mk(ap.x, ap.y, ap.z);
        }
    }
    if (lk.y >= 0) { const float4 b = child_col(lk.y); c1 = mk(b.x, b.y, b.z); }
    const struct { float F; } nd = {pf.w};
    f3 res;
    if (kind == NK_MIRROR) {
        res = basic + cw(ld3(m.mirror), c1);
    } else if (kind == NK_CONDUCTOR) {
        f3 rc = c1 * nd.F;
        rc = cw(ld3(m.mirror), rc);
        res = basic + rc;
    } else {
        float F = nd.F;
        float bd = norm(q0 - p);                                     // beerDistance Scene.cpp:110
        f3 beer = mk(f_exp(-m.absorption[0] * bd), f_exp(-m.absorption[1] * bd), f_exp(-m.absorption[2] * bd));
        if (kind == NK_DIEL_ENTER) {
            f3 inside = c0 * (1 - F);
            inside = cw(beer, inside);
            f3 refl = c1 * F;
            res = (basic + nan_check(inside)) + nan_check(refl);
        } else if (kind == NK_DIEL_TIR) {
            res = nan_check(cw(beer, c1));
        } else {
            f3 outside = c0 * (1 - F);
            f3 refl = c1 * F;
            refl = cw(beer, refl);
            res = nan_check(outside) + nan_check(refl);
        }
    }
    return res;
}

// Node i of `self` against its children in `child`, whose colours are already resolved.
DEV f3 resolve_node(const SceneView& sv, float4 nc, int i, const NodePlanes& self, const NodePlanes& child) {
    return resolve_with(sv, nc, i, self, [&](int c) { return child.col[c]; }, [&](int c) { return child.pnt[c]; });
}
// Node i of `self` together with its children in `child` (round 5): each non-final child is resolved
// here against its own children in `grand` (already resolved), with the same arithmetic, and its
// colour is never stored -- a child is read by its one parent only (ray trees), so the bottom-up pass
// skips writing and re-reading every other level.
DEV f3 resolve_node2(const SceneView& sv, float4 nc, int i, const NodePlanes& self, const NodePlanes& child,
                     const NodePlanes& grand) {
    return resolve_with(
        sv, nc, i, self,
        [&](int c) {
            const float4 a = child.col[c];
            if ((__float_as_int(a.w) & 0xFF) == NK_FINAL) return a;
            const f3 r = resolve_node(sv, a, c, child, grand);
            return make_float4(r.x, r.y, r.z, a.w);
        },
        [&](int c) { return child.pnt[c]; });
}

// Two levels of the bottom-up pass in one launch: the nodes of `self` and, inline, their children.
__global__ void __launch_bounds__(256) k_resolve2(const SceneView sv, const NodePlanes self, const NodePlanes child,
                                                  const NodePlanes grand, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 nc = self.col[i];
    if ((__float_as_int(nc.w) & 0xFF) == NK_FINAL) return;
    const f3 res = resolve_node2(sv, nc, i, self, child, grand);
    self.col[i] = make_float4(res.x, res.y, res.z, nc.w);
}

// One level of the bottom-up pass (levels >= 1; level 0 is resolved inside k_accumulate).
// One thread per node of the level; final nodes only read their colour's kind word.
__global__ void __launch_bounds__(256) k_resolve(const SceneView sv, const NodePlanes nodes, const NodePlanes child,
                                                 int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 nc = nodes.col[i];
    if ((__float_as_int(nc.w) & 0xFF) == NK_FINAL) return;
    const f3 res = resolve_node(sv, nc, i, nodes, child);
    nodes.col[i] = make_float4(res.x, res.y, res.z, nc.w);
}

// Scene::SingleSample / MultiSample (src/Scene.cpp:365-411): color += sample_s in sample order.
// A block takes PIX pixels: their samples' colours are staged through LDS with coalesced loads
// (the slots of a pixel are adjacent; one lane per slot), CHUNK samples per pixel at a time, then one
// lane per pixel sums them in order.  mode 2: the single sample itself; 1: first chunk (start from 0);
// 0: continue the running sum in `acc`.  32 pixels x 64 samples where level 0 is resolved here (the
// Whitted passes: 25 KB of LDS instead of 50, twice the blocks per CU for the resolve's dependent
// gathers -- round 5, `profiles/r6_ab_accumulate_pix32.jsonl`: dragon 1.38 -> 1.09 ms per frame, spheres
// 1.52 -> 1.08; 16 pixels no better); 256 x 16 otherwise -- the path tracer's radiance and passes of
// few samples (`r6_ab_accumulate256.jsonl`: bunny 1 spp 0.10 -> 0.04 ms, cornell_pt 2.30 -> 2.11 ms;
// with the resolve, dragon 1.45 -> 2.0 ms: not used there).
constexpr int kAccPix = 32, kAccChunk = 64;
constexpr int kAccPixWide = 256, kAccChunkWide = 16;
// Colours are read from the level-0 NodePlanes colour plane; `resolve` (Whitted only) evaluates
// non-final level-0 nodes against level 1 first.
// DEEP (round 5): level 1 is resolved inline too (resolve_node2, against the resolved level 2).
template <bool DEEP = false, int PIX = kAccPix, int CHUNK = kAccChunk>
__global__ void __launch_bounds__(256) k_accumulate(const SceneView sv,
                                                    const NodePlanes level0, const NodePlanes level1, bool resolve,
                                                    float* __restrict__ acc, const PassDev ps, int nx, int mode,
                                                    const NodePlanes level2) {
    constexpr int kAccPix = PIX, kAccChunk = CHUNK, kAccStride = CHUNK + 1;
    __shared__ float sr[kAccPix * kAccStride], sg[kAccPix * kAccStride], sb[kAccPix * kAccStride];
    const int p0 = blockIdx.x * kAccPix;
    const int np = min(kAccPix, ps.npass - p0);
    const int t = threadIdx.x;
    f3 a = mk(0.0f, 0.0f, 0.0f);
    size_t p = 0;
    if (t < np) {
        int x, k;
        tile_pixel(ps.p0 + p0 + t, nx, ps.rows_owned, ps.tile_h, ps.tile_s, x, k);
        p = (size_t)k * nx + x;                 // acc is in natural owned-row order
        if (mode == 0) a = mk(acc[3 * p], acc[3 * p + 1], acc[3 * p + 2]);
    }
    for (int s0 = 0; s0 < ps.ns; s0 += kAccChunk) {
        const int cs = min(kAccChunk, ps.ns - s0);
        __syncthreads();
        for (int e = t; e < np * cs; e += blockDim.x) {
            const int q = idiv(e, cs), s = e - q * cs;
            const size_t slot = (size_t)(p0 + q) * ps.ns + s0 + s;
            f3 c;
            const float4 nc = level0.col[slot];
            if (resolve && (__float_as_int(nc.w) & 0xFF) != NK_FINAL)   // level 0 of the bottom-up pass
                c = DEEP ? resolve_node2(sv, nc, (int)slot, level0, level1, level2)
                         : resolve_node(sv, nc, (int)slot, level0, level1);
            else
                c = mk(nc.x, nc.y, nc.z);
            sr[q * kAccStride + s] = c.x;
            sg[q * kAccStride + s] = c.y;
            sb[q * kAccStride + s] = c.z;
        }
        __syncthreads();
        if (t < np) {
            int s = 0;
            if (mode == 2 && s0 == 0) {         // SingleSample: the colour itself
                a = mk(sr[t * kAccStride], sg[t * kAccStride], sb[t * kAccStride]);
                s = 1;
            }
            for (; s < cs; s++) a = a + mk(sr[t * kAccStride + s], sg[t * kAccStride + s], sb[t * kAccStride + s]);
        }
    }
    if (t < np) { acc[3 * p] = a.x; acc[3 * p + 1] = a.y; acc[3 * p + 2] = a.z; }
}

__global__ void __launch_bounds__(256) k_finalize(const float* __restrict__ acc, float* __restrict__ out, int nx,
                                                  int ny, int row_offset, int row_stride, int row_block, int total) {
    int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= nx * ny) return;
    int y = pix / nx, x = pix - y * nx;
    float r = 0.0f, g = 0.0f, b = 0.0f;
    const int k = shard_owned_index(y, row_offset, row_stride, row_block);
    if (k >= 0) {
        int pl = k * nx + x;
        r = acc[3 * pl]; g = acc[3 * pl + 1]; b = acc[3 * pl + 2];
        if (total > 1) { r = r / (float)total; g = g / (float)total; b = b / (float)total; }
    }
    out[3 * pix] = r; out[3 * pix + 1] = g; out[3 * pix + 2] = b;
}

// Multi-GPU gather: frame row y comes from the shard that owns it, at that shard's compact row
// index (the rows of every shard are stacked in `recv` in rank order).
__global__ void __launch_bounds__(256) k_place_rows(const float* __restrict__ recv, float* __restrict__ frame, int nx,
                                                    int ny, int nranks, int block, const ShardPrefix pre) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // one float4 of a row
    const int row4 = (3 * nx + 3) / 4;
    if (e >= (long long)row4 * ny) return;
    const int y = (int)(e / row4), c = (int)(e - (long long)y * row4) * 4;
    const int r = (y / block) % nranks;
    const int k = shard_owned_index(y, r, nranks, block);
    const float* src = recv + ((size_t)(pre.rows[r] + k) * nx) * 3;
    float* dst = frame + ((size_t)y * nx) * 3;
    for (int q = c; q < c + 4 && q < 3 * nx; q++) dst[q] = src[q];
}

__global__ void __launch_bounds__(256) k_hit_details(const SceneView sv, const RayQ rays,
                                                     const HitRec* __restrict__ hits, rtg_hit* __restrict__ out,
                                                     const int* __restrict__ orig_prim, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    f3 ro, rd;
    float rt;
    load_ray(rays, i, ro, rd, rt);
    HitRec h = hits[i];
    rtg_hit o;
    o.full = h.obj >= 0;
    o.object = h.obj;
    o.prim = -1; o.material = 0; o.t = 0.0f;
    o.point[0] = o.point[1] = o.point[2] = 0.0f;
    o.normal[0] = o.normal[1] = o.normal[2] = 0.0f;
    if (h.obj >= 0) {
        Ret ret = hit_record(sv, ro, rd, rt, h);
        o.prim = orig_prim[h.prim];
        o.material = ret.matIndex;
        o.t = h.t;
        o.point[0] = ret.point.x; o.point[1] = ret.point.y; o.point[2] = ret.point.z;
        o.normal[0] = ret.normal.x; o.normal[1] = ret.normal.y; o.normal[2] = ret.normal.z;
    }
    out[i] = o;
}

// ------------------------------------------------------------------ launchers
static inline int nblk(int n, int b) { return (n + b - 1) / b; }

void launch_trace(const SceneView& sv, const RayQ rays, HitRec* hits, int n, int exhaustive, Counters* ctr,
                  hipStream_t st, const CameraDev* gen_cam, const PassDev* gen_ps, uint64_t seed, bool compact,
                  int nq, int gbase) {
    if (n <= 0) return;
    dim3 g(nblk(n, kTraceBlock)), b(kTraceBlock);
    const CameraDev cam = gen_cam ? *gen_cam : CameraDev{};
    const PassDev ps = gen_ps ? *gen_ps : PassDev{};
    const bool tl = sv.tlas_root >= 0;
#define RTG_TRACE(EX, STA, GEN)                                                                                   \
    do {                                                                                                          \
        if (tl) hipLaunchKernelGGL((k_trace<EX, STA, GEN, true>), g, b, 0, st, sv, rays, hits, n, ctr, cam, ps, seed, compact, nq, gbase); \
        else hipLaunchKernelGGL((k_trace<EX, STA, GEN, false>), g, b, 0, st, sv, rays, hits, n, ctr, cam, ps, seed, compact, nq, gbase); \
    } while (0)
    if (gen_cam) {   // primary rays generated in the kernel (rays unused)
        if (exhaustive) hipLaunchKernelGGL((k_trace<true, false, true, false>), g, b, 0, st, sv, rays, hits, n, ctr, cam, ps, seed, compact, nq, gbase);
        else if (ctr) RTG_TRACE(false, true, true);
        else RTG_TRACE(false, false, true);
        return;
    }
    if (exhaustive) hipLaunchKernelGGL((k_trace<true, false, false, false>), g, b, 0, st, sv, rays, hits, n, ctr, cam, ps, seed, compact, nq, gbase);
    else if (ctr) RTG_TRACE(false, true, false);
    else RTG_TRACE(false, false, false);
#undef RTG_TRACE
}
__global__ void k_warm() {}
void device_warm(hipStream_t st) { hipLaunchKernelGGL(k_warm, dim3(1), dim3(64), 0, st); }

void launch_shade(const SceneView& sv, const CameraDev& cam, int level, const PassDev& ps, uint64_t seed,
                  const RayQ rays, const RayMeta* meta, const HitRec* hits, NodeRec* nodes,
                  ShadowRec* shadows, int* slist, const RayQ next_rays, RayMeta* next_meta,
                  unsigned long long* qcount, int n, hipStream_t st,
                  int gen, int nq, int gbase, const unsigned char* lv_in, unsigned char* lv_out) {
    if (n <= 0) return;
    dim3 g(nblk(n, kShadeBlock)), b(kShadeBlock);
    const NodePlanes np = node_planes(nodes, n);
    const ShadowPlanes sp = shadow_planes(shadows, n, sv.num_lights);
    const bool G = gen < 0 ? rays.a == nullptr : gen != 0;   // gen < 0: a pass's level (level 0 has no queue)
#define RTG_SHADE(F, S, B, T, gr, bl)                                                                             \
    do {                                                                                                          \
        if (G)                                                                                                    \
            hipLaunchKernelGGL((k_shade<F, S, B, T, true>), gr, bl, 0, st, sv, cam, level, ps, seed, rays, meta, hits, np, sp, \
                               slist, next_rays, next_meta, qcount, n, nq, gbase, lv_in, lv_out); \
        else                                                                                                      \
            hipLaunchKernelGGL((k_shade<F, S, B, T, false>), gr, bl, 0, st, sv, cam, level, ps, seed, rays, meta, hits, np, sp, \
                               slist, next_rays, next_meta, qcount, n, nq, gbase, lv_in, lv_out); \
    } while (0)
    // full variants: SPOT = a spot or environment light (their libm code compiled in)
    if (sv.full && sv.tex && sv.heavy) RTG_SHADE(true, true, 256, true, dim3(nblk(n, 256)), dim3(256));
    else if (sv.full && sv.tex) RTG_SHADE(true, false, 256, true, dim3(nblk(n, 256)), dim3(256));
    else if (sv.full && sv.heavy) RTG_SHADE(true, true, 256, false, dim3(nblk(n, 256)), dim3(256));
    else if (sv.full)
        RTG_SHADE(true, false, kShadeLightBlock, false, dim3(nblk(n, kShadeLightBlock)), dim3(kShadeLightBlock));
    else if (sv.spot) RTG_SHADE(false, true, kShadeBlock, false, g, b);
    else RTG_SHADE(false, false, kShadeBlock, false, g, b);
#undef RTG_SHADE
}
void launch_shadow(const SceneView& sv, ShadowRec* shadows, const int* slist, const unsigned* scount, NodeRec* nodes,
                   int n, int exhaustive, Counters* ctr, unsigned* nan_queries, hipStream_t st, bool whitted, int uni_from) {
    if (n <= 0 || sv.num_lights == 0) return;
    const long long cap = (long long)n * sv.num_lights;     // upper bound of the device-side count
    dim3 g(nblk((int)cap, kTraceBlock)), b(kTraceBlock);
    const NodePlanes np = node_planes(nodes, n);
    const ShadowPlanes sp = shadow_planes(shadows, n, sv.num_lights);
    const bool lean = whitted && sv.lean_shadow && sv.num_lights == 1;
    const bool tl = sv.tlas_root >= 0;
    const PtRad z{};
    if (exhaustive) hipLaunchKernelGGL((k_shadow<true, false>), g, b, 0, st, sv, sp, lean, slist, scount, np, nan_queries, ctr, uni_from, z);
    else if (ctr && tl) hipLaunchKernelGGL((k_shadow<false, true, true>), g, b, 0, st, sv, sp, lean, slist, scount, np, nan_queries, ctr, uni_from, z);
    else if (ctr) hipLaunchKernelGGL((k_shadow<false, true>), g, b, 0, st, sv, sp, lean, slist, scount, np, nan_queries, ctr, uni_from, z);
    else if (tl) hipLaunchKernelGGL((k_shadow<false, false, true>), g, b, 0, st, sv, sp, lean, slist, scount, np, nan_queries, ctr, uni_from, z);
    else hipLaunchKernelGGL((k_shadow<false, false>), g, b, 0, st, sv, sp, lean, slist, scount, np, nan_queries, ctr, uni_from, z);
    if (sv.num_lights > 1 && whitted)
        hipLaunchKernelGGL(k_light_sum, dim3(nblk(n, 256)), dim3(256), 0, st, sv, sp, np, n);
}
void launch_pt_shadow(const SceneView& sv, ShadowRec* shadows, const int* slist, NodeRec* nodes, int n, int exhaustive,
                      Counters* ctr, unsigned* nan_queries, hipStream_t st, int uni_from, const PtRad& pr) {
    if (n <= 0 || sv.num_lights == 0) return;
    dim3 g(nblk(n, kTraceBlock)), b(kTraceBlock);           // a light's list holds at most n queries
    const NodePlanes np = node_planes(nodes, n);
    const ShadowPlanes sp = shadow_planes(shadows, n, sv.num_lights);
    const bool tl = sv.tlas_root >= 0;
    for (int li = 0; li < sv.num_lights; li++) {
        const int* sl = slist + (size_t)li * n;
        const unsigned* sc = pr.lcnt + li;
        PtRad prl = pr;
        prl.light = li;
        if (exhaustive) hipLaunchKernelGGL((k_shadow<true, false, false, true>), g, b, 0, st, sv, sp, false, sl, sc, np, nan_queries, ctr, uni_from, prl);
        else if (ctr && tl) hipLaunchKernelGGL((k_shadow<false, true, true, true>), g, b, 0, st, sv, sp, false, sl, sc, np, nan_queries, ctr, uni_from, prl);
        else if (ctr) hipLaunchKernelGGL((k_shadow<false, true, false, true>), g, b, 0, st, sv, sp, false, sl, sc, np, nan_queries, ctr, uni_from, prl);
        else if (tl) hipLaunchKernelGGL((k_shadow<false, false, true, true>), g, b, 0, st, sv, sp, false, sl, sc, np, nan_queries, ctr, uni_from, prl);
        else hipLaunchKernelGGL((k_shadow<false, false, false, true>), g, b, 0, st, sv, sp, false, sl, sc, np, nan_queries, ctr, uni_from, prl);
    }
}
void launch_pt_shade(const SceneView& sv, const CameraDev& cam, int level, const PassDev& ps, uint64_t seed,
                     const RayQ rays, const RayMeta* meta, const HitRec* hits, PathRec* paths, NodeRec* nodes,
                     ShadowRec* shadows, int* slist, const RayQ next_rays, RayMeta* next_meta, PathRec* next_paths,
                     unsigned long long* qcount, int n, hipStream_t st, bool gen, int nq, int gbase,
                     const unsigned char* lv_in, unsigned char* lv_out, const PtRad& pr, Counters* ctr) {
    if (n <= 0) return;
    dim3 g(nblk(n, kPtBlock)), b(kPtBlock);
#define RTG_PT_LAUNCH1(F, S, B, G)                                                                                \
    hipLaunchKernelGGL((k_pt_shade<F, S, B, G>), g, b, 0, st, sv, cam, level, ps, seed, rays, meta, hits, paths, \
                       node_planes(nodes, n), \
                       shadow_planes(shadows, n, sv.num_lights), slist, next_rays, next_meta, next_paths, qcount, n, \
                       nq, gbase, lv_in, lv_out, pr, ctr)
#define RTG_PT_LAUNCH(F, S, B)                                                                                    \
    do {                                                                                                          \
        if (gen) RTG_PT_LAUNCH1(F, S, B, true);                                                                   \
        else RTG_PT_LAUNCH1(F, S, B, false);                                                                      \
    } while (0)
    // textures / area / environment lights need the full variant; BRDFs alone do not
    if (sv.full && !sv.brdf_only) {
        if (sv.heavy) RTG_PT_LAUNCH(true, true, 2); else RTG_PT_LAUNCH(true, false, 2);
    }
    else if (sv.full) {    // BRDFs only: with / without the Torrance-Sparrow models
        if (sv.spot) { if (sv.brdf_ts) RTG_PT_LAUNCH(false, true, 2); else RTG_PT_LAUNCH(false, true, 1); }
        else { if (sv.brdf_ts) RTG_PT_LAUNCH(false, false, 2); else RTG_PT_LAUNCH(false, false, 1); }
    }
    else if (sv.spot) RTG_PT_LAUNCH(false, true, 0);
    else RTG_PT_LAUNCH(false, false, 0);
#undef RTG_PT_LAUNCH
#undef RTG_PT_LAUNCH1
}
void launch_resolve2(const SceneView& sv, NodeRec* nodes, const NodeRec* child_nodes, const NodeRec* grand_nodes, int n,
                     int n_child, int n_grand, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_resolve2, dim3(nblk(n, 256)), dim3(256), 0, st, sv, node_planes(nodes, n),
                       node_planes(const_cast<NodeRec*>(child_nodes), n_child),
                       node_planes(const_cast<NodeRec*>(grand_nodes), n_grand), n);
}
void launch_resolve(const SceneView& sv, NodeRec* nodes, const NodeRec* child_nodes, int n, int n_child,
                    hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_resolve, dim3(nblk(n, 256)), dim3(256), 0, st, sv, node_planes(nodes, n),
                       node_planes(const_cast<NodeRec*>(child_nodes), n_child), n);
}
void launch_resolve_planes(const SceneView& sv, const NodePlanes& self, const NodePlanes& child, int count,
                           hipStream_t st) {
    if (count <= 0) return;
    hipLaunchKernelGGL(k_resolve, dim3(nblk(count, 256)), dim3(256), 0, st, sv, self, child, count);
}
void launch_accumulate_planes(const SceneView& sv, const NodePlanes& level0, const NodePlanes& level1, bool resolve,
                              float* acc, const PassDev& ps, int nx, int mode, hipStream_t st) {
    if (ps.npass <= 0) return;
    if (!resolve || ps.ns <= kAccChunkWide)
        hipLaunchKernelGGL((k_accumulate<false, kAccPixWide, kAccChunkWide>), dim3(nblk(ps.npass, kAccPixWide)), dim3(256),
                           0, st, sv, level0, level1, resolve, acc, ps, nx, mode, NodePlanes{});
    else
        hipLaunchKernelGGL(k_accumulate<false>, dim3(nblk(ps.npass, kAccPix)), dim3(256), 0, st, sv, level0, level1,
                           resolve, acc, ps, nx, mode, NodePlanes{});
}
void launch_accumulate(const SceneView& sv, const NodeRec* level0, const NodeRec* level1, bool resolve, float* acc,
                       const PassDev& ps, int nx, int mode, hipStream_t st, bool whitted, int n0, int n1,
                       const NodeRec* level2, int n2) {
    if (ps.npass <= 0) return;
    NodeRec* l0 = const_cast<NodeRec*>(level0);
    const NodePlanes p0 = node_planes(l0, n0);
    const NodePlanes p1 = (whitted && level1) ? node_planes(const_cast<NodeRec*>(level1), n1) : NodePlanes{};
    if (whitted && resolve && level1 && level2) {
        const NodePlanes p2 = node_planes(const_cast<NodeRec*>(level2), n2);
        if (ps.ns <= kAccChunkWide)
            hipLaunchKernelGGL((k_accumulate<true, kAccPixWide, kAccChunkWide>), dim3(nblk(ps.npass, kAccPixWide)), dim3(256),
                               0, st, sv, p0, p1, true, acc, ps, nx, mode, p2);
        else
            hipLaunchKernelGGL(k_accumulate<true>, dim3(nblk(ps.npass, kAccPix)), dim3(256), 0, st, sv, p0, p1, true, acc,
                               ps, nx, mode, p2);
    } else if (!(resolve && whitted) || ps.ns <= kAccChunkWide) {
        hipLaunchKernelGGL((k_accumulate<false, kAccPixWide, kAccChunkWide>), dim3(nblk(ps.npass, kAccPixWide)), dim3(256),
                           0, st, sv, p0, p1, resolve && whitted, acc, ps, nx, mode, NodePlanes{});
    } else {
        hipLaunchKernelGGL(k_accumulate<false>, dim3(nblk(ps.npass, kAccPix)), dim3(256), 0, st, sv, p0, p1,
                           resolve && whitted, acc, ps, nx, mode, NodePlanes{});
    }
}
void launch_finalize(const float* acc, float* out, int nx, int ny, int row_offset, int row_stride, int row_block,
                     int total, hipStream_t st) {
    int n = nx * ny;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_finalize, dim3(nblk(n, 256)), dim3(256), 0, st, acc, out, nx, ny, row_offset, row_stride,
                       row_block, total);
}
void launch_place_rows(const float* recv, float* frame, int nx, int ny, int nranks, int block, const ShardPrefix& pre,
                       hipStream_t st) {
    const long long n = (long long)((3 * nx + 3) / 4) * ny;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_place_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, recv, frame, nx, ny, nranks,
                       block, pre);
}
void launch_hit_details(const SceneView& sv, const RayQ rays, const HitRec* hits, rtg_hit* out,
                        const int* orig_prim, int n, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_hit_details, dim3(nblk(n, 256)), dim3(256), 0, st, sv, rays, hits, out, orig_prim, n);
}

}  // namespace rtg
