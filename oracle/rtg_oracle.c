/*
 * rtg_oracle.c — plain-C restatement of the badiba/raytracer-795 per-pixel render loop.
 *
 * TEST INFRASTRUCTURE ONLY (see rtg_oracle.h): the checker for librtg.so and the CPU
 * baseline of bench.py.  It restates the reference algorithm function by function,
 * literally (recursive visit-both-children BVH, linear object loop, recursive shading),
 * so it is deliberately slow.  Every function cites the reference file:line it follows
 * (paths relative to the reference's repository root).
 *
 * PARITY UNPINNED — the reference has no tests/fixtures and is not buildable here.
 *
 * Arithmetic conventions:
 *  - float ops in the reference's evaluation order; compile with -ffp-contract=off.
 *  - Eigen 3-vector reductions (dot, squaredNorm) sum as x0 + (x1 + x2); normalized()
 *    returns the input unchanged when the squared norm is not > 0 (Eigen >= 3.3).
 *  - glm mat4*vec4 is (c0*x + c1*y) + (c2*z + c3*w); mat4*mat4 columns sum left to right;
 *    glm dot(vec3) is (x + y) + z.
 *  - Every transcendental the reference evaluates (float or double libm) is evaluated as
 *    (float)f64(x) — the correctly rounded value; the reference's glibc float functions
 *    agree with it to <= 1 ulp.  pow(float,int) is a double pow, as in the reference.
 *  - Undefined behaviour is given a fixed meaning: a miss's hit point is (0,0,0)
 *    (src/Helper.cpp:21 `ReturnVal nearestRet = {}` leaves Eigen storage uninitialised);
 *    Ray::gett falling off its end returns NaN (src/Ray.cpp:21-36); stand-alone
 *    triangles/spheres have textureOffset 0; out-of-range texcoords read (0,0).
 *  - RNG: the reference draws from std::mt19937 seeded by std::random_device (racing
 *    threads, src/Scene.cpp:502-503, Camera.cpp:59-60, Light.cpp:523-528, 555-556).  This restatement
 *    replaces every draw by a counter-based Philox4x32-10 value keyed by
 *    (seed, pixel, sample, ray-tree node, purpose, light, iteration), mapped to float the
 *    way libstdc++'s generate_canonical<float,24> maps one 32-bit draw.
 */
#include "rtg_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI_D 3.14159265358979323846

/* ------------------------------------------------------------------ vectors */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } v2;
typedef struct { float c[4][4]; } mat4;   /* glm column-major: c[col][row] */

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline v3 vmul(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 vcw(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
/* Eigen redux order x0 + (x1 + x2) */
static inline float vdot(v3 a, v3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
static inline float vsqn(v3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
static inline float vnorm(v3 a) { return sqrtf(vsqn(a)); }
static inline v3 vnormalized(v3 a) {
    float z = vsqn(a);
    if (z > 0.0f) return vdivs(a, sqrtf(z));
    return a;
}
static inline v3 vcross(v3 a, v3 b) {
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline int visnan(v3 a) { return a.x != a.x || a.y != a.y || a.z != a.z; }
static inline float vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void setc(v3* a, int i, float v) { if (i == 0) a->x = v; else if (i == 1) a->y = v; else a->z = v; }
/* std::max(0.0f, x) = (0 < x) ? x : 0 ; std::min(a,b) = (b < a) ? b : a */
static inline float fmax0(float x) { return (0.0f < x) ? x : 0.0f; }
static inline float stdmin(float a, float b) { return (b < a) ? b : a; }

/* transcendental convention: correctly rounded float of the double function */
static inline float f_acos(float x) { return (float)acos((double)x); }
static inline float f_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
static inline float f_cos(float x) { return (float)cos((double)x); }
static inline float f_sin(float x) { return (float)sin((double)x); }
static inline float f_tan(float x) { return (float)tan((double)x); }
static inline float f_exp(float x) { return (float)exp((double)x); }

/* ------------------------------------------------------------------ glm mat4 */
static mat4 m_identity(void) {
    mat4 m; memset(&m, 0, sizeof m);
    m.c[0][0] = m.c[1][1] = m.c[2][2] = m.c[3][3] = 1.0f;
    return m;
}
/* glm operator*(mat4, vec4): (c0*x + c1*y) + (c2*z + c3*w) */
static void m_mulv(const mat4* m, const float v[4], float out[4]) {
    for (int r = 0; r < 4; r++) {
        float a0 = m->c[0][r] * v[0];
        float a1 = m->c[1][r] * v[1];
        float add0 = a0 + a1;
        float a2 = m->c[2][r] * v[2];
        float a3 = m->c[3][r] * v[3];
        float add1 = a2 + a3;
        out[r] = add0 + add1;
    }
}
/* glm operator*(mat4, mat4): Result[i] = A0*B[i][0] + A1*B[i][1] + A2*B[i][2] + A3*B[i][3] */
static mat4 m_mul(const mat4* A, const mat4* B) {
    mat4 R;
    for (int i = 0; i < 4; i++)
        for (int r = 0; r < 4; r++)
            R.c[i][r] = ((A->c[0][r] * B->c[i][0] + A->c[1][r] * B->c[i][1]) + A->c[2][r] * B->c[i][2]) +
                        A->c[3][r] * B->c[i][3];
    return R;
}
/* glm::translate (matrix_transform.inl): Result[3] = m0*v0 + m1*v1 + m2*v2 + m3 */
static mat4 m_translate(const mat4* m, v3 v) {
    mat4 R = *m;
    for (int r = 0; r < 4; r++)
        R.c[3][r] = ((m->c[0][r] * v.x + m->c[1][r] * v.y) + m->c[2][r] * v.z) + m->c[3][r];
    return R;
}
static mat4 m_scale(const mat4* m, v3 v) {
    mat4 R = *m;
    for (int r = 0; r < 4; r++) {
        R.c[0][r] = m->c[0][r] * v.x;
        R.c[1][r] = m->c[1][r] * v.y;
        R.c[2][r] = m->c[2][r] * v.z;
    }
    return R;
}
/* glm::rotate(m, angle, axis) (matrix_transform.inl) */
static mat4 m_rotate(const mat4* m, float angle, v3 v) {
    float c = f_cos(angle), s = f_sin(angle);
    float d = (v.x * v.x + v.y * v.y) + v.z * v.z;          /* glm dot */
    float inv = 1.0f / sqrtf(d);                              /* inversesqrt */
    v3 axis = V(v.x * inv, v.y * inv, v.z * inv);
    float omc = 1.0f - c;
    v3 temp = V(omc * axis.x, omc * axis.y, omc * axis.z);
    float R00 = c + temp.x * axis.x, R01 = temp.x * axis.y + s * axis.z, R02 = temp.x * axis.z - s * axis.y;
    float R10 = temp.y * axis.x - s * axis.z, R11 = c + temp.y * axis.y, R12 = temp.y * axis.z + s * axis.x;
    float R20 = temp.z * axis.x + s * axis.y, R21 = temp.z * axis.y - s * axis.x, R22 = c + temp.z * axis.z;
    mat4 R;
    for (int r = 0; r < 4; r++) {
        R.c[0][r] = (m->c[0][r] * R00 + m->c[1][r] * R01) + m->c[2][r] * R02;
        R.c[1][r] = (m->c[0][r] * R10 + m->c[1][r] * R11) + m->c[2][r] * R12;
        R.c[2][r] = (m->c[0][r] * R20 + m->c[1][r] * R21) + m->c[2][r] * R22;
        R.c[3][r] = m->c[3][r];
    }
    return R;
}
/* glm::inverse (func_matrix.inl compute_inverse<4,4>) */
static mat4 m_inverse(const mat4* M) {
    const float (*m)[4] = M->c;
    float Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float Fac0[4] = {Coef00, Coef00, Coef02, Coef03};
    float Fac1[4] = {Coef04, Coef04, Coef06, Coef07};
    float Fac2[4] = {Coef08, Coef08, Coef10, Coef11};
    float Fac3[4] = {Coef12, Coef12, Coef14, Coef15};
    float Fac4[4] = {Coef16, Coef16, Coef18, Coef19};
    float Fac5[4] = {Coef20, Coef20, Coef22, Coef23};
    float Vec0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]};
    float Vec1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    float Vec2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]};
    float Vec3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    float Inv0[4], Inv1[4], Inv2[4], Inv3[4];
    for (int i = 0; i < 4; i++) {
        Inv0[i] = (Vec1[i] * Fac0[i] - Vec2[i] * Fac1[i]) + Vec3[i] * Fac2[i];
        Inv1[i] = (Vec0[i] * Fac0[i] - Vec2[i] * Fac3[i]) + Vec3[i] * Fac4[i];
        Inv2[i] = (Vec0[i] * Fac1[i] - Vec1[i] * Fac3[i]) + Vec3[i] * Fac5[i];
        Inv3[i] = (Vec0[i] * Fac2[i] - Vec1[i] * Fac4[i]) + Vec2[i] * Fac5[i];
    }
    const float SignA[4] = {+1, -1, +1, -1}, SignB[4] = {-1, +1, -1, +1};
    mat4 Inverse;
    for (int i = 0; i < 4; i++) {
        Inverse.c[0][i] = Inv0[i] * SignA[i];
        Inverse.c[1][i] = Inv1[i] * SignB[i];
        Inverse.c[2][i] = Inv2[i] * SignA[i];
        Inverse.c[3][i] = Inv3[i] * SignB[i];
    }
    float Row0[4] = {Inverse.c[0][0], Inverse.c[1][0], Inverse.c[2][0], Inverse.c[3][0]};
    float Dot0[4];
    for (int i = 0; i < 4; i++) Dot0[i] = m[0][i] * Row0[i];
    float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
    float OneOverDeterminant = 1.0f / Dot1;
    mat4 R;
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) R.c[c][r] = Inverse.c[c][r] * OneOverDeterminant;
    return R;
}
/* glm::inverseTranspose (gtc/matrix_inverse.inl, mat4 case) */
static mat4 m_inverse_transpose(const mat4* M) {
    const float (*m)[4] = M->c;
    float S00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float S01 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float S02 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float S03 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float S04 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float S05 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float S06 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float S07 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S08 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float S09 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float S10 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float S11 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S12 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float S13 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float S14 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float S15 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float S16 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float S17 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float S18 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    mat4 I;
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
    float Det = ((m[0][0] * I.c[0][0] + m[0][1] * I.c[0][1]) + m[0][2] * I.c[0][2]) + m[0][3] * I.c[0][3];
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) I.c[c][r] = I.c[c][r] / Det;
    return I;
}

/* ------------------------------------------------------------------ Philox RNG */
enum { RNG_CAMERA = 1, RNG_ROUGH = 2, RNG_AREA = 3, RNG_ENV = 4, RNG_PT_BOUNCE = 5, RNG_PT_EMIT = 6 };

static inline void philox_round(uint32_t c[4], const uint32_t k[2]) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k[0], n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}
/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox4x32_R(10)) */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    uint32_t k[2] = {key[0], key[1]};
    for (int r = 0; r < 10; r++) {
        philox_round(c, k);
        k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u;
    }
    memcpy(out, c, sizeof c);
}
static void rng4(uint64_t seed, uint32_t pixel, uint32_t sample, uint64_t path, uint32_t purpose,
                 uint32_t light, uint32_t iter, float out[4]) {
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(path >> 32)};
    uint32_t c[4] = {pixel, sample, (uint32_t)path, (purpose << 28) | ((light & 0xFFFu) << 16) | (iter & 0xFFFFu)};
    orc_philox4x32_10(c, k, c);
    for (int i = 0; i < 4; i++) {
        /* libstdc++ generate_canonical<float,24>: (float)u / 2^32, clamped below 1 */
        float f = (float)c[i] / 4294967296.0f;
        out[i] = (f >= 1.0f) ? 0x1.fffffep-1f : f;
    }
}
float orc_rng_uniform(uint64_t seed, uint32_t pixel, uint32_t sample, uint64_t path,
                      uint32_t purpose, uint32_t light, uint32_t iter, int lane) {
    float o[4];
    rng4(seed, pixel, sample, path, purpose, light, iter, o);
    return o[lane & 3];
}

typedef struct { uint64_t seed; uint32_t pixel, sample; } RngCtx;

/* ------------------------------------------------------------------ scene records */
typedef struct { v3 origin, direction; float time; } Ray;   /* src/Ray.h:10-12 */
static inline Ray R(v3 o, v3 d, float t) { Ray r = {o, d, t}; return r; }
static inline v3 ray_point(const Ray* r, float t) { return vadd(r->origin, vmul(r->direction, t)); } /* Ray.cpp:15-19 */
/* Ray::gett (src/Ray.cpp:21-36); falling off the end -> NaN */
static inline float ray_gett(const Ray* r, v3 p) {
    float t = (p.x - r->origin.x) / r->direction.x;
    if (t == t) return t;
    t = (p.y - r->origin.y) / r->direction.y;
    if (t == t) return t;
    t = (p.z - r->origin.z) / r->direction.z;
    return t;
}

typedef struct {              /* ReturnVal, src/defs.h:13-22 (+ debug ids) */
    v3 point, normal;
    int full;
    int matIndex;
    int dm;
    v3 textureColor;
    float textureNormalizer;
    int obj, prim;
    float t;
} RetVal;
static RetVal ret_empty(void) { RetVal r; memset(&r, 0, sizeof r); r.obj = -1; r.prim = -1; return r; }

typedef struct { v3 mn, mx; int start, end; int left, right; } BNode;

typedef struct {
    int type;                 /* rtg_object_type */
    int id, matIndex, ntex, tex[2], texOffset, smooth;
    v3 blur;
    mat4 model, inv, invT;
    /* primitives in BVH order */
    int nprims;
    int* pface;               /* original primitive index at BVH position */
    int* pv;                  /* 3 per prim: 1-based vertex indices (sphere: center) */
    int* psmooth;             /* Triangle::isSmooth per prim */
    float R;                  /* sphere radius */
    BNode* nodes; int nnodes; int root;
} Obj;

typedef struct { int base; int matIndex; int reset; v3 blur; mat4 model, inv, invT; } Inst;

typedef struct {
    int kind, decal, interp, nc, normalizer;
    float noise_scale, bump;
    int w, h;
    float* texels;
} Tex;

typedef struct {
    int type;
    v3 pos, dir, inten;
    float coverage, fall, size;
    v3 normal, u, v;
    int tex;
} Lgt;

struct orc_scene {
    int maxDepth;
    float shadowEps, intEps;
    v3 background, ambientLight;
    int bgTexture, envLight;
    int nv; v3* vertices; v3* vnormals;
    int ntc; v2* texcoords;
    int nobj; Obj* objs;
    int ninst; Inst* insts;
    int nmat; rtg_material_desc* mats;
    int ntex; Tex* texs;
    int nlight; Lgt* lights;
    /* hw7 object lights (path tracer only): emitters in object order */
    int nemit; struct Emit* emits;
    v3* etris;                /* world-space triangles of mesh emitters, 3 vertices each */
    float* ecdf;              /* running float sum of their areas, per emitter range */
    uint64_t counts[3];
    int canon_on;             /* orc_canonical_counts enabled */
    uint64_t canon[8];
};
typedef struct Emit {
    int obj;                  /* object index */
    int sphere;
    v3 Le;
    float area;               /* mesh: total world area (last cdf entry) */
    int tri_first, tri_count;
    v3 center; float radius;  /* sphere: world centre, radius * |model column 0| */
} Emit;

/* per-thread render context */
typedef struct {
    struct orc_scene* s;
    RngCtx rng;
    uint64_t n_primary, n_secondary, n_shadow;
    uint64_t canon[8];        /* orc_canonical_counts: see canon_count() */
} Ctx;

/* ------------------------------------------------------------------ textures (src/Texture.cpp) */
/* Texture::GetColorAtPixel, src/Texture.cpp:41-74 */
static v3 tex_pixel(const Tex* t, int i, int j) {
    if (i < 0) i = 0; else if (i >= t->w) i = t->w - 1;
    if (j < 0) j = 0; else if (j >= t->h) j = t->h - 1;
    const float* p = t->texels + ((size_t)j * t->w + i) * 3;
    return V(p[0], p[1], p[2]);
}
/* Texture::GetColorAtCoordinates, src/Texture.cpp:111-131 */
static v3 tex_color(const Tex* t, float u, float v) {
    u = u - floorf(u);
    v = v - floorf(v);
    float i = u * (float)t->w;
    float j = v * (float)t->h;
    if (t->interp == RTG_INTERP_NN) return tex_pixel(t, (int)i, (int)j);
    int li = (int)floorf(i), lj = (int)floorf(j);
    float a = i - (float)li, b = j - (float)lj;
    v3 c00 = tex_pixel(t, li, lj), c01 = tex_pixel(t, li, lj + 1);
    v3 c10 = tex_pixel(t, li + 1, lj), c11 = tex_pixel(t, li + 1, lj + 1);
    float w00 = (1 - a) * (1 - b), w01 = (1 - a) * b, w10 = a * (1 - b), w11 = a * b;
    return vadd(vadd(vadd(vmul(c00, w00), vmul(c01, w01)), vmul(c10, w10)), vmul(c11, w11));
}
/* Texture::GetChangeAtCoordinates, src/Texture.cpp:76-109 */
static v2 tex_change(const Tex* t, float u, float v) {
    u = u - floorf(u);
    v = v - floorf(v);
    int i = (int)(u * (float)t->w);
    int j = (int)(v * (float)t->h);
    if (i < 0) i = 0; else if (i >= t->w - 1) i = t->w - 2;
    if (j < 0) j = 0; else if (j >= t->h - 1) j = t->h - 2;
    v3 a = tex_pixel(t, i + 1, j), b = tex_pixel(t, i, j), c = tex_pixel(t, i, j + 1);
    float dede = ((a.x + a.y) + a.z) / 3.0f;
    float nene = ((b.x + b.y) + b.z) / 3.0f;
    v3 dv = vsub(c, b);
    v2 r = {dede - nene, ((dv.x + dv.y) + dv.z) / 3.0f};
    return r;
}

/* ------------------------------------------------------------------ Perlin (src/Perlin.cpp) */
static const float PERLIN_TABLE[16][3] = {
    {1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1}, {1, 0, -1}, {-1, 0, -1},
    {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1}, {1, 1, 0}, {-1, 1, 0}, {0, -1, 1}, {0, -1, -1}};
static const int PERLIN_SHUFFLED[16] = {12, 7, 15, 6, 11, 0, 4, 9, 13, 3, 14, 8, 2, 5, 1, 10};
static int perlin_P(int i) { int idx = i % 16; if (idx < 0) idx += 16; return PERLIN_SHUFFLED[idx]; } /* Perlin.cpp:86-97 */
static float perlin_weight(float x) {                                   /* Perlin.cpp:27-30 */
    double xd = (double)fabsf(x);
    return (float)((((-6) * pow(xd, 5)) + (15 * pow(xd, 4))) - (10 * pow(xd, 3)) + 1);
}
static float perlin_compute(v3 p, float scale, int nc) {                /* Perlin.cpp:52-84 */
    v3 pt = vmul(p, scale);
    int ii = (int)floorf(pt.x), jj = (int)floorf(pt.y), kk = (int)floorf(pt.z);
    float value = 0;
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                int lx = ii + i, ly = jj + j, lz = kk + k;
                int idx = perlin_P(lx + perlin_P(ly + perlin_P(lz)));
                v3 g = V(PERLIN_TABLE[idx][0], PERLIN_TABLE[idx][1], PERLIN_TABLE[idx][2]);
                v3 l = vsub(pt, V((float)lx, (float)ly, (float)lz));
                float w = (perlin_weight(l.x) * perlin_weight(l.y)) * perlin_weight(l.z);
                value += vdot(g, l) * w;
            }
    if (nc == RTG_NC_LINEAR) value = (value + 1) * 0.5f;
    else if (nc == RTG_NC_ABSVAL) value = fabsf(value);
    return value;
}
static v3 perlin_gradient(v3 p, float scale, int nc) {                  /* Perlin.cpp:36-50 */
    const float eps = 0.001f;
    v3 xe = p, ye = p, ze = p;
    xe.x += eps; ye.y += eps; ze.z += eps;
    float o = perlin_compute(p, scale, nc);
    float x = (perlin_compute(xe, scale, nc) - o) / eps;
    float y = (perlin_compute(ye, scale, nc) - o) / eps;
    float z = (perlin_compute(ze, scale, nc) - o) / eps;
    return V(x, y, z);
}

/* ------------------------------------------------------------------ geometry helpers */
/* GeometryHelpers::GetAbsSmallestIndex / GetOrthonormalUVector, src/Helper.cpp:322-342 */
static v3 ortho_u(v3 v) {
    float a0 = fabsf(v.x), a1 = fabsf(v.y), a2 = fabsf(v.z);
    int idx = 2;
    if (a0 <= a1 && a0 <= a2) idx = 0;
    else if (a1 <= a0 && a1 <= a2) idx = 1;
    v3 nl = v;
    setc(&nl, idx, 1.0f);
    return vnormalized(vcross(v, nl));
}
/* glm mat4 * (v, w) -> vec3 */
static v3 m_xform(const mat4* m, v3 v, float w) {
    float in[4] = {v.x, v.y, v.z, w}, out[4];
    m_mulv(m, in, out);
    return V(out[0], out[1], out[2]);
}
/* Transforming::TransformRay, src/Helper.cpp:110-133 */
static Ray transform_ray(const Ray* ray, const mat4* M, v3 blur) {
    v3 b = V(blur.x * ray->time, blur.y * ray->time, blur.z * ray->time);
    v3 o = ray->origin;
    o.x -= b.x; o.y -= b.y; o.z -= b.z;
    Ray r;
    r.time = ray->time;
    r.origin = m_xform(M, o, 1.0f);
    r.direction = m_xform(M, ray->direction, 0.0f);
    return r;
}
/* Transforming::TransformNormal, src/Helper.cpp:100-108 (w = 1) */
static v3 transform_normal(v3 n, const mat4* IT) { return vnormalized(m_xform(IT, n, 1.0f)); }

/* ------------------------------------------------------------------ primitive intersection */
/* Eigen 3x3 determinant (Determinant.h bruteforce_det3_helper, row-0 expansion) of the
   matrix with columns c0, c1, c2. */
static inline float det3(v3 c0, v3 c1, v3 c2) {
    float h0 = c0.x * (c1.y * c2.z - c1.z * c2.y);
    float h1 = c1.x * (c0.y * c2.z - c0.z * c2.y);
    float h2 = c2.x * (c0.y * c1.z - c0.z * c1.y);
    return (h0 - h1) + h2;
}

static v2 texcoord(const struct orc_scene* s, int idx) {
    if (idx < 0 || idx >= s->ntc) { v2 z = {0, 0}; return z; }
    return s->texcoords[idx];
}

/* Sphere::TextureComputation, src/Shape.cpp:400-503 (object-space point/normal) */
static void sphere_texture(const struct orc_scene* s, const Obj* o, v3 c, float Rr, RetVal* ret) {
    ret->dm = RTG_DECAL_NONE;
    for (int i = 0; i < o->ntex; i++) {
        const Tex* t = &s->texs[o->tex[i] - 1];
        if (t->kind == RTG_TEX_IMAGE) {
            v3 lc = vsub(ret->point, c);
            float theta = f_acos(lc.y / Rr);
            float phi = f_atan2(lc.z, lc.x);
            float tu = (float)((-(double)phi + PI_D) / (2 * PI_D));
            float tv = (float)((double)theta / PI_D);
            if (t->decal == RTG_DECAL_REPLACE_KD || t->decal == RTG_DECAL_BLEND_KD || t->decal == RTG_DECAL_REPLACE_ALL) {
                ret->dm = t->decal;
                ret->textureColor = tex_color(t, tu, tv);
                ret->textureNormalizer = (float)t->normalizer;
            } else if (t->decal == RTG_DECAL_REPLACE_NORMAL || t->decal == RTG_DECAL_BUMP_NORMAL) {
                float pi = (float)PI_D;
                v3 dpdu = V((lc.z * 2) * pi, 0, (lc.x * (-2)) * pi);
                v3 dpdv = V((lc.y * f_cos(phi)) * pi, (((-1) * Rr) * f_sin(theta)) * pi, (lc.y * f_sin(phi)) * pi);
                if (t->decal == RTG_DECAL_REPLACE_NORMAL) {
                    v3 rn = vdivs(tex_color(t, tu, tv), 255.0f);
                    rn = vnormalized(vsub(rn, V(0.5f, 0.5f, 0.5f)));
                    v3 T = vnormalized(dpdu), B = vnormalized(dpdv), N = ret->normal;
                    /* TBN * rn : row i = T_i*r0 + (B_i*r1 + N_i*r2) */
                    ret->normal = V(T.x * rn.x + (B.x * rn.y + N.x * rn.z), T.y * rn.x + (B.y * rn.y + N.y * rn.z),
                                    T.z * rn.x + (B.z * rn.y + N.z * rn.z));
                } else {
                    v2 dd = tex_change(t, tu, tv);
                    dd.x = dd.x * t->bump; dd.y = dd.y * t->bump;
                    v3 dpu = vadd(dpdu, vmul(ret->normal, dd.x));
                    v3 dpv = vadd(dpdv, vmul(ret->normal, dd.y));
                    v3 nn = vnormalized(vcross(dpv, dpu));
                    ret->normal = (vdot(ret->normal, nn) > 0) ? nn : vneg(nn);
                }
            }
        } else {
            if (t->decal == RTG_DECAL_REPLACE_KD) {
                ret->dm = t->decal;
                float p = perlin_compute(ret->point, t->noise_scale, t->nc);
                ret->textureColor = V(p, p, p);
                ret->textureNormalizer = 1;
            } else if (t->decal == RTG_DECAL_BUMP_NORMAL) {
                v3 g = perlin_gradient(ret->point, t->noise_scale, t->nc);
                v3 gpar = vmul(ret->normal, vdot(g, ret->normal));
                v3 nn = vsub(ret->normal, vmul(vsub(g, gpar), t->bump));
                ret->normal = (vdot(ret->normal, nn) > 0) ? nn : vneg(nn);
                ret->normal = vnormalized(ret->normal);
            }
        }
    }
}

/* Triangle::TextureComputation, src/Shape.cpp:505-616 */
static void triangle_texture(const struct orc_scene* s, const Obj* o, const int* vi, v3 e1, v3 e2,
                             float beta, float gamma, RetVal* ret) {
    ret->dm = RTG_DECAL_NONE;
    if (o->ntex == 0) return;
    float alpha = (1 - beta) - gamma;
    v2 uv0 = texcoord(s, vi[0] - 1 + o->texOffset);
    v2 uv1 = texcoord(s, vi[1] - 1 + o->texOffset);
    v2 uv2 = texcoord(s, vi[2] - 1 + o->texOffset);
    v2 uv = {(uv0.x * alpha + uv1.x * beta) + uv2.x * gamma, (uv0.y * alpha + uv1.y * beta) + uv2.y * gamma};
    for (int i = 0; i < o->ntex; i++) {
        const Tex* t = &s->texs[o->tex[i] - 1];
        if (t->kind == RTG_TEX_IMAGE) {
            if (t->decal == RTG_DECAL_REPLACE_KD || t->decal == RTG_DECAL_BLEND_KD || t->decal == RTG_DECAL_REPLACE_ALL) {
                ret->dm = t->decal;
                ret->textureColor = tex_color(t, uv.x, uv.y);
                ret->textureNormalizer = (float)t->normalizer;
            } else if (t->decal == RTG_DECAL_REPLACE_NORMAL || t->decal == RTG_DECAL_BUMP_NORMAL) {
                /* A = [[uv1-uv0],[uv2-uv0]] (rows); TB = A^-1 * E, E rows e1,e2 (Eigen 2x2 inverse) */
                float a00 = uv1.x - uv0.x, a01 = uv1.y - uv0.y, a10 = uv2.x - uv0.x, a11 = uv2.y - uv0.y;
                float invdet = 1.0f / (a00 * a11 - a10 * a01);
                float i00 = a11 * invdet, i10 = -a10 * invdet, i01 = -a01 * invdet, i11 = a00 * invdet;
                v3 T = V(i00 * e1.x + i01 * e2.x, i00 * e1.y + i01 * e2.y, i00 * e1.z + i01 * e2.z);
                v3 B = V(i10 * e1.x + i11 * e2.x, i10 * e1.y + i11 * e2.y, i10 * e1.z + i11 * e2.z);
                if (t->decal == RTG_DECAL_REPLACE_NORMAL) {
                    v3 rn = vdivs(tex_color(t, uv.x, uv.y), 255.0f);
                    rn = vnormalized(vsub(rn, V(0.5f, 0.5f, 0.5f)));
                    v3 N = ret->normal;
                    ret->normal = V(T.x * rn.x + (B.x * rn.y + N.x * rn.z), T.y * rn.x + (B.y * rn.y + N.y * rn.z),
                                    T.z * rn.x + (B.z * rn.y + N.z * rn.z));
                } else {
                    v2 dd = tex_change(t, uv.x, uv.y);
                    dd.x = dd.x * t->bump; dd.y = dd.y * t->bump;
                    v3 dpu = vadd(T, vmul(ret->normal, dd.x));
                    v3 dpv = vadd(B, vmul(ret->normal, dd.y));
                    v3 nn = vnormalized(vcross(dpv, dpu));
                    ret->normal = (vdot(ret->normal, nn) > 0) ? nn : vneg(nn);
                }
            }
        } else {
            if (t->decal == RTG_DECAL_REPLACE_KD) {
                ret->dm = t->decal;
                float p = perlin_compute(ret->point, t->noise_scale, t->nc);
                ret->textureColor = V(p, p, p);
                ret->textureNormalizer = 1;
            } else if (t->decal == RTG_DECAL_BUMP_NORMAL) {
                v3 g = perlin_gradient(ret->point, t->noise_scale, t->nc);
                v3 gpar = vmul(ret->normal, vdot(g, ret->normal));
                v3 nn = vsub(ret->normal, vmul(vsub(g, gpar), t->bump));
                ret->normal = (vdot(ret->normal, nn) > 0) ? nn : vneg(nn);
                ret->normal = vnormalized(ret->normal);
            }
        }
    }
}

/* Triangle::bvhIntersect, src/Shape.cpp:297-345 */
static RetVal triangle_intersect(const struct orc_scene* s, const Obj* o, int k, const Ray* ray) {
    const int* vi = o->pv + 3 * k;
    v3 a = s->vertices[vi[0] - 1], b = s->vertices[vi[1] - 1], c = s->vertices[vi[2] - 1];
    v3 amb = vsub(a, b), amc = vsub(a, c), amo = vsub(a, ray->origin), d = ray->direction;
    RetVal ret = ret_empty();
    float det = det3(amb, amc, d);
    float beta = det3(amo, amc, d) / det;
    float gamma = det3(amb, amo, d) / det;
    float t = det3(amb, amc, amo) / det;
    v3 normal;
    if (o->psmooth[k]) {
        float alpha = (1 - beta) - gamma;
        v3 n1 = s->vnormals[vi[0] - 1], n2 = s->vnormals[vi[1] - 1], n3 = s->vnormals[vi[2] - 1];
        normal = vadd(vadd(vmul(n1, alpha), vmul(n2, beta)), vmul(n3, gamma));
    } else {
        normal = vcross(vsub(c, b), vsub(a, b));
    }
    float eps = s->intEps;
    if (t >= -eps && (beta + gamma <= 1) && beta >= -eps && gamma >= -eps) {
        ret.normal = vdivs(normal, vnorm(normal));
        ret.point = ray_point(ray, t);
        triangle_texture(s, o, vi, vsub(b, a), vsub(c, a), beta, gamma, &ret);
        ret.full = 1;
    }
    return ret;
}

/* Sphere::bvhIntersect, src/Shape.cpp:347-398 */
static RetVal sphere_intersect(const struct orc_scene* s, const Obj* o, int k, const Ray* ray) {
    v3 d = ray->direction, og = ray->origin, c = s->vertices[o->pv[3 * k] - 1];
    float Rr = o->R;
    RetVal ret = ret_empty();
    v3 oc = vsub(og, c);
    float dd = vdot(d, oc);
    float disc = dd * dd - vdot(d, d) * (vdot(oc, oc) - Rr * Rr);
    if (disc < s->intEps) return ret;
    float sq = sqrtf(disc);
    float t1 = (-dd + sq) / vdot(d, d);
    float t2 = (-dd - sq) / vdot(d, d);
    v3 ip;
    if (t1 >= 0 && t2 < 0) ip = ray_point(ray, t1);
    else if (t2 >= 0 && t1 < 0) ip = ray_point(ray, t2);
    else if (t1 < 0 && t2 < 0) return ret;
    else ip = (t1 < t2) ? ray_point(ray, t1) : ray_point(ray, t2);
    ret.point = ip;
    v3 pc = vsub(ip, c);
    ret.normal = vdivs(pc, vnorm(pc));
    sphere_texture(s, o, c, Rr, &ret);
    ret.full = 1;
    return ret;
}

static RetVal prim_intersect(const struct orc_scene* s, const Obj* o, int k, const Ray* ray) {
    RetVal r = (o->type == RTG_OBJ_SPHERE) ? sphere_intersect(s, o, k, ray) : triangle_intersect(s, o, k, ray);
    r.prim = o->pface[k];
    return r;
}

/* ------------------------------------------------------------------ BVH (src/BVH.cpp) */
static float minOfThree(float a, float b, float c) {          /* Helper.cpp ShapeHelpers / BVH.cpp:10-22 */
    if (a <= b && a <= c) return a;
    else if (b <= a && b <= c) return b;
    return c;
}
static float maxOfThree(float a, float b, float c) {
    if (a >= b && a >= c) return a;
    else if (b >= a && b >= c) return b;
    return c;
}
static float minOfTwo(float a, float b) { return (a <= b) ? a : b; }   /* BVH.cpp:305-313 */
static float maxOfTwo(float a, float b) { return (a >= b) ? a : b; }

typedef struct { struct orc_scene* s; Obj* o; int* prims; int nn, cap; } Builder;

static v3 prim_center(const struct orc_scene* s, const Obj* o, int face) {
    if (o->type == RTG_OBJ_SPHERE) return s->vertices[o->pv[0] - 1];   /* Shape.cpp:64-67 */
    const int* vi = o->pv + 3 * face;                                   /* Shape.cpp:180-190 */
    v3 a = s->vertices[vi[0] - 1], b = s->vertices[vi[1] - 1], c = s->vertices[vi[2] - 1];
    return V(((a.x + b.x) + c.x) / 3.0f, ((a.y + b.y) + c.y) / 3.0f, ((a.z + b.z) + c.z) / 3.0f);
}
static void prim_box(const struct orc_scene* s, const Obj* o, int face, v3* mn, v3* mx) {
    if (o->type == RTG_OBJ_SPHERE) {                                    /* Shape.cpp:55-62 */
        v3 c = s->vertices[o->pv[0] - 1];
        float Rr = o->R;
        *mn = V(c.x - Rr, c.y - Rr, c.z - Rr);
        *mx = V(c.x + Rr, c.y + Rr, c.z + Rr);
        return;
    }
    const int* vi = o->pv + 3 * face;                                   /* Shape.cpp:162-178 */
    v3 a = s->vertices[vi[0] - 1], b = s->vertices[vi[1] - 1], c = s->vertices[vi[2] - 1];
    *mn = V(minOfThree(a.x, b.x, c.x), minOfThree(a.y, b.y, c.y), minOfThree(a.z, b.z, c.z));
    *mx = V(maxOfThree(a.x, b.x, c.x), maxOfThree(a.y, b.y, c.y), maxOfThree(a.z, b.z, c.z));
}
static int cmp_float(const void* a, const void* b) {
    float x = *(const float*)a, y = *(const float*)b;
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}
static int new_node(Builder* B) {
    if (B->nn == B->cap) {
        B->cap = B->cap ? B->cap * 2 : 64;
        B->o->nodes = (BNode*)realloc(B->o->nodes, sizeof(BNode) * B->cap);
    }
    return B->nn++;
}
/* BVH::ConstructionHelper, src/BVH.cpp:64-110 ; FindMedian BVH.cpp:117-135 ; ComputeBoundingBox BVH.cpp:268-283 */
static int construct(Builder* B, int start, int end, int splitType, int depth) {
    if (start == end - 1 || depth >= 30) {
        int n = new_node(B);
        BNode* N = &B->o->nodes[n];
        N->start = start; N->end = end; N->left = N->right = -1;
        /* leaves carry no tested box; record the range box for introspection only */
        v3 mn = V(FLT_MAX, FLT_MAX, FLT_MAX), mx = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
        for (int i = start; i < end; i++) {
            v3 a, b;
            prim_box(B->s, B->o, B->prims[i], &a, &b);
            mn = V(minOfTwo(mn.x, a.x), minOfTwo(mn.y, a.y), minOfTwo(mn.z, a.z));
            mx = V(maxOfTwo(mx.x, b.x), maxOfTwo(mx.y, b.y), maxOfTwo(mx.z, b.z));
        }
        B->o->nodes[n].mn = mn; B->o->nodes[n].mx = mx;
        return n;
    }
    if (start == end) return -1;
    if (splitType > 2) splitType = 0;
    v3 mn = V(FLT_MAX, FLT_MAX, FLT_MAX), mx = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = start; i < end; i++) {
        v3 a, b;
        prim_box(B->s, B->o, B->prims[i], &a, &b);
        mn = V(minOfTwo(mn.x, a.x), minOfTwo(mn.y, a.y), minOfTwo(mn.z, a.z));
        mx = V(maxOfTwo(mx.x, b.x), maxOfTwo(mx.y, b.y), maxOfTwo(mx.z, b.z));
    }
    int n = new_node(B);
    B->o->nodes[n].mn = mn; B->o->nodes[n].mx = mx;
    B->o->nodes[n].start = start; B->o->nodes[n].end = end;
    /* FindMedian */
    int len = end - start;
    float* cs = (float*)malloc(sizeof(float) * len);
    for (int i = start; i < end; i++) cs[i - start] = vget(prim_center(B->s, B->o, B->prims[i]), splitType);
    qsort(cs, len, sizeof(float), cmp_float);
    int mi = len / 2;
    float split = (len % 2 == 0) ? (cs[mi - 1] + cs[mi]) * 0.5f : cs[mi];
    free(cs);
    int swapIndex = start;
    for (int i = start; i < end; i++) {
        float center = vget(prim_center(B->s, B->o, B->prims[i]), splitType);
        if (center < split) {
            int tmp = B->prims[swapIndex];
            B->prims[swapIndex] = B->prims[i];
            B->prims[i] = tmp;
            swapIndex++;
        }
    }
    int l = construct(B, start, swapIndex, splitType + 1, depth + 1);
    int r = construct(B, swapIndex, end, splitType + 1, depth + 1);
    B->o->nodes[n].left = l;
    B->o->nodes[n].right = r;
    return n;
}

/* BVH::RayBBoxIntersection, src/BVH.cpp:212-266 */
static int box_test(const Ray* ray, v3 mn, v3 mx) {
    float dx = ray->direction.x, dy = ray->direction.y, dz = ray->direction.z;
    float txe, txl, tye, tyl, tze, tzl;
    if (dx > 0) { txe = (mn.x - ray->origin.x) / dx; txl = (mx.x - ray->origin.x) / dx; }
    else { txe = (mx.x - ray->origin.x) / dx; txl = (mn.x - ray->origin.x) / dx; }
    if (dy > 0) { tye = (mn.y - ray->origin.y) / dy; tyl = (mx.y - ray->origin.y) / dy; }
    else { tye = (mx.y - ray->origin.y) / dy; tyl = (mn.y - ray->origin.y) / dy; }
    if (dz > 0) { tze = (mn.z - ray->origin.z) / dz; tzl = (mx.z - ray->origin.z) / dz; }
    else { tze = (mx.z - ray->origin.z) / dz; tzl = (mn.z - ray->origin.z) / dz; }
    float tSmallestL = minOfThree(txl, tyl, tzl);
    float tLargestE = maxOfThree(txe, tye, tze);
    if (tSmallestL < tLargestE) return 0;
    return 1;
}

/* BVH::FindIntersectionWithBVH, src/BVH.cpp:137-210 (literal: visits both children) */
static RetVal bvh_find(const struct orc_scene* s, const Obj* o, const Ray* ray, int node) {
    if (node < 0) return ret_empty();
    const BNode* N = &o->nodes[node];
    if (N->left < 0 && N->right < 0) {
        RetVal nearest = ret_empty();
        float nearestPoint = FLT_MAX;
        for (int i = N->start; i < N->end; i++) {
            RetVal r = prim_intersect(s, o, i, ray);
            if (r.full) {
                float d = vnorm(vsub(r.point, ray->origin));
                if (d < nearestPoint) {
                    nearestPoint = d;
                    nearest = r;
                    nearest.matIndex = o->matIndex;
                }
            }
        }
        return nearest;
    }
    if (box_test(ray, N->mn, N->mx)) {
        RetVal L = bvh_find(s, o, ray, N->left);
        RetVal Rr = bvh_find(s, o, ray, N->right);
        if (L.full && !Rr.full) return L;
        else if (!L.full && Rr.full) return Rr;
        else if (L.full && Rr.full) {
            float dl = vnorm(vsub(L.point, ray->origin));
            float dr = vnorm(vsub(Rr.point, ray->origin));
            return (dl < dr) ? L : Rr;
        }
    }
    return ret_empty();
}

/* BVHMethods::FindIntersection, src/Helper.cpp:18-80 */
static RetVal find_intersection(const struct orc_scene* s, const Ray* ray) {
    RetVal nearest = ret_empty();
    float nearestDistance = FLT_MAX;
    const mat4* IT = NULL;
    if (visnan(ray->origin) || visnan(ray->direction)) return nearest;
    for (int i = 0; i < s->nobj; i++) {
        const Obj* o = &s->objs[i];
        Ray tr = transform_ray(ray, &o->inv, o->blur);
        RetVal r = bvh_find(s, o, &tr, o->root);
        if (r.full) {
            float distance = ray_gett(&tr, r.point);
            if (distance < nearestDistance && distance > 0) {
                nearestDistance = distance;
                IT = &o->invT;
                r.point = ray_point(ray, distance);
                r.obj = i;
                r.t = distance;
                nearest = r;
            }
        }
    }
    for (int i = 0; i < s->ninst; i++) {
        const Inst* in = &s->insts[i];
        const Obj* o = &s->objs[in->base];
        Ray tr = transform_ray(ray, &in->inv, in->blur);
        RetVal r = bvh_find(s, o, &tr, o->root);
        if (r.full) {
            float distance = ray_gett(&tr, r.point);
            if (distance < nearestDistance && distance > 0) {
                nearestDistance = distance;
                IT = &in->invT;
                r.matIndex = in->matIndex;
                r.point = ray_point(ray, distance);
                r.obj = s->nobj + i;
                r.t = distance;
                nearest = r;
            }
        }
    }
    if (nearest.full) nearest.normal = transform_normal(nearest.normal, IT);
    return nearest;
}

/* ------------------------------------------------------------------ lights (src/Light.cpp) */
static const rtg_material_desc* MAT(const struct orc_scene* s, int matIndex) { return &s->mats[matIndex - 1]; }
static v3 mv(const float f[3]) { return V(f[0], f[1], f[2]); }

/* Scene::ConductorFresnel, src/Scene.cpp:135-146 (the same formula as Light::Fresnel, src/Light.cpp:18-28) */
static float conductor_fresnel(float n_t, float k_t, v3 ray, v3 normal) {
    float cos_t = -vdot(ray, normal);
    float twoNtCost = (2 * n_t) * cos_t;
    float cosSquared = (float)pow((double)cos_t, 2);
    float ntk = (float)(pow((double)n_t, 2) + pow((double)k_t, 2));
    float rs = ((ntk - twoNtCost) + cosSquared) / ((ntk + twoNtCost) + cosSquared);
    float rp = ((ntk * cosSquared - twoNtCost) + 1) / ((ntk * cosSquared + twoNtCost) + 1);
    return 0.5f * (rs + rp);
}
/* Light::GeometryTS Light.cpp:49-60, DistributionTS Light.cpp:12-16 */
static float geometry_ts(v3 wi, v3 wo, v3 wh, v3 n) {
    float left = (2.0f * vdot(n, wh)) * vdot(n, wo);
    left = left / vdot(wo, wh);
    float right = (2.0f * vdot(n, wh)) * vdot(n, wi);
    right = right / vdot(wi, wh);
    float x = stdmin(left, right);
    return stdmin(1.0f, x);
}
static float distribution_ts(float cosAlpha, int phongExp) {
    float x = (float)((double)((float)phongExp + 2.0f) / (double)(2.0f * PI_D));
    x = (float)((double)x * pow((double)cosAlpha, phongExp));
    return x;
}
/* Light::TermBRDF, src/Light.cpp:62-155 */
static v3 term_brdf(v3 wi, v3 wo, const RetVal* ret, const rtg_material_desc* m) {
    v3 n = ret->normal, kd = mv(m->diffuse), ks = mv(m->specular);
    int p = m->phong_exp;
    switch (m->brdf) {
    case RTG_BRDF_MP:
    case RTG_BRDF_OP:
    case RTG_BRDF_MPN: {
        float n_wi = vdot(n, wi);
        v3 wr = vadd(vneg(wi), vmul(vmul(n, 2), n_wi));
        wr = vdivs(wr, vnorm(wr));
        float cosAngle = fmax0(vdot(wr, wo));
        if (m->brdf == RTG_BRDF_MP) return vadd(kd, vmul(ks, (float)pow((double)cosAngle, p)));
        if (m->brdf == RTG_BRDF_OP) {
            float cti = fmax0(vdot(wi, n));
            if (cti < 0.001f) return V(0, 0, 0);
            return vadd(kd, vdivs(vmul(ks, (float)pow((double)cosAngle, p)), cti));
        }
        v3 dp = vdivs(kd, (float)PI_D);
        v3 sp = vmul(vmul(ks, (float)((p + 2) / (2 * PI_D))), (float)pow((double)cosAngle, p));
        return vadd(dp, sp);
    }
    case RTG_BRDF_MBP:
    case RTG_BRDF_OBP:
    case RTG_BRDF_MBPN: {
        v3 h = vnormalized(vadd(wo, wi));
        float nh = vdot(n, h);
        float cosAngle = fmax0(nh);
        if (m->brdf == RTG_BRDF_MBP) return vadd(kd, vmul(ks, (float)pow((double)cosAngle, p)));
        if (m->brdf == RTG_BRDF_OBP) {
            float cti = fmax0(vdot(wi, n));
            if (cti < 0.001f) return V(0, 0, 0);
            return vadd(kd, vdivs(vmul(ks, (float)pow((double)cosAngle, p)), cti));
        }
        v3 dp = vdivs(kd, (float)PI_D);
        v3 sp = vmul(vmul(ks, (float)((p + 8) / (8 * PI_D))), (float)pow((double)cosAngle, p));
        return vadd(dp, sp);
    }
    case RTG_BRDF_TS:
    case RTG_BRDF_TSF: {
        v3 wh = vnormalized(vadd(wo, wi));
        float f = 0;
        v3 dp = vdivs(kd, (float)PI_D);
        if (m->brdf == RTG_BRDF_TSF) {
            f = conductor_fresnel(m->refraction_index, m->absorption_index, vneg(wo), n);
            dp = vmul(dp, 1 - f);
        }
        float cosAlpha = vdot(wh, n), cosTheta = vdot(wi, n), cosPhi = vdot(wo, n);
        float g = geometry_ts(wi, wo, wh, n);
        float d = distribution_ts(cosAlpha, p);
        v3 sp = vmul(vmul(ks, g), d);
        sp = vdivs(sp, (4.0f * cosPhi) * cosTheta);
        if (m->brdf == RTG_BRDF_TSF) sp = vmul(sp, f);
        return vadd(dp, sp);
    }
    default:
        return V(0, 0, 0);
    }
}
/* Light::BRDF Light.cpp:157-162 */
static v3 brdf(v3 wi, v3 wo, const RetVal* ret, v3 radiance, const rtg_material_desc* m) {
    v3 t = term_brdf(wi, wo, ret, m);
    float cosAngle = fmax0(vdot(wi, ret->normal));
    return vmul(vcw(radiance, t), cosAngle);
}
/* Diffuse kd selection shared by all lights (e.g. PointLight::Diffuse Light.cpp:206-223) */
static v3 diffuse_term(v3 LC, const RetVal* ret, const rtg_material_desc* m, float alpha) {
    if (ret->dm == RTG_DECAL_REPLACE_KD)
        return vcw(LC, vmul(vdivs(ret->textureColor, ret->textureNormalizer), alpha));
    if (ret->dm == RTG_DECAL_BLEND_KD) {
        v3 bl = vmul(vadd(mv(m->diffuse), vdivs(ret->textureColor, ret->textureNormalizer)), 0.5f);
        return vcw(LC, vmul(bl, alpha));
    }
    return vcw(LC, vmul(mv(m->diffuse), alpha));
}
static v3 specular_term(v3 LC, v3 wo, v3 wi, const RetVal* ret, const rtg_material_desc* m) {
    v3 s = vadd(wo, wi);
    v3 h = vdivs(s, vnorm(s));
    float alpha = fmax0(vdot(ret->normal, h));
    return vcw(LC, vmul(mv(m->specular), (float)pow((double)alpha, m->phong_exp)));
}

/* ------------------------------------------------------------------ SURVEY §8(d) yardstick
   Not the reference's algorithm: the canonical ordered, early-exit traversal a GPU closest-hit
   kernel would run over the SAME scene and the reference's median-split trees, used only to
   count the algorithmic work per ray that §8(d)'s byte model prices
   (B = 64 + 32 N_node + 36 N_tri + 16 N_sphere): N_node = 32-byte child records read (both
   children's boxes of every interior node popped, the root box once), N_tri / N_sphere =
   primitive tests.  Closest-hit rays (primary + secondary) keep the nearest accepted t (> 0) as
   the far end of every box interval; shadow rays stop at the first hit in (0, tmax) (any hit).
   The top level is the reference's object / instance loop (src/Helper.cpp:32-73). */
static int canon_box(const Ray* r, v3 mn, v3 mx, float tmax, float* tentry) {
    float t0 = 0.0f, t1 = tmax;
    for (int a = 0; a < 3; a++) {
        float o = vget(r->origin, a), d = vget(r->direction, a), lo = vget(mn, a), hi = vget(mx, a);
        float ta = (lo - o) / d, tb = (hi - o) / d;
        if (ta != ta || tb != tb) continue;          /* 0 * inf: the slab does not constrain */
        if (ta > tb) { float x = ta; ta = tb; tb = x; }
        if (ta > t0) t0 = ta;
        if (tb < t1) t1 = tb;
    }
    *tentry = t0;
    return t0 <= t1;
}
/* one object in its own space: returns the nearest accepted t in (0, tmax) or tmax */
static float canon_object(const struct orc_scene* s, const Obj* o, const Ray* r, float tmax, int any, uint64_t* c) {
    float best = tmax;
    int done = 0;
    if (o->type == RTG_OBJ_SPHERE) {
        c[3]++;
        RetVal h = prim_intersect(s, o, 0, r);
        if (h.full) { float t = ray_gett(r, h.point); if (t > 0 && t < best) best = t; }
        return best;
    }
    int stack[64], sp = 0;
    int node = o->root;
    if (node < 0) return best;
    const BNode* N = &o->nodes[node];
    if (N->left >= 0 || N->right >= 0) {
        float te;
        c[1]++;
        if (!canon_box(r, N->mn, N->mx, best, &te)) return best;
    }
    stack[sp++] = node;
    while (sp > 0 && !done) {
        N = &o->nodes[stack[--sp]];
        if (N->left < 0 && N->right < 0) {
            for (int k = N->start; k < N->end && !done; k++) {
                c[2]++;
                RetVal h = prim_intersect(s, o, k, r);
                if (!h.full) continue;
                float t = ray_gett(r, h.point);
                if (t > 0 && t < best) { best = t; done = any; }
            }
            continue;
        }
        int kid[2] = {N->left, N->right}, hit[2] = {0, 0};
        float te[2] = {0, 0};
        for (int q = 0; q < 2; q++) {
            if (kid[q] < 0) continue;
            c[1]++;
            hit[q] = canon_box(r, o->nodes[kid[q]].mn, o->nodes[kid[q]].mx, best, &te[q]);
        }
        if (hit[0] && hit[1]) {                  /* nearer child on top */
            int nearq = te[1] < te[0];
            stack[sp++] = kid[1 - nearq];
            stack[sp++] = kid[nearq];
        } else if (hit[0]) stack[sp++] = kid[0];
        else if (hit[1]) stack[sp++] = kid[1];
    }
    return best;
}
static void canon_count(Ctx* cx, const Ray* r, int kind, float tmax) {
    const struct orc_scene* s = cx->s;
    if (visnan(r->origin) || visnan(r->direction)) return;
    uint64_t* c = cx->canon + (kind == 2 ? 4 : 0);
    c[0]++;
    float best = tmax;
    for (int i = 0; i < s->nobj + s->ninst; i++) {
        const Obj* o = i < s->nobj ? &s->objs[i] : &s->objs[s->insts[i - s->nobj].base];
        Ray tr = i < s->nobj ? transform_ray(r, &o->inv, o->blur)
                             : transform_ray(r, &s->insts[i - s->nobj].inv, s->insts[i - s->nobj].blur);
        best = canon_object(s, o, &tr, best, kind == 2, c);
        if (kind == 2 && best < tmax) return;    /* shadow: first blocker ends the query */
    }
}

static RetVal trace_bounded(Ctx* cx, const Ray* r, int kind, float tmax) {
    if (!(visnan(r->origin) || visnan(r->direction))) {
        if (kind == 0) cx->n_primary++; else if (kind == 1) cx->n_secondary++; else cx->n_shadow++;
    }
    if (cx->s->canon_on) canon_count(cx, r, kind, tmax);
    return find_intersection(cx->s, r);
}
static RetVal trace(Ctx* cx, const Ray* r, int kind) { return trace_bounded(cx, r, kind, FLT_MAX); }

/* distance-compared shadow test of Point/Spot/Area lights, e.g. PointLight::IsShadow Light.cpp:188-204 */
static int shadow_towards(Ctx* cx, const Ray* prime, const RetVal* ret, v3 L) {
    struct orc_scene* s = cx->s;
    v3 dir = vsub(L, ret->point);
    Ray ray = R(vadd(ret->point, vmul(ret->normal, s->shadowEps)), vdivs(dir, vnorm(dir)), prime->time);
    RetVal nr = trace_bounded(cx, &ray, 2, vnorm(vsub(L, ray.origin)));
    if (nr.full) return vnorm(vsub(ret->point, L)) > vnorm(vsub(ret->point, nr.point));
    return 0;
}
static int shadow_dir(Ctx* cx, const Ray* prime, const RetVal* ret, v3 dir) {
    struct orc_scene* s = cx->s;
    Ray ray = R(vadd(ret->point, vmul(ret->normal, s->shadowEps)), dir, prime->time);
    RetVal nr = trace(cx, &ray, 2);
    return nr.full;
}

/* EnvironmentLight::ComputeLightContribution Light.cpp:563-575 */
static v3 env_radiance(const struct orc_scene* s, const Lgt* L, v3 direction) {
    float theta = f_acos(direction.y);
    float phi = f_atan2(direction.z, direction.x);
    float tu = (float)((-(double)phi + PI_D) / (2 * PI_D));
    float tv = (float)((double)theta / PI_D);
    v3 rad = tex_color(&s->texs[L->tex], tu, tv);
    return vmul(vmul(rad, 2), (float)PI_D);
}

static v3 light_shading(Ctx* cx, int li, const Ray* prime, const RetVal* ret, const rtg_material_desc* m,
                        uint64_t path) {
    struct orc_scene* s = cx->s;
    const Lgt* L = &s->lights[li];
    v3 wo = vneg(prime->direction);
    switch (L->type) {
    case RTG_LIGHT_POINT: {                                   /* PointLight::BasicShading Light.cpp:238-250 */
        if (shadow_towards(cx, prime, ret, L->pos)) return V(0, 0, 0);
        float dist = vnorm(vsub(ret->point, L->pos));
        v3 LC = vdivs(L->inten, dist * dist);
        v3 wi = vnormalized(vsub(L->pos, ret->point));
        if (m->brdf != RTG_BRDF_NONE) return brdf(wi, wo, ret, LC, m);
        float alpha = fmax0(vdot(ret->normal, wi));
        return vadd(diffuse_term(LC, ret, m, alpha), specular_term(LC, wo, wi, ret, m));
    }
    case RTG_LIGHT_DIRECTIONAL: {                             /* DirectionalLight::BasicShading Light.cpp:309-321 */
        v3 wi = vneg(L->dir);
        if (shadow_dir(cx, prime, ret, wi)) return V(0, 0, 0);
        if (m->brdf != RTG_BRDF_NONE) return brdf(wi, wo, ret, L->inten, m);
        float alpha = fmax0(vdot(ret->normal, wi));
        return vadd(diffuse_term(L->inten, ret, m, alpha), specular_term(L->inten, wo, wi, ret, m));
    }
    case RTG_LIGHT_SPOT: {                                    /* SpotLight::BasicShading Light.cpp:409-436 */
        if (shadow_towards(cx, prime, ret, L->pos)) return V(0, 0, 0);
        v3 dtp = vnormalized(vsub(ret->point, L->pos));
        float angle = f_acos(vdot(dtp, L->dir));
        if (!(angle < L->fall) && !(angle < L->coverage)) return V(0, 0, 0);
        float dist = vnorm(vsub(ret->point, L->pos));
        v3 LC = vdivs(L->inten, dist * dist);
        v3 wi = vnormalized(vsub(L->pos, ret->point));
        v3 c;
        if (m->brdf != RTG_BRDF_NONE) c = brdf(wi, wo, ret, LC, m);
        else {
            float alpha = fmax0(vdot(ret->normal, wi));
            c = vadd(diffuse_term(LC, ret, m, alpha), specular_term(LC, wo, wi, ret, m));
        }
        if (angle < L->fall) return c;
        float cf = f_cos(L->fall), cc = f_cos(L->coverage);
        float fo = (float)pow((cos((double)angle) - (double)cc) / (double)(cf - cc), 4);   /* FallOf Light.cpp:343-348 */
        return vmul(c, fo);
    }
    case RTG_LIGHT_AREA: {                                    /* AreaLight::BasicShading Light.cpp:522-545 */
        float xi[4];
        rng4(cx->rng.seed, cx->rng.pixel, cx->rng.sample, path, RNG_AREA, (uint32_t)li, 0, xi);
        float uChi = xi[0] - 0.5f, vChi = xi[1] - 0.5f;
        v3 sample = vadd(vadd(L->pos, vmul(vmul(L->u, L->size), uChi)), vmul(vmul(L->v, L->size), vChi));
        if (shadow_towards(cx, prime, ret, sample)) return V(0, 0, 0);
        /* FindAreaFactor Light.cpp:457-463 */
        v3 pms = vsub(ret->point, sample);
        float cosTheta = fabsf(vdot(vnormalized(pms), L->normal));
        float dSq = vnorm(pms);
        dSq = dSq * dSq;
        v3 LC = vmul(L->inten, (L->size * L->size) * (cosTheta / dSq));
        v3 wi = vnormalized(vsub(sample, ret->point));
        if (m->brdf != RTG_BRDF_NONE) return brdf(wi, wo, ret, LC, m);
        float alpha = fmax0(vdot(ret->normal, wi));
        return vadd(diffuse_term(LC, ret, m, alpha), specular_term(LC, wo, wi, ret, m));
    }
    case RTG_LIGHT_ENVIRONMENT: {                             /* EnvironmentLight::BasicShading Light.cpp:628-660 */
        v3 n = ret->normal;
        v3 u = ortho_u(n);
        v3 w = vcross(n, u);
        v3 direction;
        for (uint32_t it = 0;; it++) {
            float xi[4];
            rng4(cx->rng.seed, cx->rng.pixel, cx->rng.sample, path, RNG_ENV, (uint32_t)li, it, xi);
            float x = xi[0] * 2 - 1.0f, y = xi[1] * 2 - 1.0f, z = xi[2] * 2 - 1.0f;
            v3 sample = vadd(vadd(vadd(ret->point, vmul(u, x)), vmul(n, y)), vmul(w, z));
            direction = vsub(sample, ret->point);
            if (vdot(direction, n) > 0 && vnorm(direction) <= 1) { direction = vnormalized(direction); break; }
            if (it > 1000000u) { direction = n; break; }   /* degenerate normal guard */
        }
        if (shadow_dir(cx, prime, ret, direction)) return V(0, 0, 0);
        v3 LC = env_radiance(s, L, direction);
        if (m->brdf != RTG_BRDF_NONE) return brdf(direction, wo, ret, LC, m);
        float alpha = fmax0(vdot(n, direction));
        return vadd(diffuse_term(LC, ret, m, alpha), specular_term(LC, wo, direction, ret, m));
    }
    }
    return V(0, 0, 0);
}

/* Scene::BasicShading Scene.cpp:243-267 with Scene::ambient Scene.cpp:22-30 */
static v3 basic_shading(Ctx* cx, const Ray* ray, const RetVal* ret, const rtg_material_desc* m, uint64_t path) {
    struct orc_scene* s = cx->s;
    v3 raw = vadd(V(0, 0, 0), vcw(s->ambientLight, mv(m->ambient)));
    for (int i = 0; i < s->nlight; i++) raw = vadd(raw, light_shading(cx, i, ray, ret, m, path));
    return raw;
}

/* ------------------------------------------------------------------ integrator (src/Scene.cpp) */
typedef struct { Ray ray; RetVal ret; } ShadeComp;

/* Scene::MirrorReflectance Scene.cpp:32-55 (path = node whose reflection this is) */
static ShadeComp mirror_reflectance(Ctx* cx, const Ray* ray, const RetVal* ret, const rtg_material_desc* m,
                                    uint64_t path) {
    struct orc_scene* s = cx->s;
    v3 wo = vneg(ray->direction);
    float n_wo = vdot(ret->normal, wo);
    v3 wr = vadd(vneg(wo), vmul(vmul(ret->normal, 2), n_wo));
    wr = vdivs(wr, vnorm(wr));
    if (m->is_rough) {
        v3 u = ortho_u(wr);
        v3 v = vcross(wr, u);
        float xi[4];
        rng4(cx->rng.seed, cx->rng.pixel, cx->rng.sample, path, RNG_ROUGH, 0, 0, xi);
        float uChi = xi[0] - 0.5f, vChi = xi[1] - 0.5f;
        wr = vnormalized(vadd(wr, vmul(vadd(vmul(u, uChi), vmul(v, vChi)), m->roughness)));
    }
    ShadeComp sc;
    sc.ray = R(vadd(ret->point, vmul(ret->normal, s->shadowEps)), wr, ray->time);
    sc.ret = trace(cx, &sc.ray, 1);
    return sc;
}

static v3 nan_check(v3 c) { return visnan(c) ? V(0, 0, 0) : c; }   /* Scene.cpp:221-228 */

static v3 recursive_shading(Ctx* cx, const Ray* ray, const RetVal* ret, int depth, uint64_t path);

/* Scene::DielectricRefraction Scene.cpp:57-118 + FresnelReflectance Scene.cpp:120-128 + BeerLaw Scene.cpp:130-133 */
static v3 dielectric(Ctx* cx, const Ray* ray, const RetVal* ret, const rtg_material_desc* m, int depth, uint64_t path) {
    struct orc_scene* s = cx->s;
    float dp = vdot(ray->direction, ret->normal);
    float nt = m->refraction_index;
    float snell, n_t, n_i;
    v3 normal;
    int entering;
    if (dp < 0) { snell = 1.0f / nt; normal = ret->normal; n_t = nt; n_i = 1; entering = 1; }
    else { snell = nt; normal = vneg(ret->normal); n_t = 1; n_i = nt; entering = 0; }
    float cosTheta = -vdot(ray->direction, normal);
    v3 leftPart = vmul(vadd(ray->direction, vmul(normal, cosTheta)), snell);
    float srp = (float)(1 - pow((double)snell, 2) * (1 - pow((double)cosTheta, 2)));
    int isTir = srp < 0;
    srp = sqrtf(srp);
    v3 tdir = vnormalized(vsub(leftPart, vmul(normal, srp)));
    Ray tRay = R(vsub(ret->point, vmul(normal, s->shadowEps)), tdir, ray->time);
    RetVal tret = trace(cx, &tRay, 1);
    float cos_t = -vdot(tRay.direction, normal);
    float cos_i = -vdot(ray->direction, normal);
    float rPar = (n_t * cos_i - n_i * cos_t) / (n_t * cos_i + n_i * cos_t);
    float rPer = (n_i * cos_i - n_t * cos_t) / (n_i * cos_i + n_t * cos_t);
    float F = (float)(0.5f * (pow((double)rPar, 2) + pow((double)rPer, 2)));
    float bd = vnorm(vsub(tret.point, ret->point));
    v3 sig = mv(m->absorption_coeff);
    v3 beer = V(f_exp(-sig.x * bd), f_exp(-sig.y * bd), f_exp(-sig.z * bd));

    uint64_t refrPath = 2 * path, reflPath = 2 * path + 1;
    if (entering) {
        v3 inside = recursive_shading(cx, &tRay, &tret, depth - 1, refrPath);
        inside = vmul(inside, 1 - F);
        inside = vcw(beer, inside);
        ShadeComp sc = mirror_reflectance(cx, ray, ret, m, path);
        v3 refl = recursive_shading(cx, &sc.ray, &sc.ret, depth - 1, reflPath);
        refl = vmul(refl, F);
        inside = nan_check(inside);
        refl = nan_check(refl);
        return vadd(vadd(basic_shading(cx, ray, ret, m, path), inside), refl);
    }
    if (isTir) {
        ShadeComp sc = mirror_reflectance(cx, ray, ret, m, path);
        v3 ir = recursive_shading(cx, &sc.ray, &sc.ret, depth - 1, reflPath);
        ir = vcw(beer, ir);
        return nan_check(ir);
    }
    v3 outside = recursive_shading(cx, &tRay, &tret, depth - 1, refrPath);
    outside = vmul(outside, 1 - F);
    ShadeComp sc = mirror_reflectance(cx, ray, ret, m, path);
    v3 refl = recursive_shading(cx, &sc.ray, &sc.ret, depth - 1, reflPath);
    refl = vmul(refl, F);
    refl = vcw(beer, refl);
    outside = nan_check(outside);
    refl = nan_check(refl);
    return vadd(outside, refl);
}

/* Scene::RecursiveShading Scene.cpp:148-219 */
static v3 recursive_shading(Ctx* cx, const Ray* ray, const RetVal* ret, int depth, uint64_t path) {
    if (!ret->full) return V(0, 0, 0);
    const rtg_material_desc* m = MAT(cx->s, ret->matIndex);
    if (m->type == RTG_MAT_NORMAL || depth <= 0) return basic_shading(cx, ray, ret, m, path);
    if (m->type == RTG_MAT_MIRROR) {
        ShadeComp sc = mirror_reflectance(cx, ray, ret, m, path);
        v3 rc = recursive_shading(cx, &sc.ray, &sc.ret, depth - 1, 2 * path + 1);
        rc = vcw(mv(m->mirror), rc);
        return vadd(basic_shading(cx, ray, ret, m, path), rc);
    }
    if (m->type == RTG_MAT_DIELECTRIC) return dielectric(cx, ray, ret, m, depth, path);
    /* conductor */
    float f = conductor_fresnel(m->refraction_index, m->absorption_index, ray->direction, ret->normal);
    ShadeComp sc = mirror_reflectance(cx, ray, ret, m, path);
    v3 rc = recursive_shading(cx, &sc.ray, &sc.ret, depth - 1, 2 * path + 1);
    rc = vmul(rc, f);
    rc = vcw(mv(m->mirror), rc);
    return vadd(basic_shading(cx, ray, ret, m, path), rc);
}

/* Scene::Shading Scene.cpp:230-241 */
static v3 shading(Ctx* cx, const Ray* ray, const RetVal* ret) {
    if (ret->dm == RTG_DECAL_REPLACE_ALL) return ret->textureColor;
    return recursive_shading(cx, ray, ret, cx->s->maxDepth, 1);
}

/* Scene::GetBackgroundColor Scene.cpp:413-435 */
static v3 background(const struct orc_scene* s, int row, int col, int nx, int ny, const Ray* ray) {
    if (s->envLight != -1) {
        const Lgt* L = &s->lights[s->envLight];
        if (L->type != RTG_LIGHT_ENVIRONMENT) return s->background;
        float theta = f_acos(ray->direction.y);
        float phi = f_atan2(ray->direction.z, ray->direction.x);
        float tu = (float)((-(double)phi + PI_D) / (2 * PI_D));
        float tv = (float)((double)theta / PI_D);
        return tex_color(&s->texs[L->tex], tu, tv);
    }
    if (s->bgTexture == -1) return s->background;
    float u = ((float)col) / (float)nx;
    float v = ((float)row) / (float)ny;
    return tex_color(&s->texs[s->bgTexture], u, v);
}

/* ------------------------------------------------------------------ hw7 path tracer
 * No reference code exists (pages/Page7.md describes it in prose only).
 * This is the integrator DESIGN.md §8 specifies; librtg.so's wavefront must match it bit
 * for bit.  Per sample: throughput T, radiance L; at each vertex L += T (x) v where v is
 *   - the emitter radiance on an object-light hit (counted at the camera vertex, without
 *     NEE, or after a specular bounce — Page7.md:135-141), which ends the path;
 *   - else Scene::BasicShading (ambient + every light in order, shadowed) plus, with NEE,
 *     one sample of every object light (Page7.md:143-147 distance-checked shadow test);
 * then the path continues by one sampled direction (diffuse: uniform / cosine hemisphere,
 * mirror / conductor: reflection, dielectric: reflect or refract chosen by Fresnel).
 * Russian roulette continues with probability |n . w_next| (Page7.md:41-45) and lifts the
 * MaxRecursionDepth cap (RTG_PT_MAX_BOUNCES bounds the path instead). */
static int is_emitter(const struct orc_scene* s, const RetVal* r, const Emit** out) {
    if (r->obj < 0 || r->obj >= s->nobj) return 0;
    for (int k = 0; k < s->nemit; k++)
        if (s->emits[k].obj == r->obj) { *out = &s->emits[k]; return 1; }
    return 0;
}

/* light response used everywhere: the material's BRDF (Light::BRDF) or the reference's
   non-BRDF Blinn-Phong diffuse + specular terms, for incident radiance LC */
static v3 surface_response(v3 LC, v3 wo, v3 wi, const RetVal* ret, const rtg_material_desc* m) {
    if (m->brdf != RTG_BRDF_NONE) return brdf(wi, wo, ret, LC, m);
    float alpha = fmax0(vdot(ret->normal, wi));
    return vadd(diffuse_term(LC, ret, m, alpha), specular_term(LC, wo, wi, ret, m));
}

/* NEE: one sample of emitter k (light slot nlight + k) */
static v3 emitter_shading(Ctx* cx, int k, const Ray* prime, const RetVal* ret, const rtg_material_desc* m,
                          uint64_t path) {
    struct orc_scene* s = cx->s;
    const Emit* E = &s->emits[k];
    const uint32_t li = (uint32_t)(s->nlight + k);
    float xi[4];
    rng4(cx->rng.seed, cx->rng.pixel, cx->rng.sample, path, RNG_PT_EMIT, li, 0, xi);
    v3 p = ret->point, wo = vneg(prime->direction);
    v3 q, wi, LC;
    float dist;
    if (E->sphere) {
        /* uniform in the cone the sphere subtends; from inside, uniform over all directions */
        v3 dv = vsub(E->center, p);
        float dd = vnorm(dv);
        int inside = !(dd > E->radius);
        float cosmax = -1.0f;
        if (!inside) {
            float sin2 = (E->radius * E->radius) / (dd * dd);
            cosmax = sqrtf(fmax0(1.0f - sin2));
        }
        float cosT = 1.0f - xi[0] * (1.0f - cosmax);
        float sinT = sqrtf(fmax0(1.0f - cosT * cosT));
        float phi = (float)(2 * PI_D) * xi[1];
        v3 dn = dd > 0.0f ? vdivs(dv, dd) : V(0, 1, 0);
        v3 u = ortho_u(dn), w = vcross(dn, u);
        wi = vnormalized(vadd(vadd(vmul(u, sinT * f_cos(phi)), vmul(w, sinT * f_sin(phi))), vmul(dn, cosT)));
        v3 oc = vsub(p, E->center);
        float b = vdot(wi, oc);
        float disc = b * b - (vsqn(oc) - E->radius * E->radius);
        float t = inside ? -b + sqrtf(fmax0(disc)) : -b - sqrtf(fmax0(disc));
        q = vadd(p, vmul(wi, t));
        dist = vnorm(vsub(p, q));
        LC = vmul(E->Le, (float)(2 * PI_D) * (1.0f - cosmax));
    } else {
        const float* cdf = s->ecdf + E->tri_first;
        float target = xi[0] * E->area;
        int lo = 0, hi = E->tri_count - 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (target < cdf[mid]) hi = mid; else lo = mid + 1;
        }
        const v3* T = s->etris + 3 * (size_t)(E->tri_first + lo);
        float sq = sqrtf(xi[1]);
        q = vadd(vadd(vmul(T[0], 1.0f - sq), vmul(T[1], sq * (1.0f - xi[2]))), vmul(T[2], sq * xi[2]));
        v3 nl = vnormalized(vcross(vsub(T[1], T[0]), vsub(T[2], T[0])));
        v3 dv = vsub(q, p);
        dist = vnorm(dv);
        wi = vdivs(dv, dist);
        float cosl = fabsf(vdot(wi, nl));
        LC = vmul(E->Le, (cosl * E->area) / (dist * dist));
    }
    v3 c = surface_response(LC, wo, wi, ret, m);
    if (c.x == 0.0f && c.y == 0.0f && c.z == 0.0f) return V(0, 0, 0);   /* nothing to shadow: no ray */
    Ray ray = R(vadd(p, vmul(ret->normal, s->shadowEps)), wi, prime->time);
    RetVal nr = trace_bounded(cx, &ray, 2, dist);
    if (nr.full && vnorm(vsub(p, nr.point)) < dist - (s->shadowEps + 1e-4f * dist)) return V(0, 0, 0);
    return c;
}

static v3 pt_sample(Ctx* cx, Ray ray, int flags, v3 bg) {
    struct orc_scene* s = cx->s;
    v3 L = V(0, 0, 0), T = V(1, 1, 1);
    int spec = 1, medium = 0, depth = s->maxDepth;
    for (int b = 0;; b++) {
        const uint64_t path = (uint64_t)b + 1;
        RetVal ret = trace(cx, &ray, b == 0 ? 0 : 1);
        if (!ret.full) {
            if (b == 0) L = vadd(L, vcw(T, bg));
            break;
        }
        if (medium) {                                   /* Beer's law over the segment inside */
            v3 sig = mv(MAT(s, medium)->absorption_coeff);
            float bd = vnorm(vsub(ret.point, ray.origin));
            T = vcw(T, V(f_exp(-sig.x * bd), f_exp(-sig.y * bd), f_exp(-sig.z * bd)));
        }
        const Emit* E;
        if (is_emitter(s, &ret, &E)) {
            if (b == 0 || !(flags & RTG_PT_NEE) || spec) L = vadd(L, vcw(T, E->Le));
            break;
        }
        if (b == 0 && ret.dm == RTG_DECAL_REPLACE_ALL) { L = vadd(L, vcw(T, ret.textureColor)); break; }
        const rtg_material_desc* m = MAT(s, ret.matIndex);
        /* dielectric geometry (Scene::DielectricRefraction Scene.cpp:57-118) */
        int entering = 1, isTir = 0;
        float F = 0.0f;
        v3 tdir = V(0, 0, 0), torg = V(0, 0, 0);
        if (m->type == RTG_MAT_DIELECTRIC) {
            float dp = vdot(ray.direction, ret.normal);
            float nt = m->refraction_index;
            float snell, n_t, n_i;
            v3 normal;
            if (dp < 0) { snell = 1.0f / nt; normal = ret.normal; n_t = nt; n_i = 1; entering = 1; }
            else { snell = nt; normal = vneg(ret.normal); n_t = 1; n_i = nt; entering = 0; }
            float cosTheta = -vdot(ray.direction, normal);
            v3 leftPart = vmul(vadd(ray.direction, vmul(normal, cosTheta)), snell);
            float srp = (float)(1 - pow((double)snell, 2) * (1 - pow((double)cosTheta, 2)));
            isTir = srp < 0;
            srp = sqrtf(srp);
            tdir = vnormalized(vsub(leftPart, vmul(normal, srp)));
            torg = vsub(ret.point, vmul(normal, s->shadowEps));
            float cos_t = -vdot(tdir, normal);
            float cos_i = -vdot(ray.direction, normal);
            float rPar = (n_t * cos_i - n_i * cos_t) / (n_t * cos_i + n_i * cos_t);
            float rPer = (n_i * cos_i - n_t * cos_t) / (n_i * cos_i + n_t * cos_t);
            F = (float)(0.5f * (pow((double)rPar, 2) + pow((double)rPer, 2)));
        }
        if (entering) {
            v3 v = basic_shading(cx, &ray, &ret, m, path);
            if (flags & RTG_PT_NEE)
                for (int k = 0; k < s->nemit; k++) v = vadd(v, emitter_shading(cx, k, &ray, &ret, m, path));
            L = vadd(L, vcw(T, v));
        }
        int cont = (flags & RTG_PT_RUSSIAN_ROULETTE) ? (b + 1 < RTG_PT_MAX_BOUNCES) : (depth > 0);
        if (!cont) break;
        float xi[4];
        rng4(cx->rng.seed, cx->rng.pixel, cx->rng.sample, path, RNG_PT_BOUNCE, 0, 0, xi);
        v3 w = V(1, 1, 1);
        Ray next;
        int nspec = 1, nmedium = medium;
        if (m->type == RTG_MAT_NORMAL) {
            v3 n = ret.normal, u = ortho_u(n), bt = vcross(n, u);
            float phi = (float)(2 * PI_D) * xi[0];
            float cosT = (flags & RTG_PT_IMPORTANCE) ? sqrtf(1.0f - xi[1]) : xi[1];
            float sinT = sqrtf(fmax0(1.0f - cosT * cosT));
            v3 wi = vnormalized(vadd(vadd(vmul(u, sinT * f_cos(phi)), vmul(n, cosT)), vmul(bt, sinT * f_sin(phi))));
            v3 fc = surface_response(V(1, 1, 1), vneg(ray.direction), wi, &ret, m);
            if (flags & RTG_PT_IMPORTANCE) w = cosT > 0.0f ? vmul(fc, (float)PI_D / cosT) : V(0, 0, 0);
            else w = vmul(fc, (float)(2 * PI_D));
            next = R(vadd(ret.point, vmul(n, s->shadowEps)), wi, ray.time);
            nspec = 0;
        } else if (m->type == RTG_MAT_DIELECTRIC && !isTir && !(xi[3] < F)) {
            next = R(torg, tdir, ray.time);
            nmedium = entering ? ret.matIndex : 0;
        } else {
            /* mirror / conductor / dielectric reflection: Scene::MirrorReflectance Scene.cpp:32-55 */
            v3 wo = vneg(ray.direction);
            float n_wo = vdot(ret.normal, wo);
            v3 wr = vadd(vneg(wo), vmul(vmul(ret.normal, 2), n_wo));
            wr = vdivs(wr, vnorm(wr));
            if (m->is_rough) {
                v3 u = ortho_u(wr), v = vcross(wr, u);
                float xr[4];
                rng4(cx->rng.seed, cx->rng.pixel, cx->rng.sample, path, RNG_ROUGH, 0, 0, xr);
                float uChi = xr[0] - 0.5f, vChi = xr[1] - 0.5f;
                wr = vnormalized(vadd(wr, vmul(vadd(vmul(u, uChi), vmul(v, vChi)), m->roughness)));
            }
            next = R(vadd(ret.point, vmul(ret.normal, s->shadowEps)), wr, ray.time);
            if (m->type == RTG_MAT_MIRROR) w = mv(m->mirror);
            else if (m->type == RTG_MAT_CONDUCTOR)
                w = vmul(mv(m->mirror), conductor_fresnel(m->refraction_index, m->absorption_index, ray.direction, ret.normal));
        }
        if (visnan(next.origin) || visnan(next.direction)) break;
        if (flags & RTG_PT_RUSSIAN_ROULETTE) {
            float qc = fabsf(vdot(ret.normal, next.direction));
            if (!(xi[2] < qc)) break;
            w = vdivs(w, qc);
        }
        T = vcw(T, w);
        if (T.x == 0.0f && T.y == 0.0f && T.z == 0.0f) break;
        ray = next; spec = nspec; medium = nmedium; depth--;
    }
    return L;
}

/* ------------------------------------------------------------------ camera (src/Camera.cpp) */
typedef struct {
    v3 pos, gaze, up, right;
    float l, r, b, t, dist;
    int nx, ny;
    float nxDA, nyDA, pw, ph, sw, sh;
    int sampleCount, total;
    int dof; float focus, aperture;
} Cam;

static void cam_init(Cam* c, const rtg_camera_desc* d) {          /* Camera::Camera Camera.cpp:7-61 */
    int i = 1;
    c->sampleCount = 1;
    while (i < 1000) { if (i * i >= d->num_samples) { c->sampleCount = i; break; } i++; }
    v3 gz = mv(d->gaze), up = mv(d->up);
    c->gaze = vnormalized(gz);
    v3 w = d->left_handed ? vnormalized(gz) : vnormalized(vneg(gz));
    c->right = vnormalized(vcross(up, w));
    c->up = vcross(w, c->right);
    c->pos = mv(d->position);
    c->l = d->left; c->r = d->right; c->b = d->bottom; c->t = d->top; c->dist = d->near_distance;
    c->nx = d->nx; c->ny = d->ny;
    c->nxDA = 1.0f / (float)d->nx;
    c->nyDA = 1.0f / (float)d->ny;
    c->pw = (c->r - c->l) * c->nxDA;
    c->ph = (c->t - c->b) * c->nyDA;
    c->sw = c->pw / (float)c->sampleCount;
    c->sh = c->ph / (float)c->sampleCount;
    c->total = d->num_samples;
    c->dof = d->is_dof; c->focus = d->focus_distance; c->aperture = d->aperture_size;
}
static Ray cam_primary(const Cam* c, int col, int row) {          /* getPrimaryRay Camera.cpp:63-72 */
    float u = c->l + ((c->r - c->l) * (col + 0.5f)) * c->nxDA;
    float v = c->t - ((c->t - c->b) * (row + 0.5f)) * c->nyDA;
    v3 m = vadd(c->pos, vmul(c->gaze, c->dist));
    m = vadd(m, vmul(c->right, u));
    m = vadd(m, vmul(c->up, v));
    v3 d = vsub(m, c->pos);
    return R(c->pos, vdivs(d, vnorm(d)), 0);
}
static v3 cam_lb(const Cam* c, int row, int col) {                /* PixelLBCorner Camera.cpp:84-92 */
    float u = c->l + (float)col * c->pw;
    float v = c->t - (float)(row + 1) * c->ph;
    v3 m = vadd(c->pos, vmul(c->gaze, c->dist));
    m = vadd(m, vmul(c->right, u));
    m = vadd(m, vmul(c->up, v));
    return m;
}
static Ray cam_sample(const Cam* c, v3 lb, int si, const float xi[4]) {   /* getSampleRay Camera.cpp:94-113 */
    int i = si % c->sampleCount, j = si / c->sampleCount;
    v3 m = lb;
    m = vadd(m, vmul(c->right, ((float)i + xi[0]) * c->sw));
    m = vadd(m, vmul(c->up, ((float)j + xi[1]) * c->sh));
    v3 d = vsub(m, c->pos);
    Ray ray = R(c->pos, vdivs(d, vnorm(d)), 0);
    if (c->dof) {                                                   /* AddDepthOfField Camera.cpp:119-139 */
        float xa = xi[2] - 0.5f, xb = xi[3] - 0.5f;
        v3 q = c->pos;
        q = vadd(q, vmul(c->right, c->aperture * xa));
        q = vadd(q, vmul(c->up, c->aperture * xb));
        v3 dir = vnormalized(vsub(m, c->pos));
        float tfd = c->focus / vdot(dir, c->gaze);
        v3 p = ray_point(&ray, tfd);
        return R(q, vnormalized(vsub(p, q)), 0);
    }
    ray.time = xi[2];
    return ray;
}

/* ------------------------------------------------------------------ scene construction */
static mat4 compose(const rtg_scene_desc* d, int first, int count) {   /* Helper.cpp:146-183 */
    mat4 M = m_identity();
    for (int j = count - 1; j >= 0; j--) {
        const rtg_xform_ref* x = &d->xform_refs[first + j];
        int k = x->index - 1;
        if (x->type == RTG_XF_TRANSLATION)
            M = m_translate(&M, V(d->translations[3 * k], d->translations[3 * k + 1], d->translations[3 * k + 2]));
        else if (x->type == RTG_XF_SCALING)
            M = m_scale(&M, V(d->scalings[3 * k], d->scalings[3 * k + 1], d->scalings[3 * k + 2]));
        else if (x->type == RTG_XF_ROTATION) {
            const float* rr = d->rotations + 4 * k;
            float rad = rr[0] * (float)0.01745329251994329576923690768489;     /* glm::radians */
            M = m_rotate(&M, rad, V(rr[1], rr[2], rr[3]));
        } else if (x->type == RTG_XF_COMPOSITE) {
            memcpy(M.c, d->composites + 16 * k, sizeof(float) * 16);
        }
    }
    return M;
}

static void obj_free(Obj* o) { free(o->pface); free(o->pv); free(o->psmooth); free(o->nodes); }

void orc_scene_destroy(orc_scene* s) {
    if (!s) return;
    for (int i = 0; i < s->nobj; i++) obj_free(&s->objs[i]);
    free(s->objs); free(s->insts); free(s->vertices); free(s->vnormals); free(s->texcoords);
    free(s->mats);
    for (int i = 0; i < s->ntex; i++) free(s->texs[i].texels);
    free(s->texs); free(s->lights);
    free(s->emits); free(s->etris); free(s->ecdf);
    free(s);
}

int orc_scene_create(const rtg_scene_desc* d, orc_scene** out) {
    if (!d || !out) return RTG_ERR_INVALID;
    struct orc_scene* s = (struct orc_scene*)calloc(1, sizeof *s);
    s->maxDepth = d->max_recursion_depth;
    s->shadowEps = d->shadow_ray_eps;
    s->intEps = d->intersection_test_eps;
    s->background = mv(d->background);
    s->ambientLight = mv(d->ambient_light);
    s->bgTexture = d->background_texture;
    s->envLight = d->environment_light;
    s->nv = d->num_vertices;
    s->vertices = (v3*)malloc(sizeof(v3) * (s->nv ? s->nv : 1));
    for (int i = 0; i < s->nv; i++) s->vertices[i] = V(d->vertices[3 * i], d->vertices[3 * i + 1], d->vertices[3 * i + 2]);
    s->ntc = d->num_texcoords;
    s->texcoords = (v2*)malloc(sizeof(v2) * (s->ntc ? s->ntc : 1));
    for (int i = 0; i < s->ntc; i++) { s->texcoords[i].x = d->texcoords[2 * i]; s->texcoords[i].y = d->texcoords[2 * i + 1]; }
    s->nmat = d->num_materials;
    s->mats = (rtg_material_desc*)malloc(sizeof(rtg_material_desc) * (s->nmat ? s->nmat : 1));
    memcpy(s->mats, d->materials, sizeof(rtg_material_desc) * s->nmat);
    s->ntex = d->num_textures;
    s->texs = (Tex*)calloc(s->ntex ? s->ntex : 1, sizeof(Tex));
    for (int i = 0; i < s->ntex; i++) {
        const rtg_texture_desc* t = &d->textures[i];
        Tex* T = &s->texs[i];
        T->kind = t->kind; T->decal = t->decal; T->interp = t->interp; T->nc = t->noise_conv;
        T->normalizer = t->normalizer; T->noise_scale = t->noise_scale; T->bump = t->bump_factor;
        T->w = t->width; T->h = t->height;
        size_t n = (size_t)t->width * t->height * 3;
        T->texels = (float*)malloc(sizeof(float) * (n ? n : 3));
        if (n && t->texels) memcpy(T->texels, t->texels, sizeof(float) * n);
    }
    /* lights (constructors, src/Light.cpp) */
    s->nlight = d->num_lights;
    s->lights = (Lgt*)calloc(s->nlight ? s->nlight : 1, sizeof(Lgt));
    for (int i = 0; i < s->nlight; i++) {
        const rtg_light_desc* l = &d->lights[i];
        Lgt* L = &s->lights[i];
        L->type = l->type; L->pos = mv(l->position); L->inten = mv(l->intensity); L->tex = l->texture;
        L->size = l->size;
        if (l->type == RTG_LIGHT_DIRECTIONAL || l->type == RTG_LIGHT_SPOT) L->dir = vnormalized(mv(l->direction));
        if (l->type == RTG_LIGHT_SPOT) {                             /* SpotLight ctor Light.cpp:327-336 */
            L->coverage = (float)((double)(l->coverage_deg * 0.5f) * (PI_D / 180.0f));
            L->fall = (float)((double)(l->falloff_deg * 0.5f) * (PI_D / 180.0f));
        }
        if (l->type == RTG_LIGHT_AREA) {                             /* AreaLight ctor Light.cpp:442-455 */
            L->normal = vnormalized(mv(l->direction));
            L->u = ortho_u(L->normal);
            L->v = vcross(L->normal, L->u);
        }
    }
    /* objects */
    s->nobj = d->num_objects;
    s->objs = (Obj*)calloc(s->nobj ? s->nobj : 1, sizeof(Obj));
    for (int i = 0; i < s->nobj; i++) {
        const rtg_object_desc* od = &d->objects[i];
        Obj* o = &s->objs[i];
        o->type = od->type; o->id = od->id; o->matIndex = od->material;
        o->ntex = od->num_textures; o->tex[0] = od->textures[0]; o->tex[1] = od->textures[1];
        o->texOffset = (od->type == RTG_OBJ_MESH) ? od->texture_offset : 0;
        o->smooth = od->smooth;
        o->blur = mv(od->blur);
        o->R = od->radius;
        if (od->type == RTG_OBJ_MESH) {
            o->nprims = od->face_count;
            o->pv = (int*)malloc(sizeof(int) * 3 * (o->nprims ? o->nprims : 1));
            memcpy(o->pv, d->faces + 3 * od->face_first, sizeof(int) * 3 * o->nprims);
        } else {
            o->nprims = 1;
            o->pv = (int*)malloc(sizeof(int) * 3);
            if (od->type == RTG_OBJ_SPHERE) { o->pv[0] = od->center; o->pv[1] = o->pv[2] = 0; }
            else { o->pv[0] = od->v[0]; o->pv[1] = od->v[1]; o->pv[2] = od->v[2]; }
        }
        o->model = compose(d, od->xform_first, od->xform_count);
        o->inv = m_inverse(&o->model);
        o->invT = m_inverse_transpose(&o->model);
    }
    s->ninst = d->num_instances;
    s->insts = (Inst*)calloc(s->ninst ? s->ninst : 1, sizeof(Inst));
    for (int i = 0; i < s->ninst; i++) {
        const rtg_instance_desc* id = &d->instances[i];
        Inst* in = &s->insts[i];
        in->base = id->base_object; in->matIndex = id->material; in->reset = id->reset_transform;
        in->blur = mv(id->blur);
        in->model = compose(d, id->xform_first, id->xform_count);
        if (!in->reset) in->model = m_mul(&in->model, &s->objs[in->base].model);   /* Helper.cpp:216-218 */
        in->inv = m_inverse(&in->model);
        in->invT = m_inverse_transpose(&in->model);
    }
    /* hw7 object lights (no reference code): world-space emitter geometry,
       sampled at time 0 (motion blur of emitters is ignored by the light sampler) */
    {
        int ntri = 0;
        for (int i = 0; i < s->nobj; i++)
            if (d->objects[i].is_light) { s->nemit++; if (d->objects[i].type != RTG_OBJ_SPHERE) ntri += s->objs[i].nprims; }
        s->emits = (Emit*)calloc(s->nemit ? s->nemit : 1, sizeof(Emit));
        s->etris = (v3*)malloc(sizeof(v3) * 3 * (size_t)(ntri ? ntri : 1));
        s->ecdf = (float*)malloc(sizeof(float) * (size_t)(ntri ? ntri : 1));
        int e = 0, t = 0;
        for (int i = 0; i < s->nobj; i++) {
            const rtg_object_desc* od = &d->objects[i];
            if (!od->is_light) continue;
            Obj* o = &s->objs[i];
            Emit* E = &s->emits[e++];
            E->obj = i;
            E->Le = mv(od->radiance);
            E->sphere = od->type == RTG_OBJ_SPHERE;
            if (E->sphere) {
                E->center = m_xform(&o->model, s->vertices[od->center - 1], 1.0f);
                E->radius = od->radius * vnorm(V(o->model.c[0][0], o->model.c[0][1], o->model.c[0][2]));
                continue;
            }
            E->tri_first = t;
            E->tri_count = o->nprims;
            float acc = 0.0f;
            for (int k = 0; k < o->nprims; k++, t++) {      /* original (parse) face order */
                const int* vi = o->pv + 3 * k;
                v3 a = m_xform(&o->model, s->vertices[vi[0] - 1], 1.0f);
                v3 b = m_xform(&o->model, s->vertices[vi[1] - 1], 1.0f);
                v3 c = m_xform(&o->model, s->vertices[vi[2] - 1], 1.0f);
                s->etris[3 * t] = a; s->etris[3 * t + 1] = b; s->etris[3 * t + 2] = c;
                acc = acc + 0.5f * vnorm(vcross(vsub(b, a), vsub(c, a)));
                s->ecdf[t] = acc;
            }
            E->area = acc;
        }
    }
    /* smooth vertex normals, src/Scene.cpp:302-318, Shape.cpp:262-290 */
    s->vnormals = (v3*)calloc(s->nv ? s->nv : 1, sizeof(v3));
    for (int i = 0; i < s->nobj; i++) {
        Obj* o = &s->objs[i];
        int isTri = (o->type == RTG_OBJ_TRIANGLE), isMesh = (o->type == RTG_OBJ_MESH);
        if (!isTri && !(isMesh && o->smooth)) continue;
        for (int k = 0; k < o->nprims; k++) {
            const int* vi = o->pv + 3 * k;
            v3 a = s->vertices[vi[0] - 1], b = s->vertices[vi[1] - 1], c = s->vertices[vi[2] - 1];
            v3 n = vnormalized(vcross(vsub(c, b), vsub(a, b)));
            for (int q = 0; q < 3; q++) s->vnormals[vi[q] - 1] = vadd(s->vnormals[vi[q] - 1], n);
        }
    }
    for (int i = 0; i < s->nv; i++) s->vnormals[i] = vnormalized(s->vnormals[i]);
    /* BVH per object (Scene.cpp:320-323; BVH(Shape*) BVH.cpp:53-62) */
    for (int i = 0; i < s->nobj; i++) {
        Obj* o = &s->objs[i];
        int n = o->nprims;
        int* prims = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
        for (int k = 0; k < n; k++) prims[k] = k;
        /* centers/boxes are looked up through the original face index: keep pv in parse
           order while building, permute afterwards */
        Builder B = {s, o, prims, 0, 0};
        int* pvOrig = o->pv;
        o->root = construct(&B, 0, n, 0, 0);
        o->nnodes = B.nn;
        o->pface = prims;
        o->pv = (int*)malloc(sizeof(int) * 3 * (size_t)(n > 0 ? n : 1));
        o->psmooth = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
        for (int k = 0; k < n; k++) {
            memcpy(o->pv + 3 * k, pvOrig + 3 * prims[k], sizeof(int) * 3);
            o->psmooth[k] = (o->type == RTG_OBJ_TRIANGLE) ? 1 : (o->type == RTG_OBJ_MESH ? o->smooth : 0);
        }
        free(pvOrig);
    }
    *out = s;
    return RTG_OK;
}

/* ------------------------------------------------------------------ API */
int orc_render(orc_scene* s, const rtg_camera_desc* cd, uint64_t seed, int nthreads, int row_offset,
               int row_stride, int row_block, int row_begin, int row_end, float* rgb, int32_t* pobj,
               int32_t* pprim, float* pt) {
    if (!s || !cd || !rgb) return RTG_ERR_INVALID;
    Cam cam;
    cam_init(&cam, cd);
    int nx = cd->nx, ny = cd->ny;
    if (row_stride <= 0) row_stride = 1;
    if (row_block <= 0) row_block = 1;
    if (row_end <= 0 || row_end > ny) row_end = ny;
    if (row_begin < 0) row_begin = 0;
    uint64_t np = 0, nsec = 0, nsh = 0;
    uint64_t canon[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int pathT = cd->integrator == RTG_INTEGRATOR_PATH;
    if (pathT && pobj) for (int k = 0; k < nx * ny; k++) { pobj[k] = -1; pprim[k] = -1; pt[k] = 0; }
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : np, nsec, nsh)
    for (int y = row_begin; y < row_end; y++) {
        if ((y / row_block) % row_stride != row_offset % row_stride) continue;
        Ctx cx = {s, {seed, 0, 0}, 0, 0, 0, {0, 0, 0, 0, 0, 0, 0, 0}};
        for (int x = 0; x < nx; x++) {
            uint32_t pixel = (uint32_t)(y * nx + x);
            cx.rng.pixel = pixel;
            v3 color;
            if (cam.total > 1) {                          /* Scene::MultiSample Scene.cpp:386-411 */
                v3 lb = cam_lb(&cam, y, x);
                color = V(0, 0, 0);
                for (int i = 0; i < cam.total; i++) {
                    cx.rng.sample = (uint32_t)i;
                    float xi[4];
                    rng4(seed, pixel, (uint32_t)i, 1, RNG_CAMERA, 0, 0, xi);
                    Ray r = cam_sample(&cam, lb, i, xi);
                    if (pathT) {
                        color = vadd(color, pt_sample(&cx, r, cd->pt_flags, background(s, y, x, nx, ny, &r)));
                        continue;
                    }
                    RetVal nr = trace(&cx, &r, 0);
                    if (i == 0 && pobj) { pobj[pixel] = nr.full ? nr.obj : -1; pprim[pixel] = nr.full ? nr.prim : -1; pt[pixel] = nr.full ? nr.t : 0; }
                    if (nr.full) color = vadd(color, shading(&cx, &r, &nr));
                    else color = vadd(color, background(s, y, x, nx, ny, &r));
                }
                color = vdivs(color, (float)cam.total);
            } else {                                      /* Scene::SingleSample Scene.cpp:365-384 (row=x, col=y) */
                cx.rng.sample = 0;
                Ray r = cam_primary(&cam, x, y);
                if (pathT) {
                    color = pt_sample(&cx, r, cd->pt_flags, background(s, x, y, nx, ny, &r));
                    float* o = rgb + (size_t)pixel * 3;
                    o[0] = color.x; o[1] = color.y; o[2] = color.z;
                    continue;
                }
                RetVal nr = trace(&cx, &r, 0);
                if (pobj) { pobj[pixel] = nr.full ? nr.obj : -1; pprim[pixel] = nr.full ? nr.prim : -1; pt[pixel] = nr.full ? nr.t : 0; }
                if (nr.full) color = shading(&cx, &r, &nr);
                else color = background(s, x, y, nx, ny, &r);
            }
            float* o = rgb + (size_t)pixel * 3;
            o[0] = color.x; o[1] = color.y; o[2] = color.z;
        }
        np += cx.n_primary; nsec += cx.n_secondary; nsh += cx.n_shadow;
        if (s->canon_on) {
#pragma omp critical
            for (int k = 0; k < 8; k++) canon[k] += cx.canon[k];
        }
    }
    s->counts[0] = np; s->counts[1] = nsec; s->counts[2] = nsh;
    memcpy(s->canon, canon, sizeof canon);
    return RTG_OK;
}

void orc_canonical_counts(orc_scene* s, int enable, uint64_t out[8]) {
    if (out) memcpy(out, s->canon, sizeof s->canon);
    s->canon_on = enable;
}

void orc_last_ray_counts(const orc_scene* s, uint64_t counts[3]) {
    counts[0] = s->counts[0]; counts[1] = s->counts[1]; counts[2] = s->counts[2];
}

int orc_trace(orc_scene* s, const rtg_ray* rays, int n, rtg_hit* hits) {
    if (!s || (n && (!rays || !hits))) return RTG_ERR_INVALID;
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < n; i++) {
        Ray r = R(V(rays[i].origin[0], rays[i].origin[1], rays[i].origin[2]),
                  V(rays[i].direction[0], rays[i].direction[1], rays[i].direction[2]), rays[i].time);
        RetVal nr = find_intersection(s, &r);
        rtg_hit* h = &hits[i];
        memset(h, 0, sizeof *h);
        h->full = nr.full;
        h->object = nr.full ? nr.obj : -1;
        h->prim = nr.full ? nr.prim : -1;
        h->material = nr.full ? nr.matIndex : 0;
        h->t = nr.full ? nr.t : 0;
        h->point[0] = nr.point.x; h->point[1] = nr.point.y; h->point[2] = nr.point.z;
        h->normal[0] = nr.normal.x; h->normal[1] = nr.normal.y; h->normal[2] = nr.normal.z;
    }
    return RTG_OK;
}

int orc_object_bvh(const orc_scene* s, int object, int32_t* num_prims, int32_t* num_nodes, int32_t* perm,
                   int32_t* nodes, float* boxes) {
    if (!s || object < 0 || object >= s->nobj) return RTG_ERR_INVALID;
    const Obj* o = &s->objs[object];
    if (num_prims) *num_prims = o->nprims;
    if (num_nodes) *num_nodes = o->nnodes;
    if (perm) memcpy(perm, o->pface, sizeof(int32_t) * o->nprims);
    for (int k = 0; k < o->nnodes; k++) {
        const BNode* N = &o->nodes[k];
        if (nodes) { nodes[4 * k] = N->left; nodes[4 * k + 1] = N->right; nodes[4 * k + 2] = N->start; nodes[4 * k + 3] = N->end; }
        if (boxes) {
            boxes[6 * k] = N->mn.x; boxes[6 * k + 1] = N->mn.y; boxes[6 * k + 2] = N->mn.z;
            boxes[6 * k + 3] = N->mx.x; boxes[6 * k + 4] = N->mx.y; boxes[6 * k + 5] = N->mx.z;
        }
    }
    return RTG_OK;
}

int orc_object_matrices(const orc_scene* s, int top, float* inv16, float* invT16) {
    if (!s || top < 0 || top >= s->nobj + s->ninst) return RTG_ERR_INVALID;
    const mat4 *a, *b;
    if (top < s->nobj) { a = &s->objs[top].inv; b = &s->objs[top].invT; }
    else { a = &s->insts[top - s->nobj].inv; b = &s->insts[top - s->nobj].invT; }
    if (inv16) memcpy(inv16, a->c, 64);
    if (invT16) memcpy(invT16, b->c, 64);
    return RTG_OK;
}

int orc_vertex_normals(const orc_scene* s, float* normals) {
    if (!s || !normals) return RTG_ERR_INVALID;
    for (int i = 0; i < s->nv; i++) {
        normals[3 * i] = s->vnormals[i].x; normals[3 * i + 1] = s->vnormals[i].y; normals[3 * i + 2] = s->vnormals[i].z;
    }
    return RTG_OK;
}

/* ------------------------------------------------------------------ hw5 tone mapping
 * pages/Page5.md:47-53 describes a global operator; src/ has no code.  The Photographic TMO
 * of DESIGN.md §11 (Reinhard et al. 2002, global), restated plainly: luminance, log-average in
 * double (index order), scale, burn rank by sorting, Reinhard curve, saturation, gamma. */
static float tm_lum(const float* c) {
    float y = (0.2126f * c[0] + 0.7152f * c[1]) + 0.0722f * c[2];
    return (isfinite(y) && y > 0.0f) ? y : 0.0f;
}
static int cmp_f(const void* a, const void* b) {
    float x = *(const float*)a, y = *(const float*)b;
    return (x > y) - (x < y);
}
int orc_tonemap(const float* hdr, int nx, int ny, const rtg_tonemap_desc* tm, float* out) {
    if (!hdr || !out || !tm || nx < 1 || ny < 1) return RTG_ERR_INVALID;
    size_t n = (size_t)nx * ny;
    float* Y = (float*)malloc(sizeof(float) * n);
    float* L = (float*)malloc(sizeof(float) * n);
    double sum = 0.0;
    for (size_t i = 0; i < n; i++) { Y[i] = tm_lum(hdr + 3 * i); sum += log(1e-5 + (double)Y[i]); }
    double lw = exp(sum / (double)n);
    float k = (float)((double)tm->key / lw);
    for (size_t i = 0; i < n; i++) L[i] = k * Y[i];
    qsort(L, n, sizeof(float), cmp_f);
    size_t widx = n - 1;
    if (tm->burn_percent > 0.0f) {
        double f = 1.0 - (double)tm->burn_percent / 100.0;
        if (f < 0.0) f = 0.0;
        long long idx = (long long)floor((double)(n - 1) * f);
        widx = idx < 0 ? 0 : (idx > (long long)n - 1 ? n - 1 : (size_t)idx);
    }
    float white = L[widx];
    double ig = 1.0 / (double)tm->gamma;
    for (size_t i = 0; i < n; i++) {
        float y = Y[i], l = k * y;
        float ld = white > 0.0f ? (l * (1.0f + l / (white * white))) / (1.0f + l) : l / (1.0f + l);
        for (int c = 0; c < 3; c++) {
            float v = 0.0f;
            if (y > 0.0f) {
                float ch = hdr[3 * i + c] > 0.0f ? hdr[3 * i + c] : 0.0f;
                v = ld * (float)pow((double)(ch / y), (double)tm->saturation);
            }
            v = v > 0.0f ? (v < 1.0f ? v : 1.0f) : 0.0f;
            out[3 * i + c] = 255.0f * (float)pow((double)v, ig);
        }
    }
    free(Y); free(L);
    return RTG_OK;
}

