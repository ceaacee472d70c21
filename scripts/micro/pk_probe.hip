// Hardware check of the packed-fp32 instruction forms the compiler emits for rtg_device.hip when
// packed ops are allowed (find why the candidate gate went wrong with them).  The forms
// are the operand / modifier patterns of the v_pk_* census of that build's ISA; each
// runs on 2^16 input pairs mixing normal, denormal, zero, infinite and NaN operands and is compared
// bitwise with the same arithmetic one float at a time (v_mul_f32 / v_add_f32, denormals on).
//   hipcc --offload-arch=gfx950 -O2 -fno-gpu-flush-denormals-to-zero scripts/micro/pk_probe.hip -o scripts/micro/pk_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kForms = 12;
__device__ __noinline__ float smul(float a, float b) { return a * b; }
__device__ __noinline__ float sadd(float a, float b) { return a + b; }

__global__ void k_probe(const f2* a, const f2* b, f2 s, f2* got, f2* want, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f2 x = a[i], y = b[i];
    f2 r[kForms], w[kForms];
    asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(r[0]) : "v"(x), "v"(y));
    w[0] = f2{smul(x.x, y.x), smul(x.y, y.y)};
    asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r[1]) : "v"(x), "v"(y));
    w[1] = f2{sadd(x.x, -y.x), sadd(x.y, -y.y)};
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r[2]) : "v"(x), "v"(y));
    w[2] = f2{smul(x.x, y.x), smul(x.y, y.x)};
    asm volatile("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(r[3]) : "v"(x), "v"(y));
    w[3] = f2{x.y, y.x};
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r[4]) : "v"(x), "v"(y));
    w[4] = f2{smul(x.y, y.x), smul(x.x, y.y)};
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r[5]) : "v"(x), "s"(s));
    w[5] = f2{smul(x.x, s.x), smul(x.y, s.x)};
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]" : "=v"(r[6]) : "s"(s), "v"(x));
    w[6] = f2{smul(s.x, x.y), smul(s.y, x.y)};
    asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r[7]) : "s"(s), "v"(x));
    w[7] = f2{sadd(s.x, -x.x), sadd(s.y, -x.y)};
    asm volatile("v_pk_mul_f32 %0, %1, 0 op_sel_hi:[1,0]" : "=v"(r[8]) : "v"(x));
    w[8] = f2{smul(x.x, 0.0f), smul(x.y, 0.0f)};
    asm volatile("v_pk_add_f32 %0, %1, 0 neg_lo:[1,1] neg_hi:[1,1]" : "=v"(r[9]) : "v"(x));
    w[9] = f2{sadd(-x.x, -0.0f), sadd(-x.y, -0.0f)};
    asm volatile("v_pk_add_f32 %0, %1, -0.5 op_sel_hi:[1,0]" : "=v"(r[10]) : "v"(x));
    w[10] = f2{sadd(x.x, -0.5f), sadd(x.y, -0.5f)};
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r[11]) : "v"(x), "s"(s));
    w[11] = f2{smul(x.x, -s.x), smul(x.y, -s.x)};
    for (int f = 0; f < kForms; f++) {
        got[(size_t)f * n + i] = r[f];
        want[(size_t)f * n + i] = w[f];
    }
}

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint32_t rng = 12345;
static uint32_t next() { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng; }
static float pick() {
    const uint32_t k = next() % 16;
    uint32_t u = next();
    float f;
    if (k == 0) u &= 0x807FFFFFu;                      // denormal / zero
    else if (k == 1) u = (u & 0x80000000u) | 0x7F800000u;   // +-inf
    else if (k == 2) u = 0x7FC00000u | (u & 0x3FFFFFu);       // NaN
    else if (k == 3) u &= 0x80000000u;                          // +-0
    else if (k < 8) u = (u & 0x807FFFFFu) | ((1u + next() % 40) << 23);   // tiny normals (products denormal)
    else u = (u & 0x807FFFFFu) | ((100u + next() % 56) << 23);          // moderate
    memcpy(&f, &u, 4);
    return f;
}

int main() {
    const int n = 1 << 16;
    f2 *ha = new f2[n], *hb = new f2[n], *hg = new f2[(size_t)kForms * n], *hw = new f2[(size_t)kForms * n];
    for (int i = 0; i < n; i++) { ha[i] = f2{pick(), pick()}; hb[i] = f2{pick(), pick()}; }
    f2 *da, *db, *dg, *dw;
    if (hipMalloc(&da, n * sizeof(f2)) || hipMalloc(&db, n * sizeof(f2)) || hipMalloc(&dg, (size_t)kForms * n * sizeof(f2)) ||
        hipMalloc(&dw, (size_t)kForms * n * sizeof(f2))) { printf("alloc failed\n"); return 2; }
    if (hipMemcpy(da, ha, n * sizeof(f2), hipMemcpyHostToDevice) || hipMemcpy(db, hb, n * sizeof(f2), hipMemcpyHostToDevice)) return 2;
    int bad_total = 0;
    const float svals[][2] = {{1.5f, -3.25f}, {1e-30f, 7e-39f}, {-0.0f, 2.0f}, {1e30f, -1e-20f}};
    for (const auto& sv : svals) {
        k_probe<<<n / 256, 256>>>(da, db, f2{sv[0], sv[1]}, dg, dw, n);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
        if (hipMemcpy(hg, dg, (size_t)kForms * n * sizeof(f2), hipMemcpyDeviceToHost) ||
            hipMemcpy(hw, dw, (size_t)kForms * n * sizeof(f2), hipMemcpyDeviceToHost)) return 2;
        for (int f = 0; f < kForms; f++) {
            int bad = 0, first = -1;
            for (int i = 0; i < n; i++) {
                const f2 g = hg[(size_t)f * n + i], w = hw[(size_t)f * n + i];
                const uint32_t g0 = bits(g.x), g1 = bits(g.y), w0 = bits(w.x), w1 = bits(w.y);
                const bool gn0 = (g0 & 0x7FFFFFFFu) > 0x7F800000u, gn1 = (g1 & 0x7FFFFFFFu) > 0x7F800000u;
                const bool wn0 = (w0 & 0x7FFFFFFFu) > 0x7F800000u, wn1 = (w1 & 0x7FFFFFFFu) > 0x7F800000u;
                const bool ok = (gn0 ? wn0 : g0 == w0) && (gn1 ? wn1 : g1 == w1);   // any NaN matches any NaN
                if (!ok) { bad++; if (first < 0) first = i; }
            }
            if (bad) {
                const f2 g = hg[(size_t)f * n + first], w = hw[(size_t)f * n + first];
                printf("s=(%g,%g) form %d: %d of %d differ; e.g. a=(%a,%a) b=(%a,%a) got=(%a,%a) want=(%a,%a)\n", sv[0], sv[1],
                       f, bad, n, ha[first].x, ha[first].y, hb[first].x, hb[first].y, g.x, g.y, w.x, w.y);
            }
            bad_total += bad;
        }
    }
    printf("pk_probe: %d forms x 4 scalar operands x %d pairs, %d mismatches\n", kForms, n, bad_total);
    return bad_total ? 1 : 0;
}
