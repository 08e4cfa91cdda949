// Layout probe for the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 operands), round-4
// groundwork for the panel's lo product.  Hypothesis H: lane l holds A[row l & 15]
// [k = 32 (l >> 4) + i] in byte i of its 8 registers and B[k = 32 (l >> 4) + i][col l & 15], i.e. the
// K-group of a lane pairs with the same K-group of the other operand (so any K permutation applied to
// both operands alike leaves C unchanged); C as every 16x16 MFMA (col = l & 15, row = 4 (l >> 4) + r).
// Also: the scale operands (E8M0, 127 = 1.0) and the conversion v_cvt_scalef32_pk_fp8_f32.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_f8_probe.hip -o tools/_mfma_f8_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

__global__ void k_mfma(const unsigned char* A, const unsigned char* B, float* C, int sa, int sb) {
    const int l = threadIdx.x;
    i32x8 a, b;
    memcpy(&a, A + 32 * l, 32);
    memcpy(&b, B + 32 * l, 32);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, sb);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}
// per-lane scale operands: lane l passes sa[l] / sb[l] (VGPRs) -- does lane l's scale apply to its own
// row (A) / column (B) K-group, i.e. C[r][c] = sum_g 2^(sa[r + 16 g] + sb[c + 16 g] - 254) sum_i a b ?
__global__ void k_mfma_lane(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* C) {
    const int l = threadIdx.x;
    i32x8 a, b;
    memcpy(&a, A + 32 * l, 32);
    memcpy(&b, B + 32 * l, 32);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa[l], 0, sb[l]);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__global__ void k_cvt_bf16(const float* x, float scale, unsigned* y) {
    const int l = threadIdx.x;
    s16x2 old = {0, 0};
    bf16x2 v = {(__bf16)x[2 * l], (__bf16)x[2 * l + 1]};
    s16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, v, scale, false);
    unsigned u;
    memcpy(&u, &r, 4);
    y[l] = u;
}
__global__ void k_cvt(const float* x, float scale, unsigned* y) {
    const int l = threadIdx.x;
    s16x2 old = {0, 0};
    s16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(old, x[2 * l], x[2 * l + 1], scale, false);
    unsigned u;
    memcpy(&u, &r, 4);
    y[l] = u;
}

static unsigned char enc(int v) {   // small integers in OCP e4m3fn (bias 7)
    if (v == 0) return 0;
    unsigned char s = v < 0 ? 0x80 : 0;
    int a = abs(v), e = 0;
    while ((a >> e) > 1) ++e;                 // a = 2^e * (1 + m/8)
    const int m = ((a << 3) >> e) - 8;        // exact for the values used (|v| <= 4)
    return s | (unsigned char)(((e + 7) << 3) | m);
}
static float dec(unsigned char b) {
    const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
    const float v = e ? ldexpf(1.f + m / 8.f, e - 7) : ldexpf(m / 8.f, -6);
    return s ? -v : v;
}

int main() {
    unsigned char hA[64 * 32], hB[64 * 32];
    int vA[16][128], vB[128][16];
    srand(7);
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 32; ++i) {
            const int a = rand() % 7 - 3, b = rand() % 7 - 3;
            vA[l & 15][32 * (l >> 4) + i] = a;
            vB[32 * (l >> 4) + i][l & 15] = b;
            hA[32 * l + i] = enc(a);
            hB[32 * l + i] = enc(b);
        }
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 32; ++i)
            if (dec(hA[32 * l + i]) != (float)vA[l & 15][32 * (l >> 4) + i]) { printf("encode error\n"); return 1; }
    unsigned char *dA, *dB;
    float* dC;
    (void)hipMalloc(&dA, sizeof hA);
    (void)hipMalloc(&dB, sizeof hB);
    (void)hipMalloc(&dC, 256 * 4);
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    const int sc[3][2] = {{127, 127}, {128, 127}, {127, 125}};
    for (auto& s : sc) {
        hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dC, s[0], s[1]);
        float hC[256];
        (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
        const double f = ldexp(1.0, (s[0] - 127) + (s[1] - 127));
        int bad = 0;
        for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
                double ref = 0;
                for (int k = 0; k < 128; ++k) ref += vA[r][k] * vB[k][c];
                if (hC[r * 16 + c] != (float)(ref * f)) ++bad;
            }
        printf("scale_a %d scale_b %d: hypothesis H %s (%d of 256 outputs differ; C[0][0] %g)\n", s[0], s[1],
               bad ? "REJECTED" : "holds", bad, hC[0]);
    }
    {   // per-lane scales
        int hsa[64], hsb[64];
        for (int l = 0; l < 64; ++l) { hsa[l] = 127 + (l % 3) - 1; hsb[l] = 127 + ((l * 7) % 5) - 2; }
        int *dsa, *dsb;
        (void)hipMalloc(&dsa, sizeof hsa);
        (void)hipMalloc(&dsb, sizeof hsb);
        (void)hipMemcpy(dsa, hsa, sizeof hsa, hipMemcpyHostToDevice);
        (void)hipMemcpy(dsb, hsb, sizeof hsb, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_mfma_lane, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
        float hC[256];
        (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
                double ref = 0;
                for (int g = 0; g < 4; ++g) {
                    double part = 0;
                    for (int i = 0; i < 32; ++i) part += vA[r][32 * g + i] * vB[32 * g + i][c];
                    ref += part * ldexp(1.0, hsa[r + 16 * g] - 127 + hsb[c + 16 * g] - 127);
                }
                if (hC[r * 16 + c] != (float)ref) ++bad;
            }
        printf("per-lane scales (lane l: row/col l & 15, K-group l >> 4): %s (%d of 256 differ)\n",
               bad ? "REJECTED" : "holds", bad);
    }
    float hx[128];
    for (int i = 0; i < 128; ++i) hx[i] = (i % 2 ? -1.f : 1.f) * (float)(1 + (i % 5));
    float* dx;
    unsigned* dy;
    (void)hipMalloc(&dx, sizeof hx);
    (void)hipMalloc(&dy, 64 * 4);
    (void)hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
    for (float scale : {1.f, 2.f, 0.5f}) {
        hipLaunchKernelGGL(k_cvt, dim3(1), dim3(64), 0, 0, dx, scale, dy);
        unsigned hy[64];
        (void)hipMemcpy(hy, dy, sizeof hy, hipMemcpyDeviceToHost);
        printf("cvt_scalef32_pk_fp8_f32 scale %g: x = %g, %g -> bytes %02x %02x (decoded %g, %g)\n", scale, hx[0], hx[1],
               hy[0] & 255, (hy[0] >> 8) & 255, dec(hy[0] & 255), dec((hy[0] >> 8) & 255));
    }
    {   // bf16 input: exact grid values round-trip; overflow (x / scale > 448) saturates or not
        float hb[128];
        for (int i = 0; i < 128; ++i) hb[i] = 0.f;
        hb[0] = 0.3125f; hb[1] = -448.f; hb[2] = 1000.f; hb[3] = -1000.f; hb[4] = 0.001953125f; hb[5] = 0.0009765625f;
        hb[6] = 3.0f * 0.0078125f; hb[7] = 1.0f / 1024.0f * 3.0f;
        (void)hipMemcpy(dx, hb, sizeof hb, hipMemcpyHostToDevice);
        for (float scale : {1.f, 0.25f}) {
            hipLaunchKernelGGL(k_cvt_bf16, dim3(1), dim3(64), 0, 0, dx, scale, dy);
            unsigned hy[64];
            (void)hipMemcpy(hy, dy, sizeof hy, hipMemcpyDeviceToHost);
            printf("cvt_scalef32_pk_fp8_bf16 scale %g:", scale);
            for (int i = 0; i < 8; ++i) {
                const unsigned char bb = (hy[i / 2] >> (8 * (i % 2))) & 255;
                printf(" %g->%02x(%g)", hb[i], bb, dec(bb) * scale);
            }
            printf("\n");
        }
    }
    return 0;
}
