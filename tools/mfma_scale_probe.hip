// Where do the per-lane scale operands of v_mfma_scale_f32_16x16x128_f8f6f4 apply?  (round 4; the
// hypothesis "lane l's scale multiplies its own row / column K-group" was rejected by
// tools/mfma_f8_probe.hip.)  A[r][32 g] = 1, B[32 g][c] = 2^g, everything else 0, so with unit
// scales C[r][c] = 15 and a doubled (row r, K-group g) block adds 2^g: the set of doubled blocks of
// row r is the bit pattern of C[r][c] - 15.  For each lane L the A scale of lane L alone is doubled
// (all four bytes), then the B scale; then every lane's scale word gets one byte doubled, per byte
// and per op_sel, to see which byte the hardware reads.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/_mfma_scale_probe tools/mfma_scale_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int OPA, int OPB>
__global__ void k_mfma(const unsigned char* A, const unsigned char* B, const unsigned* sa, const unsigned* sb,
                       float* C) {
    const int l = threadIdx.x;
    i32x8 a, b;
    memcpy(&a, A + 32 * l, 32);
    memcpy(&b, B + 32 * l, 32);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, OPA, (int)sa[l], OPB, (int)sb[l]);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

// fp6 (e2m3): 32 bf16 values per lane (lane l: A[row l & 15][k = 32 (l >> 4) + i], B[k][col l & 15] as
// for e4m3) packed by v_cvt_scalef32_pk32_fp6_bf16 into 6 dwords, MFMA format 2 on both sides
typedef __bf16 bf16x32 __attribute__((ext_vector_type(32)));
typedef int i32x6 __attribute__((ext_vector_type(6)));
__global__ void k_mfma6(const float* A, const float* B, float* C) {
    const int l = threadIdx.x;
    bf16x32 av, bv;
    for (int i = 0; i < 32; ++i) {
        av[i] = (__bf16)A[32 * l + i];
        bv[i] = (__bf16)B[32 * l + i];
    }
    const i32x6 a6 = __builtin_amdgcn_cvt_scalef32_pk32_fp6_bf16(av, 1.0f);
    const i32x6 b6 = __builtin_amdgcn_cvt_scalef32_pk32_fp6_bf16(bv, 1.0f);
    i32x8 a = {a6[0], a6[1], a6[2], a6[3], a6[4], a6[5], 0, 0};
    i32x8 b = {b6[0], b6[1], b6[2], b6[3], b6[4], b6[5], 0, 0};
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 2, 2, 0, 127, 0, 127);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

int main() {
    unsigned char hA[64 * 32] = {}, hB[64 * 32] = {};
    const unsigned char pow2[4] = {0x38, 0x40, 0x48, 0x50};   // e4m3fn 1, 2, 4, 8
    for (int l = 0; l < 64; ++l) {
        hA[32 * l] = 0x38;              // A[row l & 15][32 (l >> 4)] = 1
        hB[32 * l] = pow2[l >> 4];      // B[32 (l >> 4)][col l & 15] = 2^(l >> 4)
    }
    unsigned char *dA, *dB;
    unsigned *dsa, *dsb;
    float* dC;
    (void)hipMalloc(&dA, sizeof hA);
    (void)hipMalloc(&dB, sizeof hB);
    (void)hipMalloc(&dsa, 256);
    (void)hipMalloc(&dsb, 256);
    (void)hipMalloc(&dC, 1024);
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    unsigned one[64], var[64];
    for (int l = 0; l < 64; ++l) one[l] = 0x7f7f7f7fu;
    float hC[256];
    auto run = [&](const unsigned* sa, const unsigned* sb, int op) {
        (void)hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
        (void)hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
        switch (op) {
            case 0: hipLaunchKernelGGL((k_mfma<0, 0>), dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC); break;
            case 1: hipLaunchKernelGGL((k_mfma<1, 1>), dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC); break;
            case 2: hipLaunchKernelGGL((k_mfma<2, 2>), dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC); break;
            default: hipLaunchKernelGGL((k_mfma<3, 3>), dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC); break;
        }
        (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    };
    run(one, one, 0);
    printf("unit scales: C[0][0] %g C[15][15] %g (expect 15)\n", hC[0], hC[255]);
    // per lane, A side: which (row, group) blocks double
    for (int side = 0; side < 2; ++side) {
        printf("%s scale of lane L doubled -> doubled blocks as row:groupmask (C[r][c] - 15, over all r and c):\n",
               side ? "B" : "A");
        for (int L = 0; L < 64; ++L) {
            for (int l = 0; l < 64; ++l) var[l] = l == L ? 0x80808080u : 0x7f7f7f7fu;
            run(side ? one : var, side ? var : one, 0);
            printf(" L%-2d:", L);
            int any = 0;
            for (int r = 0; r < 16; ++r)
                for (int c = 0; c < 16; ++c) {
                    const int d = (int)(hC[r * 16 + c] - 15.0f);
                    if (d) { printf(" (%d,%d):%x", r, c, d); ++any; if (any > 6) { printf(" ..."); r = 16; break; } }
                }
            printf("\n");
        }
    }
    // byte selection: every lane's word has byte q = 128 (x2), the others 127
    for (int op = 0; op < 4; ++op)
        for (int q = 0; q < 4; ++q) {
            for (int l = 0; l < 64; ++l) var[l] = 0x7f7f7f7fu ^ ((0x7fu ^ 0x80u) << (8 * q));
            run(var, one, op);
            printf("op_sel %d, A word byte %d doubled: C[0][0] %g C[5][9] %g\n", op, q, hC[0], hC[5 * 16 + 9]);
        }
    {   // fp6 layout: exact small integers (e2m3 holds -7.5 .. 7.5, integers to 7 exactly)
        float hA6[64 * 32], hB6[64 * 32];
        int vA[16][128], vB[128][16];
        unsigned st = 12345;
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 32; ++i) {
                st = st * 1103515245u + 12345u;
                const int a = (int)((st >> 16) % 7) - 3;
                st = st * 1103515245u + 12345u;
                const int bb = (int)((st >> 16) % 7) - 3;
                vA[l & 15][32 * (l >> 4) + i] = a;
                vB[32 * (l >> 4) + i][l & 15] = bb;
                hA6[32 * l + i] = (float)a;
                hB6[32 * l + i] = (float)bb;
            }
        float *d6a, *d6b;
        (void)hipMalloc(&d6a, sizeof hA6);
        (void)hipMalloc(&d6b, sizeof hB6);
        (void)hipMemcpy(d6a, hA6, sizeof hA6, hipMemcpyHostToDevice);
        (void)hipMemcpy(d6b, hB6, sizeof hB6, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_mfma6, dim3(1), dim3(64), 0, 0, d6a, d6b, dC);
        (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
                double ref = 0;
                for (int k = 0; k < 128; ++k) ref += vA[r][k] * vB[k][c];
                if (hC[r * 16 + c] != (float)ref) ++bad;
            }
        printf("fp6 e2m3 via cvt_scalef32_pk32_fp6_bf16, same-lane K pairing: %s (%d of 256 differ; C[0][0] %g)\n",
               bad ? "REJECTED" : "holds", bad, hC[0]);
    }
    return 0;
}
