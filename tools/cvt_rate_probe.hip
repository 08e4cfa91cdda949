// Issue cost of the conversions and MFMAs a lo-product redesign would use (round 4): per-SIMD
// cycles of v_cvt_scalef32_pk_fp8_bf16 (2 values), v_cvt_scalef32_pk32_fp6_bf16 (32 values),
// v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 / e2m3 operands, v_mfma_scale_f32_32x32x64_f8f6f4,
// and v_mfma_f32_16x16x32_bf16 / 32x32x16_bf16, each in a loop of independent instructions on
// 256 blocks x 8 waves (2 waves per SIMD, the panel passes' occupancy); and mixes of them.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_cvt_rate_probe tools/cvt_rate_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x32 __attribute__((ext_vector_type(32)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef int i32x6 __attribute__((ext_vector_type(6)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int ITERS = 4096;

template <int V>
__global__ __launch_bounds__(512) void k(const float* in, float* out, float sc) {
    const int l = threadIdx.x;
    bf16x32 x;
    for (int i = 0; i < 32; ++i) x[i] = (__bf16)in[(l + i) & 1023];
    bf16x8 xa = {x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]};
    i32x8 acc8 = {0, 0, 0, 0, 0, 0, 0, 0};
    f32x4 c[4] = {};
    f32x16 d[2] = {};
    i32x8 op = {l, l + 1, l + 2, l + 3, l + 4, l + 5, 0, 0};
    bf16x8 xs[4] = {xa, xa, xa, xa};
    for (int it = 0; it < ITERS; ++it) {
        if constexpr (V == 9 || V == 10 || V == 11 || V == 12) {
            // throughput forms: the inputs are "rewritten" by empty asm each iteration (no instruction,
            // no dependency chain) and every result is consumed by empty asm
#pragma unroll
            for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(xs[q]));
        }
        if constexpr (V == 9 || V == 11) {   // 16 x cvt_pk_fp8 (32 values)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
                    s16x2 r = {0, 0};
                    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, bf16x2{xs[q][2 * e], xs[q][2 * e + 1]}, sc, false);
                    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, bf16x2{xs[q][2 * e + 2], xs[q][2 * e + 3]}, sc, true);
                    asm volatile("" ::"v"(r));
                }
            }
        }
        if constexpr (V == 10 || V == 12) {   // 1 x pk32_fp6
            bf16x32 y;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 8; ++e) y[8 * q + e] = xs[q][e];
            const i32x6 r = __builtin_amdgcn_cvt_scalef32_pk32_fp6_bf16(y, sc);
            asm volatile("" ::"v"(r));
        }
        if constexpr (V == 11 || V == 12) {   // + 4 bf16 MFMAs
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, xa, c[q], 0, 0, 0);
        }
        if constexpr (V == 0) {   // 16 x cvt_pk_fp8 (32 values)
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                s16x2 r = {0, 0};
                r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, bf16x2{x[4 * q], x[4 * q + 1]}, sc, false);
                r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, bf16x2{x[4 * q + 2], x[4 * q + 3]}, sc, true);
                acc8[q] ^= __builtin_bit_cast(int, r);
            }
            x[it & 31] = (__bf16)(float)acc8[0];
        } else if constexpr (V == 1) {   // 1 x pk32_fp6 (32 values)
            const i32x6 r = __builtin_amdgcn_cvt_scalef32_pk32_fp6_bf16(x, sc);
#pragma unroll
            for (int q = 0; q < 6; ++q) acc8[q] ^= r[q];
            x[it & 31] = (__bf16)(float)acc8[0];
        } else if constexpr (V == 2) {   // 4 x 16x16x128 e4m3 MFMA (independent accumulators)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                c[q] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(op, op, c[q], 0, 0, 0, 127, 0, 127);
        } else if constexpr (V == 3) {   // 4 x 16x16x128 e2m3 MFMA
#pragma unroll
            for (int q = 0; q < 4; ++q)
                c[q] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(op, op, c[q], 2, 2, 0, 127, 0, 127);
        } else if constexpr (V == 4) {   // 4 x 16x16x32 bf16 MFMA
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, xa, c[q], 0, 0, 0);
        } else if constexpr (V == 5) {   // 2 x 32x32x64 e2m3 MFMA
#pragma unroll
            for (int q = 0; q < 2; ++q)
                d[q] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(op, op, d[q], 2, 2, 0, 127, 0, 127);
        } else if constexpr (V == 6) {   // 2 x 32x32x16 bf16 MFMA
#pragma unroll
            for (int q = 0; q < 2; ++q) d[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, xa, d[q], 0, 0, 0);
        } else if constexpr (V == 7) {   // mix: 4 bf16 16x16x32 MFMA + 1 pk32_fp6
            const i32x6 r = __builtin_amdgcn_cvt_scalef32_pk32_fp6_bf16(x, sc);
#pragma unroll
            for (int q = 0; q < 6; ++q) acc8[q] ^= r[q];
            x[it & 31] = (__bf16)(float)acc8[0];
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, xa, c[q], 0, 0, 0);
        } else if constexpr (V == 8) {   // mix: 4 bf16 16x16x32 MFMA + 16 cvt_pk_fp8
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                s16x2 r = {0, 0};
                r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, bf16x2{x[4 * q], x[4 * q + 1]}, sc, false);
                r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, bf16x2{x[4 * q + 2], x[4 * q + 3]}, sc, true);
                acc8[q] ^= __builtin_bit_cast(int, r);
            }
            x[it & 31] = (__bf16)(float)acc8[0];
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa, xa, c[q], 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int q = 0; q < 8; ++q) s += (float)acc8[q];
    for (int q = 0; q < 4; ++q) s += c[q][0] + c[q][3];
    for (int q = 0; q < 2; ++q) s += d[q][0] + d[q][15];
    out[blockIdx.x * 512 + l] = s;
}

int main() {
    float *in, *out;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&out, 256 * 512 * 4);
    (void)hipMemset(in, 0, 4096 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[] = {"16 x cvt_scalef32_pk_fp8_bf16 (32 values)", "1 x cvt_scalef32_pk32_fp6_bf16 (32 values)",
                           "4 x mfma_scale 16x16x128 e4m3", "4 x mfma_scale 16x16x128 e2m3",
                           "4 x mfma 16x16x32 bf16", "2 x mfma_scale 32x32x64 e2m3", "2 x mfma 32x32x16 bf16",
                           "4 x mfma 16x16x32 bf16 + 1 x pk32_fp6", "4 x mfma 16x16x32 bf16 + 16 x cvt_pk_fp8",
                           "throughput: 16 x cvt_pk_fp8", "throughput: 1 x pk32_fp6",
                           "throughput: 16 x cvt_pk_fp8 + 4 x mfma bf16", "throughput: 1 x pk32_fp6 + 4 x mfma bf16"};
    for (int v = 0; v < 13; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            switch (v) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 7: hipLaunchKernelGGL(k<7>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 8: hipLaunchKernelGGL(k<8>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 9: hipLaunchKernelGGL(k<9>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 10: hipLaunchKernelGGL(k<10>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                case 11: hipLaunchKernelGGL(k<11>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
                default: hipLaunchKernelGGL(k<12>, dim3(256), dim3(512), 0, 0, in, out, 0.5f); break;
            }
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            // 2 waves per SIMD; per-SIMD ns per loop iteration (both waves' work)
            if (rep) printf("%-44s %8.3f ms  %7.2f ns per SIMD per iteration (2 waves)\n", names[v], ms,
                            ms * 1e6 / ITERS);
        }
    }
    return 0;
}
