// Re-read probe (diagnostics only): what does a second pass over a just-streamed tile
// cost while the rest of the chip streams HBM?  This decides whether an iteration can
// read A from HBM once (A d, then A^T s from the on-chip copy) instead of twice.
//
// 1024 blocks (4 waves) walk tiles of `rows` x 4 KiB (1024 fp32) of a [m][lda] matrix,
// tile t = block + k * gridDim.  kind 0: one non-temporal read per tile; kind 1: one
// plain read; kind 2: plain read then plain re-read; kind 3: plain read, non-temporal
// re-read; kind 4: NT read then plain re-read.  fp64 FMA consumes every element.
#include <hip/hip_runtime.h>

typedef float nf4 __attribute__((ext_vector_type(4)));

template <bool NTL>
__device__ __forceinline__ float4 ld(const float4* p) {
    if (NTL) {
        nf4 t = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p));
        return make_float4(t.x, t.y, t.z, t.w);
    }
    return *p;
}

template <bool NTL>
__device__ __forceinline__ double tile_pass(const float4* base, long long lda4, int rows, int wave, int lane,
                                            double acc) {
    for (int r = wave; r < rows; r += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ld<NTL>(base + r * lda4 + u * 64 + lane);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            acc = fma((double)v[u].x, 1.0001, fma((double)v[u].y, 0.9999, fma((double)v[u].z, 1.0, fma((double)v[u].w, 0.5, acc))));
    }
    return acc;
}

template <int KIND>
__global__ __launch_bounds__(256) void reread(const float4* __restrict__ a, long long lda4, long long m, int rows,
                                               double* __restrict__ sink) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long nseg = lda4 / 256;
    const long long ntiles = nseg * (m / rows);
    double acc = 0.0;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long seg = t % nseg, rc = t / nseg;
        const float4* base = a + rc * rows * lda4 + seg * 256;
        if (KIND == 0) acc = tile_pass<true>(base, lda4, rows, wave, lane, acc);
        if (KIND == 1) acc = tile_pass<false>(base, lda4, rows, wave, lane, acc);
        if (KIND == 2) { acc = tile_pass<false>(base, lda4, rows, wave, lane, acc); __syncthreads();
                         acc = tile_pass<false>(base, lda4, rows, wave, lane, acc * 0.5); }
        if (KIND == 3) { acc = tile_pass<false>(base, lda4, rows, wave, lane, acc); __syncthreads();
                         acc = tile_pass<true>(base, lda4, rows, wave, lane, acc * 0.5); }
        if (KIND == 4) { acc = tile_pass<true>(base, lda4, rows, wave, lane, acc); __syncthreads();
                         acc = tile_pass<false>(base, lda4, rows, wave, lane, acc * 0.5); }
    }
    if (acc == 12345.0) sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" double reread_run(int kind, int blocks, const void* a, long long lda_floats, long long m, int rows,
                             double* sink, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const long long lda4 = lda_floats / 4;
    auto run = [&]() {
        switch (kind) {
            case 0: hipLaunchKernelGGL(reread<0>, dim3(blocks), dim3(256), 0, 0, (const float4*)a, lda4, m, rows, sink); break;
            case 1: hipLaunchKernelGGL(reread<1>, dim3(blocks), dim3(256), 0, 0, (const float4*)a, lda4, m, rows, sink); break;
            case 2: hipLaunchKernelGGL(reread<2>, dim3(blocks), dim3(256), 0, 0, (const float4*)a, lda4, m, rows, sink); break;
            case 3: hipLaunchKernelGGL(reread<3>, dim3(blocks), dim3(256), 0, 0, (const float4*)a, lda4, m, rows, sink); break;
            default: hipLaunchKernelGGL(reread<4>, dim3(blocks), dim3(256), 0, 0, (const float4*)a, lda4, m, rows, sink); break;
        }
    };
    run();
    hipEventRecord(e0, 0);
    for (int k = 0; k < iters; ++k) run();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return (double)ms / iters;
}
