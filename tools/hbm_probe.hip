// HBM streaming-read ceiling probe (diagnostics only, not part of the product).
// Measures what a pure read stream reaches on this MI355X for the access
// shapes the solver's passes use, so the roofline fraction of k_colpass /
// k_rowpass can be compared with an achievable ceiling, not just the spec.
//
//   kind 0: grid-stride float4 reads, fp32 add                (pure read)
//   kind 1: grid-stride float4 reads, f32->f64 convert + fma    (colpass arithmetic)
//   kind 2: kind 0 with non-temporal loads
//   kind 3: row-segment walk like k_colpass: each wave reads 4 KiB of a row,
//           next row 'lda' away; fp64 fma
//   kind 4: float4 copy (read + write), the guide's reference stream
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float nf4 __attribute__((ext_vector_type(4)));

template <int KIND, int UNR>
__global__ __launch_bounds__(256) void probe(const float4* __restrict__ a, float4* __restrict__ o,
                                              long long n4, double* __restrict__ sink, long long lda4,
                                              long long rows) {
    const long long tid = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long nth = (long long)gridDim.x * 256;
    if (KIND == 3) {
        // columns: each wave owns a 4 KiB (256 float4) segment; rows split across waves
        const int lane = threadIdx.x & 63;
        const long long wave = tid >> 6, nwave = nth >> 6;
        const long long nseg = lda4 / 256;
        double acc = 0.0;
        for (long long wv = wave; wv < nseg * (rows / 32); wv += nwave) {
            const long long seg = wv % nseg, rc = wv / nseg;
            const float4* base = a + rc * 32 * lda4 + seg * 256 + lane;
#pragma unroll 2
            for (int r = 0; r < 32; ++r) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = base[r * lda4 + u * 64];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    acc = fma((double)v[u].x, 1.0001, fma((double)v[u].y, 0.9999, fma((double)v[u].z, 1.0, fma((double)v[u].w, 0.5, acc))));
            }
        }
        if (acc == 12345.0) sink[tid] = acc;
        return;
    }
    float facc = 0.f;
    double dacc = 0.0;
    long long i = tid;
    for (; i + (UNR - 1) * nth < n4; i += UNR * nth) {
        float4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (KIND == 2) {
                nf4 t = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(a + i + u * nth));
                v[u] = make_float4(t.x, t.y, t.z, t.w);
            }
            else v[u] = a[i + u * nth];
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (KIND == 4) o[i + u * nth] = v[u];
            else if (KIND == 1) dacc = fma((double)v[u].x, 1.0001, fma((double)v[u].y, 0.9999, fma((double)v[u].z, 1.0, fma((double)v[u].w, 0.5, dacc))));
            else facc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
        }
    }
    for (; i < n4; i += nth) {
        float4 v = a[i];
        if (KIND == 4) o[i] = v;
        else facc += v.x;
    }
    if (facc == 12345.f || dacc == 12345.0) sink[tid] = facc + dacc;
}

template <int KIND, int UNR>
static void launch(int blocks, const float4* a, float4* o, long long n4, double* sink, long long lda4, long long rows,
                   hipStream_t s) {
    hipLaunchKernelGGL((probe<KIND, UNR>), dim3(blocks), dim3(256), 0, s, a, o, n4, sink, lda4, rows);
}

extern "C" double probe_run(int kind, int unroll, int blocks, const void* a, void* o, long long bytes, double* sink,
                            long long lda_floats, int iters) {
    const long long n4 = bytes / 16;
    const long long lda4 = lda_floats / 4;
    const long long rows = bytes / (lda_floats * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&]() {
#define L(K, U) launch<K, U>(blocks, (const float4*)a, (float4*)o, n4, sink, lda4, rows, 0)
        if (kind == 0) { if (unroll == 4) L(0, 4); else if (unroll == 8) L(0, 8); else L(0, 16); }
        if (kind == 1) { if (unroll == 4) L(1, 4); else if (unroll == 8) L(1, 8); else L(1, 16); }
        if (kind == 2) { if (unroll == 4) L(2, 4); else if (unroll == 8) L(2, 8); else L(2, 16); }
        if (kind == 3) L(3, 4);
        if (kind == 4) { if (unroll == 4) L(4, 4); else L(4, 8); }
#undef L
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
