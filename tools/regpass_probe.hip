// Register-resident two-phase streaming probe (diagnostics only).
//
// The streaming half of a one-HBM-pass iteration built like k_colpass: each wave walks
// rows i = wave, wave + 4, ... of a (row chunk x 1024-column segment) tile with
// non-temporal 16-byte loads, keeps NBUF row segments in VGPRs (PF of them in flight),
// computes the row partial of A d (phase 1, wave-reduced) and, LAG rows later,
// U += A^T s for that row from the same registers (phase 2).  s is a stand-in derived
// from the row's own partial: no exchange, so this bounds what the streaming structure
// can do at 1-2 blocks per CU.  Checked against a host formula for the same stand-in.
#include <hip/hip_runtime.h>

typedef float nf4 __attribute__((ext_vector_type(4)));

template <int NBUF, int PF>
__global__ __launch_bounds__(256) void regpass(const float* __restrict__ A, long long lda, long long m,
                                               int nseg, int R, const double* __restrict__ D,
                                               double* __restrict__ part, double* __restrict__ Us) {
    constexpr int LAG = NBUF - PF - 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int seg = blockIdx.x % nseg, chunk = blockIdx.x / nseg;
    const long long col = (long long)seg * 1024 + lane * 4;
    double d[16], u[16];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) { d[4 * k + e] = D[col + 256 * k + e]; u[4 * k + e] = 0.0; }
    const long long r0 = (long long)chunk * R;
    const int nrows = R / 4;                       // rows of this wave: r0 + wave + 4 q
    nf4 buf[NBUF][4];
    double sp[NBUF];
    auto load = [&](int q, nf4 (&dst)[4]) {
        const int qq = q < nrows ? q : nrows - 1;
        const float* p = A + (r0 + wave + 4ll * qq) * lda + col;
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p + 256 * k));
    };
#pragma unroll
    for (int q = 0; q < PF; ++q) load(q, buf[q]);
    for (int base = 0; base < nrows + LAG; base += NBUF) {
#pragma unroll
        for (int q = 0; q < NBUF; ++q) {
            const int r = base + q;
            load(r + PF, buf[(q + PF) % NBUF]);    // slot held row r + PF - NBUF = r - LAG - 1
            if (r < nrows) {                        // phase 1
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    s = fma((double)buf[q][k].x, d[4 * k + 0], s);
                    s = fma((double)buf[q][k].y, d[4 * k + 1], s);
                    s = fma((double)buf[q][k].z, d[4 * k + 2], s);
                    s = fma((double)buf[q][k].w, d[4 * k + 3], s);
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                sp[q] = s;
                if (lane == 0) part[(r0 + wave + 4ll * r) * nseg + seg] = s;
            }
            const int r2 = r - LAG;
            if (r2 >= 0 && r2 < nrows) {            // phase 2 on the registers of row r2
                constexpr int dummy = 0;
                (void)dummy;
                const int qs = (q - LAG + NBUF) % NBUF;
                const double sr = sp[qs] * 1e-3;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    u[4 * k + 0] = fma((double)buf[qs][k].x, sr, u[4 * k + 0]);
                    u[4 * k + 1] = fma((double)buf[qs][k].y, sr, u[4 * k + 1]);
                    u[4 * k + 2] = fma((double)buf[qs][k].z, sr, u[4 * k + 2]);
                    u[4 * k + 3] = fma((double)buf[qs][k].w, sr, u[4 * k + 3]);
                }
            }
        }
    }
    // per-wave U partial: Us[chunk][wave][cols]
    double* dst = Us + ((long long)chunk * 4 + wave) * (nseg * 1024) + col;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[256 * k + e] = u[4 * k + e];
}

extern "C" double regpass_run(const void* A, long long lda, long long m, long long n, int nchunk, const void* D,
                              void* part, void* Us, int iters, int variant) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nseg = (int)(n / 1024);
    const int R = (int)(m / nchunk);
    const dim3 grid((unsigned)(nseg * nchunk));
    auto run = [&]() {
        switch (variant) {
            case 0: hipLaunchKernelGGL((regpass<8, 3>), grid, dim3(256), 0, 0, (const float*)A, lda, m, nseg, R,
                                       (const double*)D, (double*)part, (double*)Us); break;
            case 1: hipLaunchKernelGGL((regpass<8, 4>), grid, dim3(256), 0, 0, (const float*)A, lda, m, nseg, R,
                                       (const double*)D, (double*)part, (double*)Us); break;
            case 2: hipLaunchKernelGGL((regpass<6, 2>), grid, dim3(256), 0, 0, (const float*)A, lda, m, nseg, R,
                                       (const double*)D, (double*)part, (double*)Us); break;
            default: hipLaunchKernelGGL((regpass<10, 4>), grid, dim3(256), 0, 0, (const float*)A, lda, m, nseg, R,
                                        (const double*)D, (double*)part, (double*)Us); break;
        }
    };
    run();
    (void)hipEventRecord(e0, 0);
    for (int k = 0; k < iters; ++k) run();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (double)ms / iters;
}
