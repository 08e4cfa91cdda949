// One-HBM-pass probe v5 (diagnostics only): deep register delay line + one-hop exchange.
//
// Streaming as in regpass_probe.hip (tile = row chunk x 1024-column segment; wave q of a
// block walks rows q, q+4, ... with non-temporal 16-byte loads).  The row ring buf[NBUF]
// holds PF rows in flight and LAG = NBUF - PF - 1 rows between phase 1 (S partial) and
// phase 2 (U += row * S): at NBUF ~ 20 it exceeds the 256 arch VGPRs, and with one wave per
// SIMD (launch bounds 256 x 1) the compiler keeps the cold rows in AGPRs.
// Exchange, one hop: phase 1 of row r publishes the wave's fp64 partial with its low 8
// mantissa bits replaced by the launch tag (one 8-byte agent-scope store); phase 2 of r
// reads all nseg granules of r (lane = segment), checks the tags and sums them in the
// xor-butterfly order, which gives the same bits in every lane and every block.  The
// granule load is issued PF steps before its use, beside the row prefetch of that step, so
// it rides the in-order vmcnt queue without draining it; only a late granule re-polls.
// Every poll is bounded: on timeout the error word is set and the kernel still finishes.
#include <hip/hip_runtime.h>

typedef float nf4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

__device__ __forceinline__ u64 ld_sc1(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// MODE (diagnostic bisection): 0 full exchange; 1 granule stores + loads, never checked or
// used (stand-in S); 2 no exchange traffic at all (stand-in S); 3 stores only; 4 loads only;
// 5 stores + loads of a disjoint, never-written buffer
// CW: 16-byte loads per lane per row (segment = 256 CW columns)
template <int NBUF, int PF, int MODE, int OCC, int CW>
__global__ __launch_bounds__(256, OCC) void onepass5(const float* __restrict__ A, long long lda, int nseg, int R,
                                                   const double* __restrict__ D, u64* PG,
                                                   double* __restrict__ Sout, double* __restrict__ Us,
                                                   unsigned tag, unsigned* err) {
    constexpr int LAG = NBUF - PF - 1;
    static_assert(LAG > PF, "granules are read PF steps before phase 2");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int seg = blockIdx.x % nseg, chunk = blockIdx.x / nseg;
    const long long col = (long long)seg * (256 * CW) + lane * 4;
    const u64 t8 = tag & 0xffu;
    double d[4 * CW], u[4 * CW];
#pragma unroll
    for (int k = 0; k < CW; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) { d[4 * k + e] = D[col + 256 * k + e]; u[4 * k + e] = 0.0; }
    const long long r0 = (long long)chunk * R + wave;   // row of step t: r0 + 4 t
    const int nrows = R / 4;
    const int glane = lane < nseg ? lane : 0;
    nf4 buf[NBUF][CW];
    u64 gv[NBUF];
    double sp[NBUF];
    auto load = [&](int t, int slot) {
        const int tc = t < nrows ? t : nrows - 1;
        const float* p = A + (r0 + 4ll * tc) * lda + col;
#pragma unroll
        for (int k = 0; k < CW; ++k) buf[slot][k] = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p + 256 * k));
    };
    // granules consumed at step t (phase 2 of row t - LAG)
    auto gload = [&](int t, int slot) {
        if (MODE <= 1 || MODE >= 4) {
            int t2 = t - LAG;
            t2 = t2 < 0 ? 0 : (t2 >= nrows ? nrows - 1 : t2);
            gv[slot] = ld_sc1(PG + (MODE == 5 ? 8192ll * 64 : 0ll) + (r0 + 4ll * t2) * nseg + glane);
        }
    };
    unsigned polls = 1u << 16;
    bool failed = false;
#pragma unroll
    for (int q = 0; q < PF; ++q) { gload(q, q); load(q, q); }
    for (int base = 0; base < nrows + LAG; base += NBUF) {
#pragma unroll
        for (int q = 0; q < NBUF; ++q) {
            const int t = base + q;
            constexpr int dummy = 0;
            (void)dummy;
            const int qn = (q + PF) % NBUF;
            gload(t + PF, qn);
            load(t + PF, qn);
            if (t < nrows) {   // phase 1
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < CW; ++k) {
                    s = fma((double)buf[q][k].x, d[4 * k + 0], s);
                    s = fma((double)buf[q][k].y, d[4 * k + 1], s);
                    s = fma((double)buf[q][k].z, d[4 * k + 2], s);
                    s = fma((double)buf[q][k].w, d[4 * k + 3], s);
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                sp[q] = s;
                if ((MODE <= 1 || MODE == 3 || MODE == 5) && lane == 0)
                    st_sc1(PG + (r0 + 4ll * t) * nseg + seg, ((u64)__double_as_longlong(s) & ~0xffull) | t8);
            }
            const int t2 = t - LAG;
            if (t2 >= 0 && t2 < nrows) {   // phase 2 of row t2 (slot of t2)
                const int qs = (q - LAG + NBUF) % NBUF;
                double sr;
                if (MODE == 0) {
                    u64 v = gv[q];
                    auto ready = [&](u64 w) { return lane >= nseg || (w & 0xffull) == t8; };
                    if (!__all(ready(v))) {   // late: re-poll (drains this wave's queue; rare)
                        const u64* src = PG + (r0 + 4ll * t2) * nseg + glane;
                        do {
                            if (polls == 0) { failed = true; break; }
                            --polls;
                            __builtin_amdgcn_s_sleep(2);
                            v = ld_sc1(src);
                        } while (!__all(ready(v)));
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        asm volatile("" : "+v"(v));
                    }
                    double x = lane < nseg ? __longlong_as_double((long long)(v & ~0xffull)) : 0.0;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
                    sr = x;
                    if (seg == 0 && lane == 0) Sout[r0 + 4ll * t2] = x;
                } else {
                    sr = sp[qs] * 1e-3;
                    if (MODE == 1 || MODE >= 4) sr += (double)(gv[q] & 1) * 1e-300;
                }
#pragma unroll
                for (int k = 0; k < CW; ++k) {
                    u[4 * k + 0] = fma((double)buf[qs][k].x, sr, u[4 * k + 0]);
                    u[4 * k + 1] = fma((double)buf[qs][k].y, sr, u[4 * k + 1]);
                    u[4 * k + 2] = fma((double)buf[qs][k].z, sr, u[4 * k + 2]);
                    u[4 * k + 3] = fma((double)buf[qs][k].w, sr, u[4 * k + 3]);
                }
            }
        }
    }
    if (failed && lane == 0) atomicOr(err, 1u);
    double* dst = Us + ((long long)chunk * 4 + wave) * ((long long)nseg * (256 * CW)) + col;
#pragma unroll
    for (int k = 0; k < CW; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[256 * k + e] = u[4 * k + e];
}

// (variant, NBUF, PF, MODE, blocks per CU, CW)
#define OP5_VARIANTS(X)                                                                                          \
    X(0, 12, 3, 0, 1, 4) X(1, 12, 3, 1, 1, 4) X(2, 12, 3, 2, 1, 4) X(3, 12, 3, 5, 1, 4) X(4, 12, 3, 1, 1, 4)      \
    X(5, 12, 3, 0, 1, 4) X(6, 12, 3, 3, 1, 4) X(7, 12, 3, 4, 1, 4) X(8, 8, 2, 0, 1, 4) X(9, 12, 3, 0, 1, 4)

extern "C" double onepass5_run(const void* A, long long lda, long long m, long long n, int nchunk, const void* D,
                               void* PG, void* S, void* Us, unsigned* err, int iters, unsigned tag0, int variant,
                               int* resident) {
    const int cwv[] = {4, 4, 4, 4, 4, 4, 4, 4, 4, 4};
    if (variant < 0 || variant > 9) return -2.0;
    const int nseg = (int)(n / (256 * cwv[variant]));
    const int R = (int)(m / nchunk);
    const dim3 grid((unsigned)(nseg * nchunk));
    int nb = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const void* fn = nullptr;
#define OP5_FN(V, NB, P, MD, OC, CW) if (variant == V) fn = (const void*)onepass5<NB, P, MD, OC, CW>;
    OP5_VARIANTS(OP5_FN)
#undef OP5_FN
    if (!fn) return -2.0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, 0);
    *resident = nb * cus;
    if ((long long)nseg * nchunk > (long long)nb * cus) return -1.0;   // the exchange needs every block resident
    unsigned tag = tag0;
    auto run = [&]() {
        if ((tag & 0xffu) == 0) ++tag;   // tag 0 = never written
#define OP5_RUN(V, NB, P, MD, OC, CW)                                                                                   \
    if (variant == V)                                                                                             \
        hipLaunchKernelGGL((onepass5<NB, P, MD, OC, CW>), grid, dim3(256), 0, 0, (const float*)A, lda, nseg, R,           \
                           (const double*)D, (u64*)PG, (double*)S, (double*)Us, tag, err);
        OP5_VARIANTS(OP5_RUN)
#undef OP5_RUN
        ++tag;
    };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
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
