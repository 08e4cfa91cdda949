// One-HBM-pass probe v3 (diagnostics only): wave-specialised exchange + LDS delay line.
//
// Block (row chunk, 1024-column segment), 4 waves, one block per CU, grid = resident capacity.
//   waves 0-2 stream the chunk's rows (wave c: rows c, c+3, ...) with non-temporal loads,
//     PF rows in flight in VGPRs; phase 1 (row partial of A d, wave-reduced) is published as
//     two tagged 8-byte granules PG[row][seg] (sc1 stores); the row segment is then parked in
//     an LDS ring (LAGR rows per wave) and read back LAGR steps later for phase 2
//     (U += row * S[row]), S[row] coming from the block's LDS S array.  Their vector-memory
//     queue holds only row loads and fire-and-forget stores, so the stream never waits on
//     the exchange.
//   wave 3 exchanges: it gathers and sums the 64 partials of the rows this segment sums
//     ("summer" rows: (row >> 2) % nseg == seg), publishes S[row] as a tagged pair SG[row],
//     and copies every row's published SG into the LDS S array, polling with s_sleep.
// Polls are bounded: on timeout the error word is set and every wave still finishes.
#include <hip/hip_runtime.h>

typedef float nf4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

#ifndef OP_CW
#define OP_CW 4
#endif
constexpr int kCW = OP_CW;         // streaming waves per block (+1 exchange wave)
constexpr int kSR = 512;           // circular LDS S array (rows)

__device__ __forceinline__ u64 ld_sc1(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// MODE (diagnostic): 0 full; 1 streaming waves never wait for S (the exchange still runs);
// 2 as 1 with the exchange wave idle
template <int PF, int LAGR, int MODE>
__global__ __launch_bounds__(64 * (OP_CW + 1)) void onepass3(const float* __restrict__ A, long long lda, long long m, int nseg,
                                                int R, const double* __restrict__ D, u64* PG, u64* SG,
                                                double* __restrict__ Sout, double* __restrict__ Us, unsigned tag,
                                                unsigned* err) {
    constexpr int NB = PF + 1;
    __shared__ __attribute__((aligned(16))) float ring[kCW][LAGR][1024];   // parked row segments
    __shared__ double sl_val[kSR];                                      // S of chunk rows, circular,
    __shared__ int sl_row[kSR];                                         // tagged with the row they hold
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int seg = blockIdx.x % nseg, chunk = blockIdx.x / nseg;
    const long long rbase = (long long)chunk * R;
    const u64 th = (u64)(2u * tag) << 32, tl = (u64)(2u * tag + 1u) << 32;
    const u64 tmask = 0xffffffff00000000ull;
    for (int i = threadIdx.x; i < kSR; i += blockDim.x) { sl_val[i] = 0.0; sl_row[i] = -1; }
    __syncthreads();
    unsigned polls = 1u << 18;
    bool failed = false;

    if (wave < kCW) {
        const long long col = (long long)seg * 1024 + lane * 4;
        double d[16], u[16];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) { d[4 * k + e] = D[col + 256 * k + e]; u[4 * k + e] = 0.0; }
        const int nrows = (R - wave + kCW - 1) / kCW;                     // rows wave, wave + 3, ...
        auto rloc = [&](int t) { return wave + kCW * t; };
        nf4 buf[NB][4];
        auto load = [&](int t, nf4 (&dst)[4]) {
            const int tt = t < nrows ? t : nrows - 1;
            const float* p = A + (rbase + rloc(tt)) * lda + col;
#pragma unroll
            for (int k = 0; k < 4; ++k) dst[k] = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p + 256 * k));
        };
#pragma unroll
        for (int t = 0; t < PF; ++t) load(t, buf[t]);
        float* myring = &ring[wave][0][0];
        for (int base = 0; base < nrows + LAGR; base += NB) {
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int t = base + q;
                load(t + PF, buf[(q + PF) % NB]);
                // phase 2 of row t - LAGR (its slot is then rewritten by row t)
                const int t2 = t - LAGR;
                if (t2 >= 0 && t2 < nrows) {
                    const int rl = rloc(t2);
                    int have = __hip_atomic_load(&sl_row[rl % kSR], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (MODE == 0 && have != rl) {
                        do {
                            if (polls == 0) { failed = true; break; }
                            --polls;
                            __builtin_amdgcn_s_sleep(1);
                            have = __hip_atomic_load(&sl_row[rl % kSR], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        } while (have != rl);
                    }
                    const double sr = sl_val[rl % kSR];
                    const float* slot = myring + (t2 % LAGR) * 1024;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const float4 v = *reinterpret_cast<const float4*>(slot + 256 * k + lane * 4);
                        u[4 * k + 0] = fma((double)v.x, sr, u[4 * k + 0]);
                        u[4 * k + 1] = fma((double)v.y, sr, u[4 * k + 1]);
                        u[4 * k + 2] = fma((double)v.z, sr, u[4 * k + 2]);
                        u[4 * k + 3] = fma((double)v.w, sr, u[4 * k + 3]);
                    }
                }
                // phase 1 of row t: publish, park
                if (t < nrows) {
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
                    if (lane == 0) {
                        const float hi = (float)s, lo = (float)(s - (double)hi);
                        u64* dst = PG + 2 * ((rbase + rloc(t)) * nseg + seg);
                        st_sc1(dst, th | __float_as_uint(hi));
                        st_sc1(dst + 1, tl | __float_as_uint(lo));
                    }
                    float* slot = myring + (t % LAGR) * 1024;
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        *reinterpret_cast<float4*>(slot + 256 * k + lane * 4) =
                            make_float4(buf[q][k].x, buf[q][k].y, buf[q][k].z, buf[q][k].w);
                }
            }
        }
        double* dst = Us + ((long long)chunk * kCW + wave) * ((long long)nseg * 1024) + col;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) dst[256 * k + e] = u[4 * k + e];
    } else if (MODE != 2) {
        // exchange wave: each pass issues the summer gather and the delivery poll together
        int s_front = 0;                  // next chunk row whose SG is copied to LDS
        int g_front = 0;                  // row within the current summer group
        const int ngroups = R / 4;        // groups of 4 rows; group k is summed by segment k % nseg
        int my_group = seg;               // current group this segment sums
        while (s_front < R || my_group < ngroups) {
            const bool sum_on = my_group < ngroups;
            const int rs = 4 * my_group + g_front;
            const u64* gsrc = PG + 2 * ((rbase + (sum_on ? rs : 0)) * nseg + (lane < nseg ? lane : 0));
            // deliver at most kSR - 64 rows ahead of the slowest consumer: rows below s_front - kSR
            // + 64 are consumed once every streaming wave is past them (LAGR slack) -- the ring
            // index is reused only after kSR rows
            const int rl = s_front + lane;
            const bool in = rl < R;
            const u64* dsrc = SG + 2 * (rbase + (in ? rl : 0));
            const u64 ga = ld_sc1(gsrc), gb = ld_sc1(gsrc + 1);
            const u64 da = ld_sc1(dsrc), db = ld_sc1(dsrc + 1);
            bool progress = false;
            if (sum_on) {
                const bool ok = lane >= nseg || ((ga & tmask) == th && (gb & tmask) == tl);
                if (__all(ok)) {
                    double x = lane < nseg ? (double)__uint_as_float((unsigned)ga) + (double)__uint_as_float((unsigned)gb) : 0.0;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
                    if (lane == 0) {
                        const float hi = (float)x, lo = (float)(x - (double)hi);
                        st_sc1(SG + 2 * (rbase + rs), th | __float_as_uint(hi));
                        st_sc1(SG + 2 * (rbase + rs) + 1, tl | __float_as_uint(lo));
                        Sout[rbase + rs] = x;
                    }
                    if (++g_front == 4) { g_front = 0; my_group += nseg; }
                    progress = true;
                }
            }
            if (s_front < R) {
                const bool ok = in && (da & tmask) == th && (db & tmask) == tl;
                const unsigned long long okmask = __ballot(ok);
                const int prefix = okmask == ~0ull ? 64 : __builtin_ctzll(~okmask);
                if (lane < prefix && in) {
                    sl_val[rl % kSR] = (double)__uint_as_float((unsigned)da) + (double)__uint_as_float((unsigned)db);
                    __hip_atomic_store(&sl_row[rl % kSR], rl, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if (prefix > 0) { s_front += prefix; progress = true; }
            }
            if (!progress) {
                if (polls == 0) { failed = true; break; }
                --polls;
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    if (failed && lane == 0) atomicOr(err, 1u);
}

extern "C" double onepass3_run(const void* A, long long lda, long long m, long long n, int nchunk, const void* D,
                               void* PG, void* SG, void* S, void* Us, unsigned* err, int iters, unsigned tag0,
                               int variant, int* resident) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nseg = (int)(n / 1024);
    const int R = (int)(m / nchunk);
    const dim3 grid((unsigned)(nseg * nchunk));
    int nb = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const void* fn = (const void*)onepass3<4, 8, 0>;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 64 * (kCW + 1), 0);
    *resident = nb * cus;
    if ((long long)nseg * nchunk > (long long)nb * cus) return -1.0;   // the exchange needs every block resident
    unsigned tag = tag0;
    auto run = [&]() {
#define OP3(P, LG, MD) hipLaunchKernelGGL((onepass3<P, LG, MD>), grid, dim3(64 * (kCW + 1)), 0, 0, (const float*)A, lda, m, \
                                          nseg, R, (const double*)D, (u64*)PG, (u64*)SG, (double*)S, (double*)Us, tag, err)
        switch (variant) {
            case 0: OP3(4, 8, 0); break;
            case 1: OP3(4, 8, 1); break;
            case 2: OP3(4, 8, 2); break;
            case 3: OP3(3, 8, 0); break;
            default: OP3(6, 8, 0); break;
        }
#undef OP3
        ++tag;
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
