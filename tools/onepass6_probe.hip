// One-HBM-pass probe v6 (diagnostics only): block-combined partials, XCD-local row groups.
//
// v5 (onepass5_probe.hip) shows the one-hop exchange itself is cheap unless the granule
// lines are written and read at the same time by many CUs: 64 producers and 64 readers
// per row cost ~100 us per pass.  v6 cuts both by 4-16x:
//   * a block's 4 waves walk the SAME rows, each over its own 1024 columns (block = 4096
//     columns, 16 segment blocks per row chunk at n = 65536);
//   * phase 1 of row t writes each wave's partial into an LDS slot (tagged with t in its low
//     mantissa byte); wave t % 4 later folds the 4 slots in a fixed order and publishes ONE
//     tagged granule per block and row (16 per row = one 128-byte line);
//   * phase 2 of row t: every wave reads the 16 granules of t (lanes 0..15) PF steps ahead,
//     checks the launch tag and folds them in the xor-butterfly order (same bits everywhere);
//   * the 16 segment blocks of a row chunk sit on one XCD (blockIdx % 8 = XCD).
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
__device__ __forceinline__ u64 stuff(double x, unsigned tag) {
    return ((u64)__double_as_longlong(x) & ~0xffull) | (tag & 0xffu);
}
__device__ __forceinline__ double unstuff(u64 g) { return __longlong_as_double((long long)(g & ~0xffull)); }

// DPP lane exchange (VALU, no LDS round trip): with one wave per SIMD the ds_bpermute
// latency of __shfl_xor chains is not hidden by other waves
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum over each 16-lane row, the same bits in every lane of the row (each level adds a
// partner's equal-shaped group: commutative, so both partners get identical sums)
__device__ __forceinline__ double row_sum16(double x) {
    x += dpp<0xb1>(x);    // quad_perm [1,0,3,2]
    x += dpp<0x4e>(x);    // quad_perm [2,3,0,1]
    x += dpp<0x141>(x);   // row_half_mirror
    x += dpp<0x140>(x);   // row_mirror
    return x;
}
__device__ __forceinline__ double lane_val(double x, int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// wave sum in a fixed order, uniform result: rows by DPP, then ((r0 + r1) + (r2 + r3))
__device__ __forceinline__ double wave_sum64(double x) {
    x = row_sum16(x);
    return (lane_val(x, 0) + lane_val(x, 16)) + (lane_val(x, 32) + lane_val(x, 48));
}

constexpr int kSB = 16;     // segment blocks per row chunk (n = 65536)
constexpr int kLS = 32;     // LDS partial slots (rows)

// MODE: 0 full exchange; 2 no exchange (stand-in S = own block partial); XL: XCD-local chunks
template <int NBUF, int PF, int DELTA, int MODE, int XL, int DPP>
__global__ __launch_bounds__(256, 1) void onepass6(const float* __restrict__ A, long long lda, int R,
                                                   const double* __restrict__ D, u64* PG,
                                                   double* __restrict__ Sout, double* __restrict__ Us,
                                                   unsigned tag, unsigned* err, unsigned long long* stats) {
    const u64 tk0 = __builtin_amdgcn_s_memrealtime();
    u64 n_late = 0, w_late = 0, n_pub = 0, w_pub = 0;
    constexpr int LAG = NBUF - PF - 1;
    static_assert(LAG > PF + DELTA, "granules are read PF steps before phase 2");
    __shared__ u64 part[kLS][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const int nchunk = gridDim.x / kSB;
    int chunk, sb;
    if (XL) { chunk = (b & 7) + 8 * ((b >> 3) / kSB); sb = (b >> 3) % kSB; }
    else { chunk = b / kSB; sb = b % kSB; }
    (void)nchunk;
    const long long col = (long long)sb * 4096 + wave * 1024 + lane * 4;
    const unsigned t8 = tag & 0xffu;
    for (int i = threadIdx.x; i < kLS * 4; i += 256) (&part[0][0])[i] = 0xffull;   // tag 255: no row
    __syncthreads();
    double d[16], u[16];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) { d[4 * k + e] = D[col + 256 * k + e]; u[4 * k + e] = 0.0; }
    const long long r0 = (long long)chunk * R;   // row of step t: r0 + t
    const int nrows = R;
    const int glane = lane < kSB ? lane : 0;
    nf4 buf[NBUF][4];
    u64 gv[NBUF];
    double sp[NBUF];
    auto load = [&](int t, int slot) {
        const int tc = t < nrows ? t : nrows - 1;
        const float* p = A + (r0 + tc) * lda + col;
#pragma unroll
        for (int k = 0; k < 4; ++k) buf[slot][k] = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p + 256 * k));
    };
    auto gload = [&](int t, int slot) {   // granules consumed at step t (phase 2 of row t - LAG)
        if (MODE == 0) {
            int t2 = t - LAG;
            t2 = t2 < 0 ? 0 : (t2 >= nrows ? nrows - 1 : t2);
            gv[slot] = ld_sc1(PG + (r0 + t2) * kSB + glane);
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
            const int qn = (q + PF) % NBUF;
            gload(t + PF, qn);
            load(t + PF, qn);
            if (t < nrows) {   // phase 1: wave partial of row t into LDS
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    s = fma((double)buf[q][k].x, d[4 * k + 0], s);
                    s = fma((double)buf[q][k].y, d[4 * k + 1], s);
                    s = fma((double)buf[q][k].z, d[4 * k + 2], s);
                    s = fma((double)buf[q][k].w, d[4 * k + 3], s);
                }
                if (DPP) {
                    s = wave_sum64(s);
                } else {
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                }
                sp[q] = s;
                if (MODE == 0 && lane == 0)
                    __hip_atomic_store(&part[t % kLS][wave], stuff(s, (unsigned)t), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const int tp = t - DELTA;   // publication of row tp by wave tp % 4
            if (MODE == 0 && tp >= 0 && tp < nrows && (tp & 3) == wave) {
                u64 w = 0;
                const unsigned want = (unsigned)tp & 0xffu;
                const u64 tw0 = __builtin_amdgcn_s_memrealtime();
                bool spun = false;
                while (true) {
                    w = lane < 4 ? __hip_atomic_load(&part[tp % kLS][lane], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
                    if (__all(lane >= 4 || (unsigned)(w & 0xff) == want)) break;
                    if (polls == 0) { failed = true; break; }
                    --polls;
                    spun = true;
                    __builtin_amdgcn_s_sleep(1);
                }
                if (spun) { ++n_pub; w_pub += __builtin_amdgcn_s_memrealtime() - tw0; }
                const double p0 = lane_val(unstuff(w), 0), p1 = lane_val(unstuff(w), 1);
                const double p2 = lane_val(unstuff(w), 2), p3 = lane_val(unstuff(w), 3);
                if (lane == 0) st_sc1(PG + (r0 + tp) * kSB + sb, stuff((p0 + p1) + (p2 + p3), t8));
            }
            const int t2 = t - LAG;
            if (t2 >= 0 && t2 < nrows) {   // phase 2 of row t2
                const int qs = (q - LAG + NBUF) % NBUF;
                double sr;
                if (MODE == 0) {
                    u64 v = gv[q];
                    auto ready = [&](u64 w) { return lane >= kSB || (unsigned)(w & 0xffull) == t8; };
                    if (!__all(ready(v))) {   // late: re-poll (drains this wave's queue; rare)
                        const u64 tw0 = __builtin_amdgcn_s_memrealtime();
                        const u64* src = PG + (r0 + t2) * kSB + glane;
                        do {
                            if (polls == 0) { failed = true; break; }
                            --polls;
                            __builtin_amdgcn_s_sleep(2);
                            v = ld_sc1(src);
                        } while (!__all(ready(v)));
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        asm volatile("" : "+v"(v));
                        ++n_late;
                        w_late += __builtin_amdgcn_s_memrealtime() - tw0;
                    }
                    double x = lane < kSB ? unstuff(v) : 0.0;
                    if (DPP) {
                        x = lane_val(row_sum16(x), 0);
                    } else {
#pragma unroll
                        for (int o = 1; o < kSB; o <<= 1) x += __shfl_xor(x, o);
                        x = __shfl(x, 0);   // lanes >= kSB summed zeros
                    }
                    sr = x;
                    if (sb == 0 && wave == 0 && lane == 0) Sout[r0 + t2] = x;
                } else {
                    sr = sp[qs] * 1e-3;
                }
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
    if (failed && lane == 0) atomicOr(err, 1u);
    if (lane == 0) {
        atomicAdd(stats + 0, n_late);
        atomicAdd(stats + 1, w_late);
        atomicAdd(stats + 2, n_pub);
        atomicAdd(stats + 3, w_pub);
        atomicAdd(stats + 4, __builtin_amdgcn_s_memrealtime() - tk0);
        atomicMax(stats + 5, __builtin_amdgcn_s_memrealtime() - tk0);
    }
    double* dst = Us + (long long)chunk * (kSB * 4096) + col;   // one U partial row per chunk
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[256 * k + e] = u[4 * k + e];
}

// (variant, NBUF, PF, DELTA, MODE, XCD-local, DPP reductions)
#define OP6_VARIANTS(X)                                                                                          \
    X(0, 14, 3, 1, 0, 1, 1) X(1, 14, 3, 1, 0, 0, 1) X(2, 16, 3, 1, 0, 1, 1) X(3, 16, 3, 1, 0, 0, 1)             \
    X(4, 16, 4, 1, 0, 1, 1) X(5, 18, 4, 1, 0, 1, 1) X(6, 14, 3, 1, 2, 1, 1) X(7, 18, 5, 1, 0, 1, 1)

extern "C" double onepass6_run(const void* A, long long lda, long long m, long long n, const void* D, void* PG,
                               void* S, void* Us, unsigned* err, int iters, unsigned tag0, int variant,
                               int* resident, void* stats) {
    if (n != kSB * 4096) return -3.0;
    int nb = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus;                       // one per CU
    if (blocks % (8 * kSB) != 0 && blocks % kSB != 0) return -4.0;
    const int nchunk = blocks / kSB;
    if (m % nchunk) return -5.0;
    const int R = (int)(m / nchunk);
    const void* fn = nullptr;
#define OP6_FN(V, NB, P, DL, MD, XL, DP) if (variant == V) fn = (const void*)onepass6<NB, P, DL, MD, XL, DP>;
    OP6_VARIANTS(OP6_FN)
#undef OP6_FN
    if (!fn) return -2.0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, 0);
    *resident = nb * cus;
    if (blocks > nb * cus) return -1.0;   // the exchange needs every block resident
    unsigned tag = tag0;
    auto run = [&]() {
        if ((tag & 0xffu) == 0) ++tag;   // tag 0 = never written
#define OP6_RUN(V, NB, P, DL, MD, XL, DP)                                                                          \
    if (variant == V)                                                                                            \
        hipLaunchKernelGGL((onepass6<NB, P, DL, MD, XL, DP>), dim3(blocks), dim3(256), 0, 0, (const float*)A, lda, R, \
                           (const double*)D, (u64*)PG, (double*)S, (double*)Us, tag, err, (u64*)stats);
        OP6_VARIANTS(OP6_RUN)
#undef OP6_RUN
        ++tag;
    };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    run();
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
