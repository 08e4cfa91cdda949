// bpgl device kernels (gfx950 / CDNA4) of the single-right-hand-side path.
// Included by bpgl.hip only (non-template kernels are defined here).
//
// Hot path of one block update (reference lasso.py:102-157):
//   k_colpass   partial  g = A_b^T r  over a (row chunk x column segment) tile,
//               fp64 accumulation, cross-wave LDS reduction, one fp64 slab row
//               per row chunk (replaces K1 mul_mat_t_vec_diffsize,
//               gpu_calculation.py:20-55, whose partials were summed on the host)
//   k_shrink    fixed-order split-K sum of the slab, s14/s15 best response,
//               direction D, l1 norms and the error criterion
//               (lasso.py:114-119, cpu_calculation.py:5-20)
//   k_rowpass   partial  s23 = A_b D  per (row, column segment), wave-level
//               transposed butterfly reduction (replaces K2 mul_mat_vec_diffsize,
//               gpu_calculation.py:58-91, whose lanes were strided by a row)
//   k_rowreduce fixed-order sum over column segments + l1/err partials into
//               the all-reduce buffer
//   k_step      exact line search and stopping rule (lasso.py:129-150), 1 block
//   k_update    x_b += gamma D, Ax_b += gamma s23, s11 = sum_k Ax_k - b
//               (lasso.py:153-155, :105)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bpgl_device.h"

namespace bpgl {

constexpr int kU = 4;           // 16-byte loads per lane per row segment (= kWaves)

struct DevState {
    long long t;          // index of the next iteration
    long long done;       // stopping rule fired
    long long block_cnt;  // lasso.py:144-150
    long long t_last;     // last t reached (the reference's loop variable)
    long long cur_mb;     // block updated by the current iteration
    long long t_base;     // wall clock (100 MHz) at reset
    double gamma;         // step size of the last iteration
    double err;           // error criterion of the last iteration
    double r1, r2;        // line-search numerators (diagnostics)
    long long iters;      // iterations completed (update applied or stop reached)
    unsigned long long op_ran;   // one-pass mode: k_onepass ran in this iteration (advances op_epoch)
    long long op_epoch;   // one-pass mode: launches so far (tag of the row-partial hand-off)
    long long op_fail;    // one-pass mode: a hand-off poll ran out (blocks not co-resident)
    unsigned long long op_cnt;   // one-pass mode: row-group arrivals (k_onepass line search)
    long long op_base;    // one-pass mode: op_epoch at the solver reset (row direction = parity since)
};

struct Params {
    const void* A;
    long long lda, block_stride;
    long long m, w, wp;
    int nblock, nseg, nchunk, R;
    int nparts, nranks, rank, has_comm;
    double* slab_g;   // [nchunk][wp]
    double* slab_s;   // [nseg][m]
    double* D;        // [wp]
    double* parts;    // [nparts][4]   shrink partials (sum |Bx|, sum |x|, max err)
    double* parts2;   // [m/64][2]     rowreduce partials (sum r s23, sum s23^2)
    int reverse_rows;  // rowpass walks each chunk's rows bottom-up (Infinity Cache reuse)
    int tail_permille; // with NT loads: share of each chunk read last with allocating loads
    double* comm;     // [m + 2 + nranks]
    double* r;        // [m]   residual s11 = sum_k Ax_k - b
    double* Ax;       // [nblock][m]
    const double* b;  // [m]
    double* x;        // [nblock][wp]
    const double* diag;  // [nblock][wp]
    const double* rec;   // [nblock][wp]  1 / diag (lasso.py:29-30)
    const int* order;    // [order_len] or null
    long long order_len;
    double* err_iter;
    double* time_iter;
    long long rec_len;
    DevState* st;
    double mu, err_bound;
    double wall_tick_s;   // seconds per wall_clock64() tick
};

// ---------------------------------------------------------------------------
// 16-byte vector loads of A, widened to fp64
// ---------------------------------------------------------------------------
template <typename T> struct VecT;
template <> struct VecT<float> {
    static constexpr int N = 4;
    using raw = float4;
    __device__ static inline void cvt(const raw& v, double (&o)[N]) {
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    }
};
template <> struct VecT<double> {
    static constexpr int N = 2;
    using raw = double2;
    __device__ static inline void cvt(const raw& v, double (&o)[N]) { o[0] = v.x; o[1] = v.y; }
};
struct bf16_t { unsigned short u; };
template <> struct VecT<bf16_t> {
    static constexpr int N = 8;
    using raw = uint4;
    __device__ static inline double one(unsigned int h) { return (double)__uint_as_float(h << 16); }
    __device__ static inline void cvt(const raw& v, double (&o)[N]) {
        o[0] = one(v.x & 0xffffu); o[1] = one(v.x >> 16);
        o[2] = one(v.y & 0xffffu); o[3] = one(v.y >> 16);
        o[4] = one(v.z & 0xffffu); o[5] = one(v.z >> 16);
        o[6] = one(v.w & 0xffffu); o[7] = one(v.w >> 16);
    }
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <typename T, bool NT = false>
__device__ __forceinline__ typename VecT<T>::raw ldv(const T* p) {
    using raw = typename VecT<T>::raw;
    if constexpr (NT) {
        // non-temporal 16-byte load (streamed-once A)
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        raw o;
        __builtin_memcpy(&o, &v, sizeof(raw));
        return o;
    } else {
        return *reinterpret_cast<const raw*>(p);
    }
}

__device__ __forceinline__ int cur_block(const Params& p) {
    const long long t = p.st->t;
    if (p.order) return p.order[t < p.order_len ? t : p.order_len - 1];
    return (int)(t % p.nblock);
}


// ---------------------------------------------------------------------------
// colpass: slab[chunk][col] = sum_{i in chunk} A_b[i][col] * vec[i]   (MODE 0)
//          slab[chunk][col] = sum_{i in chunk} A_b[i][col]^2           (MODE 1)
// grid = nseg * nchunk blocks of 256; block (seg, chunk) owns SEGW columns and
// R rows; the 4 waves split the rows (wave q: rows q, q+4, ...) and sum their
// fp64 partials through LDS in a fixed order.
// ---------------------------------------------------------------------------
// One "trip" of a wave in k_colpass: RPT rows (i, i+4, ..., i+4(RPT-1)), kU
// sixteen-byte loads per row.  Rows at or past i1 are clamped to row i (in
// bounds) and get a zero weight.
template <typename T, int MODE, bool NT, int RPT>
__device__ __forceinline__ void colpass_load(const T* __restrict__ Ab, long long lda, const long long (&col)[kU],
                                             const double* __restrict__ vec, long long i, long long i1,
                                             typename VecT<T>::raw (&a)[RPT][kU], double (&sc)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        long long r = i + k * kWaves;
        const bool ok = r < i1;
        r = ok ? r : i;
        sc[k] = (MODE == 0) ? vec[r] : 1.0;
        sc[k] = ok ? sc[k] : 0.0;
#pragma unroll
        for (int u = 0; u < kU; ++u) a[k][u] = ldv<T, NT>(Ab + r * lda + col[u]);
    }
}
template <typename T, int MODE, int RPT>
__device__ __forceinline__ void colpass_fma(const typename VecT<T>::raw (&a)[RPT][kU], const double (&sc)[RPT],
                                            double (&acc)[kU][VecT<T>::N]) {
    constexpr int V = VecT<T>::N;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            double v[V];
            VecT<T>::cvt(a[k][u], v);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                if (MODE == 0) acc[u][e] = fma(v[e], sc[k], acc[u][e]);
                else acc[u][e] = fma(v[e] * sc[k], v[e], acc[u][e]);
            }
        }
    }
}

// rows [i, istop) of one wave, RPT rows per trip.  PIPE: the next trip's loads
// are issued before the current trip's FMAs (2 x RPT x kU loads in flight per
// lane, at a higher register cost).  Every accumulator sees its rows in
// increasing order, so results depend on neither RPT nor PIPE.
template <typename T, int MODE, bool NT, int RPT, bool PIPE>
__device__ __forceinline__ void colpass_span(const T* __restrict__ Ab, long long lda, const long long (&col)[kU],
                                             const double* __restrict__ vec, long long& i, long long istop,
                                             long long i1, double (&acc)[kU][VecT<T>::N]) {
    using raw = typename VecT<T>::raw;
    constexpr long long step = (long long)RPT * kWaves;
    if (i >= istop) return;
    if constexpr (!PIPE) {
        for (; i < istop; i += step) {
            raw a[RPT][kU];
            double sa[RPT];
            colpass_load<T, MODE, NT, RPT>(Ab, lda, col, vec, i, i1, a, sa);
            colpass_fma<T, MODE, RPT>(a, sa, acc);
        }
    } else {
        raw a[RPT][kU], b[RPT][kU];
        double sa[RPT], sb[RPT];
        colpass_load<T, MODE, NT, RPT>(Ab, lda, col, vec, i, i1, a, sa);
        for (;;) {
            if (i + step >= istop) { colpass_fma<T, MODE, RPT>(a, sa, acc); i += step; return; }
            colpass_load<T, MODE, NT, RPT>(Ab, lda, col, vec, i + step, i1, b, sb);
            colpass_fma<T, MODE, RPT>(a, sa, acc);
            i += step;
            if (i + step >= istop) { colpass_fma<T, MODE, RPT>(b, sb, acc); i += step; return; }
            colpass_load<T, MODE, NT, RPT>(Ab, lda, col, vec, i + step, i1, a, sa);
            colpass_fma<T, MODE, RPT>(b, sb, acc);
            i += step;
        }
    }
}

// Diagnostic builds only (tools/stamp_diag.sh, -DBPGL_STAMP=1): per-block start/end times
// (s_memrealtime, 100 MHz) of the last k_colpass / k_rowpass launch, to measure ramp and tail.
#ifndef BPGL_STAMP
#define BPGL_STAMP 0
#endif
#if BPGL_STAMP
// [colpass, rowpass, onepass][0 start, 1 end (after a barrier), 2-4 wave-0 marks (k_onepass: first
// row computed, last row's phase 1, kernel end)][block]
__device__ unsigned long long g_stamps[3][5][16384];
#define BPGL_STAMP_AT(kern, se)                                                                   \
    do {                                                                                          \
        if ((se) == 1) __syncthreads();                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 16384)                                               \
            g_stamps[kern][se][blockIdx.x] = __builtin_amdgcn_s_memrealtime();                    \
    } while (0)
#else
#define BPGL_STAMP_AT(kern, se) do { } while (0)
#endif

// one (chunk, seg) tile of the A^T vec pass: rows [chunk R, +R) x the segment's columns,
// fp64 partials written to slab row `chunk`.  `red` is the block's LDS reduction buffer.
template <typename T, int MODE, bool NT, int RPT, bool PIPE>
__device__ __forceinline__ void colpass_tile(const Params& p, const T* __restrict__ Ab, const double* __restrict__ vec,
                                             double* __restrict__ slab, int seg, int chunk,
                                             double (&red)[kWaves][kU * VecT<T>::N][64]) {
    constexpr int V = VecT<T>::N;
    constexpr int SEGW = 64 * V * kU;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    long long col[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const long long c = (long long)seg * SEGW + u * 64 * V + lane * V;
        col[u] = c < p.wp ? c : 0;  // clamped: loads stay in bounds, the column is dropped below
    }
    double acc[kU][V];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[u][e] = 0.0;

    const long long i0 = (long long)chunk * p.R;
    const long long i1 = (i0 + p.R < p.m) ? i0 + p.R : p.m;
    // the rows this wave reads last (the bottom `tail` of the chunk) use plain,
    // cache-allocating loads: k_rowpass reads them first.  Everything else is
    // a non-temporal stream.
    long long i = i0 + wave;
    if (NT) {
        const long long isplit = i1 - ((i1 - i0) * p.tail_permille) / 1000;
        colpass_span<T, MODE, true, RPT, PIPE>(Ab, p.lda, col, vec, i, isplit, i1, acc);
    }
    colpass_span<T, MODE, false, RPT, PIPE>(Ab, p.lda, col, vec, i, i1, i1, acc);
    // cross-wave reduction in a fixed order (wave 0 + 1 + 2 + 3)
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) red[wave][u * V + e][lane] = acc[u][e];
    __syncthreads();
    // wave q finalises column group u = q: V consecutive fp64 per lane
    const int q = wave;
    const long long c = (long long)seg * SEGW + q * 64 * V + lane * V;
    if (c < p.wp) {
        double o[V];
#pragma unroll
        for (int e = 0; e < V; ++e)
            o[e] = ((red[0][q * V + e][lane] + red[1][q * V + e][lane]) + red[2][q * V + e][lane]) +
                   red[3][q * V + e][lane];
        double* dst = slab + (long long)chunk * p.wp + c;
#pragma unroll
        for (int e = 0; e < V; e += 2) *reinterpret_cast<double2*>(dst + e) = make_double2(o[e], o[e + 1]);
    }
}

template <typename T, int MODE, bool NT, int RPT, bool PIPE>
__global__ __launch_bounds__(kThreads) void k_colpass(Params p, const double* __restrict__ vec,
                                                      double* __restrict__ slab, int fixed_block) {
    if (fixed_block < 0 && p.st->done) return;
    BPGL_STAMP_AT(0, 0);
    const int mb = fixed_block >= 0 ? fixed_block : cur_block(p);
    const T* Ab = reinterpret_cast<const T*>(p.A) + (long long)mb * p.block_stride;
    __shared__ double red[kWaves][kU * VecT<T>::N][64];
    colpass_tile<T, MODE, NT, RPT, PIPE>(p, Ab, vec, slab, blockIdx.x % p.nseg, blockIdx.x / p.nseg, red);
    BPGL_STAMP_AT(0, 1);
}

// ---------------------------------------------------------------------------
// colreduce: out[j] = sum_{c < nchunk} slab[c][j]   (fixed order)   -- diag / mtv API
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_colreduce(const double* __restrict__ slab, long long wp,
                                                        int nchunk, double* __restrict__ out,
                                                        double* __restrict__ rec_out) {
    const long long j = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (j >= wp) return;
    double s = 0.0;
    for (int c = 0; c < nchunk; ++c) s += slab[(long long)c * wp + j];
    out[j] = s;
    if (rec_out) rec_out[j] = 1.0 / s;
}

// ---------------------------------------------------------------------------
// shrink (s14/s15 + error criterion), one thread per column of block mb
// ---------------------------------------------------------------------------

// block = 64 columns x 4 waves: wave q sums row chunks q, q+4, ... of the slab
// for its 64 columns, the 4 wave sums are added in a fixed order, wave 0 runs
// the best-response epilogue.  grid = nparts = w_pad / 64.
constexpr int kColsPerShrink = 64;
__global__ __launch_bounds__(kThreads) void k_shrink(Params p) {
    if (p.st->done) return;
    const int mb = cur_block(p);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long j = (long long)blockIdx.x * kColsPerShrink + lane;
    const long long jj = j < p.wp ? j : p.wp - 1;
    // wave 0 issues its epilogue operands (diag, 1/diag, x) with the slab loads
    double d_e = 0.0, rec_e = 0.0, x_e = 0.0;
    if (wave == 0) {
        const long long kx = (long long)mb * p.wp + jj;
        d_e = p.diag[kx];
        rec_e = p.rec[kx];
        x_e = p.x[kx];
    }
    double acc = 0.0;
    {
        int c = wave;
#pragma unroll 4
        for (; c + 3 * kWaves < p.nchunk; c += 4 * kWaves) {
            const double a0 = p.slab_g[(long long)c * p.wp + jj];
            const double a1 = p.slab_g[(long long)(c + kWaves) * p.wp + jj];
            const double a2 = p.slab_g[(long long)(c + 2 * kWaves) * p.wp + jj];
            const double a3 = p.slab_g[(long long)(c + 3 * kWaves) * p.wp + jj];
            acc = (((acc + a0) + a1) + a2) + a3;
        }
        for (; c < p.nchunk; c += kWaves) acc += p.slab_g[(long long)c * p.wp + jj];
    }
    __shared__ double red[kWaves][64];
    red[wave][lane] = acc;
    __syncthreads();
    if (wave != 0) return;
    double abx = 0.0, ax = 0.0, err = 0.0;
    if (j < p.wp) {
        const double g = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
        double Dj = 0.0;
        if (j < p.w) {
            const double d = d_e, xj = x_e;
            const double rx = d * xj - g;                     // lasso.py:114
            const double bx = rec_e * soft_thr(rx, p.mu);     // lasso.py:115-117
            Dj = bx - xj;                                     // lasso.py:119
            abx = fabs(bx);
            ax = fabs(xj);
            err = fabs(g - proj(g - xj, -p.mu, p.mu));        // cpu_calculation.py:15-20
        }
        p.D[j] = Dj;
    }
    abx = wave_sum(abx);
    ax = wave_sum(ax);
    err = wave_max(err);
    if (lane == 0) {
        double* dst = p.parts + 4ll * blockIdx.x;
        dst[0] = abx; dst[1] = ax; dst[2] = err; dst[3] = 0.0;
    }
}

// ---------------------------------------------------------------------------
// rowpass: slab_s[seg][i] = sum_{j in seg} A_b[i][j] * d[j]
// Each wave owns rows wave, wave+4, ... of the chunk, four rows per trip; the
// four per-lane partials are reduced with a transposed butterfly (7 fp64
// shuffles per 4 rows instead of 24): lanes 0/16/32/48 end with rows 0..3.
// ---------------------------------------------------------------------------
// one 16-row group of k_rowpass: rows ib, ib+4, ib+8, ib+12 of this wave
template <typename T, bool NT>
__device__ __forceinline__ void rowpass_group(const T* __restrict__ Ab, long long lda, const long long (&col)[kU],
                                          const double (&dv)[kU][VecT<T>::N], long long ib, long long i1,
                                          double* __restrict__ out, int lane) {
    constexpr int V = VecT<T>::N;
    using raw = typename VecT<T>::raw;
    long long rows[4];
    const T* rp[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rows[k] = ib + k * kWaves;
        rp[k] = Ab + (rows[k] < i1 ? rows[k] : ib) * lda;
    }
    raw a[4][kU];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int u = 0; u < kU; ++u) a[k][u] = ldv<T, NT>(rp[k] + col[u]);
    double ps[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            double v[V];
            VecT<T>::cvt(a[k][u], v);
#pragma unroll
            for (int e = 0; e < V; ++e) s = fma(v[e], dv[u][e], s);
        }
        ps[k] = s;
    }
    // transposed butterfly over the 64 lanes
    const bool up = lane & 32;
    const double k0 = up ? ps[2] : ps[0], k1 = up ? ps[3] : ps[1];
    const double s0 = up ? ps[0] : ps[2], s1 = up ? ps[1] : ps[3];
    const double q0 = k0 + __shfl_xor(s0, 32);
    const double q1 = k1 + __shfl_xor(s1, 32);
    const bool hb = lane & 16;
    double v = (hb ? q1 : q0) + __shfl_xor(hb ? q0 : q1, 16);
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 1);
    if ((lane & 15) == 0) {
        const int k = (up ? 2 : 0) + (hb ? 1 : 0);
        const long long row = ib + k * kWaves;
        if (row < i1) out[row] = v;
    }
}

// one (chunk, seg) tile of the A d pass: the segment's d in registers, the chunk's rows,
// fp64 row partials to out[seg][rows]
template <typename T, bool NT>
__device__ __forceinline__ void rowpass_tile(const Params& p, const T* __restrict__ Ab, const double* __restrict__ d,
                                             double* __restrict__ slab, int seg, int chunk) {
    constexpr int V = VecT<T>::N;
    constexpr int SEGW = 64 * V * kU;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    long long col[kU];
    double dv[kU][V];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const long long c = (long long)seg * SEGW + u * 64 * V + lane * V;
        const bool ok = c < p.wp;
        col[u] = ok ? c : 0;
#pragma unroll
        for (int e = 0; e < V; ++e) dv[u][e] = d[col[u] + e];
#pragma unroll
        for (int e = 0; e < V; ++e) dv[u][e] = ok ? dv[u][e] : 0.0;
    }
    const long long i0 = (long long)chunk * p.R;
    const long long i1 = (i0 + p.R < p.m) ? i0 + p.R : p.m;
    double* out = slab + (long long)seg * p.m;
    // reverse_rows: walk the chunk's 16-row groups bottom-up, so the first rows
    // read are the ones k_colpass (top-down) read last with cache-allocating
    // loads; the groups read last (the top `tail`) are loaded the same way for
    // the next iteration's k_colpass.
    const long long ngroups = (i1 - i0 + 4 * kWaves - 1) / (4 * kWaves);
    const long long glate = NT ? ngroups - (ngroups * p.tail_permille) / 1000 : 0;
    long long gi = 0;
    for (; gi < glate; ++gi) {
        const long long grp = p.reverse_rows ? ngroups - 1 - gi : gi;
        rowpass_group<T, true>(Ab, p.lda, col, dv, i0 + grp * 4 * kWaves + wave, i1, out, lane);
    }
    for (; gi < ngroups; ++gi) {
        const long long grp = p.reverse_rows ? ngroups - 1 - gi : gi;
        rowpass_group<T, false>(Ab, p.lda, col, dv, i0 + grp * 4 * kWaves + wave, i1, out, lane);
    }
}

template <typename T, bool NT>
__global__ __launch_bounds__(kThreads) void k_rowpass(Params p, const double* __restrict__ d,
                                                      double* __restrict__ slab, int fixed_block) {
    if (fixed_block < 0 && p.st->done) return;
    BPGL_STAMP_AT(1, 0);
    const int mb = fixed_block >= 0 ? fixed_block : cur_block(p);
    const T* Ab = reinterpret_cast<const T*>(p.A) + (long long)mb * p.block_stride;
    rowpass_tile<T, NT>(p, Ab, d, slab, blockIdx.x % p.nseg, blockIdx.x / p.nseg);
    BPGL_STAMP_AT(1, 1);
}

// ---------------------------------------------------------------------------
// line search + stopping rule on fully reduced scalars (lasso.py:129-150)
// ---------------------------------------------------------------------------
__device__ void finish_step(const Params& p, double rs, double ss, double l1bx, double l1x, double err) {
    const double r1 = rs + p.mu * (l1bx - l1x);           // lasso.py:129-131
    const double r2 = ss;                                 // lasso.py:132
    const double gamma = (r2 == 0.0) ? 0.0 : proj(-r1 / r2, 0.0, 1.0);   // lasso.py:133-136
    DevState* st = p.st;
    const long long t = st->t;
    const int mb = cur_block(p);
    if (p.err_iter && t < p.rec_len) p.err_iter[t] = err;
    st->r1 = r1;
    st->r2 = r2;
    st->err = err;
    st->t_last = t;
    st->cur_mb = mb;
    if (p.err_bound >= 0.0) {                             // lasso.py:141-150
        if (err < p.err_bound) st->block_cnt += 1;
        if (mb == p.nblock - 1) {
            if (st->block_cnt == p.nblock) {
                st->done = 1;
                st->gamma = 0.0;
                st->iters = t + 1;
                return;
            }
            st->block_cnt = 0;
        }
    }
    st->gamma = gamma;
    st->t = t + 1;
}

// write-through (sc1) accesses of 8-byte scalars: agent-scope relaxed atomics.
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// fold the shrink partials (fixed order) : sum |Bx|, sum |x|, max err
__device__ void fold_parts(const Params& p, int count, double& a, double& b, double& e) {
    __shared__ double sred[3][kWaves];
    a = 0.0; b = 0.0; e = 0.0;
    int k = threadIdx.x;
    for (; k + 3 * kThreads < count; k += 4 * kThreads) {   // 4 partials' loads in flight, adds in order
        double v[4][3];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < 3; ++c) v[u][c] = p.parts[4ll * (k + u * kThreads) + c];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a += v[u][0];
            b += v[u][1];
            e = (v[u][2] > e || v[u][2] != v[u][2]) ? v[u][2] : e;
        }
    }
    for (; k < count; k += kThreads) {
        a += p.parts[4ll * k];
        b += p.parts[4ll * k + 1];
        const double ek = p.parts[4ll * k + 2];
        e = (ek > e || ek != ek) ? ek : e;
    }
    a = wave_sum(a);
    b = wave_sum(b);
    e = wave_max(e);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { sred[0][wave] = a; sred[1][wave] = b; sred[2][wave] = e; }
    __syncthreads();
    a = ((sred[0][0] + sred[0][1]) + sred[0][2]) + sred[0][3];
    b = ((sred[1][0] + sred[1][1]) + sred[1][2]) + sred[1][3];
    e = sred[2][0];
    for (int q = 1; q < kWaves; ++q) e = (sred[2][q] > e || sred[2][q] != sred[2][q]) ? sred[2][q] : e;
}

// ---------------------------------------------------------------------------
// rowreduce: out[i] = sum_{q < nseg} slab_s[q][i].  Block = 64 rows x 4 waves,
// wave w sums segments w, w+4, ... in batches of BATCH loads issued before the
// fixed-order adds; grid-stride over 64-row groups.
//   mode 0 : plain reduction (bpgl_mv API)
//   mode 1 : solver, one rank: also this block's share of r.s23 and s23.s23
//            into parts2[block] (k_linesearch folds them)
//   mode 2 : solver, several ranks: out = this rank's share of s23; block 0
//            adds [sum |Bx|, sum |x|, err slot] for the all-reduce (k_step)
// ---------------------------------------------------------------------------
constexpr int kRowsPerReduce = 64;
constexpr int kMaxReduceBlocks = 2048;
template <int BATCH>
__global__ __launch_bounds__(kThreads) void k_rowreduce(Params p, const double* __restrict__ slab,
                                                        double* __restrict__ out, int mode) {
    if (mode && p.st->done) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ double red[kWaves][64];
    const long long ngroups = (p.m + kRowsPerReduce - 1) / kRowsPerReduce;
    double rs = 0.0, ss = 0.0;
    for (long long grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const long long i = grp * kRowsPerReduce + lane;
        const long long ii = i < p.m ? i : p.m - 1;
        double acc = 0.0;
        for (int q0 = wave; q0 < p.nseg; q0 += BATCH * kWaves) {
            double v[BATCH];
#pragma unroll
            for (int k = 0; k < BATCH; ++k) {
                const int q = q0 + k * kWaves;
                v[k] = slab[(long long)(q < p.nseg ? q : q0) * p.m + ii];
            }
#pragma unroll
            for (int k = 0; k < BATCH; ++k) acc += (q0 + k * kWaves < p.nseg) ? v[k] : 0.0;
        }
        red[wave][lane] = acc;
        __syncthreads();
        if (wave == 0 && i < p.m) {
            const double s = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
            out[i] = s;
            if (mode == 1) {
                rs = fma(p.r[i], s, rs);
                ss = fma(s, s, ss);
            }
        }
        __syncthreads();
    }
    if (mode == 1 && wave == 0) {
        rs = wave_sum(rs);
        ss = wave_sum(ss);
        if (lane == 0) {
            p.parts2[2ll * blockIdx.x] = rs;
            p.parts2[2ll * blockIdx.x + 1] = ss;
        }
    }
    if (mode == 2 && blockIdx.x == 0) {
        double a, b, e;
        fold_parts(p, p.nparts, a, b, e);
        if (threadIdx.x == 0) {
            out[p.m] = a;
            out[p.m + 1] = b;
            for (int r = 0; r < p.nranks; ++r) out[p.m + 2 + r] = (r == p.rank) ? e : 0.0;
        }
    }
}

// ---------------------------------------------------------------------------
// linesearch (one rank): fold the rowreduce and shrink partials in a fixed
// order and run the line search + stopping rule.  One block.
// ---------------------------------------------------------------------------
// `pf` (row shards, fp32 exchange): the summed scalars as hi + lo fp32 pairs [rs_hi, rs_lo,
// ss_hi, ss_lo] instead of the fp64 parts2 partials.
__global__ __launch_bounds__(kThreads) void k_linesearch(Params p, int nblocks_rr, const float* __restrict__ pf) {
    if (p.st->done) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double rs = 0.0, ss = 0.0;
    if (pf) {
        if (threadIdx.x == 0) { rs = (double)pf[0] + (double)pf[1]; ss = (double)pf[2] + (double)pf[3]; }
        nblocks_rr = 0;
    }
#pragma unroll 8
    for (int k = threadIdx.x; k < nblocks_rr; k += kThreads) {
        rs += p.parts2[2ll * k];
        ss += p.parts2[2ll * k + 1];
    }
    __shared__ double sr[kWaves], sq[kWaves];
    rs = wave_sum(rs);
    ss = wave_sum(ss);
    if (lane == 0) { sr[wave] = rs; sq[wave] = ss; }
    __syncthreads();
    rs = ((sr[0] + sr[1]) + sr[2]) + sr[3];
    ss = ((sq[0] + sq[1]) + sq[2]) + sq[3];
    double a, b, e;
    fold_parts(p, p.nparts, a, b, e);
    if (threadIdx.x == 0) finish_step(p, rs, ss, a, b, e);
}

// ---------------------------------------------------------------------------
// step (multi rank): after the all-reduce of [s23 | sum|Bx| | sum|x| | err slots]
// one block of 1024 threads; fixed-order reductions.
// ---------------------------------------------------------------------------
constexpr int kStepThreads = 1024;
__global__ __launch_bounds__(kStepThreads) void k_step(Params p) {
    if (p.st->done) return;
    const double* s23 = p.comm;
    double a = 0.0, b = 0.0;
    for (long long i = threadIdx.x; i < p.m; i += kStepThreads) {
        const double s = s23[i];
        a = fma(p.r[i], s, a);
        b = fma(s, s, b);
    }
    a = wave_sum(a);
    b = wave_sum(b);
    __shared__ double sa[kStepThreads / 64], sb[kStepThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { sa[wave] = a; sb[wave] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double rs = 0.0, ss = 0.0;
        for (int q = 0; q < kStepThreads / 64; ++q) { rs += sa[q]; ss += sb[q]; }
        double err = s23[p.m + 2];
        for (int r = 1; r < p.nranks; ++r) {
            const double e = s23[p.m + 2 + r];
            err = (e > err || e != e) ? e : err;
        }
        finish_step(p, rs, ss, s23[p.m], s23[p.m + 1], err);
    }
}

// ---------------------------------------------------------------------------
// update: x_b += gamma D (lasso.py:153), Ax_b += gamma s23 (lasso.py:155),
// next residual s11 = sum_k Ax_k - b (lasso.py:105)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_update(Params p) {
    if (p.st->done) return;
    const double gamma = p.st->gamma;
    const int mb = (int)p.st->cur_mb;
    const long long n = p.wp > p.m ? p.wp : p.m;
    for (long long k = (long long)blockIdx.x * kThreads + threadIdx.x; k < n;
         k += (long long)gridDim.x * kThreads) {
        if (k < p.w) p.x[(long long)mb * p.wp + k] += gamma * p.D[k];
        if (k < p.m) {
            p.Ax[(long long)mb * p.m + k] += gamma * p.comm[k];
            double acc = p.Ax[k];
            for (int q = 1; q < p.nblock; ++q) acc += p.Ax[(long long)q * p.m + k];
            p.r[k] = acc - p.b[k];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const long long t = p.st->t - 1;
        p.st->iters = t + 1;
        if (p.time_iter && t < p.rec_len)
            p.time_iter[t + 1] = (double)(wall_clock64() - p.st->t_base) * p.wall_tick_s;
    }
}

// residual from scratch: r = sum_k Ax_k - b; state init
__global__ __launch_bounds__(kThreads) void k_reset(Params p) {
    for (long long k = (long long)blockIdx.x * kThreads + threadIdx.x; k < p.m;
         k += (long long)gridDim.x * kThreads) {
        double acc = p.Ax[k];
        for (int q = 1; q < p.nblock; ++q) acc += p.Ax[(long long)q * p.m + k];
        p.r[k] = acc - p.b[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        DevState* st = p.st;
        st->t = 0; st->done = 0; st->block_cnt = 0; st->t_last = -1; st->cur_mb = 0;
        st->gamma = 0.0; st->err = 0.0; st->r1 = 0.0; st->r2 = 0.0; st->iters = 0; st->op_fail = 0;
        st->op_cnt = 0;
        st->op_base = st->op_epoch;
        st->t_base = (long long)wall_clock64();
        if (p.time_iter) p.time_iter[0] = 0.0;
    }
}

}  // namespace bpgl
