// bpgl fused solver iteration: two launches per block update (one rank), or
// two launches + RCCL all-reduce + k_step (column-sharded ranks).
//
//   k_iter_a  = k_colpass over every (row chunk, column segment) tile, with
//               the previous iteration's update applied on the fly, and the
//               shrink (lasso.py:114-119) run by the LAST block to finish
//               each column segment over that segment's columns.
//   k_iter_b  = k_rowpass over every tile; the LAST block of each row chunk
//               sums that chunk's rows (s23), applies the previous update to
//               Ax, and forms its share of r.s23 and s23.s23; the last of those
//               runs the line search and the stopping rule (lasso.py:129-150).
//   k_finalize applies the pending update at the end of a batch of iterations.
//
// Deferred update.  Iteration t ends with gamma_t known but x_m, Ax_m not yet
// updated ("pending").  Iteration t+1 applies it where it needs it:
//   * residual   s11_{t+1,i} = sum_k Ax_k,i - b_i with Ax_{m_t} + gamma_t s23_t,
//                computed per row by every k_iter_a wave that reads row i, and
//                stored once (column segment 0) for k_iter_b;
//   * Ax_{m_t}   updated by the row-chunk finishers of k_iter_b(t+1), each for
//                its own rows, before s23 is overwritten with s23_{t+1};
//   * x_{m_t}    updated by the segment finishers of k_iter_a(t+1) when
//                m_{t+1} == m_t (they read x there), else by all k_iter_a
//                blocks, a slice each, from the parity-(t & 1) copy of D.
// The arithmetic is the reference's (x += gamma D; Ax_m += gamma s23; s11 =
// sum_k Ax_k - b); only where it happens moves.
//
// Inter-workgroup hand-offs (MI355X_MICROARCH.md "Valid forms", row 1): the
// split-K partials are stored write-through (agent-scope relaxed atomic
// stores = sc1), every storing wave drains with s_waitcnt vmcnt(0), the block
// barriers, ONE lane adds to the arrival counter (agent scope); the block whose
// add completes a multiple of the expected count reads the partials with sc1
// loads only.  Counters are monotonic (never reset) and every launch adds the
// same count to each, so "last" = (old + 1) % expected == 0.
#pragma once
#include "bpgl_kernels.h"


namespace bpgl {

// every storing wave drains, block barrier, one lane arrives; true in every
// thread of the block that completed the count.
__device__ __forceinline__ bool arrive_last(unsigned long long* cnt, unsigned long long expected) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long old = __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = ((old + 1) % expected) == 0;
    }
    __syncthreads();
    return last != 0;
}

// The residual entry s11_i the current iteration sees (lasso.py:105), with the
// pending update of the previous iteration folded in (lasso.py:155).
struct Resid {
    const double* Ax;
    const double* s23;
    const double* b;
    double* rout;       // non-null in one block per row chunk: store s11 once
    long long m;
    int nblock, mbp, pend, lane;
    double gp;
    __device__ __forceinline__ double operator()(long long i) const {
        double acc = 0.0;
        for (int k = 0; k < nblock; ++k) {
            double a = Ax[(long long)k * m + i];
            if (pend && k == mbp) a += gp * s23[i];
            acc = (k == 0) ? a : acc + a;
        }
        const double r = acc - b[i];
        if (rout && lane == 0) rout[i] = r;
        return r;
    }
};

// rows [i, istop) of one wave, A^T s11 with s11 from `f`
template <typename T, bool NT, typename F>
__device__ __forceinline__ void colpass_span_f(const T* __restrict__ Ab, long long lda, const long long (&col)[kU],
                                               const F& f, long long& i, long long istop, long long i1,
                                               double (&acc)[kU][VecT<T>::N]) {
    constexpr int V = VecT<T>::N;
    using raw = typename VecT<T>::raw;
    for (; i < istop; i += 2 * kWaves) {
        const bool two = i + kWaves < i1;
        const long long i2 = two ? i + kWaves : i;
        const T* r0 = Ab + i * lda;
        const T* r1 = Ab + i2 * lda;
        raw a0[kU], a1[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) a0[u] = ldv<T, NT>(r0 + col[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) a1[u] = ldv<T, NT>(r1 + col[u]);
        const double s0 = f(i);
        double s1 = f(i2);              // i2 == i when !two: in bounds, no branch around loads
        s1 = two ? s1 : 0.0;
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            double v0[V], v1[V];
            VecT<T>::cvt(a0[u], v0);
            VecT<T>::cvt(a1[u], v1);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                acc[u][e] = fma(v0[e], s0, acc[u][e]);
                acc[u][e] = fma(v1[e], s1, acc[u][e]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_iter_a: A^T s11 tiles + segment finishers (shrink)
// ---------------------------------------------------------------------------
template <typename T, bool NT>
__global__ __launch_bounds__(kThreads) void k_iter_a(Params p) {
    constexpr int V = VecT<T>::N;
    constexpr int SEGW = 64 * V * kU;
    if (p.st->done) return;
    const long long t = p.st->t;
    const int mb = cur_block(p);
    const int pend = (int)p.st->pending;
    const int mbp = (int)p.st->cur_mb;
    const double gp = p.st->gamma;
    const double* Dprev = p.Dbuf + ((t + 1) & 1) * p.wp;    // direction of iteration t-1
    double* Dcur = p.Dbuf + (t & 1) * p.wp;
    const int seg = blockIdx.x % p.nseg;
    const int chunk = blockIdx.x / p.nseg;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const T* Ab = reinterpret_cast<const T*>(p.A) + (long long)mb * p.block_stride;

    // pending x update of a different block: spread over all blocks
    if (pend && mbp != mb) {
        for (long long j = (long long)blockIdx.x * kThreads + threadIdx.x; j < p.w;
             j += (long long)gridDim.x * kThreads)
            p.x[(long long)mbp * p.wp + j] += gp * Dprev[j];
    }

    long long col[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const long long c = (long long)seg * SEGW + u * 64 * V + lane * V;
        col[u] = c < p.wp ? c : 0;
    }
    double acc[kU][V];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[u][e] = 0.0;

    const Resid f{p.Ax, p.comm, p.b, seg == 0 ? p.r : nullptr, p.m, p.nblock, mbp, pend, lane, gp};
    const long long i0 = (long long)chunk * p.R;
    const long long i1 = (i0 + p.R < p.m) ? i0 + p.R : p.m;
    long long i = i0 + wave;
    if (NT) {
        const long long isplit = i1 - ((i1 - i0) * p.tail_permille) / 1000;
        colpass_span_f<T, true>(Ab, p.lda, col, f, i, isplit, i1, acc);
    }
    colpass_span_f<T, false>(Ab, p.lda, col, f, i, i1, i1, acc);

    // fixed-order combine of the 4 waves, then a write-through slab row
    __shared__ double red[kWaves][kU * V][64];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) red[wave][u * V + e][lane] = acc[u][e];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rslab = rsrc(p.slab_g, 8ll * p.nchunk * p.wp);
    {
        const int q = wave;
        const long long c = (long long)seg * SEGW + q * 64 * V + lane * V;
        if (c < p.wp) {
            double o[V];
#pragma unroll
            for (int e = 0; e < V; ++e)
                o[e] = ((red[0][q * V + e][lane] + red[1][q * V + e][lane]) + red[2][q * V + e][lane]) +
                       red[3][q * V + e][lane];
            const long long off = 8 * ((long long)chunk * p.wp + c);
#pragma unroll
            for (int e = 0; e < V; e += 2) bst2_sc1(rslab, off + 8 * e, o[e], o[e + 1]);
        }
    }
    if (!arrive_last(p.cnt_seg + seg, (unsigned long long)p.nchunk)) return;

    // ---- segment finisher: g, best response, D, norms, error (lasso.py:114-119)
    // thread k owns the V columns seg * SEGW + k * V ... + V - 1
    double abx = 0.0, ax = 0.0, err = 0.0;
    const long long j0 = (long long)seg * SEGW + threadIdx.x * V;
    if (j0 < p.wp) {
        double g[V];
#pragma unroll
        for (int e = 0; e < V; ++e) g[e] = 0.0;
        for (int c = 0; c < p.nchunk; ++c) {
            const long long off = 8 * ((long long)c * p.wp + j0);
#pragma unroll
            for (int e = 0; e < V; e += 2) {
                double a0, a1;
                bld2_sc1(rslab, off + 8 * e, a0, a1);
                g[e] += a0;
                g[e + 1] += a1;
            }
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const long long j = j0 + e;
            p.g[j] = g[e];
            double Dj = 0.0;
            if (j < p.w) {
                const long long kx = (long long)mb * p.wp + j;
                double xj = p.x[kx];
                if (pend && mbp == mb) {                       // lasso.py:153 of the previous iteration
                    xj += gp * Dprev[j];
                    p.x[kx] = xj;
                }
                const double rx = p.diag[kx] * xj - g[e];       // lasso.py:114
                const double bx = p.rec[kx] * soft_thr(rx, p.mu);   // lasso.py:115-117
                Dj = bx - xj;                                   // lasso.py:119
                abx += fabs(bx);
                ax += fabs(xj);
                const double ee = fabs(g[e] - proj(g[e] - xj, -p.mu, p.mu));   // cpu_calculation.py:15-20
                err = (ee > err || ee != ee) ? ee : err;
            }
            Dcur[j] = Dj;
        }
    }
    __shared__ double sred[3][kWaves];
    abx = wave_sum(abx);
    ax = wave_sum(ax);
    err = wave_max(err);
    if (lane == 0) { sred[0][wave] = abx; sred[1][wave] = ax; sred[2][wave] = err; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double e = sred[2][0];
        for (int q = 1; q < kWaves; ++q) e = (sred[2][q] > e || sred[2][q] != sred[2][q]) ? sred[2][q] : e;
        double* dst = p.parts + 4ll * seg;
        dst[0] = ((sred[0][0] + sred[0][1]) + sred[0][2]) + sred[0][3];
        dst[1] = ((sred[1][0] + sred[1][1]) + sred[1][2]) + sred[1][3];
        dst[2] = e;
        dst[3] = 0.0;
    }
}

// one 16-row group of the A D pass, partials stored write-through
template <typename T, bool NT>
__device__ __forceinline__ void rowpass_group_sc1(const T* __restrict__ Ab, long long lda, const long long (&col)[kU],
                                                  const double (&dv)[kU][VecT<T>::N], long long ib, long long i1,
                                                  __amdgpu_buffer_rsrc_t rout, long long out_off, int lane) {
    constexpr int V = VecT<T>::N;
    using raw = typename VecT<T>::raw;
    const T* rp[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const long long row = ib + k * kWaves;
        rp[k] = Ab + (row < i1 ? row : ib) * lda;
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
        if (row < i1) bst1_sc1(rout, 8 * (out_off + row), v);
    }
}

// ---------------------------------------------------------------------------
// k_iter_b: A D tiles + row-chunk finishers + (one rank) the line search
// ---------------------------------------------------------------------------
template <typename T, bool NT>
__global__ __launch_bounds__(kThreads) void k_iter_b(Params p) {
    constexpr int V = VecT<T>::N;
    constexpr int SEGW = 64 * V * kU;
    if (p.st->done) return;
    const long long t = p.st->t;
    const int pend = (int)p.st->pending;
    const int mbp = (int)p.st->cur_mb;
    const double gp = p.st->gamma;
    const int mb = cur_block(p);
    const double* d = p.Dbuf + (t & 1) * p.wp;
    const int seg = blockIdx.x % p.nseg;
    const int chunk = blockIdx.x / p.nseg;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const T* Ab = reinterpret_cast<const T*>(p.A) + (long long)mb * p.block_stride;

    long long col[kU];
    double dv[kU][V];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const long long c = (long long)seg * SEGW + u * 64 * V + lane * V;
        const bool ok = c < p.wp;
        col[u] = ok ? c : 0;
#pragma unroll
        for (int e = 0; e < V; ++e) dv[u][e] = ok ? d[col[u] + e] : 0.0;
    }
    const long long i0 = (long long)chunk * p.R;
    const long long i1 = (i0 + p.R < p.m) ? i0 + p.R : p.m;
    const __amdgpu_buffer_rsrc_t rslab = rsrc(p.slab_s, 8ll * p.nseg * p.m);
    const long long out_off = (long long)seg * p.m;
    const long long ngroups = (i1 - i0 + 4 * kWaves - 1) / (4 * kWaves);
    const long long glate = NT ? ngroups - (ngroups * p.tail_permille) / 1000 : 0;
    long long gi = 0;
    for (; gi < glate; ++gi) {
        const long long grp = p.reverse_rows ? ngroups - 1 - gi : gi;
        rowpass_group_sc1<T, true>(Ab, p.lda, col, dv, i0 + grp * 4 * kWaves + wave, i1, rslab, out_off, lane);
    }
    for (; gi < ngroups; ++gi) {
        const long long grp = p.reverse_rows ? ngroups - 1 - gi : gi;
        rowpass_group_sc1<T, false>(Ab, p.lda, col, dv, i0 + grp * 4 * kWaves + wave, i1, rslab, out_off, lane);
    }
    if (!arrive_last(p.cnt_chunk + chunk, (unsigned long long)p.nseg)) return;

    // ---- row-chunk finisher: s23 rows, pending Ax update, r.s23 / s23.s23 shares
    const bool multi = p.nranks > 1 || p.has_comm;   // the exchange + k_step_fused finish the step
    double rs = 0.0, ss = 0.0;
    for (long long i = i0 + threadIdx.x; i < i1; i += kThreads) {
        double s = 0.0;
        for (int q = 0; q < p.nseg; ++q) s += bld1_sc1(rslab, 8 * ((long long)q * p.m + i));
        if (pend) p.Ax[(long long)mbp * p.m + i] += gp * p.comm[i];    // lasso.py:155, iteration t-1
        p.comm[i] = s;                  // one rank: s23; several: this rank's share, all-reduced next
        if (!multi) {
            rs = fma(p.r[i], s, rs);
            ss = fma(s, s, ss);
        }
    }
    const unsigned long long nfin = (unsigned long long)p.nchunk;
    if (multi) {
        // the last chunk finisher adds the norms and this rank's error slot
        if (!arrive_last(&p.st->cnt_all, nfin)) return;
        double a, b, e;
        fold_parts(p, p.nseg, a, b, e);
        if (threadIdx.x == 0) {
            p.comm[p.m] = a;
            p.comm[p.m + 1] = b;
            for (int r = 0; r < p.nranks; ++r) p.comm[p.m + 2 + r] = (r == p.rank) ? e : 0.0;
        }
        return;
    }
    __shared__ double sr[kWaves], sq[kWaves];
    rs = wave_sum(rs);
    ss = wave_sum(ss);
    if (lane == 0) { sr[wave] = rs; sq[wave] = ss; }
    __syncthreads();
    if (threadIdx.x == 0) {
        st_sc1(p.parts2 + 2ll * chunk, ((sr[0] + sr[1]) + sr[2]) + sr[3]);
        st_sc1(p.parts2 + 2ll * chunk + 1, ((sq[0] + sq[1]) + sq[2]) + sq[3]);
    }
    if (!arrive_last(&p.st->cnt_all, nfin)) return;

    // ---- last finisher: line search + stopping rule (lasso.py:129-150)
    double a, b, e;
    fold_parts(p, p.nseg, a, b, e);
    if (threadIdx.x == 0) {
        double r1 = 0.0, r2 = 0.0;
        for (int c = 0; c < p.nchunk; ++c) {
            r1 += ld_sc1(p.parts2 + 2ll * c);
            r2 += ld_sc1(p.parts2 + 2ll * c + 1);
        }
        finish_step(p, r1, r2, a, b, e);
        p.st->pending = p.st->done ? 0 : 1;
        if (p.time_iter && t < p.rec_len)
            p.time_iter[t + 1] = (double)(wall_clock64() - p.st->t_base) * p.wall_tick_s;
        p.st->iters = p.st->done ? p.st->iters : t + 1;
    }
}

// k_step for the fused multi-rank path: after the all-reduce; sets pending
__global__ __launch_bounds__(kStepThreads) void k_step_fused(Params p) {
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
        const long long t = p.st->t;
        finish_step(p, rs, ss, s23[p.m], s23[p.m + 1], err);
        p.st->pending = p.st->done ? 0 : 1;
        if (p.time_iter && t < p.rec_len)
            p.time_iter[t + 1] = (double)(wall_clock64() - p.st->t_base) * p.wall_tick_s;
        p.st->iters = p.st->done ? p.st->iters : t + 1;
    }
}

// apply the pending update (end of a batch): x_m += gamma D, Ax_m += gamma s23,
// s11 = sum_k Ax_k - b.  Reads the state words only; `pending` is cleared by
// the last block to finish (agent counter in cnt_all is not used: a separate
// one-block clear kernel follows).
__global__ __launch_bounds__(kThreads) void k_finalize(Params p) {
    if (!p.st->pending) return;
    const double gamma = p.st->gamma;
    const int mb = (int)p.st->cur_mb;
    const long long t = p.st->t;                      // iteration t-1 is the pending one
    const double* D = p.Dbuf + ((t + 1) & 1) * p.wp;
    const long long n = p.wp > p.m ? p.wp : p.m;
    for (long long k = (long long)blockIdx.x * kThreads + threadIdx.x; k < n;
         k += (long long)gridDim.x * kThreads) {
        if (k < p.w) p.x[(long long)mb * p.wp + k] += gamma * D[k];
        if (k < p.m) {
            p.Ax[(long long)mb * p.m + k] += gamma * p.comm[k];
            double acc = p.Ax[k];
            for (int q = 1; q < p.nblock; ++q) acc += p.Ax[(long long)q * p.m + k];
            p.r[k] = acc - p.b[k];
        }
    }
}
__global__ void k_clear_pending(Params p) {
    if (threadIdx.x == 0) p.st->pending = 0;
}

}  // namespace bpgl
