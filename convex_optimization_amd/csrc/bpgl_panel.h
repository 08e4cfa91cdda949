// bpgl panel path: k right-hand sides at once (BASELINE configs[4]) with bf16 A
// on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16).
//
// k independent lasso problems share A (m x n, bf16, nblock feature blocks of
// width w); each iteration updates one block for all of them:
//   G   = A_m^T R                       (w x k)   pass 1, MFMA, fused shrink
//   D   = S_mu(diag x - G)/diag - x     per column and RHS (lasso.py:114-119)
//   S   = A_m D                         (m x k)   pass 2, MFMA, split over columns
//   gamma_j = clip(-(r_j.s_j + mu_j(|Bx_j|_1 - |x_j|_1)) / |s_j|^2, 0, 1)   per RHS
//   x_j += gamma_j D_j ;  Ax_j += gamma_j S_j ;  R = sum_b Ax_b - B
//
// Operands.  A is resident twice (row-major A for pass 2, its transpose At for
// pass 1) so each pass loads its MFMA A-operand fragments straight from HBM as
// 16-byte rows -- every A byte is still read once per pass.  R and D enter the
// MFMA as hi + lo bf16 pairs (a ~16-bit mantissa); the direction actually used
// is D' = Dh + Dl, with S = A D' and |x + D'|_1 in the line search, so the exact
// line search of the reference still guarantees descent.  Accumulation: fp32
// inside a block's MFMA chain, fp64 across pass-2 column chunks and in every
// reduction after that.
//
// Tiles.  A wave owns 32 rows of its output (2 MFMA M-tiles of 16) for all k
// RHS (NT = k/16 N-tiles); a block is 4 waves = 128 output rows.  The k-wide
// operand tile of each 32-deep K step (hi and lo) is staged once per block in
// LDS (double-buffered, registers -> LDS) and read with ds_read_b128; the A
// fragments stream from HBM through a PF-deep register ring.
#pragma once
#include <hip/hip_runtime.h>

#include "bpgl_kernels.h"

namespace bpgl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kPanelRows = 128;   // output rows per block (4 waves x 32)
constexpr int kPanelK = 32;       // K depth per MFMA step
constexpr int kPanelPad = 40;     // LDS row length (elements) of a staged K step: 80 B
constexpr int kPanelPF = 4;       // A-fragment prefetch depth (K steps)

struct PanelState {
    long long t;        // next iteration
    long long iters;
    double last_err;
    long long cur_mb;   // block of the iteration being finished (set by k_panel_step)
    long long pad[4];
};

struct PanelParams {
    const __bf16* A;    // [m][lda]   block b at column offset b * w
    const __bf16* At;   // [n][ldt]   block b at row offset b * w
    long long lda, ldt;
    long long m, w;
    int nblock, k;
    int kchunks;        // pass-2 split of the block's w columns
    __bf16* Rh;         // [k][m]
    __bf16* Rl;
    __bf16* Dh;         // [k][w]
    __bf16* Dl;
    float* X;           // [nblock][k][w]
    double* Ax;         // [nblock][k][m]
    const double* B;    // [k][m]
    double* R;          // [k][m]  residual, fp64
    const double* diag; // [nblock][w]
    const double* rec;  // [nblock][w]
    float* Sslab;       // [kchunks][k][m]
    double* S;          // [k][m]
    double* norms;      // [w / kPanelRows][k][4]  pass-1 block partials: sum|Bx|, sum|x|, max err
    double* lsp;        // [m / kLspRows][k][2]    line-search partials: r.s, s.s
    const double* mu;   // [k]
    double* gamma;      // [k]
    double* err_rhs;    // [k]  error criterion of the last iteration, per RHS
    double* err_iter;   // [rec_len] max over RHS per iteration (nullable)
    long long rec_len;
    PanelState* st;
};

constexpr int kLspRows = 1024;    // rows per line-search partial

__device__ __forceinline__ __bf16 to_bf16(float v) { return (__bf16)v; }

// stage one K step of a [k][len] bf16 hi/lo operand pair into LDS buffer `buf`:
// elements [hl][rhs][0..31] <- src_hl[rhs * ld + k0 + 0..31]
template <int NT>
__device__ __forceinline__ void panel_stage_load(const __bf16* __restrict__ hi, const __bf16* __restrict__ lo,
                                                 long long ld, long long k0, uint4 (&regs)[NT]) {
    // 2 (hi/lo) x k rows x 4 sixteen-byte parts = 8k chunks; 256 threads -> NT chunks each (k = 16 NT)
#pragma unroll
    for (int s = 0; s < NT; ++s) {
        const int c = threadIdx.x + kThreads * s;
        const int hl = c / (64 * NT);
        const int rem = c % (64 * NT);
        const int rhs = rem >> 2, part = rem & 3;
        const __bf16* src = (hl ? lo : hi) + (long long)rhs * ld + k0 + part * 8;
        regs[s] = *reinterpret_cast<const uint4*>(src);
    }
}
template <int NT>
__device__ __forceinline__ void panel_stage_store(__bf16* lds, int buf, const uint4 (&regs)[NT]) {
#pragma unroll
    for (int s = 0; s < NT; ++s) {
        const int c = threadIdx.x + kThreads * s;
        const int hl = c / (64 * NT);
        const int rem = c % (64 * NT);
        const int rhs = rem >> 2, part = rem & 3;
        __bf16* dst = lds + ((long long)((buf * 2 + hl) * (16 * NT) + rhs)) * kPanelPad + part * 8;
        *reinterpret_cast<uint4*>(dst) = regs[s];
    }
}
// B fragment (16x16x32 layout: lane l holds B[k = 8(l>>4)+j][n = l&15])
template <int NT>
__device__ __forceinline__ bf16x8 panel_bfrag(const __bf16* lds, int buf, int hl, int nt, int lane) {
    const __bf16* p = lds + ((long long)((buf * 2 + hl) * (16 * NT) + nt * 16 + (lane & 15))) * kPanelPad +
                      8 * (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(p);
}

// One block-tile GEMM: acc[mt][nt] (rows = this wave's 32 output rows, cols = k RHS)
//   = sum over K steps s of  Arows[row][K0 + 32 s + ...] . (Bh + Bl)[rhs][K0 + 32 s + ...]
// Arows: row-major bf16 operand whose row `r` starts at arow_base + r * ldarow.
template <int NT>
__device__ __forceinline__ void panel_gemm(const __bf16* __restrict__ arow_base, long long ldarow,
                                           const __bf16* __restrict__ bh, const __bf16* __restrict__ bl,
                                           long long ldb, long long K0, int nsteps, __bf16* lds,
                                           f32x4 (&acc)[2][NT]) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // A fragment of M-tile mt at step s: row (wave*32 + mt*16 + (lane&15)), K (K0 + 32 s + 8(lane>>4))
    const __bf16* ap[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
        ap[mt] = arow_base + (long long)(wave * 32 + mt * 16 + (lane & 15)) * ldarow + K0 + 8 * (lane >> 4);
    bf16x8 ring[kPanelPF][2];
#pragma unroll
    for (int u = 0; u < kPanelPF; ++u)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) ring[u][mt] = *reinterpret_cast<const bf16x8*>(ap[mt] + u * kPanelK);
    uint4 stage[NT];
    panel_stage_load<NT>(bh, bl, ldb, K0, stage);
    panel_stage_store<NT>(lds, 0, stage);
    __syncthreads();
    for (int s0 = 0; s0 < nsteps; s0 += kPanelPF) {
#pragma unroll
        for (int u = 0; u < kPanelPF; ++u) {
            const int s = s0 + u;
            const int buf = u & 1;               // kPanelPF even: parity of s
            // stage the next step (the last step re-stages itself: no branch around the loads)
            const int snext = (s + 1 < nsteps) ? s + 1 : s;
            panel_stage_load<NT>(bh, bl, ldb, K0 + (long long)snext * kPanelK, stage);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const bf16x8 b_hi = panel_bfrag<NT>(lds, buf, 0, nt, lane);
                const bf16x8 b_lo = panel_bfrag<NT>(lds, buf, 1, nt, lane);
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[u][mt], b_hi, acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[u][mt], b_lo, acc[mt][nt], 0, 0, 0);
                }
            }
            {
                const int sr = (s + kPanelPF < nsteps) ? s + kPanelPF : s;   // clamp: no branch around loads
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
                    ring[u][mt] = *reinterpret_cast<const bf16x8*>(ap[mt] + (long long)sr * kPanelK);
            }
            panel_stage_store<NT>(lds, buf ^ 1, stage);
            __syncthreads();
        }
    }
}

__device__ __forceinline__ void split_bf16(double v, __bf16& hi, __bf16& lo) {
    const float f = (float)v;
    hi = to_bf16(f);
    lo = to_bf16((float)(v - (double)(float)hi));
}

// ---------------------------------------------------------------------------
// pass 1: G = A_m^T R (EPI 0: write G [k][w] fp64 -- API), or the fused shrink
// epilogue (EPI 1: D' split, norms per RHS).  grid = w / 128 blocks of 256.
// ---------------------------------------------------------------------------
template <int NT, int EPI>
__global__ __launch_bounds__(kThreads) void k_panel_pass1(PanelParams p, int fixed_block, double* __restrict__ Gout) {
    __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 2 * 16 * NT * kPanelPad];
    const int mb = fixed_block >= 0 ? fixed_block : (int)(p.st->t % p.nblock);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long c0 = (long long)blockIdx.x * kPanelRows;             // first column of this block
    const __bf16* arow = p.At + ((long long)mb * p.w + c0) * p.ldt;      // At rows = A columns
    f32x4 acc[2][NT];
    panel_gemm<NT>(arow, p.ldt, p.Rh, p.Rl, p.m, 0, (int)(p.m / kPanelK), lds, acc);

    // C layout: row = (lane>>4)*4 + r (A column), col = lane & 15 (RHS)
    if (EPI == 0) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int rhs = nt * 16 + (lane & 15);
                const long long j = c0 + wave * 32 + mt * 16 + (lane >> 4) * 4;
#pragma unroll
                for (int r = 0; r < 4; ++r) Gout[(long long)rhs * p.w + j + r] = (double)acc[mt][nt][r];
            }
        return;
    }
    __shared__ double nred[kWaves][16 * NT][3];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int rhs = nt * 16 + (lane & 15);
        const double mu = p.mu[rhs];
        double sbx = 0.0, sx = 0.0, err = 0.0;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const long long j = c0 + wave * 32 + mt * 16 + (lane >> 4) * 4;   // 4 consecutive columns
            float* xp = p.X + ((long long)mb * p.k + rhs) * p.w + j;
            const float4 x4 = *reinterpret_cast<const float4*>(xp);
            const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
            __bf16 dh[4], dl[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double g = (double)acc[mt][nt][r];
                const double x = (double)xs[r];
                const long long kx = (long long)mb * p.w + j + r;
                const double bx = p.rec[kx] * soft_thr(p.diag[kx] * x - g, mu);
                split_bf16(bx - x, dh[r], dl[r]);
                const double dprime = (double)(float)dh[r] + (double)(float)dl[r];
                sbx += fabs(x + dprime);
                sx += fabs(x);
                const double e = fabs(g - proj(g - x, -mu, mu));
                err = (e > err || e != e) ? e : err;
            }
            __bf16* dhp = p.Dh + (long long)rhs * p.w + j;
            __bf16* dlp = p.Dl + (long long)rhs * p.w + j;
#pragma unroll
            for (int r = 0; r < 4; ++r) { dhp[r] = dh[r]; dlp[r] = dl[r]; }
        }
        // lanes l, l^16, l^32, l^48 share the RHS
        sbx += __shfl_xor(sbx, 16); sbx += __shfl_xor(sbx, 32);
        sx += __shfl_xor(sx, 16);   sx += __shfl_xor(sx, 32);
        { double o = __shfl_xor(err, 16); err = (o > err || o != o) ? o : err;
          o = __shfl_xor(err, 32); err = (o > err || o != o) ? o : err; }
        if (lane < 16) {
            nred[wave][rhs][0] = sbx;
            nred[wave][rhs][1] = sx;
            nred[wave][rhs][2] = err;
        }
    }
    __syncthreads();
    for (int rhs = threadIdx.x; rhs < 16 * NT; rhs += kThreads) {
        double a = 0.0, b = 0.0, e = 0.0;
        for (int q = 0; q < kWaves; ++q) {
            a += nred[q][rhs][0];
            b += nred[q][rhs][1];
            const double eq = nred[q][rhs][2];
            e = (eq > e || eq != eq) ? eq : e;
        }
        double* dst = p.norms + ((long long)blockIdx.x * p.k + rhs) * 4;
        dst[0] = a; dst[1] = b; dst[2] = e; dst[3] = 0.0;
    }
}

// ---------------------------------------------------------------------------
// pass 2: partial S over one column chunk: Sslab[chunk][rhs][row]
// grid = (m / 128) x kchunks
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(kThreads) void k_panel_pass2(PanelParams p, int fixed_block) {
    __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 2 * 16 * NT * kPanelPad];
    const int mb = fixed_block >= 0 ? fixed_block : (int)(p.st->t % p.nblock);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rb = blockIdx.x % (int)(p.m / kPanelRows);
    const int chunk = blockIdx.x / (int)(p.m / kPanelRows);
    const long long kc = p.w / p.kchunks;
    const long long r0 = (long long)rb * kPanelRows;
    const __bf16* arow = p.A + r0 * p.lda + (long long)mb * p.w;        // A rows, block mb columns
    f32x4 acc[2][NT];
    panel_gemm<NT>(arow, p.lda, p.Dh, p.Dl, p.w, chunk * kc, (int)(kc / kPanelK), lds, acc);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int rhs = nt * 16 + (lane & 15);
            const long long row = r0 + wave * 32 + mt * 16 + (lane >> 4) * 4;
            float* dst = p.Sslab + ((long long)chunk * p.k + rhs) * p.m + row;
            *reinterpret_cast<float4*>(dst) = make_float4(acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2],
                                                          acc[mt][nt][3]);
        }
}

// S = sum over chunks (fp64, fixed order); line-search partials per RHS and
// 1024-row group (mode 1), or plain output (mode 0, API).  grid = k x (m / 1024)
__global__ __launch_bounds__(kThreads) void k_panel_reduce(PanelParams p, double* __restrict__ Sout, int mode) {
    const int rhs = blockIdx.x % p.k;
    const int grp = blockIdx.x / p.k;
    const long long i0 = (long long)grp * kLspRows;
    double rs = 0.0, ss = 0.0;
    for (long long i = i0 + threadIdx.x; i < i0 + kLspRows && i < p.m; i += kThreads) {
        double s = 0.0;
        for (int c = 0; c < p.kchunks; ++c) s += (double)p.Sslab[((long long)c * p.k + rhs) * p.m + i];
        Sout[(long long)rhs * p.m + i] = s;
        if (mode) {
            rs = fma(p.R[(long long)rhs * p.m + i], s, rs);
            ss = fma(s, s, ss);
        }
    }
    if (!mode) return;
    __shared__ double sr[kWaves], sq[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    rs = wave_sum(rs);
    ss = wave_sum(ss);
    if (lane == 0) { sr[wave] = rs; sq[wave] = ss; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double* dst = p.lsp + ((long long)grp * p.k + rhs) * 2;
        dst[0] = ((sr[0] + sr[1]) + sr[2]) + sr[3];
        dst[1] = ((sq[0] + sq[1]) + sq[2]) + sq[3];
    }
}

// per-RHS line search: one block per RHS
__global__ __launch_bounds__(kThreads) void k_panel_step(PanelParams p) {
    const int rhs = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb1 = (int)(p.w / kPanelRows);
    double a = 0.0, b = 0.0, e = 0.0;
    for (int q = threadIdx.x; q < nb1; q += kThreads) {
        const double* src = p.norms + ((long long)q * p.k + rhs) * 4;
        a += src[0];
        b += src[1];
        e = (src[2] > e || src[2] != src[2]) ? src[2] : e;
    }
    __shared__ double s3[3][kWaves];
    a = wave_sum(a);
    b = wave_sum(b);
    e = wave_max(e);
    if (lane == 0) { s3[0][wave] = a; s3[1][wave] = b; s3[2][wave] = e; }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = ((s3[0][0] + s3[0][1]) + s3[0][2]) + s3[0][3];
        b = ((s3[1][0] + s3[1][1]) + s3[1][2]) + s3[1][3];
        e = s3[2][0];
        for (int q = 1; q < kWaves; ++q) e = (s3[2][q] > e || s3[2][q] != s3[2][q]) ? s3[2][q] : e;
        double rs = 0.0, ss = 0.0;
        const int ng = (int)((p.m + kLspRows - 1) / kLspRows);
        for (int g = 0; g < ng; ++g) {
            rs += p.lsp[((long long)g * p.k + rhs) * 2];
            ss += p.lsp[((long long)g * p.k + rhs) * 2 + 1];
        }
        const double r1 = rs + p.mu[rhs] * (a - b);
        p.gamma[rhs] = (ss == 0.0) ? 0.0 : proj(-r1 / ss, 0.0, 1.0);
        p.err_rhs[rhs] = e;
        if (rhs == 0) p.st->cur_mb = p.st->t % p.nblock;   // nobody else reads it in this launch
    }
}

// x_j += gamma_j D'_j ; Ax_j += gamma_j S_j ; R = sum_b Ax_b - B ; split R.
// One thread per element of the larger of [k][w] and [k][m]; also bumps t.
__global__ __launch_bounds__(kThreads) void k_panel_update(PanelParams p) {
    const int mb = (int)p.st->cur_mb;   // p.st->t is advanced by block 0 of this launch
    const long long nx = (long long)p.k * p.w, nr = (long long)p.k * p.m;
    const long long n = nx > nr ? nx : nr;
    for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < n; e += (long long)gridDim.x * kThreads) {
        if (e < nx) {
            const int rhs = (int)(e / p.w);
            const double dp = (double)(float)p.Dh[e] + (double)(float)p.Dl[e];
            float* xp = p.X + (long long)mb * nx + e;
            *xp = (float)((double)*xp + p.gamma[rhs] * dp);
        }
        if (e < nr) {
            const int rhs = (int)(e / p.m);
            double* ap = p.Ax + (long long)mb * nr + e;
            *ap += p.gamma[rhs] * p.S[e];
            double acc = p.Ax[e];
            for (int q = 1; q < p.nblock; ++q) acc += p.Ax[(long long)q * nr + e];
            const double r = acc - p.B[e];
            p.R[e] = r;
            split_bf16(r, p.Rh[e], p.Rl[e]);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const long long t = p.st->t;
        double emax = 0.0;
        for (int j = 0; j < p.k; ++j) emax = (p.err_rhs[j] > emax || p.err_rhs[j] != p.err_rhs[j]) ? p.err_rhs[j] : emax;
        if (p.err_iter && t < p.rec_len) p.err_iter[t] = emax;
        p.st->last_err = emax;
        p.st->t = t + 1;
        p.st->iters = t + 1;
    }
}

// split an fp64 [k][len] operand into hi/lo bf16; optionally R = -B (reset)
__global__ __launch_bounds__(kThreads) void k_panel_split(const double* __restrict__ src, long long n,
                                                          __bf16* __restrict__ hi, __bf16* __restrict__ lo,
                                                          double sign, double* __restrict__ copy) {
    for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < n; e += (long long)gridDim.x * kThreads) {
        const double v = sign * src[e];
        if (copy) copy[e] = v;
        split_bf16(v, hi[e], lo[e]);
    }
}

// diag(A_b^T A_b) from At rows: one wave per column
__global__ __launch_bounds__(kThreads) void k_panel_diag(PanelParams p, double* __restrict__ diag,
                                                         double* __restrict__ rec) {
    const int lane = threadIdx.x & 63;
    const long long col = (long long)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (col >= (long long)p.nblock * p.w) return;
    const __bf16* row = p.At + col * p.ldt;
    double acc = 0.0;
    for (long long i = lane; i < p.m; i += 64) {
        const double v = (double)(float)row[i];
        acc = fma(v, v, acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) {
        diag[col] = acc;
        rec[col] = 1.0 / acc;
    }
}

__global__ void k_panel_reset_state(PanelParams p) {
    if (threadIdx.x == 0) {
        p.st->t = 0;
        p.st->iters = 0;
        p.st->last_err = 0.0;
        p.st->cur_mb = 0;
    }
}

}  // namespace bpgl
