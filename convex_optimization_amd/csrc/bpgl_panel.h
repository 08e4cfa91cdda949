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
// Operands.  A is resident once, row-major bf16; every A byte is read once per
// pass.  R enters the MFMA as a hi + lo bf16 pair (a ~16-bit mantissa).  The
// direction enters as the same pair (NS = 2) or as its bf16 rounding alone
// (NS = 1, the solver's "d_split" knob): either way the direction actually used
// is the D' the MFMA sees, with S = A D' and |x + D'|_1 in the line search, so the
// exact line search of the reference is exact along the direction taken and
// still guarantees descent.  Accumulation: fp32 inside a block's MFMA chain, fp64
// across pass-2 column chunks and in every reduction after that.
//
// Tiles.  A block owns 256 output rows x all k RHS: 4 (M) x WN (N) waves, each
// 64 rows (4 MFMA M-tiles) x k/WN RHS.  K advances 64 per stage.  Both operand
// tiles of a stage travel HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4,
// full 128-B lines, XOR-swizzled through the source address); the A side is
// triple-buffered (two stages in flight), the k-wide side double-buffered, and
// one raw s_barrier per stage orders both (counted vmcnt, never 0 in the loop).
// Only row-major A is resident: pass 2 reads A fragments with ds_read_b128,
// pass 1 (which needs A^T) reads the same kind of image with the CDNA4
// transposing ds_read_b64_tr_b16.
#pragma once
#include <hip/hip_runtime.h>

#include "bpgl_device.h"

namespace bpgl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kPanelRows = 256;   // output rows per block (pass 1: A columns, pass 2: A rows)
constexpr int kPanelK = 64;       // K depth per stage
constexpr int kPanelNA = 3;       // A-side stage buffers (two stages in flight)
constexpr int kPanelNO = 2;       // k-wide-side stage buffers
constexpr int kPanelAStage = kPanelRows * kPanelK * 2;   // 32 KiB

// NS: bf16 pieces of the k-wide operand (2: hi + lo, ~16-bit mantissa; 1: hi only).  Waves along
// the RHS: 2 when NT >= 2, i.e. 8 waves = 2 per SIMD (16 waves with half the accumulators each
// measured 250-275 / 233-255 us per pass against 236-242 / 219-229, round 2; removed in round 5)
template <int NT, int NS = 2>
struct PanelGeo {
    static constexpr int WN = NT >= 2 ? 2 : 1;        // waves along the RHS
    static_assert(NT % WN == 0, "N-tiles per wave");
    static constexpr int NTW = NT / WN;               // N-tiles per wave
    static constexpr int NW = 4 * WN;                 // waves per block
    static constexpr int T = 64 * NW;                 // threads per block
    static constexpr int K = 16 * NT;                 // right-hand sides
    static constexpr int OStage = NS * K * kPanelK * 2;           // NS rows of 128 B per RHS
    static constexpr int LA = kPanelAStage / (T * 16);            // LDS-DMA per thread per A stage
    static constexpr int LO = (OStage + T * 16 - 1) / (T * 16);   // ... per k-wide stage (a wave may idle)
    static constexpr int Smem = kPanelNA * kPanelAStage + kPanelNO * OStage;
    static_assert(LA >= 1 && LO >= 1, "stage must cover every thread");
    static_assert(Smem <= 160 * 1024, "LDS budget");
};

struct PanelState {
    long long t;        // next iteration
    long long iters;
    double last_err;
    long long cur_mb;   // block of the iteration being finished (set by the line search)
    long long pending;  // one feature block: x += gamma D' of the last iteration not yet applied
    long long fail;     // k_panel_reduce_upd: a block waited for its RHS's step size in vain (not co-resident)
    long long pad[2];
};

struct PanelParams {
    const __bf16* A;    // [m][lda]   block b at column offset b * w
    long long lda;
    const __bf16* At;   // pass 2's copy of A in 256 x 64 tiles, [n / 64][m / 256][256][64] (kPanelTiled2)
    const __bf16* A1t;  // pass 1's copy of A in 64 x 256 tiles, [m / 64][n / 256][64][256] (kPanelTiled1)
    long long m, w;
    int nblock, k;
    int kchunks;        // pass-2 split of the block's w columns
    long long ldr, ldd; // leading dimensions of the bf16 operand images (m, w)
    __bf16* Rh;         // [k][ldr]
    __bf16* Rl;
    __bf16* Dh;         // [k][ldd]
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
    unsigned long long* cnt;   // [k] k_panel_reduce arrivals per RHS (monotone: launch q ends at q * groups)
    // carried gradient (the "carry_g" knob, one feature block): G_t = G_{t-1} + gamma_{t-1} A^T S_{t-1}
    float* Gc;          // [k][w]   the carried gradient (fp32)
    __bf16* Sh;         // [k][ldr] pass 1's operand in a carried iteration: bf16(V), V = gamma S + E (k_panel_update)
    float* Ec;          // [k][m]   V - bf16(V): the rounding error fed into the next carried operand
    // k_panel_reduce_upd (the reduce, line search and residual update in one launch)
    unsigned long long* ready;   // [k] per RHS: the arrival count at which its step size was published
    unsigned long long* lsdone;  // line searches finished (monotone, + k per launch): the last one bumps t
};

constexpr int kLspRows = 1024;    // rows per line-search partial

// Diagnostic builds only (tools/panel_diag.sh; never the shipped library): bit 0 drops the
// A-side LDS-DMA pieces after the prologue, bit 1 the RHS-side ones, bits 2 / 3 half / all of the
// lo operand pieces (panel_op_piece) -- wrong results, used to split a pass's time into MFMA + LDS
// and each stream's share.  (Round 3's bits 4-6, the lo MFMAs dropped, on e4m3 and on 32x32x16,
// went with the lo8 and mfma32 forms in rounds 4-5.)
#ifndef BPGL_PANEL_DIAG
#define BPGL_PANEL_DIAG 0
#endif

typedef __attribute__((address_space(3))) void* lds_void_ptr;

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}
typedef short s16x4 __attribute__((ext_vector_type(4)));

// float -> bf16, round to nearest even.  The float is made opaque first: otherwise the compiler may
// fold (bf16)(float)d into one double -> bf16 rounding in some kernels and not in others, and the
// two differ where (float)d lands on a bf16 tie (a register-ring pass-1 variant, measured and
// removed, once split one direction element differently from the LDS-DMA form that way).
__device__ __forceinline__ __bf16 to_bf16(float v) {
    asm volatile("" : "+v"(v));
    return (__bf16)v;
}

// one LDS-DMA piece: 64 lanes x 16 B from per-lane global addresses to lds_base + 16 * lane
__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)lds_base, 16, 0, 0);
}
// cache policy of the A stream, read once per pass by one block: nt (aux 2) measured 3-8 %
// faster per pass than the default policy (profiles/r01/sweeps/panel_policy.jsonl); the
// k-wide operand, which every block re-reads from L2, keeps the default (BPGL_PANEL_O_AUX)
#ifndef BPGL_PANEL_A_AUX
#define BPGL_PANEL_A_AUX 2
#endif
#ifndef BPGL_PANEL_O_AUX
#define BPGL_PANEL_O_AUX 0
#endif
__device__ __forceinline__ void glds16a(const void* src, char* lds_base) {
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)lds_base, 16, 0, BPGL_PANEL_A_AUX);
}
__device__ __forceinline__ void glds16o(const void* src, char* lds_base) {
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)lds_base, 16, 0, BPGL_PANEL_O_AUX);
}
// all but the youngest N vector-memory ops of this wave done, LDS reads retired, then barrier
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Image with 128-B rows (8 chunks of 16 B): chunk c of row r sits at 16 * (c ^ ((r >> 1) & 7)).
// ds_read_b128 of a 16x16x32 fragment (row = lane & 15, chunk = lane >> 4 (+4)) is conflict-free.
__device__ __forceinline__ int swz128(int r, int c) { return c ^ ((r >> 1) & 7); }
// Image with 512-B rows (32 chunks) read by ds_read_b64_tr_b16: chunk c of row r at
// 16 * (c ^ 2 * ((r & 3) | ((r >> 3 & 1) << 2))): the 8 rows of a 32-lane half land on
// 8 distinct 32-B bank groups.
__device__ __forceinline__ int swz512(int r, int c) { return c ^ (2 * ((r & 3) | (((r >> 3) & 1) << 2))); }

// k-wide operand stage: [hl < NS][k][64] bf16 from hi/lo [k][ld] at column ks, piece q of
// this wave (a piece = 8 image rows of 128 B).  When the stage has fewer pieces than waves
// (NS = 1 at k = 16 or 32) the spare waves issue nothing: the stage's counted wait only
// assumes that a wave's A pieces are its youngest operations, which still holds.
template <int NT, int NS>
__device__ __forceinline__ void panel_op_piece(int q, const __bf16* __restrict__ hi, const __bf16* __restrict__ lo,
                                               long long ld, long long ks, char* obuf, int wave, int lane) {
    using G = PanelGeo<NT, NS>;
    const int pc = q * G::NW + wave;
    if (pc * 8 >= NS * G::K) return;   // wave-uniform
    const int rr = pc * 8 + (lane >> 3);
    const int c = swz128(rr, lane & 7);
    const int hl = rr / G::K, rhs = rr % G::K;
    // diagnostic builds: bit 2 drops every other lo piece (3/4 of the operand bytes), bit 3 every lo
    // piece (the hi bytes alone) -- the MFMA work unchanged, results wrong
    if ((BPGL_PANEL_DIAG & 4) && NS == 2 && pc * 8 >= G::K && (pc & 1)) return;
    if ((BPGL_PANEL_DIAG & 8) && NS == 2 && pc * 8 >= G::K) return;
    glds16o((hl ? lo : hi) + (long long)rhs * ld + ks + 8 * c, obuf + pc * 1024);
}
// pass-1 A stage: rows ks..ks+63 of A, columns col0..col0+255 -> [64][512 B] (a piece = 2 rows).
// kPanelTiled1 (BPGL_PANEL_T1): from p.A1t, where the stage's 64 x 256 tile is one contiguous 32 KiB
// ([m / 64][n / 256][64][256]; `lda` is then n / 256)
#ifndef BPGL_PANEL_T1
#define BPGL_PANEL_T1 1
#endif
constexpr bool kPanelTiled1 = BPGL_PANEL_T1 != 0;
template <int NT>
__device__ __forceinline__ void panel_a1_piece(int q, const __bf16* __restrict__ A, long long lda, long long ks,
                                               long long col0, char* abuf, int wave, int lane) {
    using G = PanelGeo<NT, 2>;
    const int pc = q * G::NW + wave;
    const int row = pc * 2 + (lane >> 5);
    const int c = swz512(row, lane & 31);
    if constexpr (kPanelTiled1)
        glds16a(A + (((ks >> 6) * lda + (col0 >> 8)) << 14) + row * 256 + 8 * c, abuf + pc * 1024);
    else
        glds16a(A + (ks + row) * lda + col0 + 8 * c, abuf + pc * 1024);
}
// pass-2 A stage: rows r0..r0+255 of A, columns ks..ks+63 -> [256][128 B] (a piece = 8 rows).
// kPanelTiled2 (BPGL_PANEL_T2, default 1): from p.At, where the stage's 256 x 64 tile is one contiguous
// 32 KiB, the tiles stage-major ([n / 64][m / 256][256][64]; `lda` is then m / 256, the tiles per column
// strip): the 32 row bands of a column chunk read one contiguous 1 MiB per stage, as pass 1's blocks read
// one 8 MiB window.  Measured against 128 B from each of 256 rows 128 KiB apart (untiled) and against the
// tiles band-major (each block streaming its own 4 MiB, 256 streams 4 MiB apart): pass 2 184.4 -> 170.4
// µs, configs[4] 2583 -> 2670 it/s (round 5: profiles/r05/panel_tiles, profiles/r05/layout)
#ifndef BPGL_PANEL_T2
#define BPGL_PANEL_T2 1
#endif
constexpr bool kPanelTiled2 = BPGL_PANEL_T2 != 0;
template <int NT>
__device__ __forceinline__ void panel_a2_piece(int q, const __bf16* __restrict__ A, long long lda, long long r0,
                                               long long ks, char* abuf, int wave, int lane) {
    using G = PanelGeo<NT, 2>;
    const int pc = q * G::NW + wave;
    const int row = pc * 8 + (lane >> 3);
    const int c = swz128(row, lane & 7);
    if constexpr (kPanelTiled2)
        glds16a(A + (((ks >> 6) * lda + (r0 >> 8)) << 14) + row * 64 + 8 * c, abuf + pc * 1024);
    else
        glds16a(A + (r0 + row) * lda + ks + 8 * c, abuf + pc * 1024);
}
// a tiled copy of A: tile (band, ct) = rows TR band .., columns TC ct .. as one contiguous TR x TC block
// (32 KiB); a thread copies 128 B of it.  grid = (m / TR) x (n / TC).  Tiles in the order their pass's stages
// run: pass 1 (TR 64, TC 256) band-major -- a band is one stage --, pass 2 (TR 256, TC 64, CM) column-major
template <int TR, int TC, bool CM>
__global__ __launch_bounds__(256) void k_panel_tile(const __bf16* __restrict__ A, long long lda, long long n,
                                                    __bf16* __restrict__ At) {
    static_assert(TR * TC == 256 * 64, "32 KiB tiles");
    const long long nct = n / TC, nband = (long long)gridDim.x / nct;
    const long long band = blockIdx.x / nct, ct = blockIdx.x % nct;
    const int r = threadIdx.x / (TC / 64), c = (threadIdx.x % (TC / 64)) * 64;
    const __bf16* src = A + (band * TR + r) * lda + ct * TC + c;
    // CM: tile (band, ct) at ct * nband + band (column tiles major), else band * nct + ct
    __bf16* dst = At + ((CM ? ct * nband + band : (long long)blockIdx.x) << 14) + r * TC + c;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        *reinterpret_cast<uint4*>(dst + 8 * k) = *reinterpret_cast<const uint4*>(src + 8 * k);
}

// B fragment (lane: rhs = lane & 15 of the N-tile, K = 32h + 8(lane>>4) + 0..7)
__device__ __forceinline__ bf16x8 panel_bfrag(const char* obuf, int rr, int h, int lane) {
    return *reinterpret_cast<const bf16x8*>(obuf + rr * 128 + 16 * swz128(rr, 4 * h + (lane >> 4)));
}
// pass-2 A fragment: row of the [256][128 B] image
__device__ __forceinline__ bf16x8 panel_afrag2(const char* abuf, int row, int h, int lane) {
    return *reinterpret_cast<const bf16x8*>(abuf + row * 128 + 16 * swz128(row, 4 * h + (lane >> 4)));
}
// pass-1 A^T fragment from the [64][512 B] image: output row = column j0 + (lane & 15),
// K = 32h + 8(lane>>4) + 0..7, two transposing reads of 4 K-rows each
__device__ __forceinline__ bf16x8 panel_afrag1(const char* abuf, int j0, int h, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int c = (j0 >> 3) + (p >> 1);
    const int r0 = 32 * h + 8 * g + q;
    const int r1 = r0 + 4;
    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(abuf + r0 * 512 + 16 * swz512(r0, c) + 8 * (p & 1)));
    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(abuf + r1 * 512 + 16 * swz512(r1, c) + 8 * (p & 1)));
    const s16x4 lohalf = v0, hihalf = v1;
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = __builtin_shufflevector(lohalf, hihalf, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}

// Block-tile GEMM over nsteps stages of 64:
//   PASS 1: acc[mt][nt] += A[ks.., col0 + j]^T (Rh + Rl)[rhs][ks..]      (rows j, K = A rows)
//   PASS 2: acc[mt][nt] += A[r0 + i][colk + ks..] (Dh [+ Dl])[rhs][ks..] (rows i, K = A columns)
// `a_row0`/`a_col0`: PASS 1 -> (first A row of K, first column of the tile); PASS 2 -> (first row, first column of K).
// ILV 0: a stage's LDS-DMA pieces are issued together after the barrier; ILV 1: they
// are spread over the stage's MFMA groups (one scheduling group each).  NS: operand pieces.
template <int NT, int PASS, int ILV, int NS>
__device__ __forceinline__ void panel_mainloop(char* smem, const __bf16* __restrict__ A, long long lda,
                                               long long a_row0, long long a_col0, const __bf16* __restrict__ bh,
                                               const __bf16* __restrict__ bl, long long ldb, long long b_k0,
                                               int nsteps, f32x4 (&acc)[4][PanelGeo<NT, 2>::NTW]) {
    using G = PanelGeo<NT, NS>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 3, wn = wave >> 2;
    char* abufs = smem;
    char* obufs = smem + kPanelNA * kPanelAStage;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < G::NTW; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

    // piece i of stage (so, sa): i < LO -> k-wide piece, else A piece i - LO (this order is what
    // the counted wait below assumes: the youngest LA operations are A pieces)
    auto piece = [&](int i, int so, int bo, int sa, int ba) {
        if ((BPGL_PANEL_DIAG & 1) && i >= G::LO && (so | sa) != 0) return;
        if ((BPGL_PANEL_DIAG & 2) && i < G::LO && (so | sa) != 0) return;
        if (i < G::LO) {
            panel_op_piece<NT, NS>(i, bh, bl, ldb, b_k0 + (long long)so * kPanelK, obufs + bo * G::OStage,
                                        wave, lane);
        } else if (PASS == 1) {
            panel_a1_piece<NT>(i - G::LO, A, lda, a_row0 + (long long)sa * kPanelK, a_col0,
                                    abufs + ba * kPanelAStage, wave, lane);
        } else {
            panel_a2_piece<NT>(i - G::LO, A, lda, a_row0, a_col0 + (long long)sa * kPanelK,
                                    abufs + ba * kPanelAStage, wave, lane);
        }
    };
    auto issue_a = [&](int s, int buf) {
#pragma unroll
        for (int i = G::LO; i < G::LO + G::LA; ++i) piece(i, 0, 0, s, buf);
    };
    auto issue_o = [&](int s, int buf) {
#pragma unroll
        for (int i = 0; i < G::LO; ++i) piece(i, s, buf, 0, 0);
    };
    constexpr int NP = G::LO + G::LA;
    constexpr int NG = 2 * G::NTW;                 // MFMA groups per stage
    constexpr int PPG = (NP + NG - 1) / NG;         // pieces per group (ILV)
    // prologue: op(0), A(0), A(1) -- the loop's counted wait assumes exactly this issue order
    issue_o(0, 0);
    issue_a(0, 0);
    issue_a(nsteps > 1 ? 1 : 0, 1);
    int abuf = 0;
    for (int s = 0; s < nsteps; ++s) {
        // everything but A(s+1) has landed (op(s), A(s)); every wave is past stage s-1's reads
        wait_vm_barrier<G::LA>();
        const int so = s + 1 < nsteps ? s + 1 : nsteps - 1;     // clamped tail: loads into unread buffers
        const int sa = s + 2 < nsteps ? s + 2 : nsteps - 1;
        const int bo = (s + 1) & 1, ba = abuf == 0 ? 2 : abuf - 1;   // (s + 2) % 3
        if (!ILV) {
#pragma unroll
            for (int i = 0; i < NP; ++i) piece(i, so, bo, sa, ba);
        }
        const char* ab = abufs + abuf * kPanelAStage;
        const char* ob = obufs + (s & 1) * G::OStage;
        static_for<0, 2>([&](auto hc) {
            constexpr int h = decltype(hc)::value;
            bf16x8 af[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
                af[mt] = PASS == 1 ? panel_afrag1(ab, wm * 64 + mt * 16, h, lane)
                                   : panel_afrag2(ab, wm * 64 + mt * 16 + (lane & 15), h, lane);
            static_for<0, G::NTW>([&](auto ntc) {
                constexpr int nt = decltype(ntc)::value;
                constexpr int grp = h * G::NTW + nt;
                constexpr int p0 = grp * PPG < NP ? grp * PPG : NP;
                constexpr int p1 = (grp + 1) * PPG < NP ? (grp + 1) * PPG : NP;
                if constexpr (ILV) {
                    static_for<p0, p1>([&](auto ic) { piece(decltype(ic)::value, so, bo, sa, ba); });
                }
                const int rhs = (wn * G::NTW + nt) * 16 + (lane & 15);
                const bf16x8 b_hi = panel_bfrag(ob, rhs, h, lane);
                bf16x8 b_lo;
                if constexpr (NS == 2) b_lo = panel_bfrag(ob, G::K + rhs, h, lane);
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], b_hi, acc[mt][nt], 0, 0, 0);
                    if constexpr (NS == 2)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], b_lo, acc[mt][nt], 0, 0, 0);
                }
                if constexpr (ILV) {
                    if constexpr (p1 > p0) __builtin_amdgcn_sched_group_barrier(0x20, p1 - p0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x8, 4 * NS, 0);
                }
            });
        });
        abuf = abuf == 2 ? 0 : abuf + 1;
    }
    wait_vm_barrier<0>();   // the clamped tail loads have landed; LDS free for the epilogue
}

// Software-pipelined form of the same GEMM (interleave knob 2).  The stage barrier sits
// before a stage's LAST MFMA group: the fragments of the next stage's first group are read
// behind that group's MFMAs, and every group's fragments are read one group ahead.  Buffer
// reuse is unchanged (a stage's buffers are refilled only after the barrier that follows
// all of its reads); all LDS-DMA pieces of a stage are issued before its barrier, spread
// over the first G - 1 groups.
template <int NT, int PASS, int NS>
__device__ __forceinline__ void panel_mainloop_pipe(char* smem, const __bf16* __restrict__ A, long long lda,
                                                    long long a_row0, long long a_col0,
                                                    const __bf16* __restrict__ bh, const __bf16* __restrict__ bl,
                                                    long long ldb, long long b_k0, int nsteps,
                                                    f32x4 (&acc)[4][PanelGeo<NT, 2>::NTW]) {
    using G = PanelGeo<NT, NS>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 3, wn = wave >> 2;
    char* abufs = smem;
    char* obufs = smem + kPanelNA * kPanelAStage;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < G::NTW; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto piece = [&](int i, int so, int bo, int sa, int ba) {
        if ((BPGL_PANEL_DIAG & 1) && i >= G::LO && (so | sa) != 0) return;
        if ((BPGL_PANEL_DIAG & 2) && i < G::LO && (so | sa) != 0) return;
        if (i < G::LO) {
            panel_op_piece<NT, NS>(i, bh, bl, ldb, b_k0 + (long long)so * kPanelK, obufs + bo * G::OStage,
                                        wave, lane);
        } else if (PASS == 1) {
            panel_a1_piece<NT>(i - G::LO, A, lda, a_row0 + (long long)sa * kPanelK, a_col0,
                                    abufs + ba * kPanelAStage, wave, lane);
        } else {
            panel_a2_piece<NT>(i - G::LO, A, lda, a_row0, a_col0 + (long long)sa * kPanelK,
                                    abufs + ba * kPanelAStage, wave, lane);
        }
    };
    constexpr int NP = G::LO + G::LA;
    constexpr int NG = 2 * G::NTW;                                  // MFMA groups per stage (h, nt)
    constexpr int NGI = NG > 1 ? NG - 1 : 1;                        // groups that carry LDS-DMA pieces
    constexpr int PPG = (NP + NGI - 1) / NGI;
    auto read_a = [&](const char* ab, int h, bf16x8 (&af)[4]) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
            af[mt] = PASS == 1 ? panel_afrag1(ab, wm * 64 + mt * 16, h, lane)
                               : panel_afrag2(ab, wm * 64 + mt * 16 + (lane & 15), h, lane);
    };
    auto read_b = [&](const char* ob, int h, int nt, bf16x8& bhi, bf16x8& blo) {
        const int rhs = (wn * G::NTW + nt) * 16 + (lane & 15);
        bhi = panel_bfrag(ob, rhs, h, lane);
        if constexpr (NS == 2) blo = panel_bfrag(ob, G::K + rhs, h, lane);
    };

    // prologue: op(0), A(0), A(1), then stage 0 landed and group 0's fragments read
    for (int i = 0; i < G::LO; ++i) piece(i, 0, 0, 0, 0);
    for (int i = G::LO; i < NP; ++i) piece(i, 0, 0, 0, 0);
    for (int i = G::LO; i < NP; ++i) piece(i, 0, 0, nsteps > 1 ? 1 : 0, 1);
    wait_vm_barrier<G::LA>();
    bf16x8 af[2][4];
    bf16x8 bfr[2][2];
    read_a(abufs, 0, af[0]);
    read_b(obufs, 0, 0, bfr[0][0], bfr[0][1]);
    int abuf = 0;
    for (int s = 0; s < nsteps; ++s) {
        const int so = s + 1 < nsteps ? s + 1 : nsteps - 1;     // clamped tail: loads into unread buffers
        const int sa = s + 2 < nsteps ? s + 2 : nsteps - 1;
        const int bo = (s + 1) & 1, ba = abuf == 0 ? 2 : abuf - 1;   // (s + 2) % 3
        const int abuf_next = abuf == 2 ? 0 : abuf + 1;
        const char* ab = abufs + abuf * kPanelAStage;
        const char* ob = obufs + (s & 1) * G::OStage;
        static_for<0, NG>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            constexpr int h = g / G::NTW, nt = g % G::NTW;
            constexpr int cb = g & 1, ca = h & 1;
            constexpr int p0 = g < NGI ? (g * PPG < NP ? g * PPG : NP) : NP;
            constexpr int p1 = g < NGI ? ((g + 1) * PPG < NP ? (g + 1) * PPG : NP) : NP;
            static_for<p0, p1>([&](auto ic) { piece(decltype(ic)::value, so, bo, sa, ba); });
            if constexpr (g + 1 < NG) {
                constexpr int h1 = (g + 1) / G::NTW, nt1 = (g + 1) % G::NTW;
                if constexpr (h1 != h) read_a(ab, h1, af[h1 & 1]);
                read_b(ob, h1, nt1, bfr[cb ^ 1][0], bfr[cb ^ 1][1]);
            } else {
                // stage s + 1 landed (only A(s+2) may be outstanding); stage s's reads retired
                wait_vm_barrier<G::LA>();
                const char* abn = abufs + abuf_next * kPanelAStage;
                const char* obn = obufs + ((s + 1) & 1) * G::OStage;
                read_a(abn, 0, af[0]);   // the last group runs on af[1] (h = 1)
                read_b(obn, 0, 0, bfr[cb ^ 1][0], bfr[cb ^ 1][1]);
            }
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ca][mt], bfr[cb][0], acc[mt][nt], 0, 0, 0);
                if constexpr (NS == 2)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ca][mt], bfr[cb][1], acc[mt][nt], 0, 0, 0);
            }
        });
        abuf = abuf_next;
    }
    wait_vm_barrier<0>();   // the clamped tail loads have landed; LDS free for the epilogue
}

// Plain 16- / 8-byte stores for the outputs a kernel hands to the next launch.  (Round 2's
// write-through (sc1) variant of these stores -- the "write_through" knob -- measured <= 0.6 % and
// cost the pass-1 epilogue 18 us; removed in round 5.)
template <typename V, typename E>
__device__ __forceinline__ void put(E* base, long long e, const V& v) {
    *reinterpret_cast<V*>(base + e) = v;
}

__device__ __forceinline__ void split_bf16(double v, __bf16& hi, __bf16& lo) {
    const float f = (float)v;
    hi = to_bf16(f);
    lo = to_bf16((float)(v - (double)(float)hi));
}

// pass-1 epilogue: EPI 0 writes G
// [k][w] fp64 (API); EPI 1 is the fused shrink -- the direction D' in DS bf16 pieces, the norms
// per RHS and block.  The wave owns output rows c0 + 64 wm .. (A columns) x RHS tiles wn * NTW ..;
// T threads per block; smem holds at least 4 * k * 3 doubles and is free (after a barrier).
// GM (carried gradient, one feature block): 0 -- g is the product (A^T R); 1 -- the same, also stored as
// the carried G; 2 -- the product is U = A^T bf16(V_{t-1}) and g = G + U, stored back.  V = gamma S + E
// (k_panel_update) carries the previous roundings forward (error feedback), so the images' sum tracks
// R_t - R_exact to one bf16 rounding of the last step instead of accumulating one per step
// 16-B LDS read by inline asm: the compiler does not tie it to outstanding LDS-DMA (it cannot tell one
// buffer of the shared array from another and would wait for every DMA in flight); the caller orders
// it after the DMA it reads (s_waitcnt vmcnt + barrier) and retires it with lds_wait
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned lds_off(const void* ptr) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)ptr;
}
__device__ __forceinline__ u32x4 lds_rd128(unsigned addr) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
    return v;
}

// one (RHS tile, column group) step of the shrink epilogue: the lane's 4 columns of one RHS -- g from
// the product (+ the carried G), the prox step, D' in DS bf16 pieces, the norm / error partials
template <int DS, int GM>
__device__ __forceinline__ void panel_shrink4(const f32x4& acc, const float (&xs)[4], float (&gs)[4],
                                              const double (&dgv)[4], const double (&rcv)[4], double mu,
                                              __bf16 (&dh)[4], __bf16 (&dl)[4], double& sbx, double& sx,
                                              double& err) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        double g = (double)acc[r];
        if constexpr (GM == 2) g = (double)gs[r] + g;
        if constexpr (GM != 0) gs[r] = (float)g;
        const double x = (double)xs[r];
        const double bx = rcv[r] * soft_thr(dgv[r] * x - g, mu);
        double dprime;
        if constexpr (DS == 2) {
            split_bf16(bx - x, dh[r], dl[r]);
            dprime = (double)(float)dh[r] + (double)(float)dl[r];
        } else {
            dh[r] = to_bf16((float)(bx - x));
            dprime = (double)(float)dh[r];
        }
        sbx += fabs(x + dprime);
        sx += fabs(x);
        const double e = fabs(g - proj(g - x, -mu, mu));
        err = (e > err || e != e) ? e : err;
    }
}
// the per-RHS partials of one wave's RHS tile (lanes l, l^16, l^32, l^48 share the RHS) -> nred
__device__ __forceinline__ void panel_norms_wave(double* nred, int wm, int K, int rhs, double sbx, double sx,
                                                 double err) {
    const int lane = threadIdx.x & 63;
    sbx += __shfl_xor(sbx, 16); sbx += __shfl_xor(sbx, 32);
    sx += __shfl_xor(sx, 16);   sx += __shfl_xor(sx, 32);
    { double o = __shfl_xor(err, 16); err = (o > err || o != o) ? o : err;
      o = __shfl_xor(err, 32); err = (o > err || o != o) ? o : err; }
    if (lane < 16) {
        double* d = nred + ((long long)wm * K + rhs) * 4;
        d[0] = sbx;
        d[1] = sx;
        d[2] = err;
        d[3] = 0.0;
    }
}
// the block's norms per RHS from the four column groups' partials (after a barrier)
__device__ __forceinline__ void panel_norms_out(const PanelParams& p, const double* nred, int T) {
    const int K = p.k;
    for (int rhs = threadIdx.x; rhs < K; rhs += T) {
        double a = 0.0, b = 0.0, e = 0.0;
        for (int q = 0; q < 4; ++q) {
            const double* d = nred + ((long long)q * K + rhs) * 4;
            a += d[0];
            b += d[1];
            e = (d[2] > e || d[2] != d[2]) ? d[2] : e;
        }
        double* dst = p.norms + ((long long)blockIdx.x * p.k + rhs) * 4;
        dst[0] = a; dst[1] = b; dst[2] = e; dst[3] = 0.0;
    }
}

// BPGL_PANEL_DIAG (timing-only builds, tools/panel_diag.sh; results wrong): bit 0 -- no carried-G
// store, bit 1 -- no D' store, bit 3 -- no epilogue loop at all (the products are only kept alive)
template <int NTW, int EPI, int DS, int GM = 0, int NW = 0>
__device__ __forceinline__ void panel_pass1_epilogue(const PanelParams& p, int mb, long long c0, int wm, int wn,
                                                     int T, f32x4 (&acc)[4][NTW], char* smem,
                                                     double* __restrict__ Gout) {
    const int lane = threadIdx.x & 63;
    const int K = p.k;
    // C layout: row = (lane>>4)*4 + r (A column), col = lane & 15 (RHS)
    if (EPI == 0) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                const int rhs = (wn * NTW + nt) * 16 + (lane & 15);
                const long long j = c0 + wm * 64 + mt * 16 + (lane >> 4) * 4;
#pragma unroll
                for (int r = 0; r < 4; ++r) Gout[(long long)rhs * p.w + j + r] = (double)acc[mt][nt][r];
            }
        return;
    }
    double* nred = reinterpret_cast<double*>(smem);   // [4 wm][k][4]
    if constexpr ((BPGL_PANEL_DIAG & 8) != 0) {
        float sink = 0.f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) sink += acc[mt][nt][0] + acc[mt][nt][1] + acc[mt][nt][2] + acc[mt][nt][3];
        if (p.k < 0) p.Gc[lane] = sink;
        return;
    }
    // one feature block: the previous iteration's x += gamma D' (k_panel_update leaves it
    // pending) is applied here, from the D' this thread is about to overwrite -- the same
    // arithmetic as k_panel_update's x part, so x is bitwise unchanged by the deferral
    const bool fx = p.st->pending != 0;
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    if constexpr (NTW == 4 && NW == 8) {
        // k = 128, 8 waves: the block's X (and carried G) rows travel HBM -> LDS by LDS-DMA, 1 KiB
        // per instruction (256 columns x fp32 of one RHS), one RHS tile per phase for both wave
        // columns (32 rows), two phases in flight -- instead of per-lane 16-B loads whose round trips
        // left the epilogue latency-bound (≈31 µs of the carried pass 1, BPGL_PANEL_DIAG 8).
        // diag / rec of the block's 256 columns are staged once.  Same arithmetic, same order.
        constexpr int RS = 1024 + 16;                 // LDS row stride (+16 B: conflict-free 16-B reads)
        constexpr int NR = 32;                        // RHS rows per phase
        constexpr int BUF = (GM == 2 ? 2 : 1) * NR * RS;
        static_assert(2 * 2 * NR * RS + 6144 + 4 * 128 * 4 * 8 <= 160 * 1024, "LDS budget");
        char* dgl = smem + 2 * BUF;                   // diag [256], rec [256], mu [128], gamma [128] (fp64)
        double* nrd = reinterpret_cast<double*>(dgl + 6144);
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        __syncthreads();                              // the mainloop's last LDS reads are done
        // every operand by LDS-DMA (vmcnt retires in order: a plain load issued after the next
        // phase's DMA would make its first use wait for that phase too)
        if (wave < 4)
            glds16((wave < 2 ? p.diag : p.rec) + (long long)mb * p.w + c0 + (wave & 1) * 128 + lane * 2,
                   dgl + wave * 1024);
        else if (wave < 6)
            glds16((wave == 4 ? p.mu : p.gamma) + lane * 2, dgl + 4096 + (wave - 4) * 1024);
        auto issue = [&](int nt, char* buf) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wave * 4 + i;
                const int rhs = ((r >> 4) * 4 + nt) * 16 + (r & 15);
                glds16a(p.X + ((long long)mb * p.k + rhs) * p.w + c0 + lane * 4, buf + r * RS);
                if constexpr (GM == 2) glds16a(p.Gc + (long long)rhs * p.w + c0 + lane * 4, buf + (NR + r) * RS);
            }
        };
        // a pending x update (defer_x) with the bf16 direction: each phase's D' goes to registers just
        // before the phase's DMA, so the phase wait covers it (vmcnt retires in order)
        bf16x4 dpre[2][4] = {};
        auto lddp = [&](int nt) {
            if constexpr (DS == 1) {
                if (fx) {
                    const int rq = (wn * 4 + nt) * 16 + (lane & 15);
#pragma unroll
                    for (int mt = 0; mt < 4; ++mt)
                        dpre[nt & 1][mt] = *reinterpret_cast<const bf16x4*>(
                            p.Dh + (long long)rq * p.ldd + c0 + wm * 64 + mt * 16 + (lane >> 4) * 4);
                }
            }
        };
        lddp(0);
        issue(0, smem);
        lddp(1);
        issue(1, smem + BUF);
        constexpr int OPS = GM == 2 ? 8 : 4;          // LDS-DMA instructions of one phase per wave
        const int rl = wn * 16 + (lane & 15);         // this lane's RHS row within a phase
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            if (nt < 3) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(OPS) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            const char* buf = smem + (nt & 1) * BUF;
            const int rhs = (wn * 4 + nt) * 16 + (lane & 15);
            const double mu = reinterpret_cast<const double*>(dgl + 4096)[rhs];
            const double gprev = fx ? reinterpret_cast<const double*>(dgl + 5120)[rhs] : 0.0;
            double sbx = 0.0, sx = 0.0, err = 0.0;
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int cc = wm * 64 + mt * 16 + (lane >> 4) * 4;   // column within the block
                const long long j = c0 + cc;
                u32x4 vx = lds_rd128(lds_off(buf + rl * RS + cc * 4)), vg = {0u, 0u, 0u, 0u};
                if constexpr (GM == 2) vg = lds_rd128(lds_off(buf + (NR + rl) * RS + cc * 4));
                u32x4 vd0 = lds_rd128(lds_off(dgl + cc * 8)), vd1 = lds_rd128(lds_off(dgl + cc * 8 + 16));
                u32x4 vr0 = lds_rd128(lds_off(dgl + 2048 + cc * 8)), vr1 = lds_rd128(lds_off(dgl + 2048 + cc * 8 + 16));
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vx), "+v"(vg), "+v"(vd0), "+v"(vd1), "+v"(vr0), "+v"(vr1));
                const float4 x4 = __builtin_bit_cast(float4, vx);
                float gs[4] = {0.f, 0.f, 0.f, 0.f};
                if constexpr (GM == 2) {
                    const float4 g4 = __builtin_bit_cast(float4, vg);
                    gs[0] = g4.x; gs[1] = g4.y; gs[2] = g4.z; gs[3] = g4.w;
                }
                const double2 d01 = __builtin_bit_cast(double2, vd0), d23 = __builtin_bit_cast(double2, vd1);
                const double2 r01 = __builtin_bit_cast(double2, vr0), r23 = __builtin_bit_cast(double2, vr1);
                const double dgv[4] = {d01.x, d01.y, d23.x, d23.y};
                const double rcv[4] = {r01.x, r01.y, r23.x, r23.y};
                float xs[4] = {x4.x, x4.y, x4.z, x4.w};
                if (fx) {
                    bf16x4 hq = dpre[nt & 1][mt], lq;
                    if constexpr (DS == 2) {
                        hq = *reinterpret_cast<const bf16x4*>(p.Dh + (long long)rhs * p.ldd + j);
                        lq = *reinterpret_cast<const bf16x4*>(p.Dl + (long long)rhs * p.ldd + j);
                    }
                    bool chg = false;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        double dq = (double)(float)hq[r];
                        if constexpr (DS == 2) dq += (double)(float)lq[r];
                        chg = chg || (dq != 0.0 && gprev != 0.0);
                        xs[r] = (float)((double)xs[r] + gprev * dq);
                    }
                    // x + gamma * 0 is x: columns the step left alone (most of a sparse solution's) keep
                    // their stored x, which saves a share of the 32 MiB X write at configs[4]
                    if (chg)
                        put(p.X, ((long long)mb * p.k + rhs) * p.w + j, make_float4(xs[0], xs[1], xs[2], xs[3]));
                }
                __bf16 dh[4], dl[4];
                panel_shrink4<DS, GM>(acc[mt][nt], xs, gs, dgv, rcv, mu, dh, dl, sbx, sx, err);
                if constexpr (GM != 0)   // read again only next iteration, after all of A: non-temporal
                    __builtin_nontemporal_store(f32x4{gs[0], gs[1], gs[2], gs[3]},
                                                reinterpret_cast<f32x4*>(p.Gc + (long long)rhs * p.w + j));
                put(p.Dh, (long long)rhs * p.ldd + j, bf16x4{dh[0], dh[1], dh[2], dh[3]});
                if constexpr (DS == 2)
                    put(p.Dl, (long long)rhs * p.ldd + j, bf16x4{dl[0], dl[1], dl[2], dl[3]});
            }
            panel_norms_wave(nrd, wm, K, rhs, sbx, sx, err);
            if (nt + 2 < 4) {
                __syncthreads();                      // every wave is done with this phase's buffer
                lddp(nt + 2);
                issue(nt + 2, smem + (nt & 1) * BUF);
            }
        }
        __syncthreads();
        panel_norms_out(p, nrd, T);
        return;
    }
    // every load is issued ahead of the stores it would otherwise wait behind (the compiler cannot
    // reorder loads past stores through possibly aliasing pointers, and one dependent round trip per
    // (RHS tile, column group) serialised the epilogue): mu / gamma per RHS tile up front, and X, diag,
    // rec (and the carried G) one (RHS tile, column group) step ahead of
    // their use (D' of a pending x update too with the bf16 direction; with hi + lo at the step
    // itself, for registers).  Same arithmetic, same order.
    const long long jl = c0 + wm * 64 + (lane >> 4) * 4;   // the lane's first column; + 16 mt + r
    double muv[NTW], gpv[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
        const int rhs = (wn * NTW + nt) * 16 + (lane & 15);
        muv[nt] = p.mu[rhs];
        gpv[nt] = fx ? p.gamma[rhs] : 0.0;
    }
    auto xptr = [&](int nt, int mt) {
        return p.X + ((long long)mb * p.k + (wn * NTW + nt) * 16 + (lane & 15)) * p.w + jl + mt * 16;
    };
    auto gptr = [&](int nt, int mt) {
        return p.Gc + (long long)((wn * NTW + nt) * 16 + (lane & 15)) * p.w + jl + mt * 16;
    };
    auto dptr = [&](const __bf16* base, int nt, int mt) {
        return base + (long long)((wn * NTW + nt) * 16 + (lane & 15)) * p.ldd + jl + mt * 16;
    };
    auto lddr = [&](const double* base, int mt, double2& a, double2& b) {
        const long long kx = (long long)mb * p.w + jl + mt * 16;
        a = *reinterpret_cast<const double2*>(base + kx);
        b = *reinterpret_cast<const double2*>(base + kx + 2);
    };
    double2 dq01, dq23, rq01, rq23;
    lddr(p.diag, 0, dq01, dq23);
    lddr(p.rec, 0, rq01, rq23);
    float4 xq = *reinterpret_cast<const float4*>(xptr(0, 0));
    float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (GM == 2) gq = *reinterpret_cast<const float4*>(gptr(0, 0));
    bf16x4 hq1 = {};
    if constexpr (DS == 1)
        if (fx) hq1 = *reinterpret_cast<const bf16x4*>(dptr(p.Dh, 0, 0));
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
        const int rhs = (wn * NTW + nt) * 16 + (lane & 15);
        const double mu = muv[nt];
        const double gprev = gpv[nt];
        double sbx = 0.0, sx = 0.0, err = 0.0;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            const long long j = jl + mt * 16;   // 4 consecutive columns
            // the next step's operands first
            const int q1 = nt * 4 + mt + 1, nt1 = q1 / 4, mt1 = q1 % 4;
            float4 xn = xq, gn = gq;
            bf16x4 hn1 = hq1;
            double2 dn01 = dq01, dn23 = dq23, rn01 = rq01, rn23 = rq23;
            if (q1 < NTW * 4) {
                if constexpr (DS == 1) {   // (with the hi + lo direction the registers are not there: no spills)
                    lddr(p.diag, mt1, dn01, dn23);
                    lddr(p.rec, mt1, rn01, rn23);
                }
                xn = *reinterpret_cast<const float4*>(xptr(nt1, mt1));
                if constexpr (GM == 2) gn = *reinterpret_cast<const float4*>(gptr(nt1, mt1));
                if constexpr (DS == 1)
                    if (fx) hn1 = *reinterpret_cast<const bf16x4*>(dptr(p.Dh, nt1, mt1));
            }
            float xs[4] = {xq.x, xq.y, xq.z, xq.w};
            if (fx) {
                bf16x4 hq = hq1, lq;
                if constexpr (DS == 2) hq = *reinterpret_cast<const bf16x4*>(dptr(p.Dh, nt, mt));
                if constexpr (DS == 2) lq = *reinterpret_cast<const bf16x4*>(dptr(p.Dl, nt, mt));
                bool chg = false;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double dq = (double)(float)hq[r];
                    if constexpr (DS == 2) dq += (double)(float)lq[r];
                    chg = chg || (dq != 0.0 && gprev != 0.0);
                    xs[r] = (float)((double)xs[r] + gprev * dq);
                }
                if (chg)   // x + gamma * 0 is x: unchanged columns keep their stored x
                    put(p.X, ((long long)mb * p.k + rhs) * p.w + j, make_float4(xs[0], xs[1], xs[2], xs[3]));
            }
            __bf16 dh[4], dl[4];
            if constexpr (DS == 2) {
                if (q1 > 1) {   // step 0's came with the prologue
                    lddr(p.diag, mt, dq01, dq23);
                    lddr(p.rec, mt, rq01, rq23);
                }
            }
            float gs[4] = {gq.x, gq.y, gq.z, gq.w};
            const double dgv[4] = {dq01.x, dq01.y, dq23.x, dq23.y};
            const double rcv[4] = {rq01.x, rq01.y, rq23.x, rq23.y};
            panel_shrink4<DS, GM>(acc[mt][nt], xs, gs, dgv, rcv, mu, dh, dl, sbx, sx, err);
            if constexpr (GM != 0 && (BPGL_PANEL_DIAG & 1) == 0)
                *reinterpret_cast<float4*>(p.Gc + (long long)rhs * p.w + j) = make_float4(gs[0], gs[1], gs[2], gs[3]);
            if constexpr ((BPGL_PANEL_DIAG & 2) == 0)
            put(p.Dh, (long long)rhs * p.ldd + j, bf16x4{dh[0], dh[1], dh[2], dh[3]});
            if constexpr (DS == 2)
                put(p.Dl, (long long)rhs * p.ldd + j, bf16x4{dl[0], dl[1], dl[2], dl[3]});
            xq = xn; gq = gn; hq1 = hn1;
            dq01 = dn01; dq23 = dn23; rq01 = rn01; rq23 = rn23;
        }
        panel_norms_wave(nred, wm, K, rhs, sbx, sx, err);
    }
    __syncthreads();
    panel_norms_out(p, nred, T);
}

// ---------------------------------------------------------------------------
// pass 1: G = A_m^T R (EPI 0: write G [k][w] fp64 -- API), or the fused shrink
// epilogue (EPI 1: the direction D' in DS bf16 pieces (2: Dh + Dl, 1: Dh alone), norms
// per RHS).  grid = w / 256 blocks.  R always enters as hi + lo.
// ---------------------------------------------------------------------------
template <int NT, int EPI, int ILV, int DS, int GM = 0>
__global__ __launch_bounds__((PanelGeo<NT, 2>::T)) void k_panel_pass1(PanelParams p, int fixed_block,
                                                                         double* __restrict__ Gout) {
    using G = PanelGeo<NT, 2>;
    __shared__ __attribute__((aligned(16))) char smem[G::Smem];
    const int mb = fixed_block >= 0 ? fixed_block : (int)(p.st->t % p.nblock);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 3, wn = wave >> 2;
    const long long c0 = (long long)blockIdx.x * kPanelRows;             // first column of this block (in block mb)
    const __bf16* A1 = kPanelTiled1 ? p.A1t : p.A;
    const long long ld1 = kPanelTiled1 ? (long long)p.nblock * p.w / 256 : p.lda;
    f32x4 acc[4][G::NTW];
    if constexpr (GM == 2) {   // carried iteration: U = A^T bf16(V_{t-1}), one bf16 operand
        if constexpr (ILV >= 2)
            panel_mainloop_pipe<NT, 1, 1>(smem, A1, ld1, 0, (long long)mb * p.w + c0, p.Sh, p.Sh, p.ldr, 0,
                                          (int)(p.m / kPanelK), acc);
        else
            panel_mainloop<NT, 1, ILV, 1>(smem, A1, ld1, 0, (long long)mb * p.w + c0, p.Sh, p.Sh, p.ldr, 0,
                                          (int)(p.m / kPanelK), acc);
        panel_pass1_epilogue<G::NTW, EPI, DS, 2, G::NW>(p, mb, c0, wm, wn, G::T, acc, smem, Gout);
        return;
    }
    if constexpr (ILV >= 2)
        panel_mainloop_pipe<NT, 1, 2>(smem, A1, ld1, 0, (long long)mb * p.w + c0, p.Rh, p.Rl, p.ldr, 0,
                                      (int)(p.m / kPanelK), acc);
    else
        panel_mainloop<NT, 1, ILV, 2>(smem, A1, ld1, 0, (long long)mb * p.w + c0, p.Rh, p.Rl, p.ldr, 0,
                                      (int)(p.m / kPanelK), acc);

    panel_pass1_epilogue<G::NTW, EPI, DS, GM, G::NW>(p, mb, c0, wm, wn, G::T, acc, smem, Gout);
}

// ---------------------------------------------------------------------------
// pass 2: partial S over one column chunk: Sslab[chunk][rhs][row]; the direction in NS
// bf16 pieces.  grid = (m / 256) x kchunks
// ---------------------------------------------------------------------------
template <int NT, int ILV, int NS>
__global__ __launch_bounds__((PanelGeo<NT, NS>::T)) void k_panel_pass2(PanelParams p, int fixed_block) {
    using G = PanelGeo<NT, NS>;
    __shared__ __attribute__((aligned(16))) char smem[G::Smem];
    const int mb = fixed_block >= 0 ? fixed_block : (int)(p.st->t % p.nblock);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 3, wn = wave >> 2;
    const int nrb = (int)(p.m / kPanelRows);
    // XCD-aware: blocks are dealt to the 8 XCDs round-robin (blockIdx % 8); when the chunk
    // count allows, give all row blocks of a column chunk (which share its D panel) one XCD.
    int rb = blockIdx.x % nrb, chunk = blockIdx.x / nrb;
    if (p.kchunks % 8 == 0) {                          // kchunks / 8 chunks per XCD
        const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
        chunk = xcd * (p.kchunks / 8) + slot / nrb;
        rb = slot % nrb;
    } else if (8 % p.kchunks == 0 && nrb % (8 / p.kchunks) == 0) {   // 8 / kchunks XCDs per chunk
        const int xpc = 8 / p.kchunks, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
        chunk = xcd / xpc;
        rb = (xcd % xpc) * (nrb / xpc) + slot;
    }
    const long long kc = p.w / p.kchunks;
    const long long r0 = (long long)rb * kPanelRows;
    f32x4 acc[4][G::NTW];
    const __bf16* A2 = kPanelTiled2 ? p.At : p.A;
    const long long ld2 = kPanelTiled2 ? p.m / 256 : p.lda;
    if constexpr (ILV >= 2)
        panel_mainloop_pipe<NT, 2, NS>(smem, A2, ld2, r0, (long long)mb * p.w + chunk * kc, p.Dh, p.Dl, p.ldd,
                                       chunk * kc, (int)(kc / kPanelK), acc);
    else
        panel_mainloop<NT, 2, ILV, NS>(smem, A2, ld2, r0, (long long)mb * p.w + chunk * kc, p.Dh, p.Dl, p.ldd,
                                       chunk * kc, (int)(kc / kPanelK), acc);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < G::NTW; ++nt) {
            const int rhs = (wn * G::NTW + nt) * 16 + (lane & 15);
            const long long row = r0 + wm * 64 + mt * 16 + (lane >> 4) * 4;
            put(p.Sslab, ((long long)chunk * p.k + rhs) * p.m + row,
                   make_float4(acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]));
        }
}

__device__ __forceinline__ void panel_st_sc1(double* q, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(q), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double panel_ld_sc1(const double* q) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(q),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
template <bool LSP_SC1> __device__ void panel_step_rhs(const PanelParams& p, int rhs, double a, double b, double e);
// this thread's share of the pass-1 norm partials of one RHS (tiles q = threadIdx.x, + kThreads, ...):
// sum |Bx|, sum |x|, max err -- loaded by every k_panel_reduce block before its slab loads, so the last
// block's line search does not wait for them
__device__ __forceinline__ void panel_norm_share(const PanelParams& p, int rhs, double& a, double& b, double& e) {
    const int nb1 = (int)(p.w / kPanelRows);
    a = 0.0, b = 0.0, e = 0.0;
    for (int q = threadIdx.x; q < nb1; q += kThreads) {
        const double* src = p.norms + ((long long)q * p.k + rhs) * 4;
        a += src[0];
        b += src[1];
        e = (src[2] > e || src[2] != src[2]) ? src[2] : e;
    }
}

// S = sum over chunks (fp64, fixed order); line-search partials per RHS and
// 1024-row group (mode 1), or plain output (mode 0, API).  grid = k x (m / 1024);
// a thread owns 4 consecutive rows (16-B slab loads).  Mode 1: the last block of an RHS to
// finish runs that RHS's line search (panel_step_rhs), so no separate step launch.
__global__ __launch_bounds__(kThreads) void k_panel_reduce(PanelParams p, double* __restrict__ Sout, int mode) {
    const int rhs = blockIdx.x % p.k;
    const int grp = blockIdx.x / p.k;
    const long long i = (long long)grp * kLspRows + 4 * threadIdx.x;
    double rs = 0.0, ss = 0.0;
    double na = 0.0, nb = 0.0, ne = 0.0;
    if (mode) panel_norm_share(p, rhs, na, nb, ne);
    if (i < p.m) {
        double s[4] = {0.0, 0.0, 0.0, 0.0};
        // the residual rows for the line-search partials, loaded up front (in flight with the chunk
        // loads; p.R is a valid buffer in mode 0 too, where they go unused)
        const double* rp = p.R + (long long)rhs * p.m + i;
        const double2 r01 = *reinterpret_cast<const double2*>(rp);
        const double2 r23 = *reinterpret_cast<const double2*>(rp + 2);
        const float* src = p.Sslab + (long long)rhs * p.m + i;
        const long long cstride = (long long)p.k * p.m;
        auto add = [&](const float4& v) {
            s[0] += (double)v.x;
            s[1] += (double)v.y;
            s[2] += (double)v.z;
            s[3] += (double)v.w;
        };
        // chunks in groups of 8 with every load of a group issued before its adds (one memory round
        // trip per group instead of one per chunk; no per-element condition inside a group, which
        // would make hipcc wait for each load), the adds in chunk order as before
        int c = 0;
        for (; c + 8 <= p.kchunks; c += 8) {
            float4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const float4*>(src + (c + q) * cstride);
#pragma unroll
            for (int q = 0; q < 8; ++q) add(v[q]);
        }
        for (; c < p.kchunks; ++c) add(*reinterpret_cast<const float4*>(src + c * cstride));
        const long long e = (long long)rhs * p.m + i;
        put(Sout, e, make_double2(s[0], s[1]));
        put(Sout, e + 2, make_double2(s[2], s[3]));
        if (mode) {
            rs = fma(r01.x, s[0], rs); rs = fma(r01.y, s[1], rs);
            rs = fma(r23.x, s[2], rs); rs = fma(r23.y, s[3], rs);
            ss = fma(s[0], s[0], ss); ss = fma(s[1], s[1], ss);
            ss = fma(s[2], s[2], ss); ss = fma(s[3], s[3], ss);
        }
    }
    if (!mode) return;
    __shared__ double sr[kWaves], sq[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    rs = wave_sum(rs);
    ss = wave_sum(ss);
    if (lane == 0) { sr[wave] = rs; sq[wave] = ss; }
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x == 0) {
        double* dst = p.lsp + ((long long)grp * p.k + rhs) * 2;
        panel_st_sc1(dst, ((sr[0] + sr[1]) + sr[2]) + sr[3]);
        panel_st_sc1(dst + 1, ((sq[0] + sq[1]) + sq[2]) + sq[3]);
        const unsigned long long ng = (unsigned long long)((p.m + kLspRows - 1) / kLspRows);
        // no agent fences: the partials are stored sc1 by this lane, which waits vmcnt(0) before its
        // add, and the last block reads them sc1 after its add returned (row 1 of MI355X_MICROARCH.md's
        // table of sc1 hand-offs; the fence pair measured +36 us per launch, see op_arrive_last)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long old = __hip_atomic_fetch_add(p.cnt + rhs, 1ull, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
        last = ((old + 1) % ng) == 0;
    }
    __syncthreads();
    if (last) panel_step_rhs<true>(p, rhs, na, nb, ne);
}

// per-RHS line search (lasso.py:129-136): the pass-1 norm partials and the reduce's r.s / s.s
// partials of one RHS folded in a fixed order -> gamma, err.  LSP_SC1: read the line-search
// partials write-through (they were written by other blocks of the running launch).
// a, b, e: this thread's share of the norm partials (panel_norm_share)
template <bool LSP_SC1>
__device__ void panel_step_rhs(const PanelParams& p, int rhs, double a, double b, double e) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ double s3[3][kWaves];
    a = wave_sum(a);
    b = wave_sum(b);
    e = wave_max(e);
    if (lane == 0) { s3[0][wave] = a; s3[1][wave] = b; s3[2][wave] = e; }
    // the line-search partials of the 1024-row groups: loaded in parallel (one group per
    // thread), summed by thread 0 in group order -- a serial chain of dependent loads cost ~1 us
    // per group
    __shared__ double lsr[kThreads][2];
    double rs = 0.0, ss = 0.0;
    const int ng = (int)((p.m + kLspRows - 1) / kLspRows);
    for (int g0 = 0; g0 < ng; g0 += kThreads) {
        const int g = g0 + (int)threadIdx.x;
        if (g < ng) {
            const double* q = p.lsp + ((long long)g * p.k + rhs) * 2;
            lsr[threadIdx.x][0] = LSP_SC1 ? panel_ld_sc1(q) : q[0];
            lsr[threadIdx.x][1] = LSP_SC1 ? panel_ld_sc1(q + 1) : q[1];
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int i = 0; i < kThreads && g0 + i < ng; ++i) { rs += lsr[i][0]; ss += lsr[i][1]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        a = ((s3[0][0] + s3[0][1]) + s3[0][2]) + s3[0][3];
        b = ((s3[1][0] + s3[1][1]) + s3[1][2]) + s3[1][3];
        e = s3[2][0];
        for (int q = 1; q < kWaves; ++q) e = (s3[2][q] > e || s3[2][q] != s3[2][q]) ? s3[2][q] : e;
        const double r1 = rs + p.mu[rhs] * (a - b);
        // write-through: k_panel_reduce_upd's other blocks read them in the same launch
        panel_st_sc1(p.gamma + rhs, (ss == 0.0) ? 0.0 : proj(-r1 / ss, 0.0, 1.0));
        panel_st_sc1(p.err_rhs + rhs, e);
        if (rhs == 0) p.st->cur_mb = p.st->t % p.nblock;   // nobody else reads it in this launch
    }
}

// end of an iteration (wave 0 of block 0 of the update launch): the max error over the RHS
// (one load per lane, then the wave max -- a serial loop over k dependent loads cost ~10 us),
// the error record, t + 1; `pending`: x += gamma D' is left to the next pass-1 epilogue
__device__ __forceinline__ void panel_bump_t(const PanelParams& p, bool pending) {
    double e = 0.0;
    for (int j = threadIdx.x; j < p.k; j += 64) {
        const double v = p.err_rhs[j];
        e = (v > e || v != v) ? v : e;
    }
    e = wave_max(e);
    if (threadIdx.x == 0) {
        const long long t = p.st->t;
        if (p.err_iter && t < p.rec_len) p.err_iter[t] = e;
        p.st->last_err = e;
        p.st->t = t + 1;
        p.st->iters = t + 1;
        if (pending) p.st->pending = 1;
    }
}

// carried gradient (one feature block): the next pass 1's operand V = gamma S + E (cflag & 3 == 1; 2: the
// iteration's G was exact, E restarts at 0), its bf16 image to Sh and the rounding error back to E;
// cflag & 4: R's hi / lo images are not written (no exact pass 1 reads them before the next update)
__device__ __forceinline__ void panel_put_carry(const PanelParams& p, int cflag, long long e, long long re,
                                                double g, const double2& s01, const double2& s23) {
    typedef __bf16 bf16x4c __attribute__((ext_vector_type(4)));
    float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((cflag & 3) == 1) e4 = *reinterpret_cast<const float4*>(p.Ec + e);
    const double v[4] = {(double)e4.x + g * s01.x, (double)e4.y + g * s01.y, (double)e4.z + g * s23.x,
                         (double)e4.w + g * s23.y};
    __bf16 h[4];
    float r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        h[q] = to_bf16((float)v[q]);
        r[q] = (float)(v[q] - (double)(float)h[q]);
    }
    *reinterpret_cast<bf16x4c*>(p.Sh + re) = bf16x4c{h[0], h[1], h[2], h[3]};
    *reinterpret_cast<float4*>(p.Ec + e) = make_float4(r[0], r[1], r[2], r[3]);
}

// x_j += gamma_j D'_j ; Ax_j += gamma_j S_j ; R = sum_b Ax_b - B ; split R.
// Work units: u < ux -> 8 consecutive x elements ([k][w], 16-B Dh (+ Dl when DS = 2) loads);
// ux <= u < ux + ur -> 4 consecutive residual rows ([k][m]).  Also bumps t.  k*w and k*m <
// 2^31 (checked at create), so the index math is 32-bit.
// NB1 (one feature block): R_j += gamma_j S_j directly -- R = Ax - B with a single block, so Ax
// and B need not be read or written (28 instead of 44 bytes per residual element); Ax is then not
// maintained (nothing reads it with one block).
// cflag: the carried gradient's operand and R's images (panel_put_carry; 0 none).
template <int DS, bool NB1>
__global__ __launch_bounds__(kThreads) void k_panel_update(PanelParams p, int cflag) {
    const int mb = (int)p.st->cur_mb;   // p.st->t is advanced by block 0 of this launch
    const long long nx = (long long)p.k * p.w, nr = (long long)p.k * p.m;
    const unsigned ux = (unsigned)(nx / 8), ur = (unsigned)(nr / 4);
    const unsigned nu = ux + ur;
    const unsigned w8 = (unsigned)(p.w / 8), m4 = (unsigned)(p.m / 4);
    typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
    typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
    for (unsigned u = blockIdx.x * kThreads + threadIdx.x; u < nu; u += gridDim.x * kThreads) {
        if (u < ux) {
            const long long e = 8ll * u;
            const unsigned rhs = u / w8;
            const long long de = (long long)rhs * p.ldd + (e - (long long)rhs * p.w);   // operand image index
            const double g = p.gamma[rhs];
            const bf16x8v dh = *reinterpret_cast<const bf16x8v*>(p.Dh + de);
            bf16x8v dl;
            if constexpr (DS == 2) dl = *reinterpret_cast<const bf16x8v*>(p.Dl + de);
            float* xp = p.X + (long long)mb * nx + e;
            float4 x0 = *reinterpret_cast<const float4*>(xp);
            float4 x1 = *reinterpret_cast<const float4*>(xp + 4);
            float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                double dq = (double)(float)dh[q];
                if constexpr (DS == 2) dq += (double)(float)dl[q];
                xs[q] = (float)((double)xs[q] + g * dq);
            }
            *reinterpret_cast<float4*>(xp) = make_float4(xs[0], xs[1], xs[2], xs[3]);
            *reinterpret_cast<float4*>(xp + 4) = make_float4(xs[4], xs[5], xs[6], xs[7]);
        }
        else {
            const unsigned v = u - ux;
            const long long e = 4ll * v;
            const unsigned rhs = v / m4;
            const long long re = (long long)rhs * p.ldr + (e - (long long)rhs * p.m);   // operand image index
            const double g = p.gamma[rhs];
            double r[4];
            __bf16 hi[4], lo[4];
            if constexpr (NB1) {
                const double2 r01 = *reinterpret_cast<const double2*>(p.R + e);
                const double2 r23 = *reinterpret_cast<const double2*>(p.R + e + 2);
                const double2 s01 = *reinterpret_cast<const double2*>(p.S + e);
                const double2 s23 = *reinterpret_cast<const double2*>(p.S + e + 2);
                r[0] = r01.x + g * s01.x; r[1] = r01.y + g * s01.y;
                r[2] = r23.x + g * s23.x; r[3] = r23.y + g * s23.y;
#pragma unroll
                for (int q = 0; q < 4; ++q) split_bf16(r[q], hi[q], lo[q]);
                if (cflag) panel_put_carry(p, cflag, e, re, g, s01, s23);
            } else {
                double* ap = p.Ax + (long long)mb * nr + e;
                double a[4], acc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = ap[q] + g * p.S[e + q];
#pragma unroll
                for (int q = 0; q < 4; ++q) ap[q] = a[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = mb == 0 ? a[q] : p.Ax[e + q];
                for (int b = 1; b < p.nblock; ++b)
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q] += b == mb ? a[q] : p.Ax[(long long)b * nr + e + q];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    r[q] = acc[q] - p.B[e + q];
                    split_bf16(r[q], hi[q], lo[q]);
                }
            }
            put(p.R, e, make_double2(r[0], r[1]));
            put(p.R, e + 2, make_double2(r[2], r[3]));
            if (!(cflag & 4)) {
                put(p.Rh, re, bf16x4v{hi[0], hi[1], hi[2], hi[3]});
                put(p.Rl, re, bf16x4v{lo[0], lo[1], lo[2], lo[3]});
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) panel_bump_t(p, false);
}

// One feature block: R_j += gamma_j S_j (= Ax_j + gamma_j S_j - B_j; Ax is not kept) and its
// hi/lo split; x += gamma D' is left pending for the next pass-1 epilogue (or k_panel_flush).
// A thread owns 4 consecutive residual rows.  Also bumps t.
__global__ __launch_bounds__(kThreads) void k_panel_update1(PanelParams p, int cflag) {
    const long long nr = (long long)p.k * p.m;
    const unsigned ur = (unsigned)(nr / 4), m4 = (unsigned)(p.m / 4);
    typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
    for (unsigned v = blockIdx.x * kThreads + threadIdx.x; v < ur; v += gridDim.x * kThreads) {
        const long long e = 4ll * v;
        const unsigned rhs = v / m4;
        const long long re = (long long)rhs * p.ldr + (e - (long long)rhs * p.m);   // operand image index
        const double g = p.gamma[rhs];
        const double2 r01 = *reinterpret_cast<const double2*>(p.R + e);
        const double2 r23 = *reinterpret_cast<const double2*>(p.R + e + 2);
        const double2 s01 = *reinterpret_cast<const double2*>(p.S + e);
        const double2 s23 = *reinterpret_cast<const double2*>(p.S + e + 2);
        const double r[4] = {r01.x + g * s01.x, r01.y + g * s01.y, r23.x + g * s23.x, r23.y + g * s23.y};
        if (cflag) panel_put_carry(p, cflag, e, re, g, s01, s23);
        __bf16 hi[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split_bf16(r[q], hi[q], lo[q]);
        put(p.R, e, make_double2(r[0], r[1]));
        put(p.R, e + 2, make_double2(r[2], r[3]));
        if (!(cflag & 4)) {
            put(p.Rh, re, bf16x4v{hi[0], hi[1], hi[2], hi[3]});
            put(p.Rl, re, bf16x4v{lo[0], lo[1], lo[2], lo[3]});
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) panel_bump_t(p, true);
}

// One feature block with x deferred (the default configs[4] iteration): k_panel_reduce (S = the
// fixed-order sum of the chunk slabs, the line-search partials, each RHS's last block running its
// line search) and k_panel_update1 (R += gamma S, the carried operand, R's images) in ONE launch.
// Grid = k x G, G blocks per RHS, block g of RHS j owning its U 1024-row groups; a thread owns 4
// rows per group and keeps their S, R (and E) in registers across the line search: the blocks of an
// RHS that are not last wait (bounded, one lane polling an sc1 word) for the step size its last block
// publishes, then update their own rows -- S is never stored and R, S, E are read once (the two
// kernels read R twice and wrote and re-read S).  Every sum is the two kernels' (per 1024-row group:
// the 4 rows of a lane, wave sums, the 4 waves in order; the groups in order), so the iterates are
// bitwise those of the two-kernel path.  Needs the k x G blocks co-resident (k x G <= the occupancy x
// CUs, checked at bind, where the library picks this form; nothing else runs on the stream between);
// a wait that runs out sets PanelState::fail, updates nothing, and bpgl_panel_status reports it.
// The last line search to finish (lsdone) ends the iteration as k_panel_update1 does (t + 1, the
// error record, x pending).
constexpr unsigned kPanelPolls = 1u << 20;
template <int U>
__global__ __launch_bounds__(kThreads) void k_panel_reduce_upd(PanelParams p, int cflag, int G) {
    const int rhs = blockIdx.x % p.k;
    const int g = blockIdx.x / p.k;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double na = 0.0, nb = 0.0, ne = 0.0;
    panel_norm_share(p, rhs, na, nb, ne);
    const long long cstride = (long long)p.k * p.m;
    double s[U][4], r[U][4];
    float4 ev[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long long e = (long long)rhs * p.m + (long long)(g * U + u) * kLspRows + 4 * threadIdx.x;
        const double2 r01 = *reinterpret_cast<const double2*>(p.R + e);
        const double2 r23 = *reinterpret_cast<const double2*>(p.R + e + 2);
        r[u][0] = r01.x; r[u][1] = r01.y; r[u][2] = r23.x; r[u][3] = r23.y;
        ev[u] = (cflag & 3) == 1 ? *reinterpret_cast<const float4*>(p.Ec + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float* src = p.Sslab + e;
#pragma unroll
        for (int q = 0; q < 4; ++q) s[u][q] = 0.0;
        int c = 0;
        for (; c + 8 <= p.kchunks; c += 8) {   // 8 loads in flight, the adds in chunk order
            float4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const float4*>(src + (c + q) * cstride);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                s[u][0] += (double)v[q].x; s[u][1] += (double)v[q].y; s[u][2] += (double)v[q].z; s[u][3] += (double)v[q].w;
            }
        }
        for (; c < p.kchunks; ++c) {
            const float4 v = *reinterpret_cast<const float4*>(src + c * cstride);
            s[u][0] += (double)v.x; s[u][1] += (double)v.y; s[u][2] += (double)v.z; s[u][3] += (double)v.w;
        }
    }
    // per-group line-search partials, in k_panel_reduce's order
    __shared__ double sr[U][kWaves], sq[U][kWaves];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        double rs = 0.0, ss = 0.0;
        rs = fma(r[u][0], s[u][0], rs); rs = fma(r[u][1], s[u][1], rs);
        rs = fma(r[u][2], s[u][2], rs); rs = fma(r[u][3], s[u][3], rs);
        ss = fma(s[u][0], s[u][0], ss); ss = fma(s[u][1], s[u][1], ss);
        ss = fma(s[u][2], s[u][2], ss); ss = fma(s[u][3], s[u][3], ss);
        rs = wave_sum(rs);
        ss = wave_sum(ss);
        if (lane == 0) { sr[u][wave] = rs; sq[u][wave] = ss; }
    }
    __syncthreads();
    __shared__ int last, ok;
    __shared__ unsigned long long target;
    __shared__ double gsh;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            double* dst = p.lsp + ((long long)(g * U + u) * p.k + rhs) * 2;
            panel_st_sc1(dst, ((sr[u][0] + sr[u][1]) + sr[u][2]) + sr[u][3]);
            panel_st_sc1(dst + 1, ((sq[u][0] + sq[u][1]) + sq[u][2]) + sq[u][3]);
        }
        // the sc1 hand-off of k_panel_reduce (no agent fences; see op_arrive_last)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long old = __hip_atomic_fetch_add(p.cnt + rhs, 1ull, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
        last = ((old + 1) % (unsigned long long)G) == 0;
        target = (old / (unsigned long long)G + 1) * (unsigned long long)G;
        ok = 1;
    }
    __syncthreads();
    if (last) {
        panel_step_rhs<true>(p, rhs, na, nb, ne);   // gamma, err_rhs (sc1)
        if (threadIdx.x == 0) {
            gsh = panel_ld_sc1(p.gamma + rhs);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(p.ready + rhs, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long d = __hip_atomic_fetch_add(p.lsdone, 1ull, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT);
            last = ((d + 1) % (unsigned long long)p.k) == 0 ? 2 : 1;   // 2: the last line search of the launch
        }
    } else if (threadIdx.x == 0) {
        unsigned n = kPanelPolls;
        while (__hip_atomic_load(p.ready + rhs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (n-- == 0) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        if (ok) gsh = panel_ld_sc1(p.gamma + rhs);
        else __hip_atomic_store(reinterpret_cast<unsigned long long*>(&p.st->fail), 1ull, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!ok) return;   // block-uniform: nothing is updated (bpgl_panel_status reports the failure)
    const double gm = gsh;
    typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long long e = (long long)rhs * p.m + (long long)(g * U + u) * kLspRows + 4 * threadIdx.x;
        const long long re = (long long)rhs * p.ldr + (e - (long long)rhs * p.m);
        double rn[4];
        __bf16 hi[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rn[q] = r[u][q] + gm * s[u][q];
        if (cflag) {   // the carried operand V = E + gamma S (panel_put_carry, E preloaded)
            const float e4[4] = {ev[u].x, ev[u].y, ev[u].z, ev[u].w};
            __bf16 h[4];
            float rr[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double v = (double)e4[q] + gm * s[u][q];
                h[q] = to_bf16((float)v);
                rr[q] = (float)(v - (double)(float)h[q]);
            }
            *reinterpret_cast<bf16x4v*>(p.Sh + re) = bf16x4v{h[0], h[1], h[2], h[3]};
            *reinterpret_cast<float4*>(p.Ec + e) = make_float4(rr[0], rr[1], rr[2], rr[3]);
        }
        put(p.R, e, make_double2(rn[0], rn[1]));
        put(p.R, e + 2, make_double2(rn[2], rn[3]));
        if (!(cflag & 4)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) split_bf16(rn[q], hi[q], lo[q]);
            put(p.Rh, re, bf16x4v{hi[0], hi[1], hi[2], hi[3]});
            put(p.Rl, re, bf16x4v{lo[0], lo[1], lo[2], lo[3]});
        }
    }
    if (last == 2 && threadIdx.x < 64) {   // every RHS's err_rhs is published (sc1): end the iteration
        double e = 0.0;
        for (int j = threadIdx.x; j < p.k; j += 64) {
            const double v = panel_ld_sc1(p.err_rhs + j);
            e = (v > e || v != v) ? v : e;
        }
        e = wave_max(e);
        if (threadIdx.x == 0) {
            const long long t = p.st->t;
            if (p.err_iter && t < p.rec_len) p.err_iter[t] = e;
            p.st->last_err = e;
            p.st->t = t + 1;
            p.st->iters = t + 1;
            p.st->pending = 1;
        }
    }
}

// apply a pending x += gamma D' (one feature block) -- the end of every bpgl_panel_step, so the
// iterates the caller reads are current; a no-op when nothing is pending
template <int DS>
__global__ __launch_bounds__(kThreads) void k_panel_flush(PanelParams p) {
    if (p.st->pending == 0) return;
    const long long nx = (long long)p.k * p.w;
    typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
    const unsigned w8 = (unsigned)(p.w / 8);
    for (unsigned u = blockIdx.x * kThreads + threadIdx.x; u < (unsigned)(nx / 8); u += gridDim.x * kThreads) {
        const long long e = 8ll * u;
        const unsigned rhs = u / w8;
        const long long de = (long long)rhs * p.ldd + (e - (long long)rhs * p.w);   // operand image index
        const double g = p.gamma[rhs];
        const bf16x8v dh = *reinterpret_cast<const bf16x8v*>(p.Dh + de);
        bf16x8v dl;
        if constexpr (DS == 2) dl = *reinterpret_cast<const bf16x8v*>(p.Dl + de);
        float* xp = p.X + e;
        float4 x0 = *reinterpret_cast<const float4*>(xp);
        float4 x1 = *reinterpret_cast<const float4*>(xp + 4);
        float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            double dq = (double)(float)dh[q];
            if constexpr (DS == 2) dq += (double)(float)dl[q];
            xs[q] = (float)((double)xs[q] + g * dq);
        }
        *reinterpret_cast<float4*>(xp) = make_float4(xs[0], xs[1], xs[2], xs[3]);
        *reinterpret_cast<float4*>(xp + 4) = make_float4(xs[4], xs[5], xs[6], xs[7]);
    }
}
__global__ void k_panel_clear_pending(PanelParams p) {
    if (threadIdx.x == 0) p.st->pending = 0;
}

// split an fp64 [k][len] operand into hi/lo bf16 images [k][ld]; optionally R = -B (reset)
__global__ __launch_bounds__(kThreads) void k_panel_split(const double* __restrict__ src, long long n, long long len,
                                                          long long ld, __bf16* __restrict__ hi,
                                                          __bf16* __restrict__ lo, double sign,
                                                          double* __restrict__ copy) {
    for (long long e = (long long)blockIdx.x * kThreads + threadIdx.x; e < n; e += (long long)gridDim.x * kThreads) {
        const double v = sign * src[e];
        if (copy) copy[e] = v;
        const long long row = e / len;
        const long long d = row * ld + (e - row * len);
        split_bf16(v, hi[d], lo[d]);
    }
}

// diag(A^T A) from row-major A: a block owns 512 columns (64 lanes x 8), its 4
// waves take every 4th row; fixed-order fp64 combine.  grid = n / 512
__global__ __launch_bounds__(kThreads) void k_panel_diag(PanelParams p, double* __restrict__ diag,
                                                         double* __restrict__ rec) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long n = (long long)p.nblock * p.w;
    const long long col = (long long)blockIdx.x * 512 + lane * 8;
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (long long i = wave; i < p.m && col < n; i += kWaves) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(p.A + i * p.lda + col);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const double d = (double)(float)v[e];
            acc[e] = fma(d, d, acc[e]);
        }
    }
    __shared__ double part[kWaves][512];
#pragma unroll
    for (int e = 0; e < 8; ++e) part[wave][lane * 8 + e] = acc[e];
    __syncthreads();
    for (int c = threadIdx.x; c < 512 && blockIdx.x * 512LL + c < n; c += kThreads) {
        const double s = ((part[0][c] + part[1][c]) + part[2][c]) + part[3][c];
        diag[blockIdx.x * 512 + c] = s;
        rec[blockIdx.x * 512 + c] = 1.0 / s;
    }
}

__global__ void k_panel_reset_state(PanelParams p) {
    if (threadIdx.x == 0) {
        p.st->t = 0;
        p.st->iters = 0;
        p.st->last_err = 0.0;
        p.st->cur_mb = 0;
        p.st->pending = 0;
        p.st->fail = 0;
    }
}

}  // namespace bpgl
