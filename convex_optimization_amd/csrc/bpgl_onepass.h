// One-HBM-pass iteration (single feature block; one rank, or row shards over ranks): A is
// streamed once per iteration and yields both products the iteration needs.
//
// For one block the gradient obeys the recurrence
//     g_{t+1} = A^T r_{t+1} = A^T (r_t + gamma_t s23_t) = g_t + gamma_t A^T (A D_t)
// (the reference applies the same update to Ax, lasso.py:155).  So an iteration needs
// s23 = A D and U = A^T s23 -- two passes over A if done one after the other, but only one
// if every row's s23 is complete while the row is still on chip.  k_onepass does that:
//
//   * grid = ngroups x SB persistent blocks (one per CU, all resident): a row group of SB
//     segment blocks walks the same R rows; block sb owns 4 x WC columns, wave q of the
//     block WC of them (WC = 64 lanes x LU 16-byte loads);
//   * per row t each wave keeps the row in registers: phase 1 forms its partial of
//     s23[t] (fp64 FMA, DPP row sums), stores it in an LDS slot; wave t % 4 folds the 4
//     slots in a fixed order and publishes ONE granule per (row, block): the fp64 partial
//     with its lowest mantissa bit replaced by the launch parity, one 8-byte agent-scope
//     store (a single-copy-atomic hand-off, no fences).  One bit suffices: every launch
//     that runs rewrites every granule, so a reader sees this launch's value or the
//     previous launch's, and consecutive launches alternate parity (op_epoch advances
//     exactly when k_onepass ran);
//   * LAG rows later (the row is still in the register ring) every wave reads the SB
//     granules of row t (lane = block; the load was issued PF rows earlier beside the row
//     prefetch, so the in-order vmcnt queue is never drained), checks their tags and folds
//     them in one fixed order -> s23[t], bit-identical in every block; U += row * s23[t]
//     (SB <= 64: one granule per lane; SB <= 128: lanes l and l + 64, GPL = 2);
//   * a late granule is re-polled (bounded; on exhaustion the state's op_fail word is set
//     and the kernel still finishes).  A failed launch commits nothing: every block arrives
//     at the line-search counter after setting op_fail, so the last arrival sees every
//     failure of the launch and skips the line search (the iteration index does not
//     advance), and k_onepass_tail skips the update while op_fail is set.
//     bpgl_solver_status then re-runs the lost iterations (one rank: on the two-pass
//     kernels for the rest of the solve; row shards: the same iteration again, with the
//     failure flag summed over ranks so every rank skips the same iterations).
// Outputs: s23 (by segment block 0) and one U partial row per row group; k_onepass_tail
// folds the partials in a fixed order into g += gamma U after the line search.
//
// Row shards (several ranks, bpgl_set_shard): rank q holds rows [m_q, m_{q+1}) of A and a
// replicated copy of x, D, g (every column).  Then U = sum_q A_q^T (A_q D) and the line-search
// dot products are sums over ranks: k_onepass_fold folds the row-group partials of this rank
// into the exchange buffer [U (wp) | r.s23 | s23.s23], ONE all-reduce (SUM) of wp + 2 fp64
// follows, and every rank computes the identical gamma, g, x and next D from it.  Results are
// bitwise deterministic; the tag bit perturbs each s23 partial by <= 1 ulp (2^-52 relative).
// Measured development steps: tools/onepass*_probe.hip, DESIGN.md section 6b.
#pragma once
#include "bpgl_kernels.h"

namespace bpgl {

constexpr int kOpSlotsLog = 5;
constexpr int kOpSlots = 1 << kOpSlotsLog;   // LDS partial slots (rows); > LAG + publication delay
// an LDS slot's parity: row t and the slot's previous row t - kOpSlots differ in bit kOpSlotsLog
constexpr int kOpDelta = 1;     // rows between a row's phase 1 and its publication
constexpr int kOpMaxSB = 128;   // at most two granules per lane (GPL)
constexpr unsigned kOpPolls = 1u << 16;
#ifndef BPGL_TAIL_BLOCKS
#define BPGL_TAIL_BLOCKS 1024
#endif
constexpr int kOpTailBlocks = BPGL_TAIL_BLOCKS;   // k_onepass_tail grid cap (= its shrink partial count)
constexpr int kOpMaxGroups = 256;     // row groups (one block per CU: at most the CU count)
// k_onepass_tail sums U per lane (one 64-column tile per wave) up to this many row groups; above it
// (configs[3]: 256 groups of a 4096-column block) the 4 waves of a block split the groups of a tile
constexpr int kOpTailWaveGroups = 32;

struct OnePassArgs {
    double* G;                   // [wp]   gradient carried across iterations
    double* S;                   // [m]    s23 = A D (the solver's exchange buffer)
    double* Us;                  // [ngroups][wp] U partial of each row group
    unsigned long long* PG;      // [m][SB] tagged row partials
    int SB, ngroups, R, xl;      // segment blocks per row, row groups, rows per group, XCD-local map
    int ls;                      // 1: the last row group to finish runs the line search (one rank)
    int cache_permille;          // share of each group's rows read last with cache-allocating loads
    const float* Uf;             // row shards, fp32 exchange: the all-reduced U (read instead of Us)
    double* abe;                 // row shards: [sum|Bx|, sum|x|, max err] of the last shrink (k_onepass_fold)
    long long fail_at;           // test hook: iteration whose launch reports a hand-off failure (-1: none)
    int rowb;                    // k_onepass_tail: blocks appended after the column blocks that only run
                                 // the residual update (0: the column blocks run it first, as before)
    int rilv;                    // 1: row group g owns rows g, g + ngroups, ... (interleaved; the k_onepass<..., true>
                                 // instantiation), 0: R consecutive rows
    int tailw;                   // k_onepass_tail, one rank: every lane sums its column's U partials itself
                                 // (wave-owned 64-column tiles, no LDS fold; ngroups <= kOpTailWaveGroups)
};

typedef unsigned long long op_u64;

// a hand-off word: fp64 value with its lowest mantissa bit replaced by a parity tag
__device__ __forceinline__ op_u64 op_stuff(double x, unsigned bit) {
    return ((op_u64)__double_as_longlong(x) & ~1ull) | (bit & 1u);
}
__device__ __forceinline__ double op_unstuff(op_u64 g) { return __longlong_as_double((long long)(g & ~1ull)); }
__device__ __forceinline__ unsigned op_tag(op_u64 g) { return (unsigned)(g & 1ull); }

// DPP lane exchange: a VALU op, no LDS round trip (with one wave per SIMD the ds_bpermute
// latency of __shfl_xor chains is not hidden by other waves)
template <int CTRL>
__device__ __forceinline__ double op_dpp(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum over each 16-lane row, the same bits in every lane of the row: each level adds an
// equally shaped partner group, and fp addition is commutative
__device__ __forceinline__ double op_row_sum16(double x) {
    x += op_dpp<0xb1>(x);    // quad_perm [1,0,3,2]
    x += op_dpp<0x4e>(x);    // quad_perm [2,3,0,1]
    x += op_dpp<0x141>(x);   // row_half_mirror
    x += op_dpp<0x140>(x);   // row_mirror
    return x;
}
__device__ __forceinline__ double op_lane(double x, int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// x + (x of the partner 16-lane row: rows 0<->1, 2<->3), the same bits in both rows
// (gfx950 v_permlane16_swap; VALU, no LDS round trip, no readlane)
__device__ __forceinline__ double op_xrow16(double x) {
    const long long b = __double_as_longlong(x);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    const double p = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);   // rows (0, 0, 2, 2)
    const double q = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);   // rows (1, 1, 3, 3)
    return p + q;
}
// x + (x of the other 32-lane half), the same bits in every lane (v_permlane32_swap)
__device__ __forceinline__ double op_xhalf32(double x) {
    const long long b = __double_as_longlong(x);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    const double p = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);   // lanes 0-31 in both halves
    const double q = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);   // lanes 32-63 in both halves
    return p + q;
}
// wave sum in a fixed order ((row0 + row1) + (row2 + row3)), the same bits in every lane
__device__ __forceinline__ double op_wave_sum(double x) { return op_xhalf32(op_xrow16(op_row_sum16(x))); }
// (lanes 0 + 1) + (lanes 2 + 3) of every quad, in every lane of the quad
__device__ __forceinline__ double op_quad_sum(double x) {
    x += op_dpp<0xb1>(x);
    x += op_dpp<0x4e>(x);
    return x;
}

// The line search of a one-rank one-pass iteration (lasso.py:129-150), run by the last row
// group of k_onepass to finish: its r.s23 / s23.s23 partials (parts2, written through to
// memory by every group) and the shrink partials of the previous k_onepass_tail, folded in
// a fixed order.  Every block of the grid arrives (after publishing its failure, if any), so
// the counter only grows and launch k ends at count k * gridDim.x.
__device__ __forceinline__ bool op_failed(const Params& p) {
    return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(&p.st->op_fail), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT) != 0;
}
// The hand-off needs no agent fences: the partials the last arrival reads (parts2) are stored sc1
// (st_sc1) by one lane, every wave of the block waits vmcnt(0) before the barrier behind which one
// lane adds, and the last arrival reads them with sc1 loads (ld_sc1) after its add has returned --
// row 1 of MI355X_MICROARCH.md's table of hand-offs measured valid with sc1 loads in place of the
// acquire.  An agent release / acquire pair here writes back the XCD L2 in every block
// (buffer_wbl2 sc1): measured +3 us per k_onepass launch and +36 us per k_panel_reduce (round 5,
// profiles/r05/fences), so it is not used.
__device__ __forceinline__ bool op_arrive_last(unsigned long long* cnt, unsigned long long expected) {
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
__device__ void op_linesearch(const Params& p, int ngroups) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double rs = 0.0, ss = 0.0;
    for (int k = threadIdx.x; k < ngroups; k += kThreads) {
        rs += ld_sc1(p.parts2 + 2ll * k);
        ss += ld_sc1(p.parts2 + 2ll * k + 1);
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
    // every block set op_fail (if it failed) before it arrived: a failed launch commits nothing
    if (threadIdx.x == 0 && !op_failed(p)) finish_step(p, rs, ss, a, b, e);
}

// an fp64 scalar as an fp32 hi + lo pair (the fp32 exchange of row shards, k_onepass_fold)
__device__ __forceinline__ void op_split_f32(double v, float* dst) {
    const float hi = (float)v;
    dst[0] = hi;
    dst[1] = (float)(v - (double)hi);
}
template <int LU, typename T>
struct OnePassGeo {
    static constexpr int N = VecT<T>::N;
    static constexpr int CPL = LU * N;       // columns per lane
    static constexpr int WC = 64 * CPL;      // columns per wave
    static constexpr int BC = kWaves * WC;   // columns per segment block
};

template <typename T, int NB, int PF, int LU, int GPL, bool RILV>
__global__ __launch_bounds__(kThreads, 1) void k_onepass(Params p, OnePassArgs o) {
    if (p.st->done) return;
    using G = OnePassGeo<LU, T>;
    using raw = typename VecT<T>::raw;
    constexpr int N = G::N;
    constexpr int LAG = NB - PF - 1;
    static_assert(LAG > PF + kOpDelta && LAG + kOpDelta < kOpSlots, "ring geometry");
    __shared__ op_u64 part[kOpSlots][kWaves];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x, SB = o.SB;
    int grp, sb;
    if (o.xl) { grp = (b & 7) + 8 * ((b >> 3) / SB); sb = (b >> 3) % SB; }
    else { grp = b / SB; sb = b % SB; }
    // this group's rows: R consecutive ones, or (rilv) rows grp, grp + ngroups, ... -- the groups then
    // read adjacent rows at once (one contiguous window of A instead of ngroups streams R rows apart)
    // (a compile-time choice: the runtime stride cost the consecutive form 0.4-0.8 % -- the row step is
    // sensitive to every scalar instruction at one wave per SIMD; profiles/r05/consec)
    // (the interleaved instantiation keeps the runtime form of these expressions: written with the
    // compile-time stride it measured 0.6 % slower at configs[1])
    const bool ilv = RILV && o.rilv;
    const long long gs = ilv ? o.ngroups : 1;
    const long long i0 = ilv ? grp : (long long)grp * o.R;
    const long long i1 = i0 + o.R < p.m ? i0 + o.R : p.m;
    const int nrows = ilv ? (grp < p.m ? (int)((p.m - grp + gs - 1) / gs) : 0) : (i1 > i0 ? (int)(i1 - i0) : 0);
    auto rowat = [&](long long i) -> long long { return RILV ? i0 + i * gs : i0 + i; };   // this group's i-th row
    // launches alternate the row direction; each reads the last cache_permille of its rows with
    // cache-allocating loads, which the next launch (opposite direction) reads first from the
    // Infinity Cache (only the small tail kernel runs in between)
    const bool rev = ((p.st->op_epoch - p.st->op_base) & 1) != 0;   // per solver run: reruns repeat bits
    auto rowof = [&](int t) -> long long { return rowat(rev ? nrows - 1 - t : t); };
    if (nrows == 0) {   // the whole row group (uniform); ngroups = cdiv(m, R) makes this unreachable
        if (sb == 0 && threadIdx.x == 0) { st_sc1(p.parts2 + 2ll * grp, 0.0); st_sc1(p.parts2 + 2ll * grp + 1, 0.0); }
        if (o.ls && op_arrive_last(&p.st->op_cnt, (unsigned long long)gridDim.x)) op_linesearch(p, o.ngroups);
        return;
    }
    const unsigned tag = (unsigned)((p.st->op_epoch + 1) & 1);   // bound scratch is zero: parity 0 = unwritten
    if (b == 0 && threadIdx.x == 0) p.st->op_ran = 1;

    for (int k = threadIdx.x; k < kOpSlots * kWaves; k += kThreads) (&part[0][0])[k] = 1ull;   // rows 0..31: parity 0
    __syncthreads();
    BPGL_STAMP_AT(2, 0);

    // this lane's columns: LU 16-byte groups, 64 * N apart
    const T* __restrict__ Ab = reinterpret_cast<const T*>(p.A);
    long long col[LU];
    double d[LU][N], u[LU][N];
    bool colok[LU];
#pragma unroll
    for (int k = 0; k < LU; ++k) {
        const long long c = (long long)sb * G::BC + wave * G::WC + k * 64 * N + lane * N;
        colok[k] = c < p.wp;
        col[k] = colok[k] ? c : 0;
#pragma unroll
        for (int e = 0; e < N; ++e) {
            d[k][e] = colok[k] ? p.D[c + e] : 0.0;
            u[k][e] = 0.0;
        }
    }
    // GPL 0: one segment block per row (SB = 1, e.g. configs[3]): a row's s23 is complete inside the
    // block, so phase 2 folds the 4 wave partials straight from the LDS slots -- no granule through
    // memory, no publication step ("onepass_sb1", default on when SB = 1)
    static_assert(GPL == 0 || GPL == 1 || GPL == 2, "granules per lane");
    constexpr int NG = GPL > 0 ? GPL : 1;
    int glane[NG];   // granule k of this lane: segment block lane + 64 k
#pragma unroll
    for (int k = 0; k < NG; ++k) glane[k] = lane + 64 * k < SB ? lane + 64 * k : 0;
    raw buf[NB][LU];
    op_u64 gv[NB][NG];
    unsigned polls = kOpPolls;
    bool failed = o.fail_at >= 0 && b == 0 && p.st->t == o.fail_at;   // test hook (bpgl_set_tuning)

    const int tcache = nrows - (int)(((long long)nrows * o.cache_permille) / 1000);
    // NTL: the load policy, a compile-time choice per copy of the row loop (a runtime branch
    // around the loads makes the compiler drain the load queue at the join)
    auto load = [&](auto NTL, int t, int slot) {
        const int tc = t < nrows ? t : nrows - 1;
        const T* rp = Ab + rowof(tc) * p.lda;
#pragma unroll
        for (int k = 0; k < LU; ++k) buf[slot][k] = ldv<T, decltype(NTL)::value>(rp + col[k]);
    };
    auto gload = [&](int t, int slot) {   // granules consumed at step t (phase 2 of row t - LAG)
        if constexpr (GPL == 0) return;
        int t2 = t - LAG;
        t2 = t2 < 0 ? 0 : (t2 >= nrows ? nrows - 1 : t2);
#pragma unroll
        for (int k = 0; k < GPL; ++k)
            gv[slot][k] = __hip_atomic_load(o.PG + rowof(t2) * SB + glane[k], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    };

    // one row step: prefetch row t + PF (and the granules of its phase 2), phase 1 of row t,
    // publication of row t - 1, phase 2 of row t - LAG.  (A branch-free steady-state copy of
    // the loop made the register allocator spill: the three loop copies are not worth it.)
    auto step = [&](auto NTL, const int q, const int t) {
        const int qn = (q + PF) % NB;
        gload(t + PF, qn);
        load(NTL, t + PF, qn);
        if (t < nrows) {   // phase 1: this wave's partial of s23[t] into its LDS slot
            double acc[4] = {0.0, 0.0, 0.0, 0.0};   // 4 independent FMA chains, folded in a fixed order
#pragma unroll
            for (int k = 0; k < LU; ++k) {
                double v[N];
                VecT<T>::cvt(buf[q][k], v);
#pragma unroll
                for (int e = 0; e < N; ++e) acc[(k * N + e) & 3] = fma(v[e], d[k][e], acc[(k * N + e) & 3]);
            }
            const double s = op_wave_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
#if BPGL_STAMP
            if ((t == 0 || t == nrows - 1) && threadIdx.x == 0 && b < 16384)
                g_stamps[2][t == 0 ? 2 : 3][b] = __builtin_amdgcn_s_memrealtime() + (unsigned long long)(s != s);
#endif
            if (lane == 0)
                __hip_atomic_store(&part[t % kOpSlots][wave], op_stuff(s, (unsigned)t >> kOpSlotsLog),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const int tp = t - kOpDelta;   // publication of row tp by wave tp % 4
        if (GPL > 0 && tp >= 0 && tp < nrows && (tp & 3) == wave) {
            const unsigned want = ((unsigned)tp >> kOpSlotsLog) & 1u;
            op_u64 w = 0;
            while (true) {
                w = lane < kWaves ? __hip_atomic_load(&part[tp % kOpSlots][lane], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP)
                                  : 0;
                if (__all(lane >= kWaves || op_tag(w) == want)) break;
                if (polls == 0) { failed = true; break; }
                --polls;
                __builtin_amdgcn_s_sleep(1);
            }
            const double bsum = op_quad_sum(op_unstuff(w));   // (p0 + p1) + (p2 + p3) in lane 0
            if (lane == 0)
                __hip_atomic_store(o.PG + rowof(tp) * SB + sb, op_stuff(bsum, tag), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        const int t2 = t - LAG;
        if (GPL == 0 && t2 >= 0 && t2 < nrows) {   // phase 2, one segment block: s23[t2] from the LDS slots
            const int qs = (q - LAG + NB) % NB;
            const unsigned want = ((unsigned)t2 >> kOpSlotsLog) & 1u;
            op_u64 w = 0;
            while (true) {   // every wave wrote its partial of row t2 at its step t2 (LAG steps ago: rarely late)
                w = lane < kWaves ? __hip_atomic_load(&part[t2 % kOpSlots][lane], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP)
                                  : 0;
                if (__all(lane >= kWaves || op_tag(w) == want)) break;
                if (polls == 0) { failed = true; break; }
                --polls;
                __builtin_amdgcn_s_sleep(1);
            }
            const double x = op_lane(op_quad_sum(op_unstuff(w)), 0);   // (p0 + p1) + (p2 + p3)
            if (wave == 0 && lane == 0) o.S[rowof(t2)] = x;
#pragma unroll
            for (int k = 0; k < LU; ++k) {
                double v2[N];
                VecT<T>::cvt(buf[qs][k], v2);
#pragma unroll
                for (int e = 0; e < N; ++e) u[k][e] = fma(v2[e], x, u[k][e]);
            }
        }
        if (GPL > 0 && t2 >= 0 && t2 < nrows) {   // phase 2: U += row(t2) * s23[t2]
            const int qs = (q - LAG + NB) % NB;
            op_u64 v[NG];
#pragma unroll
            for (int k = 0; k < GPL; ++k) v[k] = gv[q][k];
            // lanes past SB read block 0's granule (glane), which is ready exactly when block 0's is:
            // no per-lane exemption needed (fewer VALU ops per row at one wave per SIMD)
            auto ready = [&]() {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < NG; ++k) ok = ok && op_tag(v[k]) == tag;
                return ok;
            };
            if (!__all(ready())) {   // late: re-poll (drains this wave's queue; rare)
                const op_u64* src = o.PG + rowof(t2) * SB;
                do {
                    if (polls == 0) { failed = true; break; }
                    --polls;
                    __builtin_amdgcn_s_sleep(2);
#pragma unroll
                    for (int k = 0; k < NG; ++k)
                        v[k] = __hip_atomic_load(src + glane[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } while (!__all(ready()));
                // settle here, so the merge with the fast path is not a pending load
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int k = 0; k < NG; ++k) asm volatile("" : "+v"(v[k]));
            }
            // GPL 2 means SB > 64: every lane's first granule is a block of its own
            double x = (GPL == 2 || lane < SB) ? op_unstuff(v[0]) : 0.0;
            if (GPL == 2) x += lane + 64 < SB ? op_unstuff(v[NG - 1]) : 0.0;   // blocks l and l + 64, then the wave
            x = SB <= 16 ? op_lane(op_row_sum16(x), 0) : op_wave_sum(x);
            if (sb == 0 && wave == 0 && lane == 0) o.S[rowof(t2)] = x;
#pragma unroll
            for (int k = 0; k < LU; ++k) {
                double v2[N];
                VecT<T>::cvt(buf[qs][k], v2);
#pragma unroll
                for (int e = 0; e < N; ++e) u[k][e] = fma(v2[e], x, u[k][e]);
            }
        }
    };

    using NTon = std::integral_constant<bool, true>;
    using NToff = std::integral_constant<bool, false>;
#pragma unroll
    for (int q = 0; q < PF; ++q) { gload(q, q); load(NTon{}, q, q); }
    int base = 0;   // stays a multiple of NB: ring slots are static
    // rows issued before tcache stream non-temporally, the rest allocate in the caches
    for (; base + NB + PF <= tcache; base += NB) {
#pragma unroll
        for (int q = 0; q < NB; ++q) step(NTon{}, q, base + q);
    }
    for (; base < nrows + LAG; base += NB) {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            // uniform: the last chunk of the ring ends with the drain, not NB-aligned -- leaving here skips
            // the up to NB - 1 empty steps after it (each still issued its prefetch loads): k_onepass
            // 330.0 -> 326.0 us at configs[1], 332.7 -> 324.8 us on the weak shard, 53.2 -> 51.7 us on the
            // N = 8 strong shard, configs[3] unchanged (round 5, profiles/r05/drain_exit)
            if (base + q >= nrows + LAG) break;
            step(NToff{}, q, base + q);
        }
    }
    BPGL_STAMP_AT(2, 1);
    if (failed && lane == 0) atomicOr((unsigned long long*)&p.st->op_fail, 1ull);
    if (sb == 0 && wave == 0) {
        // this row group's share of the line search, r.s23 and s23.s23, from the s23 rows this
        // wave wrote (fixed order: lanes stride the rows, then the wave sum) -> parts2[grp]
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __threadfence_block();
        // 8 rows per lane in flight, then their FMAs in row order (the same bits as one row at a
        // time; the compiler had waited for each row's two loads, a memory round trip per 64 rows
        // on the launch's critical path)
        double rs = 0.0, ss = 0.0;
        int i = lane;
        for (; i + 7 * 64 < nrows; i += 8 * 64) {
            double sv[8], rv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                sv[k] = o.S[rowat(i + 64 * k)];
                rv[k] = p.r[rowat(i + 64 * k)];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                rs = fma(rv[k], sv[k], rs);
                ss = fma(sv[k], sv[k], ss);
            }
        }
        for (; i < nrows; i += 64) {
            const double sv = o.S[rowat(i)];
            rs = fma(p.r[rowat(i)], sv, rs);
            ss = fma(sv, sv, ss);
        }
        rs = op_wave_sum(rs);
        ss = op_wave_sum(ss);
        if (lane == 0) { st_sc1(p.parts2 + 2ll * grp, rs); st_sc1(p.parts2 + 2ll * grp + 1, ss); }
    }
    double* dst = o.Us + (long long)grp * p.wp;
#pragma unroll
    for (int k = 0; k < LU; ++k)
        if (colok[k])
#pragma unroll
            for (int e = 0; e < N; ++e) dst[col[k] + e] = u[k][e];
    if (o.ls && op_arrive_last(&p.st->op_cnt, (unsigned long long)gridDim.x)) op_linesearch(p, o.ngroups);   // block-uniform
#if BPGL_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0 && b < 16384) g_stamps[2][4][b] = __builtin_amdgcn_s_memrealtime();
#endif
}

// Row shards: this rank's exchange contribution [sum_groups U (wp) | sum r.s23 | sum s23.s23 |
// failed] (fixed order over the row groups; `failed` = this rank's op_fail, so the sum tells
// every rank whether any rank's launch failed).  Runs whether or not the solver stopped: the
// all-reduce after it runs in every iteration of a captured graph.  `outf` (RCCL row shards,
// the "exchange_fp32" knob): the same contribution as fp32 -- U rounded, each scalar split
// into a hi + lo pair [U (wp) | rs_hi | rs_lo | ss_hi | ss_lo | failed] -- half the bytes on
// xGMI.  With one rank the pair carries the scalar to ~2^-48; RCCL sums the hi words and the
// lo words separately in fp32, so with several ranks each summed word is rounded to fp32 and
// the scalars are only fp32-accurate (~2^-24 relative).
__global__ __launch_bounds__(kThreads) void k_onepass_fold(Params p, OnePassArgs o, double* __restrict__ out,
                                                           float* __restrict__ outf) {
    const int cblocks = (int)gridDim.x - 1;   // the last block folds the scalars
    if ((int)blockIdx.x < cblocks) {
        const long long stride = (long long)cblocks * kThreads;
        for (long long j = (long long)blockIdx.x * kThreads + threadIdx.x; j < p.wp; j += stride) {
            // 8 loads in flight, then the adds in group order (the same bits as one at a time)
            double acc = 0.0;
            int q = 0;
            for (; q + 8 <= o.ngroups; q += 8) {
                double v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = o.Us[(long long)(q + k) * p.wp + j];
#pragma unroll
                for (int k = 0; k < 8; ++k) acc += v[k];
            }
            for (; q < o.ngroups; ++q) acc += o.Us[(long long)q * p.wp + j];
            if (outf) outf[j] = (float)acc;
            else out[j] = acc;
        }
        return;
    }
    // the last shrink's per-block partials (identical on every rank: x, g and D are replicated) for
    // the line search at the head of k_onepass_tail -- the fold k_linesearch ran, in the same order
    // (p.nparts = the tail's grid); the groups' [r.s23, s23.s23] staged through LDS by all lanes at
    // once, then summed by one thread in group order
    __shared__ double pr[2 * kOpMaxGroups];
    for (int k = threadIdx.x; k < 2 * o.ngroups; k += kThreads) pr[k] = p.parts2[k];
    double a = 0.0, b = 0.0, e = 0.0;
    if (o.abe) fold_parts(p, p.nparts, a, b, e);   // has a barrier
    __syncthreads();
    if (threadIdx.x == 0) {
        if (o.abe) { o.abe[0] = a; o.abe[1] = b; o.abe[2] = e; }
        double rs = 0.0, ss = 0.0;
        for (int q = 0; q < o.ngroups; ++q) { rs += pr[2 * q]; ss += pr[2 * q + 1]; }
        const bool failed = op_failed(p);
        if (outf) {
            op_split_f32(rs, outf + p.wp);
            op_split_f32(ss, outf + p.wp + 2);
            outf[p.wp + 4] = failed ? 1.0f : 0.0f;
        } else {
            out[p.wp] = rs;
            out[p.wp + 1] = ss;
            out[p.wp + 2] = failed ? 1.0 : 0.0;
        }
    }
}

// Row shards without the one-pass kernel (a failed hand-off, or "onepass" = 0): the line-search
// scalars of the two-pass row iteration -- the fixed-order sums of k_rowreduce's per-block
// [r.s23, s23.s23] partials -- into the exchange tail [.. | r.s23 | s23.s23 | failed = 0], and
// the fixed-order fold of the shrink partials for the line search at the head of
// k_onepass_tail (the U part of the buffer is zero: the next iteration recomputes g exactly).
// One block.
__global__ __launch_bounds__(kThreads) void k_rows2_fold(Params p, OnePassArgs o, double* __restrict__ out,
                                                         int nrr) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double rs = 0.0, ss = 0.0;
    for (int k = threadIdx.x; k < nrr; k += kThreads) {
        rs += p.parts2[2ll * k];
        ss += p.parts2[2ll * k + 1];
    }
    __shared__ double sr[kWaves], sq[kWaves];
    rs = wave_sum(rs);
    ss = wave_sum(ss);
    if (lane == 0) { sr[wave] = rs; sq[wave] = ss; }
    __syncthreads();
    double a, b, e;
    fold_parts(p, p.nparts, a, b, e);
    if (threadIdx.x == 0) {
        out[p.wp] = ((sr[0] + sr[1]) + sr[2]) + sr[3];
        out[p.wp + 1] = ((sq[0] + sq[1]) + sq[2]) + sq[3];
        out[p.wp + 2] = 0.0;
        o.abe[0] = a;
        o.abe[1] = b;
        o.abe[2] = e;
    }
}

// rec = 1 / diag after the column norms were summed over row shards (lasso.py:29-30)
__global__ __launch_bounds__(kThreads) void k_recip(const double* __restrict__ d, double* __restrict__ rec,
                                                    long long n) {
    const long long j = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (j < n) rec[j] = 1.0 / d[j];
}

// Tail of a one-pass iteration, one kernel.  UPDATE: x += gamma D, Ax += gamma s23,
// r = Ax - b (lasso.py:153-155, :105), g += gamma sum_groups U (fixed order); then, for every
// mode, the shrink of the next iteration from (g, x) (lasso.py:114-119, cpu_calculation.py:
// 15-20): D and per-block [sum|Bx|, sum|x|, max err] partials that
// the next line search folds (p.nparts = gridDim.x).  UPDATE = false runs the shrink alone (after a
// reset or an exact refresh of g).  UPDATE also advances the launch parity iff k_onepass ran
// (it runs in the iteration whose line search stops, too).
template <bool UPDATE>
__global__ __launch_bounds__(kThreads) void k_onepass_tail(Params p, OnePassArgs o) {
    // Every load the head needs is issued before the first decision (one memory round trip
    // instead of four dependent ones): the state words, the exchange scalars and the fold's sums
    // (row shards), and the operands of this wave's first column tile (pre-summed U).
    const bool b0 = blockIdx.x == 0 && threadIdx.x == 0;
    const long long done = p.st->done;
    const bool opf = UPDATE && op_failed(p);
    const unsigned long long ran = (UPDATE && b0) ? p.st->op_ran : 0ull;
    const long long epoch = (UPDATE && b0) ? p.st->op_epoch : 0;
    double gamma = UPDATE ? p.st->gamma : 0.0;
    double xfail = 0.0, rs = 0.0, ss = 0.0, a = 0.0, b = 0.0, e = 0.0;
    if (UPDATE && o.abe) {   // row shards
        if (o.Uf) {
            xfail = (double)o.Uf[p.wp + 4];
            rs = (double)o.Uf[p.wp] + (double)o.Uf[p.wp + 1];
            ss = (double)o.Uf[p.wp + 2] + (double)o.Uf[p.wp + 3];
        } else {
            xfail = o.Us[p.wp + 2];
            rs = o.Us[p.wp];
            ss = o.Us[p.wp + 1];
        }
        a = o.abe[0];
        b = o.abe[1];
        e = o.abe[2];
    }
    const int cb0 = (int)gridDim.x - (UPDATE ? o.rowb : 0);   // column blocks
    const int lane0 = threadIdx.x & 63, wave0 = threadIdx.x >> 6;
    // pre-summed U (row shards), or (tailw) few row-group
    // partials that each lane sums for its own column: each wave owns 64-column tiles
    const bool wtile = o.ngroups == 1 || o.tailw;
    const long long tile0 = (long long)blockIdx.x * kWaves + wave0;
    const long long j0 = tile0 * 64 + lane0;
    const bool pre = wtile && (int)blockIdx.x < cb0 && j0 < p.wp;
    // U of column j: the row groups summed in the order of the LDS fold below -- group q into
    // accumulator q % 4 (increasing q), then ((a0 + a1) + a2) + a3 -- so both forms give the same bits
    auto usum = [&](long long j) -> double {
        if (!UPDATE) return 0.0;
        if (o.Uf) return (double)o.Uf[j];
        if (o.ngroups == 1) return o.Us[j];
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        int q = 0;
        for (; q + 16 <= o.ngroups; q += 16) {   // 16 loads in flight, then the adds in group order
            double v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = o.Us[(long long)(q + k) * p.wp + j];
#pragma unroll
            for (int k = 0; k < 16; k += 4) { a0 += v[k]; a1 += v[k + 1]; a2 += v[k + 2]; a3 += v[k + 3]; }
        }
        for (; q < o.ngroups; ++q) {
            const double v = o.Us[(long long)q * p.wp + j];
            if ((q & 3) == 0) a0 += v;
            else if ((q & 3) == 1) a1 += v;
            else if ((q & 3) == 2) a2 += v;
            else a3 += v;
        }
        return ((a0 + a1) + a2) + a3;
    };
    double pg = 0.0, pu = 0.0, px = 0.0, pd = 0.0, pdg = 0.0, prc = 0.0;
    if (pre) {
        const bool col = j0 < p.w;
        pg = o.G[j0];
        pu = usum(j0);
        px = col ? p.x[j0] : 0.0;
        pd = (UPDATE && col) ? p.D[j0] : 0.0;
        pdg = col ? p.diag[j0] : 0.0;
        prc = col ? p.rec[j0] : 0.0;
    }
    // the parity advances after every k_onepass launch, a failed one too (it still published
    // every granule of its rows)
    if (UPDATE && b0 && ran) {
        p.st->op_epoch = epoch + 1;
        p.st->op_ran = 0;
    }
    if (done) return;
    // a failed k_onepass (this iteration or an earlier one not yet re-run) commits nothing
    if (UPDATE && opf) return;
    if (UPDATE && o.abe) {
        // row shards: any rank's failure, summed over ranks -> every rank skips this iteration
        if (xfail != 0.0) {   // grid-uniform
            if (b0)
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(&p.st->op_fail), 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    if (UPDATE && o.abe) {
        // row shards: the line search (lasso.py:129-150) on the all-reduced [r.s23, s23.s23] and the
        // fold's shrink sums, computed identically by every block (the same inputs, the same
        // arithmetic as k_linesearch: rs and ss are the sums of one value each).  One feature
        // block: the stop rule is err < err_bound in this iteration (block_cnt never carries).
        // Block 0 records the state (finish_step); a block that finds the rule fired updates nothing.
        const double r1 = rs + p.mu * (a - b);
        gamma = (ss == 0.0) ? 0.0 : proj(-r1 / ss, 0.0, 1.0);
        const bool stop = p.err_bound >= 0.0 && e < p.err_bound;
        if (blockIdx.x == 0 && threadIdx.x == 0) finish_step(p, rs, ss, a, b, e);
        if (stop) return;   // block-uniform
    }
    // the residual update Ax += gamma s23, r = Ax - b (lasso.py:153-155): on `rowb` blocks of its own
    // (they run beside the column blocks instead of delaying the first of them by a memory round
    // trip), or, with rowb = 0, by every block before its columns
    const int cb = (int)gridDim.x - (UPDATE ? o.rowb : 0);   // column blocks
    if (UPDATE) {
        const bool own = o.rowb > 0;
        if (!own || (int)blockIdx.x >= cb) {
            const long long stride = (long long)(own ? o.rowb : gridDim.x) * kThreads;
            const long long k0 = (long long)(own ? (int)blockIdx.x - cb : (int)blockIdx.x) * kThreads + threadIdx.x;
            for (long long k = k0; k < p.m; k += stride) {
                const double ax = p.Ax[k] + gamma * o.S[k];
                p.Ax[k] = ax;
                p.r[k] = ax - p.b[k];
            }
            if (own) return;   // block-uniform: row blocks write no shrink partials
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ double ured[kWaves][64];
    double abx = 0.0, ax1 = 0.0, err = 0.0;
    const long long ntile = (p.wp + 63) / 64;
    // the shrink of one column j with U_j already summed (u); accumulates this lane's partials
    auto shrink_col = [&](long long j, double g, double u, double xj, double dold, double dg, double rc) {
        if (UPDATE) {
            g += gamma * u;
            o.G[j] = g;
        }
        double Dj = 0.0;
        if (j < p.w) {
            if (UPDATE) {
                xj += gamma * dold;
                p.x[j] = xj;
            }
            const double rx = dg * xj - g;                        // lasso.py:114
            const double bx = rc * soft_thr(rx, p.mu);            // lasso.py:115-117
            Dj = bx - xj;                                         // lasso.py:119
            abx += fabs(bx);
            ax1 += fabs(xj);
            const double e = fabs(g - proj(g - xj, -p.mu, p.mu)); // cpu_calculation.py:15-20
            err = (e > err || e != e) ? e : err;
        }
        p.D[j] = Dj;
    };
    if (wtile) {
        // U already summed (over ranks) or summed per lane: every wave takes its own
        // 64-column tiles; the first tile's operands were loaded at the head
        // (software-pipelined: the next tile's operands are loaded before this tile's shrink stores,
        // which the compiler could not move them past -- D and x are written in place)
        const long long tstep = (long long)cb * kWaves;
        bool have = pre;
        long long j = j0;
        for (long long tile = tile0; tile < ntile; tile += tstep) {   // wave-uniform bounds
            const long long jn = j + tstep * 64;
            const bool hn = tile + tstep < ntile && jn < p.wp;
            double ng = 0.0, nu = 0.0, nx = 0.0, nd = 0.0, ndg = 0.0, nrc = 0.0;
            if (hn) {
                const bool col = jn < p.w;
                ng = o.G[jn];
                nu = usum(jn);
                nx = col ? p.x[jn] : 0.0;
                nd = (UPDATE && col) ? p.D[jn] : 0.0;
                ndg = col ? p.diag[jn] : 0.0;
                nrc = col ? p.rec[jn] : 0.0;
            }
            if (have) shrink_col(j, pg, pu, px, pd, pdg, prc);
            have = hn;
            j = jn;
            pg = ng; pu = nu; px = nx; pd = nd; pdg = ndg; prc = nrc;
        }
    } else
    // one rank: tiles of 64 (lane = column); the 4 waves split the row-group partials of U
    // (q = wave, wave + 4, ...), wave 0 adds the 4 sums in a fixed order and runs the shrink
    for (long long tile = blockIdx.x; tile < ntile; tile += cb) {   // block-uniform
        const long long j = tile * 64 + lane;
        const bool ok = j < p.wp;
        const bool col = ok && j < p.w;
        // wave 0's column operands are loaded before the U fold and its barrier, so both sets of
        // loads are in flight together (one memory round trip instead of two)
        double g = 0.0, xj = 0.0, dold = 0.0, dg = 0.0, rc = 0.0;
        if (wave == 0 && ok) {
            g = o.G[j];
            if (col) {
                xj = p.x[j];
                if (UPDATE) dold = p.D[j];
                dg = p.diag[j];
                rc = p.rec[j];
            }
        }
        if (UPDATE) {
            double acc = 0.0;
            if (ok) {
                // 16 loads in flight per lane (configs[3]: 256 row groups, 64 per wave); the adds stay
                // in group order
#pragma unroll 16
                for (int q = wave; q < o.ngroups; q += kWaves)
                    acc += o.Uf ? (double)o.Uf[j] : o.Us[(long long)q * p.wp + j];   // Uf: ngroups = 1
            }
            ured[wave][lane] = acc;
            __syncthreads();
        }
        if (wave == 0 && ok) {
            const double u = UPDATE ? ((ured[0][lane] + ured[1][lane]) + ured[2][lane]) + ured[3][lane] : 0.0;
            shrink_col(j, g, u, xj, dold, dg, rc);
        }
        if (UPDATE) __syncthreads();   // ured is rewritten by the next tile
    }
    // block partials: wave sums, then the 4 waves in a fixed order (waves 1-3 hold zeros on the
    // one-rank path, where only wave 0 runs the shrink: adding them changes no bit)
    abx = wave_sum(abx);
    ax1 = wave_sum(ax1);
    err = wave_max(err);
    __shared__ double wred[3][kWaves];
    if (lane == 0) { wred[0][wave] = abx; wred[1][wave] = ax1; wred[2][wave] = err; }
    __syncthreads();
    if (threadIdx.x == 0) {
        abx = ((wred[0][0] + wred[0][1]) + wred[0][2]) + wred[0][3];
        ax1 = ((wred[1][0] + wred[1][1]) + wred[1][2]) + wred[1][3];
        err = wred[2][0];
        for (int q = 1; q < kWaves; ++q) err = (wred[2][q] > err || wred[2][q] != wred[2][q]) ? wred[2][q] : err;
        {
            double* dst = p.parts + 4ll * blockIdx.x;
            dst[0] = abx;
            dst[1] = ax1;
            dst[2] = err;
            dst[3] = 0.0;
            if (UPDATE && blockIdx.x == 0) {
                const long long t = p.st->t - 1;
                p.st->iters = t + 1;
                if (p.time_iter && t < p.rec_len)
                    p.time_iter[t + 1] = (double)(wall_clock64() - p.st->t_base) * p.wall_tick_s;
            }
        }
    }
}

}  // namespace bpgl
