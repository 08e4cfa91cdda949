// bpgl -- C ABI (include/bpgl.h) over the gfx950 kernels of bpgl_kernels.h.
//
// Host-side responsibilities: validate shapes before any launch, carve the
// caller's scratch buffer, choose the launch geometry, enqueue the per-block
// update sequence (optionally as one captured hipGraph per iteration), drive
// the RCCL all-reduce of the column-sharded multi-GPU path, and time kernels
// with HIP events when asked.  No hipMalloc anywhere: device memory belongs to
// the caller (PyTorch).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bpgl.h"
#include "bpgl_host.h"
#include "bpgl_kernels.h"
#include "bpgl_onepass.h"

using namespace bpgl;

namespace bpgl_host {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
}  // namespace bpgl_host
using namespace bpgl_host;

namespace {
constexpr int kTimedKinds = 9;   // + 8: the exact-gradient refresh of the one-pass iteration
constexpr int kMaxRanks = 64;

int vec_elems(int dtype) { return dtype == BPGL_F32 ? 4 : dtype == BPGL_F64 ? 2 : 8; }

}  // namespace

struct bpgl_ctx {
    int device = 0, dtype = BPGL_F32;
    int64_t m = 0, n_local = 0, w = 0, wp = 0;
    int32_t nblock = 1;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // geometry
    int nseg = 0, nchunk = 0, R = 0, segw = 0, nparts = 0;
    // bound buffers
    const void* A = nullptr;
    int64_t lda = 0, block_stride = 0;
    bool bound = false, have_diag = false;
    Params p{};
    // multi-GPU
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    bool external = false;   // nranks > 1 with the exchange done by the caller
    // solver
    bool solver = false, use_graph = false;
    // gexec[j]: a hipGraph of 2^j iterations, j < kGraphLevels, 2^j <= graph_max; a run of n iterations
    // replays the largest that fits (one replay gap per graph, not per 8 iterations)
    hipGraphExec_t gexec[kGraphLevels] = {};
    int graph_max = kGraphMaxIters;   // "graph_max" knob (RCCL contexts cap it at kGraphIters)
    // timing
    bool timing = false;
    std::vector<hipEvent_t> evs;   // 2 events per (timed iteration, kind)
    std::vector<hipEvent_t> ref_evs;   // 2 events per timed exact-gradient refresh (kind 8)
    int64_t ref_timed = 0;
    int64_t timed_iters = 0;
    bool kind_used[kTimedKinds] = {};
    double wall_tick_s = 1e-8;
    int reverse_rows = 0;
    int col_mode = 1;      // k_colpass row schedule (see launch_colpass)
    int nt_loads = 1;
    int tail_permille = 120;
    // one-pass iteration (bpgl_onepass.h)
    int cus = 256;             // CUs the persistent grid is sized for (the stream's CU mask, or "cus")
    int dev_cus = 256;         // CUs of the device
    bool cu_masked = false;    // the stream carries a CU mask narrower than the device
    int onepass = -1;          // tuning: -1 when eligible, 0 off, 1 required
    // exact g = A^T r every this many iterations (0: at reset only).  The recurrence's own drift is
    // below the trajectory's rounding sensitivity: after 1024 iterations at configs[1], x is within
    // 1-2e-7 of the two-pass iterates for periods 0, 64, 256 and 1024 alike, the objective within
    // 3e-15 (profiles/r01/sweeps/onepass_refresh_drift.jsonl); 256 keeps the refresh (one A^T r pass)
    // at 0.4 % of the iteration time
    int op_refresh = 256;
    // permille of each row group read with cache-allocating loads (-1: auto, op_cache_auto)
    int op_cache = -1;
    int op_rows = -1;          // tuning "onepass_rows": -1 auto, 0 consecutive, 1 interleaved
    int op_sb1 = -1;           // tuning "onepass_sb1": -1 auto (on when SB = 1), 0 off
    bool op_shape = false;     // the shape admits it (geometry)
    bool op_on = false;        // this solver run uses it
    int op_SB = 0, op_ngroups = 0, op_R = 0, op_xl = 0, op_tail_grid = 0, op_gpl = 1;
    int op_rowb = 1;   // k_onepass_tail: residual update on blocks of its own ("tail_row_blocks" knob)
    // row shards (bpgl_set_shard): A holds this rank's rows of the single feature block; x, D, g
    // are replicated and each one-pass iteration all-reduces [U | r.s23 | s23.s23]
    bool rows = false;
    int xch32 = 0;   // row shards' per-iteration exchange in fp32 ("exchange_fp32"; opt-in, -1 = RCCL only)
    bool op_refresh_pending = false;   // external rows: phase 2 ran, phase 3 not yet
    int64_t op_t = 0;          // iterations enqueued since the solver reset
    int64_t req_t = 0;         // iterations requested since the solver reset (bpgl_solver_step)
    int64_t op_fail_at = -1;   // test hook "onepass_fail_at": the launch of this iteration reports a failure
    // counters since the solver reset (bpgl_solver_stat)
    int64_t n_refresh = 0;     // exact-gradient refreshes enqueued
    int64_t n_fallback = 0;    // one-pass solves moved to the two-pass kernels after a failure
    OnePassArgs op{};
};

namespace {

void drop_graphs(bpgl_ctx* c) {
    for (auto& g : c->gexec)
        if (g) { (void)hipGraphExecDestroy(g); g = nullptr; }
}

void geometry(bpgl_ctx* c) {
    const int V = vec_elems(c->dtype);
    c->segw = 64 * V * kU;
    c->wp = up(c->w, V);
    c->nseg = (int)cdiv(c->wp, c->segw);
    // tiles per launch (rows per chunk a multiple of 16 = 4 waves x 4 rows): one resident wave
    // of 1024 blocks for fp32; fp64 and bf16 A measured ~3 % faster at 512
    // (profiles/r01/sweeps: tile-count sweeps per storage type)
    int64_t target = c->dtype == BPGL_F32 ? 1024 : 512;
    if (const char* e = getenv("BPGL_TARGET_BLOCKS")) target = std::max<int64_t>(1, atoll(e));
    int64_t nchunk = std::max<int64_t>(1, cdiv(target, c->nseg));
    nchunk = std::min<int64_t>(nchunk, cdiv(c->m, 16));
    int64_t R = up(cdiv(c->m, nchunk), 16);
    c->R = (int)R;
    c->nchunk = (int)cdiv(c->m, R);
    c->nparts = (int)cdiv(c->wp, kColsPerShrink);
    // one-pass geometry: SB segment blocks per row, floor(CUs / SB) row groups, one block per CU
    const int bc = c->dtype == BPGL_F32 ? OnePassGeo<4, float>::BC
                 : c->dtype == BPGL_F64 ? OnePassGeo<4, double>::BC : OnePassGeo<3, bf16_t>::BC;
    const int64_t SB = cdiv(c->wp, bc);
    // op_shape: the one-pass buffers and geometry exist (one block, SB <= 128).  Whether the persistent
    // grid fits the CUs (ngroups x SB co-resident blocks) is onepass_ineligible's question: with more
    // segment blocks than CUs (a row of 524288 fp32 columns on a 64- or 32-CU partition) there is one
    // row group, the one-pass iteration is ineligible, and RCCL row shards run the two-pass row
    // iteration on these buffers
    c->op_shape = c->nblock == 1 && SB <= kOpMaxSB;
    c->op_gpl = SB > 64 ? 2 : 1;   // k_onepass<..., 2> relies on SB > 64
    if (c->op_shape) {
        int64_t ng = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(c->cus / SB, c->m), kOpMaxGroups));
        const int64_t R = cdiv(c->m, ng);
        ng = cdiv(c->m, R);
        c->op_SB = (int)SB;
        c->op_ngroups = (int)ng;
        c->op_R = (int)R;
        c->op_xl = (ng % 8 == 0) ? 1 : 0;   // each row group's blocks on one XCD (blockIdx % 8)
        // k_onepass_tail: 64-column tiles -- one per wave when U arrives summed (row shards) or each
        // lane sums its column's few row-group partials (one rank, ngroups <= kOpTailWaveGroups); one per
        // block otherwise, its 4 waves splitting the row groups -- and 256-row strides
        c->op_tail_grid = c->rows || ng <= kOpTailWaveGroups
                              ? (int)std::min<int64_t>(cdiv(c->wp, 64 * kWaves), kOpTailBlocks)
                              : (int)std::min<int64_t>(std::max(cdiv(c->m, kThreads), cdiv(c->wp, 64)), kOpTailBlocks);
    } else {
        c->op_SB = c->op_ngroups = c->op_R = c->op_xl = c->op_tail_grid = 0;
    }
}

// "onepass_cache_permille" = -1 (default): 750 when this rank's A block fits the 256 MiB Infinity
// Cache give or take a quarter (the N = 8 row shard of the 8192 x 65536 matrix: k_onepass 57.5 ->
// 52.2 us), else 0 (all non-temporal: at 512 MiB and 2 GiB cache-allocating loads cost 1-10 %).
// Launches alternate the row direction, so the rows a launch read last are the next launch's first.
// profiles/r03/strong_cache, profiles/r03/fold_sweep
int op_cache_eff(const bpgl_ctx* c) {
    if (c->op_cache >= 0) return c->op_cache;
    const int64_t bytes = c->m * c->wp * (c->dtype == BPGL_F32 ? 4 : c->dtype == BPGL_F64 ? 8 : 2);
    return bytes <= (int64_t)320 << 20 ? 750 : 0;
}

// "onepass_rows" = -1 (default): row groups own interleaved rows (g, g + ngroups, ...) when there are at
// least 8 groups of at least 128 rows over at least 16 segment blocks -- the groups then read one contiguous
// window of A instead of ngroups streams R rows apart: configs[1] (16 groups of 512 rows) k_onepass 336.7 ->
// 331.0 us, the N = 2 and N = 4 strong row shards (4096 / 2048 rows per GPU) 187.8 -> 180.5 and 108.6 ->
// 106.3 us per iteration -- and consecutive rows otherwise: even or slower at 64-row groups (the N = 8
// strong shard, 63.0 / 62.7 us on one box, 51.6 -> 52.9 us on another), with one segment block per row
// (configs[3], 2709 -> 2757 us) and at 2 groups (the weak shard, 328 -> 333.7 us); profiles/r05/layout,
// profiles/r05/rows.  Results agree to rounding (the U partials sum other rows per group).
// granules per lane of the k_onepass instantiation in use: 0 = one segment block per row with the
// LDS-only hand-off ("onepass_sb1", default on when SB = 1; round 6; an explicit "onepass_rows" = 1
// takes the granule path, whose instantiation has the interleaved form), else 1 (SB <= 64) or 2
int op_gpl_eff(const bpgl_ctx* c) {
    return (c->op_SB == 1 && c->op_sb1 != 0 && c->op_rows != 1) ? 0 : c->op_gpl;
}
int op_rows_eff(const bpgl_ctx* c) {
    if (op_gpl_eff(c) != 1) return 0;   // the interleaved kernel is instantiated for 1 < SB <= 64 only
    if (c->op_rows >= 0) return c->op_rows;
    return c->op_SB >= 16 && c->op_ngroups >= 8 && c->op_R >= 128 ? 1 : 0;
}

// scratch layout (offsets in bytes)
struct Layout {
    int64_t slab_g, slab_s, D, parts, parts2, comm, r, Ax, st, diag, rec, opG, opUs, opPG, opS, opABE, total;
};
Layout layout(const bpgl_ctx* c) {
    Carve k;
    Layout L;
    L.st = k.take(sizeof(DevState));
    L.slab_g = k.take(8 * (int64_t)c->nchunk * c->wp);
    L.slab_s = k.take(8 * (int64_t)c->nseg * c->m);
    L.D = k.take(8 * c->wp);
    L.parts = k.take(8 * 4 * (int64_t)std::max(c->nparts, c->op_tail_grid));
    L.parts2 = k.take(8 * 2 * std::max<int64_t>(kMaxReduceBlocks, c->nchunk));
    // column shards exchange [s23 (m) | 2 | err slots]; row shards [U (wp) | r.s23 | s23.s23 | failed]
    L.comm = k.take(8 * std::max<int64_t>(c->m + 2 + kMaxRanks, c->wp + 3));
    L.r = k.take(8 * c->m);
    L.Ax = k.take(8 * (int64_t)c->nblock * c->m);
    L.diag = k.take(8 * (int64_t)c->nblock * c->wp);
    L.rec = k.take(8 * (int64_t)c->nblock * c->wp);
    const bool op = c->op_shape;
    L.opG = k.take(op ? 8 * c->wp : 0);
    L.opUs = k.take(op ? 8 * (int64_t)c->op_ngroups * c->wp : 0);
    L.opPG = k.take(op ? 8 * c->m * c->op_SB : 0);
    L.opS = k.take(op && c->rows ? 8 * c->m : 0);
    L.opABE = k.take(op && c->rows ? 8 * 4 : 0);
    L.total = k.off;
    return L;
}

dim3 grid_tiles(const bpgl_ctx* c) { return dim3((unsigned)((int64_t)c->nseg * c->nchunk)); }

template <typename T, int RPT, bool PIPE>
int launch_colpass_r(bpgl_ctx* c, int mode, const double* vec, double* slab, int fixed_block) {
    if (mode == 0 && c->nt_loads)
        hipLaunchKernelGGL((k_colpass<T, 0, true, RPT, PIPE>), grid_tiles(c), dim3(kThreads), 0, c->stream, c->p, vec,
                           slab, fixed_block);
    else if (mode == 0)
        hipLaunchKernelGGL((k_colpass<T, 0, false, RPT, PIPE>), grid_tiles(c), dim3(kThreads), 0, c->stream, c->p, vec,
                           slab, fixed_block);
    else
        hipLaunchKernelGGL((k_colpass<T, 1, false, 2, false>), grid_tiles(c), dim3(kThreads), 0, c->stream, c->p, vec,
                           slab, fixed_block);
    LAUNCH_CHECK("k_colpass");
    return 0;
}
// col_mode: 0 = 2 rows per trip, 1 = 4 rows per trip, 2 = 2 rows per trip software-pipelined
template <typename T>
int launch_colpass(bpgl_ctx* c, int mode, const double* vec, double* slab, int fixed_block) {
    switch (c->col_mode) {
        case 1: return launch_colpass_r<T, 4, false>(c, mode, vec, slab, fixed_block);
        case 2: return launch_colpass_r<T, 2, true>(c, mode, vec, slab, fixed_block);
        default: return launch_colpass_r<T, 2, false>(c, mode, vec, slab, fixed_block);
    }
}
int colpass(bpgl_ctx* c, int mode, const double* vec, double* slab, int fixed_block) {
    switch (c->dtype) {
        case BPGL_F32: return launch_colpass<float>(c, mode, vec, slab, fixed_block);
        case BPGL_F64: return launch_colpass<double>(c, mode, vec, slab, fixed_block);
        default: return launch_colpass<bf16_t>(c, mode, vec, slab, fixed_block);
    }
}
template <typename T>
int launch_rowpass(bpgl_ctx* c, const double* d, double* slab, int fixed_block) {
    if (c->nt_loads)
        hipLaunchKernelGGL((k_rowpass<T, true>), grid_tiles(c), dim3(kThreads), 0, c->stream, c->p, d, slab, fixed_block);
    else
        hipLaunchKernelGGL((k_rowpass<T, false>), grid_tiles(c), dim3(kThreads), 0, c->stream, c->p, d, slab, fixed_block);
    LAUNCH_CHECK("k_rowpass");
    return 0;
}
int rowpass(bpgl_ctx* c, const double* d, double* slab, int fixed_block) {
    switch (c->dtype) {
        case BPGL_F32: return launch_rowpass<float>(c, d, slab, fixed_block);
        case BPGL_F64: return launch_rowpass<double>(c, d, slab, fixed_block);
        default: return launch_rowpass<bf16_t>(c, d, slab, fixed_block);
    }
}

unsigned rowreduce_blocks(const bpgl_ctx* c) {
    return (unsigned)std::min<int64_t>(cdiv(c->m, kRowsPerReduce), kMaxReduceBlocks);
}
int rowreduce_p(bpgl_ctx* c, const Params& q, const double* slab, double* out, int mode) {
    const dim3 g(rowreduce_blocks(c)), b(kThreads);
    // one batch of loads per wave covers the segments: 4 waves x BATCH >= nseg
    if (q.nseg <= 4) hipLaunchKernelGGL(k_rowreduce<1>, g, b, 0, c->stream, q, slab, out, mode);
    else if (q.nseg <= 16) hipLaunchKernelGGL(k_rowreduce<4>, g, b, 0, c->stream, q, slab, out, mode);
    else hipLaunchKernelGGL(k_rowreduce<16>, g, b, 0, c->stream, q, slab, out, mode);
    LAUNCH_CHECK("k_rowreduce");
    if (mode == 1) {
        hipLaunchKernelGGL(k_linesearch, dim3(1), dim3(kThreads), 0, c->stream, q, (int)rowreduce_blocks(c),
                           (const float*)nullptr);
        LAUNCH_CHECK("k_linesearch");
    }
    return 0;
}
int rowreduce(bpgl_ctx* c, const double* slab, double* out, int mode) { return rowreduce_p(c, c->p, slab, out, mode); }

// ---------------------------------------------------------------------------
// one-pass iteration (bpgl_onepass.h)
// ---------------------------------------------------------------------------
// ring slots NB and rows in flight PF per storage type; the loads per lane and row (LU: 4 KiB of
// fp32 / fp64, 3 KiB of bf16 A per wave and row) set the geometry.  Round 4 re-measured the deeper
// and shallower rings (NB 14-18, PF 3-4; bf16 NB 9-11) at 1024 x 65536 and 8192 x 65536: the
// defaults stayed best (61.6-81.5 us against 60.6 us per strong N = 8 shard,
// profiles/r04/split_model/variants_m1024); the variants were removed in round 5.  bf16 takes LU 3:
// its per-row instruction path (the same 16-24 fp64 FMAs and wave sums as fp32) limits it at LU 2
// (2.9k it/s), LU 4 spills;
// LU 3 with a 12-row ring reaches 3.4-3.5k it/s at configs[1]'s shape.
// profiles/r01/sweeps/onepass6_probe.jsonl, onepass_bf16_lu3_variants.jsonl
template <typename T> struct OpLU { static constexpr int LU = 4; };
template <> struct OpLU<bf16_t> { static constexpr int LU = 3; };
template <typename T> struct OpRing { static constexpr int NB = 16, PF = 3; };
template <> struct OpRing<bf16_t> { static constexpr int NB = 12, PF = 2; };

// the two-pass kernels' view of one-pass state: g is read from G (one slab row), s23 from S
Params op_params(const bpgl_ctx* c) {
    Params q = c->p;
    q.slab_g = c->op.G;
    q.nchunk = 1;
    q.nseg = 1;
    q.nparts = c->op_tail_grid;   // shrink partials come from k_onepass_tail
    return q;
}
// GPL: granules per lane of the row hand-off (SB <= 64: 1, SB <= 128: 2); RILV: interleaved row groups
// (instantiated for GPL 1 only: "onepass_rows" applies when SB <= 64)
template <typename T, int GPL, bool RILV>
const void* onepass_fn_g() { return (const void*)k_onepass<T, OpRing<T>::NB, OpRing<T>::PF, OpLU<T>::LU, GPL, RILV>; }
template <typename T>
const void* onepass_fn_t(int gpl, int rilv) {
    return gpl == 2 ? onepass_fn_g<T, 2, false>() : gpl == 0 ? onepass_fn_g<T, 0, false>()
                     : rilv ? onepass_fn_g<T, 1, true>() : onepass_fn_g<T, 1, false>();
}
const void* onepass_fn(int dtype, int gpl, int rilv) {
    return dtype == BPGL_F32 ? onepass_fn_t<float>(gpl, rilv) : dtype == BPGL_F64 ? onepass_fn_t<double>(gpl, rilv)
                                                                                   : onepass_fn_t<bf16_t>(gpl, rilv);
}
template <typename T, int GPL, bool RILV>
void onepass_launch_g(bpgl_ctx* c) {
    hipLaunchKernelGGL((k_onepass<T, OpRing<T>::NB, OpRing<T>::PF, OpLU<T>::LU, GPL, RILV>),
                       dim3((unsigned)(c->op_ngroups * c->op_SB)), dim3(kThreads), 0, c->stream, op_params(c), c->op);
}
template <typename T>
void onepass_launch_t(bpgl_ctx* c) {
    const int gpl = op_gpl_eff(c);
    if (gpl == 2) onepass_launch_g<T, 2, false>(c);
    else if (gpl == 0) onepass_launch_g<T, 0, false>(c);
    else if (c->op.rilv) onepass_launch_g<T, 1, true>(c);
    else onepass_launch_g<T, 1, false>(c);
}
int onepass_launch(bpgl_ctx* c) {
    switch (c->dtype) {
        case BPGL_F32: onepass_launch_t<float>(c); break;
        case BPGL_F64: onepass_launch_t<double>(c); break;
        default: onepass_launch_t<bf16_t>(c); break;
    }
    LAUNCH_CHECK("k_onepass");
    return 0;
}
// the one-pass tail's view of U: the row-group partials (one rank), or the all-reduced sum
// in the exchange buffer (row shards)
// Row shards exchange [U | r.s23 | s23.s23 | failed] in fp32 (U rounded, the scalars as hi + lo
// pairs, exact to ~2^-48 for one rank; summed over several ranks RCCL rounds each hi and lo sum
// to fp32, so the scalars are then fp32-accurate): half the all-reduce bytes; measured drift
// DESIGN.md section 6 (1.8e-7 with one rank, 1.5e-6 with eight: each rank's partial is rounded
// before the cross-rank cancellation), so it is opt-in: 1 = any row-shard exchange, -1 = RCCL
// communicators only, 0 (default) = fp64.  The exact-gradient refresh is always fp64.
bool xch_f32(const bpgl_ctx* c) {
    return c->rows && c->op_on && (c->xch32 > 0 || (c->xch32 < 0 && c->comm && !c->external));
}
OnePassArgs op_tail_args(const bpgl_ctx* c) {
    OnePassArgs o = c->op;
    if (c->rows) {
        o.Us = c->p.comm;
        o.ngroups = 1;
        if (xch_f32(c)) o.Uf = reinterpret_cast<const float*>(c->p.comm);
    } else {
        o.tailw = c->op_ngroups <= kOpTailWaveGroups ? 1 : 0;
    }
    return o;
}
template <bool UPDATE>
int onepass_tail(bpgl_ctx* c) {
    OnePassArgs o = op_tail_args(c);
    // the residual update on blocks of its own (about 2 rows per thread, at most kOpTailBlocks blocks)
    o.rowb = UPDATE && c->op_rowb ? (int)std::min<int64_t>(cdiv(c->m, 2 * kThreads), kOpTailBlocks) : 0;
    hipLaunchKernelGGL(k_onepass_tail<UPDATE>, dim3((unsigned)(c->op_tail_grid + o.rowb)), dim3(kThreads), 0,
                       c->stream, op_params(c), o);
    LAUNCH_CHECK("k_onepass_tail");
    return 0;
}
int allreduce_sum(bpgl_ctx* c, double* buf, int64_t count) {
    ncclResult_t nr = ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, c->comm, c->stream);
    if (nr != ncclSuccess) return fail(BPGL_E_RCCL, "ncclAllReduce: %s", ncclGetErrorString(nr));
    return 0;
}
// this rank's A^T r into dst (row shards: a partial over ranks)
int onepass_local_gradient(bpgl_ctx* c, double* dst) {
    int rc;
    if ((rc = colpass(c, 0, c->p.r, c->p.slab_g, -1))) return rc;
    hipLaunchKernelGGL(k_colreduce, dim3((unsigned)cdiv(c->wp, kThreads)), dim3(kThreads), 0, c->stream, c->p.slab_g,
                       c->wp, c->nchunk, dst, (double*)nullptr);
    LAUNCH_CHECK("k_colreduce");
    return 0;
}
// exact g = A^T r into G (at reset and every op_refresh iterations); row shards sum it over ranks
int onepass_refresh(bpgl_ctx* c) {
    int rc;
    if ((rc = onepass_local_gradient(c, c->op.G))) return rc;
    if (c->rows && c->comm && (rc = allreduce_sum(c, c->op.G, c->wp))) return rc;
    return onepass_tail<false>(c);   // the shrink of the next iteration from the exact g
}
// can this solver run use the one-pass iteration?  (0 yes; else the reason)
const char* onepass_ineligible(bpgl_ctx* c) {
    if (!c->op_shape) return "needs one feature block and at most 128 segment blocks per row";
    if (!c->rows && (c->nranks != 1 || c->comm || c->external))
        return "column shards need a single rank without a communicator (row shards run it on several)";
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, onepass_fn(c->dtype, op_gpl_eff(c), op_rows_eff(c)), kThreads, 0) != hipSuccess || nb < 1)
        return "kernel does not fit on a CU";
    if ((int64_t)c->op_ngroups * c->op_SB > (int64_t)nb * c->cus) return "grid exceeds the resident capacity";
    return nullptr;
}

int check_ready(const bpgl_ctx* c) {
    if (!c) return fail(BPGL_E_ARG, "null context");
    if (!c->bound) return fail(BPGL_E_STATE, "bpgl_bind has not been called");
    return 0;
}

// kinds: 0 colpass, 1 shrink, 2 rowpass, 3 rowreduce, 4 allreduce, 5 step, 6 update, 7 onepass;
// event 2 * (it * kinds + kind) + {0: start, 1: end}.  Kind 8 (the refresh, not in every
// iteration) has its own event list, 2 per refresh.
void ev_record(bpgl_ctx* c, int64_t it, int kind, int end) {
    if (!c->timing) return;
    if (kind == 8) {
        const size_t idx = 2 * (size_t)c->ref_timed + end;
        while (c->ref_evs.size() <= idx) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return;
            c->ref_evs.push_back(e);
        }
        (void)hipEventRecord(c->ref_evs[idx], c->stream);
        if (end) c->ref_timed++;
        c->kind_used[kind] = true;
        return;
    }
    const size_t idx = 2 * ((size_t)it * kTimedKinds + kind) + end;
    while (c->evs.size() <= idx) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->evs.push_back(e);
    }
    (void)hipEventRecord(c->evs[idx], c->stream);
    c->kind_used[kind] = true;
}

// phase 0: colpass, shrink, rowpass, rowreduce [, allreduce, step]; phase 1: update.
// With the caller doing the exchange (external ranks) phase 0 stops after
// rowreduce and phase 1 starts with the step.
// one-pass iteration, two kernels: k_onepass (s23 and the U partials; its row groups also
// fold r.s23 and s23.s23, and the last group to finish runs the line search); phase 1:
// k_onepass_tail (x, Ax, r, g += gamma U and the next iteration's shrink)
//
// Row shards: k_onepass, k_onepass_fold -> exchange buffer [U | r.s23 | s23.s23 | failed],
// all-reduce (RCCL); phase 1: k_onepass_tail, which runs the line search on the summed scalars
// at its head and then applies the summed U.  With the exchange done by the caller (external
// ranks) phase 0 ends after the fold and phase 1 is the tail.
int enqueue_phase_onepass_rows(bpgl_ctx* c, int64_t it, int phase) {
    int rc;
    if (phase == 0) {
        ev_record(c, it, 7, 0);
        if ((rc = onepass_launch(c))) return rc;
        ev_record(c, it, 7, 1);
        float* xf = xch_f32(c) ? reinterpret_cast<float*>(c->p.comm) : nullptr;
        ev_record(c, it, 3, 0);
        hipLaunchKernelGGL(k_onepass_fold, dim3((unsigned)std::min<int64_t>(cdiv(c->wp, kThreads), 1024) + 1),
                           dim3(kThreads), 0, c->stream, op_params(c), c->op, c->p.comm, xf);
        LAUNCH_CHECK("k_onepass_fold");
        ev_record(c, it, 3, 1);
        if (c->comm) {
            ev_record(c, it, 4, 0);
            if (xf) {
                ncclResult_t nr = ncclAllReduce(xf, xf, (size_t)(c->wp + 5), ncclFloat32, ncclSum, c->comm, c->stream);
                if (nr != ncclSuccess) return fail(BPGL_E_RCCL, "ncclAllReduce: %s", ncclGetErrorString(nr));
            } else if ((rc = allreduce_sum(c, c->p.comm, c->wp + 3))) {
                return rc;
            }
            ev_record(c, it, 4, 1);
        }
    }
    // the line search runs at the head of k_onepass_tail (o.abe: the fold pre-summed the shrink
    // partials; [r.s23, s23.s23] come from the exchange buffer)
    if (phase == 1) {
        ev_record(c, it, 6, 0);
        if ((rc = onepass_tail<true>(c))) return rc;
        ev_record(c, it, 6, 1);
    }
    return 0;
}

// Row shards on the two-pass kernels (RCCL ranks; after a failed one-pass hand-off, or with
// "onepass" = 0): phase 0 = the exact g = sum_q A_q^T r_q (colpass, colreduce, all-reduce of
// w_pad) and the shrink, s23_q = A_q D on the local rows (rowpass, rowreduce), the line-search
// partials and ONE all-reduce of [r.s23 | s23.s23 | failed] (3 fp64); phase 1 = k_onepass_tail
// (the line search at its head; U = 0).  Two passes over A_q and two all-reduces per iteration,
// but no co-residency requirement.
int enqueue_phase_rows_twopass(bpgl_ctx* c, int64_t it, int phase) {
    int rc;
    if (phase == 0) {
        ev_record(c, it, 0, 0);
        if ((rc = onepass_refresh(c))) return rc;     // exact g, then the shrink (tail<false>)
        ev_record(c, it, 0, 1);
        ev_record(c, it, 2, 0);
        if ((rc = rowpass(c, c->p.D, c->p.slab_s, -1))) return rc;
        const dim3 g(rowreduce_blocks(c)), b(kThreads);
        if (c->p.nseg <= 4) hipLaunchKernelGGL(k_rowreduce<1>, g, b, 0, c->stream, c->p, c->p.slab_s, c->op.S, 1);
        else if (c->p.nseg <= 16) hipLaunchKernelGGL(k_rowreduce<4>, g, b, 0, c->stream, c->p, c->p.slab_s, c->op.S, 1);
        else hipLaunchKernelGGL(k_rowreduce<16>, g, b, 0, c->stream, c->p, c->p.slab_s, c->op.S, 1);
        LAUNCH_CHECK("k_rowreduce");
        ev_record(c, it, 2, 1);
        ev_record(c, it, 3, 0);
        HIP_TRY(hipMemsetAsync(c->p.comm, 0, 8 * c->wp, c->stream));
        hipLaunchKernelGGL(k_rows2_fold, dim3(1), dim3(kThreads), 0, c->stream, op_params(c), c->op, c->p.comm,
                           (int)rowreduce_blocks(c));
        LAUNCH_CHECK("k_rows2_fold");
        ev_record(c, it, 3, 1);
        ev_record(c, it, 4, 0);
        if (c->comm && (rc = allreduce_sum(c, c->p.comm + c->wp, 3))) return rc;
        ev_record(c, it, 4, 1);
    } else {
        ev_record(c, it, 6, 0);
        if ((rc = onepass_tail<true>(c))) return rc;
        ev_record(c, it, 6, 1);
    }
    return 0;
}

int enqueue_phase_onepass(bpgl_ctx* c, int64_t it, int phase) {
    int rc;
    if (c->rows) return enqueue_phase_onepass_rows(c, it, phase);
    if (phase == 0) {   // k_onepass ends with the line search (its last row group)
        ev_record(c, it, 7, 0);
        if ((rc = onepass_launch(c))) return rc;
        ev_record(c, it, 7, 1);
    } else {
        ev_record(c, it, 6, 0);
        if ((rc = onepass_tail<true>(c))) return rc;
        ev_record(c, it, 6, 1);
    }
    return 0;
}

int enqueue_phase(bpgl_ctx* c, int64_t it, int phase) {
    int rc;
    if (c->op_on) return enqueue_phase_onepass(c, it, phase);
    if (c->rows) return enqueue_phase_rows_twopass(c, it, phase);
    const bool multi = c->comm != nullptr || c->external;
    if (phase == 0) {
        ev_record(c, it, 0, 0);
        if ((rc = colpass(c, 0, c->p.r, c->p.slab_g, -1))) return rc;
        ev_record(c, it, 0, 1);
        ev_record(c, it, 1, 0);
        hipLaunchKernelGGL(k_shrink, dim3((unsigned)c->nparts), dim3(kThreads), 0, c->stream, c->p);
        LAUNCH_CHECK("k_shrink");
        ev_record(c, it, 1, 1);
        ev_record(c, it, 2, 0);
        if ((rc = rowpass(c, c->p.D, c->p.slab_s, -1))) return rc;
        ev_record(c, it, 2, 1);
        ev_record(c, it, 3, 0);
        if ((rc = rowreduce(c, c->p.slab_s, c->p.comm, multi ? 2 : 1))) return rc;
        ev_record(c, it, 3, 1);
        if (c->comm) {
            ev_record(c, it, 4, 0);
            ncclResult_t nr = ncclAllReduce(c->p.comm, c->p.comm, (size_t)(c->m + 2 + c->nranks), ncclFloat64,
                                            ncclSum, c->comm, c->stream);
            if (nr != ncclSuccess) return fail(BPGL_E_RCCL, "ncclAllReduce: %s", ncclGetErrorString(nr));
            ev_record(c, it, 4, 1);
        }
    }
    if ((phase == 0 && c->comm) || (phase == 1 && c->external)) {
        ev_record(c, it, 5, 0);
        hipLaunchKernelGGL(k_step, dim3(1), dim3(kStepThreads), 0, c->stream, c->p);
        LAUNCH_CHECK("k_step");
        ev_record(c, it, 5, 1);
    }
    if (phase == 1) {
        ev_record(c, it, 6, 0);
        const int64_t nupd = std::max<int64_t>(c->wp, c->m);
        const unsigned ublocks = (unsigned)std::min<int64_t>(cdiv(nupd, kThreads), 1024);
        hipLaunchKernelGGL(k_update, dim3(ublocks), dim3(kThreads), 0, c->stream, c->p);
        LAUNCH_CHECK("k_update");
        ev_record(c, it, 6, 1);
    }
    return 0;
}

// One block update, enqueued on c->stream.  The block index and every
// iteration-dependent value are read on the device from the state words, so
// the same launch sequence (or its captured graph) serves every iteration.
int enqueue_iteration(bpgl_ctx* c, int64_t it) {
    int rc;
    if ((rc = enqueue_phase(c, it, 0))) return rc;
    return enqueue_phase(c, it, 1);
}

// largest graph a context captures: RCCL contexts keep kGraphIters (each captured iteration holds
// an all-reduce node), the others graph_max
int graph_cap(const bpgl_ctx* c) { return c->comm ? std::min(c->graph_max, kGraphIters) : c->graph_max; }

// hipGraphs of 1, 2, 4, ... graph_cap iterations (c->use_graph), uploaded to the device here so
// the first replay inside a caller's timed region pays no upload
int capture_graphs(bpgl_ctx* c) {
    drop_graphs(c);
    if (!c->use_graph) return 0;
    int rc = 0;
    const bool was_timing = c->timing;
    c->timing = false;
    for (int level = 0; level < kGraphLevels && (1 << level) <= graph_cap(c) && !rc; ++level) {
        const int iters = 1 << level;
        hipGraph_t graph = nullptr;
        HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < iters && !rc; ++k) rc = enqueue_iteration(c, 0);
        hipError_t ec = hipStreamEndCapture(c->stream, &graph);
        if (rc) { if (graph) (void)hipGraphDestroy(graph); break; }
        if (ec != hipSuccess) { rc = fail(BPGL_E_HIP, "hipStreamEndCapture: %s", hipGetErrorString(ec)); break; }
        hipGraphExec_t* dst = &c->gexec[level];
        hipError_t ei = hipGraphInstantiate(dst, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) { rc = fail(BPGL_E_HIP, "hipGraphInstantiate: %s", hipGetErrorString(ei)); break; }
        if ((ei = hipGraphUpload(*dst, c->stream)) != hipSuccess)
            rc = fail(BPGL_E_HIP, "hipGraphUpload: %s", hipGetErrorString(ei));
    }
    c->timing = was_timing;
    return rc;
}

// enqueue n_iter iterations (graph replays when captured), with the one-pass exact-gradient
// refresh every op_refresh iterations
int step_impl(bpgl_ctx* c, int64_t n_iter) {
    int rc;
    const int64_t K = c->op_on ? c->op_refresh : 0;
    for (int64_t i = 0; i < n_iter;) {
        if (K > 0 && c->op_t > 0 && c->op_t % K == 0) {
            ev_record(c, c->timed_iters, 8, 0);
            c->n_refresh++;
            if ((rc = onepass_refresh(c))) return rc;
            ev_record(c, c->timed_iters, 8, 1);
        }
        const int64_t room = K > 0 ? std::min<int64_t>(n_iter - i, K - c->op_t % K) : n_iter - i;
        int64_t k = 1;
        int level = -1;   // the largest captured graph that fits the room
        if (!c->timing)
            for (int j = kGraphLevels - 1; j >= 0 && level < 0; --j)
                if (c->gexec[j] && room >= (int64_t(1) << j)) level = j;
        if (level >= 0) {
            HIP_TRY(hipGraphLaunch(c->gexec[level], c->stream));
            k = int64_t(1) << level;
        } else {
            if ((rc = enqueue_iteration(c, c->timing ? c->timed_iters : 0))) return rc;
            if (c->timing) c->timed_iters++;
        }
        i += k;
        c->op_t += k;
    }
    return 0;
}

// A one-pass launch whose row hand-off ran out of polls (its blocks were not all resident:
// another kernel or process held CUs) commits nothing, and neither does any iteration after
// it until the flag is cleared (bpgl_onepass.h).  Re-run the iterations that were lost on the
// two-pass kernels, which need no co-residency, and stay on them for the rest of this solve:
// one rank on the ordinary two-pass iteration, RCCL row shards on the two-pass row iteration
// (every rank sees the same summed failure flag, so every rank switches at the same iteration;
// RCCL ranks must all call bpgl_solver_status at the same point).  External-exchange ranks
// get BPGL_E_EXCHANGE with the state intact.
int read_state(bpgl_ctx* c, DevState& st) {
    HIP_TRY(hipMemcpyAsync(&st, c->p.st, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}
int recover_onepass(bpgl_ctx* c, DevState& st) {
    int rc;
    while (st.op_fail) {
        HIP_TRY(hipMemsetAsync(&c->p.st->op_fail, 0, sizeof st.op_fail, c->stream));
        const int64_t t = st.t;
        c->op_fail_at = -1;   // the test hook fires once
        c->op.fail_at = -1;
        if (c->external)
            return fail(BPGL_E_EXCHANGE, "one-pass row hand-off timed out (blocks not co-resident); iterations from "
                                         "t = %lld on were not applied and the solver state is intact: run them again",
                        (long long)t);
        if (!c->op_on)   // cannot happen: only k_onepass raises the flag
            return fail(BPGL_E_EXCHANGE, "hand-off failure flag set outside the one-pass iteration at t = %lld",
                        (long long)t);
        c->op_on = false;
        c->n_fallback++;
        if ((rc = capture_graphs(c))) return rc;
        if (!st.done && c->req_t > t && (rc = step_impl(c, c->req_t - t))) return rc;
        if ((rc = read_state(c, st))) return rc;
    }
    return 0;
}

}  // namespace

extern "C" {

const char* bpgl_last_error(void) { return bpgl_host::g_err.c_str(); }
int bpgl_version(void) { return 302; }

int bpgl_stream_create(int device, const uint32_t* cu_mask, int32_t mask_words, void** out) {
    if (!out) return fail(BPGL_E_ARG, "out is null");
    *out = nullptr;
    if (cu_mask && mask_words <= 0) return fail(BPGL_E_ARG, "mask_words must be > 0");
    HIP_TRY(hipSetDevice(device));
    hipStream_t s = nullptr;
    if (cu_mask) {
        int dev_cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, device));
        if (popcount_mask(cu_mask, mask_words, dev_cus) == 0) return fail(BPGL_E_ARG, "the CU mask selects no CU");
        HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask));
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    *out = (void*)s;
    return 0;
}

int bpgl_stream_destroy(void* stream) {
    if (stream) HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return 0;
}

int bpgl_create(bpgl_ctx** out, int device, int a_dtype, int64_t m, int64_t n_local, int32_t nblock,
                void* hip_stream) {
    if (!out) return fail(BPGL_E_ARG, "out is null");
    *out = nullptr;
    if (a_dtype != BPGL_F32 && a_dtype != BPGL_F64 && a_dtype != BPGL_BF16)
        return fail(BPGL_E_ARG, "unknown dtype %d", a_dtype);
    if (m <= 0 || n_local <= 0 || nblock <= 0) return fail(BPGL_E_ARG, "m, n_local, nblock must be > 0");
    if (n_local % nblock) return fail(BPGL_E_ARG, "n_local (%lld) must be divisible by nblock (%d)",
                                      (long long)n_local, nblock);
    if (m > (int64_t)1 << 40) return fail(BPGL_E_ARG, "m too large");
    HIP_TRY(hipSetDevice(device));
    bpgl_ctx* c = new bpgl_ctx();
    c->device = device;
    c->dtype = a_dtype;
    c->m = m;
    c->n_local = n_local;
    c->nblock = nblock;
    c->w = n_local / nblock;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->cus = cus;
    c->dev_cus = c->cus;
    if (hip_stream) {
        c->stream = (hipStream_t)hip_stream;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            return fail(BPGL_E_HIP, "hipStreamCreate failed");
        }
        c->own_stream = true;
    }
    {   // a CU-masked stream (bpgl_stream_create): the persistent one-pass grid is sized to the CUs
        // the stream may use, so all of its blocks stay resident beside other masked streams
        const int n = stream_cus(c->stream, c->dev_cus);
        if (n > 0 && n < c->dev_cus) {
            c->cus = n;
            c->cu_masked = true;
        }
    }
    int rate_khz = 0;
    if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && rate_khz > 0)
        c->wall_tick_s = 1.0 / (1000.0 * rate_khz);
    geometry(c);
    if (c->nchunk > 0x7fffffff / std::max(1, c->nseg)) {
        delete c;
        return fail(BPGL_E_ARG, "grid too large");
    }
    *out = c;
    return 0;
}

void bpgl_destroy(bpgl_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);   // destroy path: nothing to report to
    drop_graphs(c);
    for (auto e : c->evs) (void)hipEventDestroy(e);
    for (auto e : c->ref_evs) (void)hipEventDestroy(e);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

void* bpgl_stream(bpgl_ctx* c) { return c ? (void*)c->stream : nullptr; }

int64_t bpgl_scratch_bytes(const bpgl_ctx* c) { return c ? layout(c).total : -1; }
int64_t bpgl_block_width_padded(const bpgl_ctx* c) { return c ? c->wp : -1; }

int bpgl_geometry(const bpgl_ctx* c, int32_t* nseg, int32_t* nchunk, int32_t* R, int32_t* segw) {
    if (!c) return fail(BPGL_E_ARG, "null context");
    if (nseg) *nseg = c->nseg;
    if (nchunk) *nchunk = c->nchunk;
    if (R) *R = c->R;
    if (segw) *segw = c->segw;
    return 0;
}

int bpgl_bind(bpgl_ctx* c, const void* A, int64_t lda, int64_t block_stride, void* scratch,
              int64_t scratch_bytes) {
    if (!c) return fail(BPGL_E_ARG, "null context");
    if (!A || !scratch) return fail(BPGL_E_ARG, "A and scratch must be non-null");
    const int V = vec_elems(c->dtype);
    if (((uintptr_t)A) % 16) return fail(BPGL_E_ARG, "A must be 16-byte aligned");
    if (((uintptr_t)scratch) % 256) return fail(BPGL_E_ARG, "scratch must be 256-byte aligned");
    if (lda < c->wp || lda % V) return fail(BPGL_E_ARG, "lda (%lld) must be >= w_pad (%lld) and a multiple of %d",
                                            (long long)lda, (long long)c->wp, V);
    if (c->nblock > 1 && (block_stride % V || block_stride < c->wp))
        return fail(BPGL_E_ARG, "block_stride (%lld) must be a multiple of %d and >= w_pad",
                    (long long)block_stride, V);
    const Layout L = layout(c);
    if (scratch_bytes < L.total)
        return fail(BPGL_E_SCRATCH, "scratch too small: %lld < %lld", (long long)scratch_bytes, (long long)L.total);
    c->A = A;
    c->lda = lda;
    c->block_stride = block_stride;
    char* s = (char*)scratch;
    Params& p = c->p;
    p = Params{};
    p.A = A;
    p.lda = lda;
    p.block_stride = block_stride;
    p.m = c->m;
    p.w = c->w;
    p.wp = c->wp;
    p.nblock = c->nblock;
    p.nseg = c->nseg;
    p.nchunk = c->nchunk;
    p.R = c->R;
    p.nparts = c->nparts;
    p.nranks = c->nranks;
    p.rank = c->rank;
    p.slab_g = (double*)(s + L.slab_g);
    p.slab_s = (double*)(s + L.slab_s);
    p.D = (double*)(s + L.D);
    p.parts = (double*)(s + L.parts);
    p.parts2 = (double*)(s + L.parts2);
    p.reverse_rows = c->reverse_rows;
    p.tail_permille = c->tail_permille;
    p.comm = (double*)(s + L.comm);
    p.r = (double*)(s + L.r);
    p.Ax = (double*)(s + L.Ax);
    p.st = (DevState*)(s + L.st);
    p.diag = (const double*)(s + L.diag);
    p.rec = (const double*)(s + L.rec);
    p.wall_tick_s = c->wall_tick_s;
    c->op = OnePassArgs{};
    if (c->op_shape) {
        c->op.G = (double*)(s + L.opG);
        // s23 goes straight into the exchange buffer k_update reads (row shards: that buffer
        // carries U, s23 stays local)
        c->op.S = c->rows ? (double*)(s + L.opS) : p.comm;
        c->op.Us = (double*)(s + L.opUs);
        c->op.PG = (unsigned long long*)(s + L.opPG);
        c->op.SB = c->op_SB;
        c->op.ngroups = c->op_ngroups;
        c->op.R = c->op_R;
        c->op.xl = c->op_xl;
        c->op.ls = c->rows ? 0 : 1;   // row shards: the line search follows the all-reduce (in the tail)
        c->op.abe = c->rows ? (double*)(s + L.opABE) : nullptr;
        c->op.cache_permille = op_cache_eff(c);
        c->op.rilv = op_rows_eff(c);
    }
    c->op.fail_at = c->op_fail_at;
    HIP_TRY(hipSetDevice(c->device));
    if (c->op_shape) {
        HIP_TRY(hipMemsetAsync(s + L.opPG, 0, 8 * c->m * c->op_SB, c->stream));   // tag 0: never written
    }
    HIP_TRY(hipMemsetAsync(s + L.st, 0, sizeof(DevState), c->stream));
    HIP_TRY(hipMemsetAsync(s + L.D, 0, 8 * c->wp, c->stream));
    if (8ll * c->nchunk * c->wp >= (1ll << 31) || 8ll * c->nseg * c->m >= (1ll << 31))
        return fail(BPGL_E_ARG, "split-K slabs exceed 2 GiB (raise BPGL_TARGET_BLOCKS granularity)");
    c->bound = true;
    c->have_diag = false;
    c->solver = false;
    drop_graphs(c);
    return 0;
}

int bpgl_diag_ata(bpgl_ctx* c, double* out) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    for (int b = 0; b < c->nblock; ++b) {
        if ((rc = colpass(c, 1, nullptr, c->p.slab_g, b))) return rc;
        double* dst = const_cast<double*>(c->p.diag) + (int64_t)b * c->wp;
        double* rdst = const_cast<double*>(c->p.rec) + (int64_t)b * c->wp;
        hipLaunchKernelGGL(k_colreduce, dim3((unsigned)cdiv(c->wp, kThreads)), dim3(kThreads), 0, c->stream,
                           c->p.slab_g, c->wp, c->nchunk, dst, rdst);
        LAUNCH_CHECK("k_colreduce");
    }
    if (c->rows && c->comm) {   // row shards: column norms are sums over ranks
        double* dg = const_cast<double*>(c->p.diag);
        if ((rc = allreduce_sum(c, dg, c->wp))) return rc;
        hipLaunchKernelGGL(k_recip, dim3((unsigned)cdiv(c->wp, kThreads)), dim3(kThreads), 0, c->stream, dg,
                           const_cast<double*>(c->p.rec), c->wp);
        LAUNCH_CHECK("k_recip");
    }
    if (out)
        HIP_TRY(hipMemcpyAsync(out, c->p.diag, 8 * (size_t)c->nblock * c->wp, hipMemcpyDeviceToDevice, c->stream));
    c->have_diag = true;
    return 0;
}

int bpgl_set_diag(bpgl_ctx* c, const double* diag) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    if (!diag) return fail(BPGL_E_ARG, "null diag");
    HIP_TRY(hipSetDevice(c->device));
    const int64_t n = (int64_t)c->nblock * c->wp;
    double* dg = const_cast<double*>(c->p.diag);
    if (diag != dg) HIP_TRY(hipMemcpyAsync(dg, diag, 8 * (size_t)n, hipMemcpyDeviceToDevice, c->stream));
    hipLaunchKernelGGL(k_recip, dim3((unsigned)cdiv(n, kThreads)), dim3(kThreads), 0, c->stream, dg,
                       const_cast<double*>(c->p.rec), n);
    LAUNCH_CHECK("k_recip");
    c->have_diag = true;
    c->solver = false;
    drop_graphs(c);
    return 0;
}

int bpgl_set_shard(bpgl_ctx* c, int mode) {
    if (!c) return fail(BPGL_E_ARG, "null context");
    if (mode != BPGL_SHARD_COLUMNS && mode != BPGL_SHARD_ROWS) return fail(BPGL_E_ARG, "unknown shard mode %d", mode);
    if (c->bound) return fail(BPGL_E_STATE, "bpgl_set_shard must precede bpgl_bind");
    if (mode == BPGL_SHARD_ROWS && c->nblock != 1) return fail(BPGL_E_ARG, "row shards need one feature block");
    c->rows = mode == BPGL_SHARD_ROWS;
    geometry(c);   // the tail's grid differs for row shards
    return 0;
}

int bpgl_mtv(bpgl_ctx* c, int32_t block, const double* r, double* g) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    if (block < 0 || block >= c->nblock) return fail(BPGL_E_ARG, "block %d out of range", block);
    if (!r || !g) return fail(BPGL_E_ARG, "null vector");
    HIP_TRY(hipSetDevice(c->device));
    if ((rc = colpass(c, 0, r, c->p.slab_g, block))) return rc;
    hipLaunchKernelGGL(k_colreduce, dim3((unsigned)cdiv(c->wp, kThreads)), dim3(kThreads), 0, c->stream,
                       c->p.slab_g, c->wp, c->nchunk, g, (double*)nullptr);
    LAUNCH_CHECK("k_colreduce");
    return 0;
}

int bpgl_mv(bpgl_ctx* c, int32_t block, const double* d, double* s) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    if (block < 0 || block >= c->nblock) return fail(BPGL_E_ARG, "block %d out of range", block);
    if (!d || !s) return fail(BPGL_E_ARG, "null vector");
    HIP_TRY(hipSetDevice(c->device));
    if ((rc = rowpass(c, d, c->p.slab_s, block))) return rc;
    return rowreduce(c, c->p.slab_s, s, 0);
}

int bpgl_comm_unique_id(void* out128) {
    if (!out128) return fail(BPGL_E_ARG, "null buffer");
    ncclUniqueId id;
    ncclResult_t nr = ncclGetUniqueId(&id);
    if (nr != ncclSuccess) return fail(BPGL_E_RCCL, "ncclGetUniqueId: %s", ncclGetErrorString(nr));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(out128, &id, 128);
    return 0;
}

int bpgl_comm_init(bpgl_ctx* c, const void* uid, int rank, int nranks) {
    if (!c || !uid) return fail(BPGL_E_ARG, "null argument");
    if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
        return fail(BPGL_E_ARG, "bad rank %d / nranks %d", rank, nranks);
    HIP_TRY(hipSetDevice(c->device));
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    c->rank = rank;
    c->nranks = nranks;
    c->p.rank = rank;
    c->p.nranks = nranks;
    {   // also for nranks == 1: an explicit request (it runs the sharded code path on one GPU)
        ncclUniqueId id;
        memcpy(&id, uid, 128);
        ncclResult_t nr = ncclCommInitRank(&c->comm, nranks, id, rank);
        if (nr != ncclSuccess) return fail(BPGL_E_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(nr));
    }
    c->p.has_comm = c->comm != nullptr;
    c->external = false;
    drop_graphs(c);
    return 0;
}

int bpgl_set_ranks(bpgl_ctx* c, int rank, int nranks) {
    if (!c) return fail(BPGL_E_ARG, "null context");
    if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
        return fail(BPGL_E_ARG, "bad rank %d / nranks %d", rank, nranks);
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    c->rank = rank;
    c->nranks = nranks;
    c->p.rank = rank;
    c->p.nranks = nranks;
    c->p.has_comm = 0;
    c->external = nranks > 1;
    drop_graphs(c);
    c->solver = false;
    return 0;
}

int bpgl_solver_phase(bpgl_ctx* c, int phase) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    if (!c->solver) return fail(BPGL_E_STATE, "bpgl_solver_reset has not been called");
    if (phase < 0 || phase > 3) return fail(BPGL_E_ARG, "phase must be 0, 1, 2 or 3");
    HIP_TRY(hipSetDevice(c->device));
    if (phase >= 2) {   // exact-gradient exchange of external row shards
        if (!(c->rows && c->external && c->op_on))
            return fail(BPGL_E_STATE, "phases 2 and 3 exist for external row shards only");
        if (phase == 2) {
            if ((rc = onepass_local_gradient(c, c->p.comm))) return rc;
            HIP_TRY(hipMemsetAsync(c->p.comm + c->wp, 0, 24, c->stream));
            c->op_refresh_pending = true;
            return 0;
        }
        if (!c->op_refresh_pending) return fail(BPGL_E_STATE, "phase 3 needs phase 2 first");
        HIP_TRY(hipMemcpyAsync(c->op.G, c->p.comm, 8 * c->wp, hipMemcpyDeviceToDevice, c->stream));
        c->op_refresh_pending = false;
        return onepass_tail<false>(c);
    }
    return enqueue_phase(c, 0, phase);
}

double* bpgl_solver_exchange_buffer(bpgl_ctx* c, int64_t* count) {
    if (!c) return nullptr;
    if (count) *count = c->rows ? c->wp + 3 : c->m + 2 + c->nranks;
    return c->p.comm;
}

int bpgl_solver_reset(bpgl_ctx* c, const double* b, double mu, double* x, const int32_t* order,
                      int64_t order_len, double err_bound, double* err_iter, double* time_iter,
                      int64_t record_len, int use_graph) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    if (!c->have_diag) return fail(BPGL_E_STATE, "bpgl_diag_ata must run before the solver");
    if (!b || !x) return fail(BPGL_E_ARG, "b and x must be non-null");
    if (order && order_len <= 0) return fail(BPGL_E_ARG, "order_len must be > 0");
    if (!(mu >= 0.0)) return fail(BPGL_E_ARG, "mu must be >= 0");
    HIP_TRY(hipSetDevice(c->device));
    Params& p = c->p;
    p.b = b;
    p.x = x;
    p.mu = mu;
    p.order = order;
    p.order_len = order ? order_len : 0;
    p.err_bound = err_bound;
    p.err_iter = err_iter;
    p.time_iter = time_iter;
    p.rec_len = (err_iter || time_iter) ? record_len : 0;
    // Ax_k = A_k x_k for the initial point (lasso.py:91 starts from 0)
    for (int k = 0; k < c->nblock; ++k) {
        if ((rc = rowpass(c, x + (int64_t)k * c->wp, p.slab_s, k))) return rc;
        if ((rc = rowreduce(c, p.slab_s, p.Ax + (int64_t)k * c->m, 0))) return rc;
    }
    if (c->comm && !c->rows) {
        // column-sharded ranks: every Ax_k is a sum over ranks (row shards: Ax rows are local)
        ncclResult_t nr = ncclAllReduce(p.Ax, p.Ax, (size_t)c->nblock * c->m, ncclFloat64, ncclSum, c->comm,
                                        c->stream);
        if (nr != ncclSuccess) return fail(BPGL_E_RCCL, "ncclAllReduce: %s", ncclGetErrorString(nr));
    }
    hipLaunchKernelGGL(k_reset, dim3((unsigned)std::min<int64_t>(cdiv(c->m, kThreads), 1024)), dim3(kThreads), 0,
                       c->stream, p);
    LAUNCH_CHECK("k_reset");
    {
        const char* why = c->onepass != 0 ? onepass_ineligible(c) : "disabled";
        if (c->onepass == 1 && why) return fail(BPGL_E_ARG, "onepass=1: %s", why);
        // row shards without one pass: the two-pass row iteration (RCCL ranks only; it needs the
        // geometry of a one-pass-shaped context for its buffers)
        if (c->rows && why && (c->external || !c->op_shape))
            return fail(BPGL_E_ARG, "external row shards run the one-pass iteration only: %s", why);
        c->op_on = c->onepass != 0 && !why;
        c->op_t = 0;
        c->op_refresh_pending = false;
        // external row shards: the caller runs the first exact gradient (phases 2 and 3)
        if (c->op_on && !(c->rows && c->external) && (rc = onepass_refresh(c))) return rc;
    }
    c->use_graph = use_graph != 0 && !c->external;
    if ((rc = capture_graphs(c))) return rc;
    c->req_t = 0;
    c->n_refresh = c->n_fallback = 0;
    c->solver = true;
    c->timed_iters = 0;
    return 0;
}

int bpgl_solver_step(bpgl_ctx* c, int64_t n_iter) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    if (!c->solver) return fail(BPGL_E_STATE, "bpgl_solver_reset has not been called");
    if (n_iter < 0) return fail(BPGL_E_ARG, "n_iter < 0");
    if (c->external) return fail(BPGL_E_STATE, "external-exchange ranks advance with bpgl_solver_phase");
    HIP_TRY(hipSetDevice(c->device));
    c->req_t += n_iter;
    return step_impl(c, n_iter);
}

int bpgl_solver_status(bpgl_ctx* c, int64_t* iters_done, int* stopped, int64_t* t_last, double* gamma,
                       double* err) {
    int rc;
    if ((rc = check_ready(c))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    DevState st;
    if ((rc = read_state(c, st))) return rc;
    if (st.op_fail && c->solver && (rc = recover_onepass(c, st))) return rc;
    if (iters_done) *iters_done = st.iters;
    if (stopped) *stopped = (int)st.done;
    if (t_last) *t_last = st.t_last;
    if (gamma) *gamma = st.gamma;
    if (err) *err = st.err;
    return 0;
}

int bpgl_solver_stat(bpgl_ctx* c, const char* key, int64_t* value) {
    if (!c || !key || !value) return fail(BPGL_E_ARG, "null argument");
    if (!strcmp(key, "onepass")) *value = c->op_on ? 1 : 0;
    else if (!strcmp(key, "refresh_period")) *value = c->op_on ? c->op_refresh : 0;
    else if (!strcmp(key, "refreshes")) *value = c->n_refresh;
    else if (!strcmp(key, "fallbacks")) *value = c->n_fallback;
    else if (!strcmp(key, "requested")) *value = c->req_t;
    else if (!strcmp(key, "enqueued")) *value = c->op_t;
    else if (!strcmp(key, "cus")) *value = c->cus;
    else if (!strcmp(key, "cu_masked")) *value = c->cu_masked ? 1 : 0;
    else if (!strcmp(key, "onepass_grid")) *value = (int64_t)c->op_ngroups * c->op_SB;
    else if (!strcmp(key, "onepass_rows")) *value = c->op_shape ? op_rows_eff(c) : 0;
    else if (!strcmp(key, "onepass_sb1")) *value = c->op_shape && op_gpl_eff(c) == 0 ? 1 : 0;
    else return fail(BPGL_E_ARG, "unknown stat '%s'", key);
    return 0;
}

const double* bpgl_solver_residual(bpgl_ctx* c) { return c ? c->p.r : nullptr; }

int bpgl_iterate(bpgl_ctx* c, int64_t n_iter, const int32_t* order, double mu, const double* b, double* x,
                 double* err_iter, double* time_iter, double err_bound, int64_t* iters_done) {
    int rc;
    if ((rc = bpgl_solver_reset(c, b, mu, x, order, order ? n_iter : 0, err_bound, err_iter, time_iter, n_iter,
                                1)))
        return rc;
    if ((rc = bpgl_solver_step(c, n_iter))) return rc;
    // always: the status call synchronises and re-runs iterations a failed one-pass launch lost
    int64_t done = 0;
    if ((rc = bpgl_solver_status(c, &done, nullptr, nullptr, nullptr, nullptr))) return rc;
    if (iters_done) *iters_done = done;
    return 0;
}

int bpgl_set_tuning(bpgl_ctx* c, const char* key, int64_t value) {
    if (!c || !key) return fail(BPGL_E_ARG, "null argument");
    if (!strcmp(key, "reverse_rows")) {
        c->reverse_rows = value != 0;
        c->p.reverse_rows = c->reverse_rows;
        drop_graphs(c);
        c->solver = false;   // a new bpgl_solver_reset re-captures the iteration
        return 0;
    }
    if (!strcmp(key, "tail_permille")) {
        if (value < 0 || value > 1000) return fail(BPGL_E_ARG, "tail_permille must be in [0, 1000]");
        c->tail_permille = (int)value;
        c->p.tail_permille = c->tail_permille;
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "col_mode")) {
        if (value < 0 || value > 2) return fail(BPGL_E_ARG, "col_mode must be 0, 1 or 2");
        c->col_mode = (int)value;
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "onepass")) {
        if (value < -1 || value > 1) return fail(BPGL_E_ARG, "onepass must be -1, 0 or 1");
        c->onepass = (int)value;
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "tail_row_blocks")) {   // speed only: where the tail's residual update runs (bitwise neutral)
        if (value != 0 && value != 1) return fail(BPGL_E_ARG, "tail_row_blocks must be 0 or 1");
        c->op_rowb = (int)value;
        drop_graphs(c);
        return 0;
    }
    if (!strcmp(key, "onepass_cache_permille")) {
        if (value < -1 || value > 1000) return fail(BPGL_E_ARG, "onepass_cache_permille must be -1 (auto) or in [0, 1000]");
        c->op_cache = (int)value;
        c->op.cache_permille = op_cache_eff(c);
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "onepass_rows")) {
        if (value < -1 || value > 1) return fail(BPGL_E_ARG, "onepass_rows must be -1 (auto), 0 or 1");
        c->op_rows = (int)value;
        if (c->op_shape) c->op.rilv = op_rows_eff(c);
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "onepass_sb1")) {
        if (value < -1 || value > 0) return fail(BPGL_E_ARG, "onepass_sb1 must be -1 (auto) or 0");
        c->op_sb1 = (int)value;
        if (c->op_shape) c->op.rilv = op_rows_eff(c);
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "exchange_fp32")) {
        if (value < -1 || value > 1) return fail(BPGL_E_ARG, "exchange_fp32 must be -1, 0 or 1");
        c->xch32 = (int)value;
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "onepass_fail_at")) {   // test hook: the one-pass launch of iteration `value` fails once
        c->op_fail_at = value < 0 ? -1 : value;
        c->op.fail_at = c->op_fail_at;
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "cus")) {   // size the persistent grids for this many CUs (the layout depends on it)
        if (c->bound) return fail(BPGL_E_STATE, "\"cus\" must be set before bpgl_bind (it sets the scratch layout)");
        if (value < 1 || value > c->dev_cus) return fail(BPGL_E_ARG, "cus must be in [1, %d]", c->dev_cus);
        c->cus = (int)value;
        geometry(c);
        return 0;
    }
    if (!strcmp(key, "onepass_refresh")) {
        if (value < 0) return fail(BPGL_E_ARG, "onepass_refresh must be >= 0");
        c->op_refresh = (int)std::min<int64_t>(value, 1 << 30);
        return 0;
    }
    if (!strcmp(key, "graph_max")) {   // speed only: the largest hipGraph of iterations (replays per run)
        if (value < 1 || value > kGraphMaxIters || (value & (value - 1)))
            return fail(BPGL_E_ARG, "graph_max must be a power of two in [1, %d]", kGraphMaxIters);
        c->graph_max = (int)value;
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    if (!strcmp(key, "nt_loads")) {
        c->nt_loads = value != 0;
        drop_graphs(c);
        c->solver = false;
        return 0;
    }
    return fail(BPGL_E_ARG, "unknown tuning key '%s'", key);
}

int bpgl_set_kernel_timing(bpgl_ctx* c, int enable) {
    if (!c) return fail(BPGL_E_ARG, "null context");
    c->timing = enable != 0;
    c->timed_iters = 0;
    c->ref_timed = 0;
    for (int k = 0; k < kTimedKinds; ++k) c->kind_used[k] = false;
    return 0;
}

int bpgl_kernel_times(bpgl_ctx* c, double* avg_ms, int64_t* samples) {
    if (!c || !avg_ms) return fail(BPGL_E_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    double sum[kTimedKinds] = {0};
    for (int64_t r = 0; r < c->ref_timed; ++r) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ref_evs[2 * r], c->ref_evs[2 * r + 1]));
        sum[8] += ms;
    }
    for (int64_t it = 0; it < c->timed_iters; ++it) {
        for (int k = 0; k < kTimedKinds - 1; ++k) {
            if (!c->kind_used[k]) continue;
            float ms = 0.f;
            const size_t i0 = 2 * ((size_t)it * kTimedKinds + k);
            if (i0 + 1 >= c->evs.size()) continue;
            HIP_TRY(hipEventElapsedTime(&ms, c->evs[i0], c->evs[i0 + 1]));
            sum[k] += ms;
        }
    }
    for (int k = 0; k < kTimedKinds; ++k) avg_ms[k] = c->timed_iters ? sum[k] / c->timed_iters : 0.0;
    if (samples) *samples = c->timed_iters;
    c->timed_iters = 0;
    c->ref_timed = 0;
    for (int k = 0; k < kTimedKinds; ++k) c->kind_used[k] = false;
    return 0;
}

}  // extern "C"

#if BPGL_STAMP
// diagnostic builds only: copy the [3][5][16384] block stamps to host memory
extern "C" int bpgl_diag_stamps(void* host_out) {
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(bpgl::g_stamps), sizeof(bpgl::g_stamps)) == hipSuccess ? 0 : -1;
}
#endif
