// bpgl panel ABI -- k right-hand sides on bf16 A (BASELINE configs[4]): the
// bpgl_panel_* entry points of include/bpgl.h over the MFMA kernels of
// bpgl_panel.h.  Same conventions as bpgl.hip: caller-owned device memory,
// validated shapes, negative codes + bpgl_last_error() on failure.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/bpgl.h"
#include "bpgl_host.h"
#include "bpgl_panel.h"

using namespace bpgl;
using namespace bpgl_host;

// ===========================================================================
// panel path (k right-hand sides, bf16 A, MFMA): BASELINE configs[4]
// ===========================================================================
constexpr int kPanelKinds = 5;   // pass1, pass2, reduce, step, update

struct bpgl_panel {
    int device = 0;
    int64_t m = 0, n = 0, w = 0;
    int32_t nblock = 1, k = 0, kchunks = 1;
    hipStream_t stream = nullptr;
    bool own_stream = false, bound = false, have_diag = false, solver = false;
    PanelParams p{};
    hipGraphExec_t gexec = nullptr;
    bool timing = false;
    std::vector<hipEvent_t> evs;
    int64_t timed_iters = 0;
    bool kind_used[kPanelKinds] = {};   // kinds recorded in the current window (step: folded into reduce)
    int interleave[2] = {2, -1};  // mainloop variant per pass (tuning knobs; -1: the measured default, panel_ilv)
    int dsplit = 1;               // bf16 pieces of the solver's direction (d_split knob; 1 since round 4)
    int defer_x = 1;              // one block: x += gamma D' in the next pass-1 epilogue ("defer_x" knob; round 4 default)
    int carry_g = 1;              // carried gradient, one feature block ("carry_g" knob; ignored for nblock > 1)
    int64_t g_period = 64;        // exact gradient every g_period iterations ("g_refresh" knob)
    int gm_cur = 0;               // pass-1 form of the launch being enqueued: 0 plain, 1 exact + store G, 2 carried
    hipGraphExec_t gexec_ref = nullptr;   // carry_g: a graph whose first iteration is the exact-gradient one
    int fuse_update = 1;          // one block, x deferred: reduce + line search + R update in one launch ("fuse_update")
    int fuse_ok = 0;              // ... and the shape and occupancy admit it (panel_fused_geo, set at bind)
    int fuse_cus = 0;             // the CUs that check counted (the stream's CU mask, or the device)
    int fuse_grid = 1024;         // its grid: at most this many blocks, k x G ("fuse_grid": 256, 512 or 1024;
                                  // 1024 measured best with 512, +0.4 % over 256: profiles/r05/panel_fused)
    int64_t t_host = 0;           // iterations enqueued since the last reset
    int64_t n_exact = 0;          // carried gradient: exact-gradient iterations since the last reset
    int64_t ldr() const { return m; }
    int64_t ldd() const { return w; }
};

namespace {

struct PanelLayout {
    int64_t st, Rh, Rl, Dh, Dl, X, Ax, B, R, diag, rec, Sslab, S, norms, lsp, mu, gamma, err_rhs, cnt, ready, lsdone, Gc,
        Sh, Ec, At, A1t, total;
};
PanelLayout panel_layout(const bpgl_panel* c) {
    Carve k;
    PanelLayout L;
    const int64_t km = (int64_t)c->k * c->m, kw = (int64_t)c->k * c->w;
    L.st = k.take(sizeof(PanelState));
    L.Rh = k.take(2 * (int64_t)c->k * c->ldr());
    L.Rl = k.take(2 * (int64_t)c->k * c->ldr());
    L.Dh = k.take(2 * (int64_t)c->k * c->ldd());
    L.Dl = k.take(2 * (int64_t)c->k * c->ldd());
    L.X = k.take(4 * kw * c->nblock);
    L.Ax = k.take(8 * km * c->nblock);
    L.B = k.take(8 * km);
    L.R = k.take(8 * km);
    L.diag = k.take(8 * c->n);
    L.rec = k.take(8 * c->n);
    L.Sslab = k.take(4 * km * c->kchunks);
    L.S = k.take(8 * km);
    L.norms = k.take(8 * 4 * (c->w / kPanelRows) * c->k);
    L.lsp = k.take(8 * 2 * cdiv(c->m, kLspRows) * c->k);
    L.mu = k.take(8 * c->k);
    L.gamma = k.take(8 * c->k);
    L.err_rhs = k.take(8 * c->k);
    L.cnt = k.take(8 * (int64_t)c->k);
    L.ready = k.take(8 * (int64_t)c->k);
    L.lsdone = k.take(8);
    // the carried gradient's state (one feature block only; ADVICE r04: not reserved otherwise)
    const bool carry = c->nblock == 1;
    L.Gc = k.take(carry ? 4 * kw : 0);                           // the carried gradient (fp32)
    L.Sh = k.take(carry ? 2 * (int64_t)c->k * c->ldr() : 0);     // the carried product's bf16 operand
    L.Ec = k.take(carry ? 4 * km : 0);                           // its rounding error, fed into the next one (fp32)
    L.At = k.take(kPanelTiled2 ? 2 * c->m * c->n : 0);            // pass 2's tiled copy of A (bf16)
    L.A1t = k.take(kPanelTiled1 ? 2 * c->m * c->n : 0);           // pass 1's tiled copy of A (bf16)
    L.total = k.off;
    return L;
}

// ns: bf16 pieces of the direction (pass 1's epilogue writes it, pass 2 reads it): the
// solver's d_split knob, 2 for the API products (bpgl_panel_mtm / _mm)
// the mainloop variant of a pass: the knob, or the measured default -- pass 1: 2 (software-pipelined);
// pass 2: 2 with the bf16 direction alone at k >= 64 (+0.7 % at k = 64 and 128), else 1 (k = 32 and the
// hi + lo direction; profiles/r04/ilv)
int panel_ilv(const bpgl_panel* c, int which, int ns) {
    const int v = c->interleave[which];
    if (v >= 0) return v;
    return which == 0 ? 2 : (ns == 1 && c->k >= 64 ? 2 : 1);
}
template <int NT, int ILV, int NS>
int panel_launch_nt(bpgl_panel* c, int which, int fixed_block, double* out, int mode) {
    switch (which) {
        case 0:
            {   // carried-gradient forms (one feature block)
                if (mode && c->gm_cur == 1) {
                    hipLaunchKernelGGL((k_panel_pass1<NT, 1, ILV, NS, 1>), dim3((unsigned)(c->w / kPanelRows)),
                                       dim3(PanelGeo<NT, 2>::T), 0, c->stream, c->p, fixed_block, out);
                    LAUNCH_CHECK("k_panel_pass1");
                    break;
                }
                if (mode && c->gm_cur == 2) {
                    hipLaunchKernelGGL((k_panel_pass1<NT, 1, ILV, NS, 2>), dim3((unsigned)(c->w / kPanelRows)),
                                       dim3(PanelGeo<NT, 2>::T), 0, c->stream, c->p, fixed_block, out);
                    LAUNCH_CHECK("k_panel_pass1");
                    break;
                }
            }
            if (mode) hipLaunchKernelGGL((k_panel_pass1<NT, 1, ILV, NS>), dim3((unsigned)(c->w / kPanelRows)),
                                         dim3(PanelGeo<NT, 2>::T), 0, c->stream, c->p, fixed_block, out);
            else hipLaunchKernelGGL((k_panel_pass1<NT, 0, ILV, 2>), dim3((unsigned)(c->w / kPanelRows)),
                                    dim3(PanelGeo<NT, 2>::T), 0, c->stream, c->p, fixed_block, out);
            LAUNCH_CHECK("k_panel_pass1");
            break;
        case 1:
            hipLaunchKernelGGL((k_panel_pass2<NT, ILV, NS>), dim3((unsigned)((c->m / kPanelRows) * c->kchunks)),
                               dim3(PanelGeo<NT, NS>::T), 0, c->stream, c->p, fixed_block);
            LAUNCH_CHECK("k_panel_pass2");
            break;
    }
    return 0;
}
template <int NT, int NS>
int panel_launch_ilv(bpgl_panel* c, int which, int fixed_block, double* out, int mode) {
    switch (panel_ilv(c, which, NS)) {
        case 0: return panel_launch_nt<NT, 0, NS>(c, which, fixed_block, out, mode);
        case 1: return panel_launch_nt<NT, 1, NS>(c, which, fixed_block, out, mode);
        default: return panel_launch_nt<NT, 2, NS>(c, which, fixed_block, out, mode);
    }
}
template <int NS>
int panel_launch_ns(bpgl_panel* c, int which, int fixed_block, double* out, int mode) {
    switch (c->k) {
        case 16: return panel_launch_ilv<1, NS>(c, which, fixed_block, out, mode);
        case 32: return panel_launch_ilv<2, NS>(c, which, fixed_block, out, mode);
        case 64: return panel_launch_ilv<4, NS>(c, which, fixed_block, out, mode);
        default: return panel_launch_ilv<8, NS>(c, which, fixed_block, out, mode);
    }
}
int panel_launch(bpgl_panel* c, int which, int fixed_block, double* out, int mode, int ns) {
    return ns == 1 ? panel_launch_ns<1>(c, which, fixed_block, out, mode)
                   : panel_launch_ns<2>(c, which, fixed_block, out, mode);
}
bool panel_carry(const bpgl_panel* c) { return c->carry_g && c->nblock == 1; }
int panel_pass(bpgl_panel* c, int which) { return panel_launch(c, which, -1, nullptr, 1, c->dsplit); }
// k_panel_reduce_upd's geometry: G blocks per RHS of U 1024-row groups each (k x G <= fuse_grid
// blocks); false when the shape does not admit it (m a multiple of 1024, U in {1, 2, 4})
bool panel_fused_geo(const bpgl_panel* c, int* G, int* U) {
    if (c->m % kLspRows) return false;
    const int64_t groups = c->m / kLspRows;
    const int64_t g = std::min<int64_t>(std::max<int64_t>(1, c->fuse_grid / c->k), groups);
    if (groups % g) return false;
    const int64_t u = groups / g;
    if (u != 1 && u != 2 && u != 4) return false;
    *G = (int)g;
    *U = (int)u;
    return true;
}
const void* panel_fused_fn(int U) {
    return U == 1 ? (const void*)k_panel_reduce_upd<1> : U == 2 ? (const void*)k_panel_reduce_upd<2>
                                                              : (const void*)k_panel_reduce_upd<4>;
}
int panel_reduce_upd(bpgl_panel* c, int cflag) {
    int G = 0, U = 0;
    (void)panel_fused_geo(c, &G, &U);
    const dim3 grid((unsigned)(c->k * G)), blk(kThreads);
    if (U == 1) hipLaunchKernelGGL(k_panel_reduce_upd<1>, grid, blk, 0, c->stream, c->p, cflag, G);
    else if (U == 2) hipLaunchKernelGGL(k_panel_reduce_upd<2>, grid, blk, 0, c->stream, c->p, cflag, G);
    else hipLaunchKernelGGL(k_panel_reduce_upd<4>, grid, blk, 0, c->stream, c->p, cflag, G);
    LAUNCH_CHECK("k_panel_reduce_upd");
    return 0;
}
// the fused reduce + update needs its k x G blocks resident together: on the CUs the stream may use
// (a CU-masked stream from bpgl_stream_create gets fewer), else the two-kernel form runs
void panel_fuse_check(bpgl_panel* c) {
    int G = 0, U = 0, nb = 0;
    c->fuse_ok = 0;
    c->fuse_cus = 0;
    if (!panel_fused_geo(c, &G, &U)) return;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, panel_fused_fn(U), kThreads, 0) != hipSuccess) {
        (void)hipGetLastError();   // the query's own error only
        return;
    }
    c->fuse_cus = usable_cus(c->stream, c->device);
    if ((int64_t)nb * c->fuse_cus >= (int64_t)c->k * G) c->fuse_ok = 1;
}
int panel_reduce(bpgl_panel* c, double* out, int mode) {
    hipLaunchKernelGGL(k_panel_reduce, dim3((unsigned)(c->k * cdiv(c->m, kLspRows))), dim3(kThreads), 0, c->stream,
                       c->p, out, mode);
    LAUNCH_CHECK("k_panel_reduce");
    return 0;
}
void panel_ev(bpgl_panel* c, int64_t it, int kind, int end) {
    if (!c->timing) return;
    c->kind_used[kind] = true;
    const size_t idx = 2 * ((size_t)it * kPanelKinds + kind) + end;
    while (c->evs.size() <= idx) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->evs.push_back(e);
    }
    (void)hipEventRecord(c->evs[idx], c->stream);
}
// exact: with the carried gradient, this iteration computes G = A^T R exactly (and stores it);
// split_r: the update writes R's hi / lo images (with the carried gradient only the exact pass 1 reads
// them, so only an iteration followed by an exact one needs to)
int panel_iteration(bpgl_panel* c, int64_t it, bool exact = false, bool split_r = true) {
    int rc;
    c->gm_cur = panel_carry(c) ? (exact ? 1 : 2) : 0;
    // the update's carried-gradient operand: 0 none, 1 V = E + gamma S, 2 V = gamma S (G is exact now);
    // + 4: skip R's hi / lo images
    const int cflag = (c->gm_cur == 0 ? 0 : c->gm_cur == 1 ? 2 : 1) | (c->gm_cur && !split_r ? 4 : 0);
    panel_ev(c, it, 0, 0);
    rc = panel_pass(c, 0);
    c->gm_cur = 0;
    if (rc) return rc;
    panel_ev(c, it, 0, 1);
    panel_ev(c, it, 1, 0);
    if ((rc = panel_pass(c, 1))) return rc;
    panel_ev(c, it, 1, 1);
    panel_ev(c, it, 2, 0);
    if (c->nblock == 1 && c->defer_x && c->fuse_update && c->fuse_ok) {   // reduce + line search + R update
        rc = panel_reduce_upd(c, cflag);
        panel_ev(c, it, 2, 1);
        return rc;
    }
    if ((rc = panel_reduce(c, c->p.S, 1))) return rc;   // its last block per RHS runs the line search
    panel_ev(c, it, 2, 1);
    panel_ev(c, it, 4, 0);
    if (c->nblock == 1 && c->defer_x) {   // R only; x += gamma D' rides on the next pass-1 epilogue (or the flush)
        const dim3 ug((unsigned)std::min<int64_t>(cdiv((int64_t)c->k * c->m / 4, kThreads), 8192));
        hipLaunchKernelGGL(k_panel_update1, ug, dim3(kThreads), 0, c->stream, c->p, cflag);
    } else {
        const int64_t n = (int64_t)c->k * c->w / 8 + (int64_t)c->k * c->m / 4;   // work units
        const dim3 ug((unsigned)std::min<int64_t>(cdiv(n, kThreads), 8192));
        const bool nb1 = c->nblock == 1;
        if (c->dsplit == 1) {
            if (nb1) hipLaunchKernelGGL((k_panel_update<1, true>), ug, dim3(kThreads), 0, c->stream, c->p, cflag);
            else hipLaunchKernelGGL((k_panel_update<1, false>), ug, dim3(kThreads), 0, c->stream, c->p, cflag);
        } else {
            if (nb1) hipLaunchKernelGGL((k_panel_update<2, true>), ug, dim3(kThreads), 0, c->stream, c->p, cflag);
            else hipLaunchKernelGGL((k_panel_update<2, false>), ug, dim3(kThreads), 0, c->stream, c->p, cflag);
        }
    }
    LAUNCH_CHECK("k_panel_update");
    panel_ev(c, it, 4, 1);
    return 0;
}
// src [k][len] fp64 -> hi/lo images [k][ld]
int panel_split(bpgl_panel* c, const double* src, int64_t len, int64_t ld, __bf16* hi, __bf16* lo, double sign,
                double* copy) {
    const int64_t n = (int64_t)c->k * len;
    hipLaunchKernelGGL(k_panel_split, dim3((unsigned)std::min<int64_t>(cdiv(n, kThreads), 2048)), dim3(kThreads), 0,
                       c->stream, src, n, len, ld, hi, lo, sign, copy);
    LAUNCH_CHECK("k_panel_split");
    return 0;
}
void drop_graphs(bpgl_panel* c) {
    if (c->gexec) { (void)hipGraphExecDestroy(c->gexec); c->gexec = nullptr; }
    if (c->gexec_ref) { (void)hipGraphExecDestroy(c->gexec_ref); c->gexec_ref = nullptr; }
}

int panel_ready(const bpgl_panel* c) {
    if (!c) return fail(BPGL_E_ARG, "null panel context");
    if (!c->bound) return fail(BPGL_E_STATE, "bpgl_panel_bind has not been called");
    return 0;
}
}  // namespace

extern "C" {

int bpgl_panel_create(bpgl_panel** out, int device, int64_t m, int64_t n, int32_t nblock, int32_t nrhs,
                      int32_t kchunks, void* hip_stream) {
    if (!out) return fail(BPGL_E_ARG, "out is null");
    *out = nullptr;
    if (nrhs != 16 && nrhs != 32 && nrhs != 64 && nrhs != 128)
        return fail(BPGL_E_ARG, "nrhs must be 16, 32, 64 or 128 (got %d)", nrhs);
    if (nblock <= 0 || n % nblock) return fail(BPGL_E_ARG, "n must be divisible by nblock");
    const int64_t w = n / nblock;
    if (m <= 0 || m % kPanelRows) return fail(BPGL_E_ARG, "m (%lld) must be a positive multiple of %d", (long long)m,
                                              kPanelRows);
    if (w <= 0 || w % kPanelRows) return fail(BPGL_E_ARG, "block width (%lld) must be a positive multiple of %d",
                                              (long long)w, kPanelRows);
    if (kchunks <= 0) {   // one pass-2 tile per CU (256), chunk width a multiple of two 64-deep stages
        kchunks = (int32_t)std::max<int64_t>(1, std::min<int64_t>(w / (2 * kPanelK), 256 / (m / kPanelRows)));
        while (kchunks > 1 && w % ((int64_t)kchunks * 2 * kPanelK)) --kchunks;
    }
    if (w % ((int64_t)kchunks * kPanelK)) return fail(BPGL_E_ARG, "w must be a multiple of 64 * kchunks");
    if ((int64_t)nrhs * w >= (1ll << 31) || (int64_t)nrhs * m >= (1ll << 31))
        return fail(BPGL_E_ARG, "nrhs * block width and nrhs * m must be below 2^31");
    HIP_TRY(hipSetDevice(device));
    bpgl_panel* c = new bpgl_panel();
    c->device = device;
    c->m = m;
    c->n = n;
    c->w = w;
    c->nblock = nblock;
    c->k = nrhs;
    c->kchunks = kchunks;
    if (hip_stream) {
        c->stream = (hipStream_t)hip_stream;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            return fail(BPGL_E_HIP, "hipStreamCreate failed");
        }
        c->own_stream = true;
    }
    *out = c;
    return 0;
}

void bpgl_panel_destroy(bpgl_panel* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);   // destroy path: nothing to report to
    drop_graphs(c);
    for (auto e : c->evs) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int64_t bpgl_panel_scratch_bytes(const bpgl_panel* c) { return c ? panel_layout(c).total : -1; }

int bpgl_panel_bind(bpgl_panel* c, const void* A, int64_t lda, void* scratch, int64_t scratch_bytes) {
    if (!c) return fail(BPGL_E_ARG, "null panel context");
    if (!A || !scratch) return fail(BPGL_E_ARG, "A and scratch must be non-null");
    if (((uintptr_t)A) % 16) return fail(BPGL_E_ARG, "A must be 16-byte aligned");
    if (((uintptr_t)scratch) % 256) return fail(BPGL_E_ARG, "scratch must be 256-byte aligned");
    if (lda < c->n || lda % 8) return fail(BPGL_E_ARG, "lda must be >= n and a multiple of 8");
    const PanelLayout L = panel_layout(c);
    if (scratch_bytes < L.total) return fail(BPGL_E_SCRATCH, "scratch too small: %lld < %lld",
                                             (long long)scratch_bytes, (long long)L.total);
    char* s = (char*)scratch;
    PanelParams& p = c->p;
    p = PanelParams{};
    p.A = (const __bf16*)A;
    p.lda = lda;
    p.m = c->m;
    p.w = c->w;
    p.nblock = c->nblock;
    p.k = c->k;
    p.kchunks = c->kchunks;
    p.ldr = c->ldr();
    p.ldd = c->ldd();
    p.st = (PanelState*)(s + L.st);
    p.Rh = (__bf16*)(s + L.Rh);
    p.Rl = (__bf16*)(s + L.Rl);
    p.Dh = (__bf16*)(s + L.Dh);
    p.Dl = (__bf16*)(s + L.Dl);
    p.X = (float*)(s + L.X);
    p.Ax = (double*)(s + L.Ax);
    p.B = (const double*)(s + L.B);
    p.R = (double*)(s + L.R);
    p.diag = (const double*)(s + L.diag);
    p.rec = (const double*)(s + L.rec);
    p.Sslab = (float*)(s + L.Sslab);
    p.S = (double*)(s + L.S);
    p.norms = (double*)(s + L.norms);
    p.lsp = (double*)(s + L.lsp);
    p.mu = (const double*)(s + L.mu);
    p.gamma = (double*)(s + L.gamma);
    p.err_rhs = (double*)(s + L.err_rhs);
    p.cnt = (unsigned long long*)(s + L.cnt);
    p.Gc = (float*)(s + L.Gc);
    p.Ec = (float*)(s + L.Ec);
    p.ready = (unsigned long long*)(s + L.ready);
    p.lsdone = (unsigned long long*)(s + L.lsdone);
    p.At = kPanelTiled2 ? (const __bf16*)(s + L.At) : nullptr;
    p.A1t = kPanelTiled1 ? (const __bf16*)(s + L.A1t) : nullptr;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemsetAsync(s, 0, L.At, c->stream));   // everything but the tiled A copies (laid out last)
    if (kPanelTiled2) {
        hipLaunchKernelGGL((k_panel_tile<256, 64, true>), dim3((unsigned)((c->m / 256) * (c->n / 64))), dim3(256), 0,
                           c->stream, p.A, p.lda, c->n, const_cast<__bf16*>(p.At));
        LAUNCH_CHECK("k_panel_tile");
    }
    if (kPanelTiled1) {
        hipLaunchKernelGGL((k_panel_tile<64, 256, false>), dim3((unsigned)((c->m / 64) * (c->n / 256))), dim3(256), 0,
                           c->stream, p.A, p.lda, c->n, const_cast<__bf16*>(p.A1t));
        LAUNCH_CHECK("k_panel_tile");
    }
    panel_fuse_check(c);
    c->bound = true;
    c->have_diag = false;
    c->solver = false;
    drop_graphs(c);
    return 0;
}

int bpgl_panel_diag(bpgl_panel* c, double* out) {
    int rc;
    if ((rc = panel_ready(c))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_panel_diag, dim3((unsigned)cdiv(c->n, 512)), dim3(kThreads), 0, c->stream, c->p,
                       const_cast<double*>(c->p.diag), const_cast<double*>(c->p.rec));
    LAUNCH_CHECK("k_panel_diag");
    if (out) HIP_TRY(hipMemcpyAsync(out, c->p.diag, 8 * c->n, hipMemcpyDeviceToDevice, c->stream));
    c->have_diag = true;
    return 0;
}

int bpgl_panel_mtm(bpgl_panel* c, int32_t block, const double* R, double* G) {
    int rc;
    if ((rc = panel_ready(c))) return rc;
    if (block < 0 || block >= c->nblock) return fail(BPGL_E_ARG, "block out of range");
    if (!R || !G) return fail(BPGL_E_ARG, "null operand");
    HIP_TRY(hipSetDevice(c->device));
    if ((rc = panel_split(c, R, c->m, c->ldr(), c->p.Rh, c->p.Rl, 1.0, nullptr))) return rc;
    c->solver = false;   // Rh/Rl now hold the caller's operand
    return panel_launch(c, 0, block, G, 0, 2);
}

int bpgl_panel_mm(bpgl_panel* c, int32_t block, const double* D, double* S) {
    int rc;
    if ((rc = panel_ready(c))) return rc;
    if (block < 0 || block >= c->nblock) return fail(BPGL_E_ARG, "block out of range");
    if (!D || !S) return fail(BPGL_E_ARG, "null operand");
    HIP_TRY(hipSetDevice(c->device));
    if ((rc = panel_split(c, D, c->w, c->ldd(), c->p.Dh, c->p.Dl, 1.0, nullptr))) return rc;
    c->solver = false;
    if ((rc = panel_launch(c, 1, block, nullptr, 0, 2))) return rc;
    return panel_reduce(c, S, 0);
}

int bpgl_panel_reset(bpgl_panel* c, const double* B, const double* mu, double* err_iter, int64_t record_len,
                     int use_graph) {
    int rc;
    if ((rc = panel_ready(c))) return rc;
    if (!c->have_diag) return fail(BPGL_E_STATE, "bpgl_panel_diag must run before the solver");
    if (!B || !mu) return fail(BPGL_E_ARG, "B and mu must be non-null");
    HIP_TRY(hipSetDevice(c->device));
    PanelParams& p = c->p;
    const int64_t km = (int64_t)c->k * c->m;
    HIP_TRY(hipMemcpyAsync(const_cast<double*>(p.B), B, 8 * km, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(const_cast<double*>(p.mu), mu, 8 * c->k, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(p.X, 0, 4 * (int64_t)c->k * c->w * c->nblock, c->stream));
    HIP_TRY(hipMemsetAsync(p.Ax, 0, 8 * km * c->nblock, c->stream));
    // x = 0 => Ax = 0, R = -B
    if ((rc = panel_split(c, p.B, c->m, c->ldr(), p.Rh, p.Rl, -1.0, p.R))) return rc;
    c->t_host = 0;
    c->n_exact = 0;
    p.err_iter = err_iter;
    p.rec_len = err_iter ? record_len : 0;
    HIP_TRY(hipMemsetAsync(p.cnt, 0, 8 * (int64_t)c->k, c->stream));   // arrival counters start at 0
    HIP_TRY(hipMemsetAsync(p.ready, 0, 8 * (int64_t)c->k, c->stream));
    HIP_TRY(hipMemsetAsync(p.lsdone, 0, 8, c->stream));
    hipLaunchKernelGGL(k_panel_reset_state, dim3(1), dim3(64), 0, c->stream, c->p);
    LAUNCH_CHECK("k_panel_reset_state");
    p.Sh = panel_carry(c) ? (__bf16*)((char*)p.st + (panel_layout(c).Sh - panel_layout(c).st)) : nullptr;
    drop_graphs(c);
    if (use_graph) {
        // kGraphIters iterations; with the carried gradient a second graph whose first iteration is
        // the exact one (bpgl_panel_step replays it at every g_period-th iteration)
        for (int g = 0; g < (panel_carry(c) ? 2 : 1); ++g) {
            hipGraph_t graph = nullptr;
            const bool was = c->timing;
            c->timing = false;
            HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
            rc = 0;
            // R's images from the graph's last iteration: the next replay may start with the exact one
            for (int k = 0; k < kGraphIters && !rc; ++k)
                rc = panel_iteration(c, 0, g == 1 && k == 0, k == kGraphIters - 1);
            hipError_t ec = hipStreamEndCapture(c->stream, &graph);
            c->timing = was;
            if (rc) { if (graph) (void)hipGraphDestroy(graph); return rc; }
            if (ec != hipSuccess) return fail(BPGL_E_HIP, "hipStreamEndCapture: %s", hipGetErrorString(ec));
            hipGraphExec_t& ge = g ? c->gexec_ref : c->gexec;
            hipError_t ei = hipGraphInstantiate(&ge, graph, nullptr, nullptr, 0);
            (void)hipGraphDestroy(graph);
            if (ei != hipSuccess) return fail(BPGL_E_HIP, "hipGraphInstantiate: %s", hipGetErrorString(ei));
            // uploaded here, so the first replay in a caller's timed region pays no upload
            if ((ei = hipGraphUpload(ge, c->stream)) != hipSuccess)
                return fail(BPGL_E_HIP, "hipGraphUpload: %s", hipGetErrorString(ei));
        }
    }
    c->solver = true;
    c->timed_iters = 0;
    return 0;
}

int bpgl_panel_step(bpgl_panel* c, int64_t n_iter) {
    int rc;
    if ((rc = panel_ready(c))) return rc;
    if (!c->solver) return fail(BPGL_E_STATE, "bpgl_panel_reset has not been called");
    HIP_TRY(hipSetDevice(c->device));
    int64_t i = 0;
    while (i < n_iter) {
        // carried gradient: every g_period-th iteration (the first included) computes G exactly
        const bool exact = panel_carry(c) && c->t_host % c->g_period == 0;
        if (!c->timing && c->gexec && i + kGraphIters <= n_iter && c->t_host % kGraphIters == 0) {
            HIP_TRY(hipGraphLaunch(exact ? c->gexec_ref : c->gexec, c->stream));
            c->n_exact += exact;
            i += kGraphIters;
            c->t_host += kGraphIters;
        } else {
            const bool next_exact = (c->t_host + 1) % c->g_period == 0;
            if ((rc = panel_iteration(c, c->timing ? c->timed_iters : 0, exact, next_exact || i + 1 == n_iter)))
                return rc;
            c->n_exact += exact;
            if (c->timing) c->timed_iters++;
            ++i;
            ++c->t_host;
        }
    }
    if (c->nblock == 1 && c->defer_x) {   // the last iteration's x update, so X is current between calls
        const dim3 fg((unsigned)std::min<int64_t>(cdiv((int64_t)c->k * c->w / 8, kThreads), 8192));
        if (c->dsplit == 1) hipLaunchKernelGGL(k_panel_flush<1>, fg, dim3(kThreads), 0, c->stream, c->p);
        else hipLaunchKernelGGL(k_panel_flush<2>, fg, dim3(kThreads), 0, c->stream, c->p);
        LAUNCH_CHECK("k_panel_flush");
        hipLaunchKernelGGL(k_panel_clear_pending, dim3(1), dim3(64), 0, c->stream, c->p);
        LAUNCH_CHECK("k_panel_clear_pending");
    }
    return 0;
}

int bpgl_panel_status(bpgl_panel* c, int64_t* iters, double* last_err) {
    int rc;
    if ((rc = panel_ready(c))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    PanelState st;
    HIP_TRY(hipMemcpyAsync(&st, c->p.st, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (iters) *iters = st.iters;
    if (last_err) *last_err = st.last_err;
    if (st.fail)
        return fail(BPGL_E_EXCHANGE, "k_panel_reduce_upd: a block waited in vain for its right-hand side's step size "
                                     "(blocks not co-resident: another kernel held CUs); the iterates are not valid -- "
                                     "reset and run with the tuning key fuse_update = 0");
    return 0;
}

const float* bpgl_panel_x(bpgl_panel* c) { return c ? c->p.X : nullptr; }

int bpgl_panel_set_kernel_timing(bpgl_panel* c, int enable) {
    if (!c) return fail(BPGL_E_ARG, "null panel context");
    c->timing = enable != 0;
    c->timed_iters = 0;
    return 0;
}

int bpgl_panel_kernel_times(bpgl_panel* c, double* avg_ms /* 5 */, int64_t* samples) {
    if (!c || !avg_ms) return fail(BPGL_E_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    double sum[kPanelKinds] = {0};
    for (int64_t it = 0; it < c->timed_iters; ++it)
        for (int k = 0; k < kPanelKinds; ++k) {
            if (!c->kind_used[k]) continue;
            const size_t i0 = 2 * ((size_t)it * kPanelKinds + k);
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, c->evs[i0], c->evs[i0 + 1]));
            sum[k] += ms;
        }
    for (int k = 0; k < kPanelKinds; ++k) avg_ms[k] = c->timed_iters ? sum[k] / c->timed_iters : 0.0;
    if (samples) *samples = c->timed_iters;
    c->timed_iters = 0;
    for (int k = 0; k < kPanelKinds; ++k) c->kind_used[k] = false;
    return 0;
}

int bpgl_panel_set_tuning(bpgl_panel* c, const char* key, int64_t value) {
    if (!c || !key) return fail(BPGL_E_ARG, "null argument");
    const bool both = !strcmp(key, "interleave");
    if (both || !strcmp(key, "interleave1") || !strcmp(key, "interleave2")) {
        if (value < 0 || value > 2) return fail(BPGL_E_ARG, "interleave must be 0, 1 or 2");
        if (both || key[10] == '1') c->interleave[0] = (int)value;
        if (both || key[10] == '2') c->interleave[1] = (int)value;
    } else if (!strcmp(key, "fuse_grid")) {
        if (value != 256 && value != 512 && value != 1024) return fail(BPGL_E_ARG, "fuse_grid must be 256, 512 or 1024");
        c->fuse_grid = (int)value;
        panel_fuse_check(c);
        c->solver = false;
    } else if (!strcmp(key, "fuse_update")) {
        if (value != 0 && value != 1) return fail(BPGL_E_ARG, "fuse_update must be 0 or 1");
        c->fuse_update = (int)value;
        c->solver = false;   // the graphs bake the launch sequence in: a reset must follow
    } else if (!strcmp(key, "defer_x")) {
        if (value != 0 && value != 1) return fail(BPGL_E_ARG, "defer_x must be 0 or 1");
        c->defer_x = (int)value;
        c->solver = false;   // the graph bakes in where x is updated (and the flush): a reset must follow
    } else if (!strcmp(key, "d_split")) {
        if (value != 1 && value != 2) return fail(BPGL_E_ARG, "d_split must be 1 or 2");
        c->dsplit = (int)value;
    } else if (!strcmp(key, "carry_g")) {
        if (value != 0 && value != 1) return fail(BPGL_E_ARG, "carry_g must be 0 or 1");
        if (value && c->nblock != 1) return fail(BPGL_E_ARG, "carry_g needs one feature block");
        c->carry_g = (int)value;
        c->solver = false;   // the graphs and the operand image depend on it: a reset must follow
    } else if (!strcmp(key, "g_refresh")) {
        if (value < kGraphIters || value % kGraphIters)
            return fail(BPGL_E_ARG, "g_refresh must be a positive multiple of %d", kGraphIters);
        c->g_period = value;
        c->solver = false;
    } else {
        return fail(BPGL_E_ARG, "unknown panel tuning key '%s'", key);
    }
    drop_graphs(c);
    return 0;
}

int bpgl_panel_get_tuning(const bpgl_panel* c, const char* key, int64_t* value) {
    if (!c || !key || !value) return fail(BPGL_E_ARG, "null argument");
    if (!strcmp(key, "interleave1")) *value = panel_ilv(c, 0, c->dsplit);
    else if (!strcmp(key, "interleave2")) *value = panel_ilv(c, 1, c->dsplit);   // the solver's pass 2
    else if (!strcmp(key, "d_split")) *value = c->dsplit;
    else if (!strcmp(key, "defer_x")) *value = c->defer_x;
    else if (!strcmp(key, "fuse_grid")) *value = c->fuse_grid;
    else if (!strcmp(key, "fuse_update")) *value = c->nblock == 1 && c->defer_x && c->fuse_update && c->fuse_ok;   // in effect
    else if (!strcmp(key, "carry_g")) *value = panel_carry(c) ? 1 : 0;   // the form in effect
    else if (!strcmp(key, "g_refresh")) *value = c->g_period;
    else return fail(BPGL_E_ARG, "unknown panel tuning key '%s'", key);
    return 0;
}

int bpgl_panel_stat(const bpgl_panel* c, const char* key, int64_t* value) {
    if (!c || !key || !value) return fail(BPGL_E_ARG, "null argument");
    if (!strcmp(key, "iters_enqueued")) *value = c->t_host;
    else if (!strcmp(key, "exact_gradients")) *value = c->n_exact;
    else if (!strcmp(key, "fuse_cus")) *value = c->fuse_cus;   // CUs the fused-update check counted
    else return fail(BPGL_E_ARG, "unknown panel stat '%s'", key);
    return 0;
}

const double* bpgl_panel_residual(bpgl_panel* c) { return c ? c->p.R : nullptr; }

int bpgl_panel_geometry(const bpgl_panel* c, int32_t* kchunks) {
    if (!c) return fail(BPGL_E_ARG, "null panel context");
    if (kchunks) *kchunks = c->kchunks;
    return 0;
}

}  // extern "C"

