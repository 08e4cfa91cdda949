/*
 * bpgl -- MI355X-native block proximal-gradient (best-response) lasso hot path.
 *
 * Flat C ABI of convex_optimization_amd/_lib/libbpgl.so.  Plain pointers and
 * sizes only; every device pointer is memory allocated by the caller (PyTorch
 * tensors on the Python side).  The library never calls hipMalloc: it borrows
 * the caller's buffers for the lifetime of a context.
 *
 * Problem (reference lasso.py:102-157, one "ISTA iteration" = one block update):
 *   minimise 1/2 ||A x - b||^2 + mu ||x||_1,  A: m x n, columns split into
 *   nblock feature blocks of width w = n / nblock.
 *
 * Device layout of A (one rank): element (i, j) of feature block b lives at
 *   A + b * block_stride + i * lda + j        (0 <= j < w_pad)
 * w_pad = w rounded up to 16 bytes worth of elements; padding columns must be 0.
 * The reference's own GPU layout (gpu_calculation.py:172-173, np.hsplit into a
 * (BLOCK, H, W) array) is block_stride = m * w_pad, lda = w_pad.
 *
 * Conventions: return 0 on success, a negative BPGL_E* code on failure; the
 * failing call's message is available from bpgl_last_error() (thread-local).
 * No C++ exception crosses this boundary.  A context is not thread-safe and is
 * bound to one device; all work is enqueued on the context's stream.
 */
#ifndef BPGL_H
#define BPGL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dtype of A (the reference's class tunable TYPE, gpu_calculation.py:146) */
enum { BPGL_F32 = 0, BPGL_F64 = 1, BPGL_BF16 = 2 };

enum {
    BPGL_OK = 0,
    BPGL_E_ARG = -1,      /* bad argument / shape / alignment            */
    BPGL_E_STATE = -2,    /* call out of order (not bound / no solver)   */
    BPGL_E_HIP = -3,      /* HIP runtime error                           */
    BPGL_E_RCCL = -4,     /* RCCL error                                  */
    BPGL_E_SCRATCH = -5,  /* scratch buffer too small                    */
    BPGL_E_EXCHANGE = -6  /* one-pass row hand-off timed out (another
                             kernel held CUs) on an external-exchange
                             rank; the failed iterations committed
                             nothing: the solver state is intact at the
                             reported t (other ranks recover, see
                             bpgl_solver_status)                          */
};

typedef struct bpgl_ctx bpgl_ctx;

/* Message of the last failing call on this thread ("" if none). */
const char* bpgl_last_error(void);

/* Library / ABI version (major * 10000 + minor * 100 + patch).
 *   100 (0.1.0): the first ABI.
 *   200 (0.2.0): + bpgl_stream_create / bpgl_stream_destroy; bpgl_iterate always synchronises
 *                the solver stream before returning; the "onepass_cache_permille" default moved
 *                from 0 to -1 (automatic: 750 when the rank's A block fits the Infinity Cache);
 *                panel tuning keys "carry_g" (default 1: the carried gradient, one feature
 *                block) and "g_refresh".
 *   300 (0.3.0): the opt-in forms measured to lose were removed:
 *                tuning keys "fused", "onepass_fold", "onepass_variant"; panel keys "lo8",
 *                "r_refresh", "write_through", "op_pad", "waves*", interleave 3; panel stat
 *                "refreshes"; bpgl_panel_refresh.
 *   301 (0.3.1): tuning key "onepass_rows" and solver stat "onepass_rows".
 *   302 (0.3.2): RCCL row shards whose row needs more segment blocks than the stream's CUs run
 *                the two-pass row iteration instead of failing at bpgl_solver_reset; the panel's
 *                fused update is admitted against the stream's CUs; panel stat "fuse_cus"; tuning
 *                key and solver stat "onepass_sb1". */
int bpgl_version(void);

/*
 * A HIP stream for a context, optionally restricted to a set of CUs
 * (hipExtStreamCreateWithCUMask; bit i of cu_mask[i / 32] enables CU i).  Several
 * processes (ranks) sharing one GPU each get disjoint CUs this way, so the
 * persistent one-pass grid of every rank stays resident beside the others.
 * bpgl_create sizes that grid to the CUs its stream may use (hipExtStreamGetCUMask;
 * the tuning key "cus" overrides it before bpgl_bind).  The mask should give
 * every XCD the same number of CUs: the python helper
 * distributed.xcd_symmetric_cu_mask builds one.  cu_mask NULL: an unrestricted
 * non-blocking stream.  No reference counterpart (pycuda used one context and
 * the default stream, gpu_calculation.py:4).
 */
int bpgl_stream_create(int device, const uint32_t* cu_mask, int32_t mask_words, void** stream_out);
int bpgl_stream_destroy(void* stream);

/*
 * Create a context for an m x n_local matrix split into nblock feature blocks.
 * Replaces GPU_Calculation.__init__ / init_cpu_array (gpu_calculation.py:148-220):
 * grid sizes and scratch needs are derived here instead of per-call numpy.
 * `hip_stream` may be NULL (the library then creates its own stream).
 */
int bpgl_create(bpgl_ctx** out, int device, int a_dtype, int64_t m, int64_t n_local,
                int32_t nblock, void* hip_stream);
void bpgl_destroy(bpgl_ctx* ctx);

/* The stream all work of this context is enqueued on. */
void* bpgl_stream(bpgl_ctx* ctx);

/* Bytes of device scratch the caller must provide to bpgl_bind. */
int64_t bpgl_scratch_bytes(const bpgl_ctx* ctx);

/* Padded block width (w rounded up to a 16-byte multiple of elements). */
int64_t bpgl_block_width_padded(const bpgl_ctx* ctx);

/*
 * Bind the device copy of A and a scratch buffer (both caller-owned).
 * Replaces init_gpu_array (gpu_calculation.py:222-236), whose H2D copy and
 * pycuda allocations become caller-side PyTorch allocations.
 */
int bpgl_bind(bpgl_ctx* ctx, const void* A, int64_t lda, int64_t block_stride,
              void* scratch, int64_t scratch_bytes);

/*
 * diag(A_b^T A_b) for every block b into out[b * w_pad + j] (device, fp64).
 * Replaces GPU_Calculation.diag_ATA + kernel get_diag_ATA
 * (gpu_calculation.py:246-261, :116-137).  Also caches 1/diag for the solver.
 */
int bpgl_diag_ata(bpgl_ctx* ctx, double* out);

/*
 * Install diag(A_b^T A_b) (device, nblock * w_pad fp64) computed elsewhere, and
 * 1/diag.  Used by external-exchange row shards, whose column norms are sums of
 * every rank's bpgl_diag_ata output (the RCCL path does that sum itself).
 */
int bpgl_set_diag(bpgl_ctx* ctx, const double* diag);

/*
 * g = A_b^T r  (device: r has m fp64 values, g receives w_pad fp64 values).
 * Replaces GPU_Calculation.mat_tMulVec_DiffSize + kernel mul_mat_t_vec_diffsize
 * (gpu_calculation.py:264-277, :20-55); the split-K reduction happens on the
 * device in a fixed order (no host partial sums, no atomics).
 */
int bpgl_mtv(bpgl_ctx* ctx, int32_t block, const double* r, double* g);

/*
 * s = A_b d  (device: d has w_pad fp64 values, s receives m fp64 values).
 * Replaces GPU_Calculation.matMulVec_DiffSize + kernel mul_mat_vec_diffsize
 * (gpu_calculation.py:280-292, :58-91).
 */
int bpgl_mv(bpgl_ctx* ctx, int32_t block, const double* d, double* s);

/*
 * Multi-GPU: column shards of every feature block across ranks (the
 * reference's P-way shards, cpu_calculation.py:23-27 / lasso.py:107-126,
 * lifted from Pool workers to GPUs).  bpgl_comm_unique_id fills 128 bytes on
 * one rank; the caller broadcasts them; every rank then calls bpgl_comm_init.
 * The solver then all-reduces (RCCL, SUM) m + 2 + nranks fp64 values per
 * iteration.
 */
int bpgl_comm_unique_id(void* out128);
int bpgl_comm_init(bpgl_ctx* ctx, const void* unique_id128, int rank, int nranks);

/*
 * Shard layout across ranks (call between bpgl_create and bpgl_bind):
 * BPGL_SHARD_COLUMNS (default) as above; BPGL_SHARD_ROWS: one feature block, rank
 * q holds rows [m_q, m_{q+1}) of A (the context's m is its row count, n_local the
 * full width), b and the residual are local, x is replicated.  Row shards run the
 * one-pass iteration (A read once per iteration): per iteration one all-reduce
 * (SUM) of [A^T A D | r.s23 | s23.s23 | failed] -- w_pad + 3 fp64, or (opt-in
 * tuning key "exchange_fp32") w_pad + 5 fp32 (U rounded, the scalars as hi + lo
 * pairs; fp32-accurate once summed over several ranks);
 * bpgl_diag_ata and every
 * exact gradient refresh all-reduce w_pad values.  There is no reference
 * counterpart: the reference shards columns only (cpu_calculation.py:23-27).
 */
enum { BPGL_SHARD_COLUMNS = 0, BPGL_SHARD_ROWS = 1 };
int bpgl_set_shard(bpgl_ctx* ctx, int mode);

/*
 * Caller-performed exchange (validation of the sharded kernels where RCCL
 * cannot run, e.g. several ranks on one GPU): bpgl_set_ranks declares this
 * context rank `rank` of `nranks` without a communicator.  Each iteration is
 * then bpgl_solver_phase(ctx, 0); the caller sums the
 * bpgl_solver_exchange_buffer (count = m + 2 + nranks fp64) over ranks and
 * writes the sum back on every rank; bpgl_solver_phase(ctx, 1).  Requires the
 * initial point x = 0.
 */
/* Row shards (count = w_pad + 3): the same two phases per iteration; in
 * addition the exact gradient g = A^T r is exchanged by phase 2 (this rank's
 * A_q^T r_q into the exchange buffer), the caller's sum, and phase 3 -- after
 * bpgl_solver_reset and again every "onepass_refresh" iterations.  With the
 * tuning key "exchange_fp32" = 1 phases 0/1 exchange w_pad + 5 fp32 at the same
 * address instead: [U (w_pad) | r.s23 hi, lo | s23.s23 hi, lo | failed]; phases
 * 2/3 stay fp64.  The `failed` slot is each rank's one-pass failure flag: a
 * nonzero sum makes every rank skip the iteration (bpgl_solver_status then
 * reports BPGL_E_EXCHANGE with the state intact, and the caller re-runs it). */
int bpgl_set_ranks(bpgl_ctx* ctx, int rank, int nranks);
int bpgl_solver_phase(bpgl_ctx* ctx, int phase);
double* bpgl_solver_exchange_buffer(bpgl_ctx* ctx, int64_t* count);

/*
 * Device-resident solver (the loop of ClassLasso.run, lasso.py:190-292, and
 * ClassLassoCB_v2.run, lasso.py:458-613, with every step on the device).
 *
 * bpgl_solver_reset: b (m, device fp64), x (nblock * w_pad, device fp64, in/out,
 *   initial point), order (device int32 block index per iteration, NULL =
 *   cyclic t % nblock as lasso.py:40-41), order_len, err_bound (< 0 disables
 *   the ERR_BOUND stopping rule of lasso.py:141-150), err_iter / time_iter
 *   (device fp64, NULL = not recorded; record_len entries of err_iter and
 *   record_len + 1 of time_iter, as lasso.py:54-62).
 * bpgl_solver_step: enqueue n_iter more iterations (asynchronous; with
 *   `use_graph`, replays of the captured hipGraphs of 1, 2, 4, ... iterations,
 *   the largest that fits each time -- tuning key "graph_max").
 * bpgl_solver_status: synchronise the stream and read (iterations done,
 *   stopped flag, last t, last step size, last error).  It also completes
 *   iterations a one-pass launch lost: a launch whose blocks were not all
 *   resident (another kernel or process held CUs) commits nothing, nor does
 *   any later iteration until this call re-runs them on the two-pass kernels,
 *   which stay in use for the rest of the solve (RCCL row shards: the two-pass
 *   row iteration, two passes over the local rows and two all-reduces per
 *   iteration; every rank switches at the same iteration, so RCCL row-shard
 *   ranks must all call it at the same point: the recovery is collective --
 *   it enqueues all-reduces, so every rank must enter bpgl_solver_status
 *   concurrently, one process or thread per rank).
 * bpgl_solver_stat: counters since the last reset -- "onepass" (1 while the
 *   one-pass iteration is in use), "refresh_period" (iterations between
 *   exact-gradient refreshes, 0 = none), "refreshes" (exact-gradient refreshes
 *   enqueued), "fallbacks" (recoveries above), "requested"
 *   (iterations asked of bpgl_solver_step), "enqueued", "cus" (CUs the
 *   persistent grid is sized for), "cu_masked" (1: narrower than the device,
 *   from the stream's CU mask), "onepass_grid" (its blocks), "onepass_rows" (1:
 *   the row groups own interleaved rows, see "onepass_rows" under bpgl_set_tuning).
 * bpgl_solver_residual: device pointer of the residual s11 = sum_k Ax_k - b (m).
 */
int bpgl_solver_reset(bpgl_ctx* ctx, const double* b, double mu, double* x,
                      const int32_t* order, int64_t order_len, double err_bound,
                      double* err_iter, double* time_iter, int64_t record_len,
                      int use_graph);
int bpgl_solver_step(bpgl_ctx* ctx, int64_t n_iter);
int bpgl_solver_status(bpgl_ctx* ctx, int64_t* iters_done, int* stopped, int64_t* t_last,
                       double* gamma, double* err);
int bpgl_solver_stat(bpgl_ctx* ctx, const char* key, int64_t* value);
const double* bpgl_solver_residual(bpgl_ctx* ctx);

/*
 * One-call form: reset, run n_iter iterations, wait (bpgl_solver_status, so lost
 * one-pass iterations are re-run whether or not iters_done is given), report.
 * The survey's bpgl_iterate.  iters_done may be NULL.
 */
int bpgl_iterate(bpgl_ctx* ctx, int64_t n_iter, const int32_t* order, double mu,
                 const double* b, double* x, double* err_iter, double* time_iter,
                 double err_bound, int64_t* iters_done);

/* Timing of the most recent bpgl_solver_step window on the context stream:
 * average duration (ms) of each kernel kind over the window, measured with
 * HIP events when profiling was enabled by bpgl_set_kernel_timing(ctx, 1).
 * kinds: 0 colpass (A^T r), 1 shrink, 2 rowpass (A D), 3 rowreduce (+ line
 * search on one rank), 4 allreduce, 5 step (multi-rank line search), 6 update
 * (+ gradient update in one-pass mode), 7 onepass (A D and A^T (A D) in one
 * pass over A), 8 refresh (the one-pass exact-gradient refresh, amortised:
 * its total time over the window's iterations).  Row shards: 3 = fold of the
 * exchange contribution (the line search runs in 6). */
int bpgl_set_kernel_timing(bpgl_ctx* ctx, int enable);
int bpgl_kernel_times(bpgl_ctx* ctx, double* avg_ms /* 9 */, int64_t* samples);

/* Runtime tuning knobs (call before bpgl_solver_reset).  These do not change
 * results:
 *   "nt_loads" (default 1): stream A with non-temporal loads.
 *   "tail_permille" (default 120): with nt_loads, the share of every row chunk
 *   each pass reads last with cache-allocating loads (Infinity Cache reuse by
 *   the other pass).
 *   "reverse_rows" (default 0): the A D pass walks each row chunk bottom-up.
 *   "tail_row_blocks" (default 1): the one-pass tail runs the residual update on
 *   blocks of its own, beside its column blocks (0: every block first).
 *   "graph_max" (default 64; a power of two, at most 8 with an RCCL communicator):
 *   the largest hipGraph of iterations bpgl_solver_reset captures (use_graph).
 * These select the iteration's arithmetic path (results agree to rounding,
 * each path is bitwise deterministic):
 *   "onepass" (default -1 = when eligible, 0 = off, 1 = required): one pass
 *   over A per iteration, the gradient carried as g += gamma A^T (A D); needs
 *   one feature block, one rank (or row shards), at most
 *   128 x 4096 columns (fp32; 128 x 6144 for bf16, 128 x 2048 for fp64) and all
 *   of its blocks resident at once (nothing else running on the device): its segment
 *   blocks per row must fit the CUs the stream may use.  When they do not (e.g. a
 *   row of 524288 fp32 columns on a 64-CU partition), auto runs two passes; RCCL
 *   row shards then run the two-pass row iteration (exact g through an all-reduce
 *   of w, s23 on the local rows) -- since ABI 302; before, such a context was refused.
 *   "onepass_cache_permille" (default -1 = auto: 750 when this rank's A block is
 *   at most 320 MiB, i.e. about the 256 MiB Infinity Cache, else 0): share of every
 *   row group the one-pass kernel reads with cache-allocating loads (launches
 *   alternate the row direction, so the next launch starts on those rows).
 *   "onepass_rows" (default -1 = auto: interleaved when there are at least 8 row
 *   groups of at least 128 rows over at least 16 segment blocks, else 0): 1 = row
 *   group g of the one-pass kernel owns rows g, g + ngroups, ... (the groups read
 *   adjacent rows at once; with at most 64 segment blocks per row, else always 0),
 *   0 = R consecutive rows; bpgl_solver_stat("onepass_rows") reports the form in use.
 *   "onepass_sb1" (default -1 = on when a row is one segment block, 0 = off): with one
 *   segment block per row (e.g. 4096 fp32 columns) the row's s23 is folded from the 4 wave
 *   partials in LDS instead of a tagged granule through memory (configs[3] +2 %; results agree
 *   with the granule path to its parity bit; an explicit "onepass_rows" = 1 selects the
 *   granule path); bpgl_solver_stat("onepass_sb1") reports it.
 *   "onepass_refresh" (default 256; 0 = only at reset): recompute g = A^T r
 *   exactly every this many iterations (bounds the recurrence's drift).
 *   "exchange_fp32" (default 0 = never, -1 = with an RCCL communicator, 1 = also for
 *   a caller-side exchange): row shards' per-iteration exchange in fp32 -- half the
 *   bytes, x within 2e-7 (1 rank) to 1.5e-6 (8 ranks, 120 iterations) of the fp64 exchange;
 *   5.7e-6 from the one-GPU path after 300 iterations at 8 ranks (round 6: kept opt-in).
 *   "onepass_fail_at" (test hook, default -1): the one-pass launch of iteration t
 *   reports a row hand-off failure once (exercises the recovery above).
 *   "cus" (before bpgl_bind only; default: the stream's CU mask, else the device):
 *   the CU count the persistent one-pass grid (row groups x segment blocks) is
 *   sized for.
 * The environment variable BPGL_TARGET_BLOCKS (read by bpgl_create) sets the
 * number of (row chunk x column segment) tiles per two-pass launch (default
 * 1024 for fp32 A, 512 for fp64 / bf16). */
int bpgl_set_tuning(bpgl_ctx* ctx, const char* key, int64_t value);

/* Launch geometry chosen for this context (diagnostics). */
int bpgl_geometry(const bpgl_ctx* ctx, int32_t* nseg, int32_t* nchunk, int32_t* rows_per_chunk,
                  int32_t* seg_width);

/* ===========================================================================
 * Panel path (BASELINE configs[4]): nrhs in {16, 32, 64, 128} right-hand sides
 * solved together, A stored once in bf16 (row-major A [m][lda], caller-owned;
 * the A^T pass reads it through transposing LDS reads), both passes on CDNA4
 * MFMA (v_mfma_f32_16x16x32_bf16) with split-bf16 operands.  The reference
 * has no batched solver: each RHS follows the single-RHS iteration of
 * lasso.py:102-157 (cyclic blocks, fixed iteration count).  m and the block
 * width must be multiples of 256.  Layouts: B, R [nrhs][m]; G, D [nrhs][w];
 * x [nblock][nrhs][w] fp32.
 * =========================================================================== */
typedef struct bpgl_panel bpgl_panel;
int bpgl_panel_create(bpgl_panel** out, int device, int64_t m, int64_t n, int32_t nblock, int32_t nrhs,
                      int32_t kchunks /* <= 0: automatic */, void* hip_stream);
void bpgl_panel_destroy(bpgl_panel* ctx);
int64_t bpgl_panel_scratch_bytes(const bpgl_panel* ctx);
/* bind COPIES A's contents into two tiled m x n bf16 images inside the scratch (one per pass: each pass's
 * 64-deep stage is then one contiguous 32 KiB), so bpgl_panel_scratch_bytes includes 4 m n bytes for
 * them on top of the vectors.  The solver passes and bpgl_panel_mtm / _mm read those copies; only
 * bpgl_panel_diag reads A itself.  A must stay valid while the context is bound, and after A's
 * contents change the context must be bound again (the copies are not refreshed).  The fused
 * reduce + update form ("fuse_update" below) is admitted at bind only if its blocks fit on the CUs
 * the context's stream may use (a CU-masked stream counts its own CUs; stat "fuse_cus"). */
int bpgl_panel_bind(bpgl_panel* ctx, const void* A /* [m][lda] bf16 */, int64_t lda, void* scratch,
                    int64_t scratch_bytes);
int bpgl_panel_diag(bpgl_panel* ctx, double* out /* nullable, n fp64 */);
/* G = A_b^T R  and  S = A_b D  (fp64 in/out, device; split-bf16 MFMA inside) */
int bpgl_panel_mtm(bpgl_panel* ctx, int32_t block, const double* R, double* G);
int bpgl_panel_mm(bpgl_panel* ctx, int32_t block, const double* D, double* S);
int bpgl_panel_reset(bpgl_panel* ctx, const double* B, const double* mu /* nrhs */, double* err_iter,
                     int64_t record_len, int use_graph);
int bpgl_panel_step(bpgl_panel* ctx, int64_t n_iter);
int bpgl_panel_status(bpgl_panel* ctx, int64_t* iters, double* last_err);
const float* bpgl_panel_x(bpgl_panel* ctx);
int bpgl_panel_set_kernel_timing(bpgl_panel* ctx, int enable);
int bpgl_panel_kernel_times(bpgl_panel* ctx, double* avg_ms /* 5: pass1, pass2, reduce (+ line search), step (0: folded into reduce), update */,
                            int64_t* samples);
/* tuning knobs.  Results are bitwise independent of these: "interleave1",
 * "interleave2" (pass 1 / pass 2; "interleave" sets both) 0/1/2 -- LDS-DMA
 * pieces issued together after each stage barrier (0), spread over the stage's
 * MFMA groups (1), or spread and software-pipelined with fragment reads one MFMA
 * group ahead across the stage barrier (2).  Defaults: pass 1 -- 2; pass 2 -- 2 with the bf16 direction
 * (d_split 1) at k >= 64, else 1 (round 4); get_tuning reports the form in use.
 * This one selects the solver's arithmetic (every choice is an exact line
 * search along the direction it takes): "d_split" 1 (default since ABI 200) --
 * the direction enters the A D pass as its bf16 rounding alone (half the
 * pass-2 MFMA work); 2 -- as a hi + lo bf16 pair (~16-bit mantissa).  Both
 * converge to the same solution: after the reference's 1000 iterations at the
 * configs[4] shape both are within 1.7-2.2e-5 of the fp64 oracle on x and 1e-11
 * on the objective (the gradient pass, hi + lo always, sets the fixed point;
 * profiles/r04/accuracy); short runs follow slightly different trajectories.
 * bpgl_panel_mtm / _mm always use hi + lo operands.  bpgl_panel_get_tuning reads
 * "interleave1", "interleave2", "d_split", "defer_x", "carry_g", "g_refresh", "fuse_update",
 * "fuse_grid".
 * "fuse_update" (0 / 1; default 1; in effect with one feature block, defer_x and m a multiple of
 * 1024 -- get_tuning reports the form in effect; a reset must follow a change): the split-K reduce, each
 * RHS's line search and R += gamma S run as ONE launch whose blocks wait for their RHS's step size
 * (bitwise the two-kernel result); it needs its blocks co-resident, which bpgl_panel_bind checks with
 * the occupancy API against the stream's usable CUs (its CU mask, else the device) -- should a wait still run out (another kernel holding CUs), nothing is updated and
 * bpgl_panel_status returns BPGL_E_EXCHANGE.  "fuse_grid" (256 / 512 / 1024, default 1024): its grid.
 * "defer_x" (0 / 1; default 1, one feature block; a reset must follow a change): the
 * update x += gamma D' of an iteration is applied by the next pass-1 epilogue (and at
 * the end of every bpgl_panel_step), bitwise the same x.
 * "carry_g" (0 / 1; default 1, in effect with one feature block only -- set to 1
 * with more blocks is an error; a reset must follow a change): the gradient is
 * carried in fp32, G_t = G_{t-1} + gamma_{t-1} A^T S_{t-1} with S_{t-1} = A D'_{t-1}
 * the previous iteration's product (its bf16 image: one MFMA product in pass 1
 * instead of the residual's two), and recomputed exactly from R (hi + lo) every
 * "g_refresh" iterations (default 64, a multiple of 8) -- the single-RHS path's
 * carried gradient.  Measured at configs[4]: pass 1
 * 226 -> 196 us, and after 1000 iterations x within 4e-6 of the oracle instead of
 * 1.9e-5 (fp32 accumulation of small updates instead of re-reading R through its
 * 2^-17 pieces).  get_tuning("carry_g") reports the form in effect. */
int bpgl_panel_set_tuning(bpgl_panel* ctx, const char* key, int64_t value);
int bpgl_panel_get_tuning(const bpgl_panel* ctx, const char* key, int64_t* value);
int bpgl_panel_geometry(const bpgl_panel* ctx, int32_t* kchunks);
/* Counters since the last reset: "iters_enqueued", "exact_gradients" (carried
 * gradient: iterations whose pass 1 computed G = A^T R exactly -- every g_refresh-th). */
int bpgl_panel_stat(const bpgl_panel* ctx, const char* key, int64_t* value);
/* The solver's fp64 residual R = A X - B, [nrhs][m] in device memory (valid after
 * the stream has drained). */
const double* bpgl_panel_residual(bpgl_panel* ctx);

#ifdef __cplusplus
}
#endif
#endif /* BPGL_H */
