/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's block best-response lasso iteration
 * (kingold5/convex_optimization).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * or as the timed CPU baseline.  The product path (convex_optimization_amd/)
 * never links or calls it.
 *
 * Parity pinning: the restatement is checked against golden vectors produced
 * by running the reference's own ClassLassoCPU (lasso.py:25-169) in the build
 * container (tests/golden/make_golden.py); see tests/test_oracle.py.
 *
 * Reference map (file:line in the reference):
 *   soft threshold        cpu_calculation.py:5-6
 *   element_proj          cpu_calculation.py:10-11
 *   error_crit            cpu_calculation.py:15-20
 *   diag(A_m^T A_m)       cpu_calculation.py:35-42 (K3 gpu_calculation.py:116-137)
 *   A_m^T r  (s12/s13)    cpu_calculation.py:30-31, lasso.py:107-111
 *   A_m D    (s22/s23)    cpu_calculation.py:45-46, lasso.py:121-126 (P shards summed)
 *   one iteration         lasso.py:102-157
 *
 * Arithmetic: every product and sum in fp64; A may be stored fp32 or fp64.
 * Results are independent of the thread count: each output element is
 * accumulated by exactly one thread in a fixed order.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define AT(A, f64, idx) ((f64) ? ((const double*)(A))[idx] : (double)((const float*)(A))[idx])

static void set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

/* diag(A_b^T A_b) for every feature block b: out[b*w + j] = sum_i A[i, b*w+j]^2 */
int oracle_diag_ata(int a_f64, const void* A, int64_t lda, int64_t m, int64_t n,
                    int32_t nblock, double* out, int nthreads) {
    if (nblock <= 0 || n % nblock) return -1;
    set_threads(nthreads);
    memset(out, 0, sizeof(double) * (size_t)n);
    const int64_t CH = 256;
#pragma omp parallel for schedule(static)
    for (int64_t j0 = 0; j0 < n; j0 += CH) {
        int64_t j1 = j0 + CH < n ? j0 + CH : n;
        for (int64_t i = 0; i < m; ++i)
            for (int64_t j = j0; j < j1; ++j) {
                double a = AT(A, a_f64, i * lda + j);
                out[j] += a * a;
            }
    }
    return 0;
}

/* g[j] = sum_i A[i, col0+j] * r[i], j < w  (row order i = 0..m-1) */
int oracle_mtv(int a_f64, const void* A, int64_t lda, int64_t m, int64_t col0,
               int64_t w, const double* r, double* g, int nthreads) {
    set_threads(nthreads);
    memset(g, 0, sizeof(double) * (size_t)w);
    const int64_t CH = 512;
#pragma omp parallel for schedule(static)
    for (int64_t j0 = 0; j0 < w; j0 += CH) {
        int64_t j1 = j0 + CH < w ? j0 + CH : w;
        for (int64_t i = 0; i < m; ++i) {
            const double ri = r[i];
            const int64_t base = i * lda + col0;
            if (a_f64) {
                const double* Ar = (const double*)A + base;
                for (int64_t j = j0; j < j1; ++j) g[j] += Ar[j] * ri;
            } else {
                const float* Ar = (const float*)A + base;
                for (int64_t j = j0; j < j1; ++j) g[j] += (double)Ar[j] * ri;
            }
        }
    }
    return 0;
}

/* s[i] = sum_{p<P} ( sum_{j in shard p} A[i, col0+j] d[j] ), shards of w/P
 * columns summed in order p = 0..P-1 (lasso.py:123-126). */
int oracle_mv(int a_f64, const void* A, int64_t lda, int64_t m, int64_t col0,
              int64_t w, int32_t P, const double* d, double* s, int nthreads) {
    if (P <= 0 || w % P) return -1;
    set_threads(nthreads);
    const int64_t ws = w / P;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < m; ++i) {
        const int64_t base = i * lda + col0;
        double tot = 0.0;
        for (int32_t p = 0; p < P; ++p) {
            double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            int64_t j = p * ws, je = (p + 1) * ws;
            if (a_f64) {
                const double* Ar = (const double*)A + base;
                for (; j + 8 <= je; j += 8)
                    for (int k = 0; k < 8; ++k) acc[k] += Ar[j + k] * d[j + k];
                for (; j < je; ++j) acc[0] += Ar[j] * d[j];
            } else {
                const float* Ar = (const float*)A + base;
                for (; j + 8 <= je; j += 8)
                    for (int k = 0; k < 8; ++k) acc[k] += (double)Ar[j + k] * d[j + k];
                for (; j < je; ++j) acc[0] += (double)Ar[j] * d[j];
            }
            double sp = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
            tot = (p == 0) ? sp : tot + sp;
        }
        s[i] = tot;
    }
    return 0;
}

static inline double soft_thr(double t, double tau) {           /* cpu_calculation.py:5-6 */
    double mag = fabs(t) - tau;
    double sg = (t > 0) ? 1.0 : ((t < 0) ? -1.0 : 0.0);
    return sg * (mag > 0 ? mag : 0.0);
}
static inline double proj(double v, double lo, double hi) {      /* cpu_calculation.py:10-11 */
    double a = v < hi ? v : hi;
    return a > lo ? a : lo;
}

/*
 * The full solver loop of ClassLassoCPU.run (lasso.py:70-169).
 *   order    : block index per iteration (nullable -> cyclic t % nblock, lasso.py:40-41)
 *   err_bound: < 0 disables the stopping rule (ERR_BOUND not a float)
 *   x        : in/out, n values (start from x0; the reference starts at 0)
 *   err_iter : nullable, iter_max values (lasso.py:54-58)
 *   t_last   : the last loop index t reached (the reference's `t` after the loop)
 *   gamma_out: nullable, step size per iteration (diagnostics)
 * When r2 == 0 the reference prints and reuses a stale step (lasso.py:133-136);
 * here gamma = 0, which is identical whenever D == 0 (the only way r2 == 0 on
 * real data) and defined at t = 0 where the reference raises.
 */
int oracle_run(int a_f64, const void* A, int64_t lda, int64_t m, int64_t n,
               int32_t nblock, int32_t P, const double* b, double mu, int64_t iter_max,
               const int32_t* order, double err_bound, double* x, double* err_iter,
               int64_t* t_last, double* gamma_out, int nthreads) {
    if (nblock <= 0 || n % nblock) return -1;
    const int64_t w = n / nblock;
    if (P <= 0 || w % P) return -2;
    double* dg = (double*)malloc(sizeof(double) * (size_t)n);
    double* Ax = (double*)calloc((size_t)(nblock * m), sizeof(double));
    double* r = (double*)malloc(sizeof(double) * (size_t)m);
    double* g = (double*)malloc(sizeof(double) * (size_t)w);
    double* Bx = (double*)malloc(sizeof(double) * (size_t)w);
    double* D = (double*)malloc(sizeof(double) * (size_t)w);
    double* s23 = (double*)malloc(sizeof(double) * (size_t)m);
    if (!dg || !Ax || !r || !g || !Bx || !D || !s23) return -3;
    oracle_diag_ata(a_f64, A, lda, m, n, nblock, dg, nthreads);
    /* initial Ax from x0 (zero in the reference) */
    for (int32_t k = 0; k < nblock; ++k) {
        int nz = 0;
        for (int64_t j = 0; j < w; ++j) nz |= x[k * w + j] != 0.0;
        if (nz) oracle_mv(a_f64, A, lda, m, k * w, w, 1, x + k * w, Ax + k * m, nthreads);
    }
    int bounded = err_bound >= 0.0;
    int64_t block_cnt = 0, t = 0;
    for (t = 0; t < iter_max; ++t) {
        int32_t mb = order ? order[t] : (int32_t)(t % nblock);
        const double* dm = dg + mb * w;
        double* xm = x + mb * w;
        /* s11 = sum_k Ax[k] - b  (lasso.py:105) */
        for (int64_t i = 0; i < m; ++i) {
            double acc = Ax[i];
            for (int32_t k = 1; k < nblock; ++k) acc += Ax[k * m + i];
            r[i] = acc - b[i];
        }
        oracle_mtv(a_f64, A, lda, m, mb * w, w, r, g, nthreads);       /* s12/s13 */
        double l1_bx = 0.0, l1_x = 0.0, err = 0.0;
        for (int64_t j = 0; j < w; ++j) {
            double rx = dm[j] * xm[j] - g[j];                          /* s14 */
            double st = soft_thr(rx, mu);
            Bx[j] = (1.0 / dm[j]) * st;                                 /* s15 */
            D[j] = Bx[j] - xm[j];
            l1_bx += fabs(Bx[j]);
            l1_x += fabs(xm[j]);
            double e = fabs(g[j] - proj(g[j] - xm[j], -mu, mu));       /* error_crit */
            if (e > err || isnan(e)) err = e;
        }
        oracle_mv(a_f64, A, lda, m, mb * w, w, P, D, s23, nthreads);    /* s21-s23 */
        double r1 = 0.0, r2 = 0.0;
        for (int64_t i = 0; i < m; ++i) { r1 += r[i] * s23[i]; r2 += s23[i] * s23[i]; }
        r1 += mu * (l1_bx - l1_x);
        double gamma = (r2 == 0.0) ? 0.0 : proj(-r1 / r2, 0.0, 1.0);
        if (gamma_out) gamma_out[t] = gamma;
        if (err_iter) err_iter[t] = err;
        if (bounded) {                                                  /* lasso.py:141-150 */
            if (err < err_bound) block_cnt++;
            if (nblock - 1 == mb) {
                if (block_cnt == nblock) break;
                block_cnt = 0;
            }
        }
        for (int64_t j = 0; j < w; ++j) xm[j] += gamma * D[j];          /* lasso.py:153 */
        for (int64_t i = 0; i < m; ++i) Ax[mb * m + i] += gamma * s23[i]; /* lasso.py:155 */
    }
    if (t == iter_max) t = iter_max - 1;
    if (t_last) *t_last = t;
    free(dg); free(Ax); free(r); free(g); free(Bx); free(D); free(s23);
    return 0;
}
