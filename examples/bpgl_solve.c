/* bpgl_solve -- a plain C caller of libbpgl (include/bpgl.h): no Python, no PyTorch.
 *
 * It does what a non-Python host binding of the reference's GPU path would do
 * (GPU_Calculation(A, Block) + ClassLassoCB_v2.run, gpu_calculation.py:148-261,
 * lasso.py:458-613): allocate device memory itself (the library never does),
 * upload A and b, compute diag(A^T A), run the device-resident solver with the
 * reference's ERR_BOUND rule (lasso.py:141-150) and read x and the error record
 * back.  tests/test_c_caller.py runs it on a reference-run fixture and compares.
 *
 * usage: bpgl_solve A.f32 b.f64 m n nblock mu iters err_bound x_out.f64 err_out.f64
 *   A.f32: m x n row-major float32; b.f64: m float64; err_bound < 0: off.
 * Writes x (n float64, the reference's block order) and err_iter (iters float64);
 * prints "iters_done stopped t_last" on stdout.  Exit 0 on success, 2 on usage,
 * 1 on a library or HIP error (message on stderr).
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bpgl.h"

#define HIP_OK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #expr, hipGetErrorString(e_));                 \
            return 1;                                                                  \
        }                                                                              \
    } while (0)
#define CHECK_BPGL(expr)                                                               \
    do {                                                                               \
        int rc_ = (expr);                                                              \
        if (rc_ != BPGL_OK) {                                                          \
            fprintf(stderr, "%s failed (%d): %s\n", #expr, rc_, bpgl_last_error());    \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

static void* read_file(const char* path, size_t bytes) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    void* buf = malloc(bytes ? bytes : 1);
    size_t got = buf ? fread(buf, 1, bytes, f) : 0;
    fclose(f);
    if (got != bytes) { free(buf); return NULL; }
    return buf;
}

static int write_file(const char* path, const void* buf, size_t bytes) {
    FILE* f = fopen(path, "wb");
    if (!f) return 1;
    size_t put = fwrite(buf, 1, bytes, f);
    fclose(f);
    return put != bytes;
}

int main(int argc, char** argv) {
    if (argc != 11) {
        fprintf(stderr, "usage: %s A.f32 b.f64 m n nblock mu iters err_bound x_out.f64 err_out.f64\n", argv[0]);
        return 2;
    }
    const int64_t m = atoll(argv[3]), n = atoll(argv[4]);
    const int32_t nblock = atoi(argv[5]);
    const double mu = atof(argv[6]);
    const int64_t iters = atoll(argv[7]);
    const double err_bound = atof(argv[8]);
    if (m <= 0 || n <= 0 || nblock <= 0 || n % nblock || iters <= 0) {
        fprintf(stderr, "bad shape or iteration count\n");
        return 2;
    }
    float* A = (float*)read_file(argv[1], (size_t)(m * n) * sizeof(float));
    double* b = (double*)read_file(argv[2], (size_t)m * sizeof(double));
    if (!A || !b) {
        fprintf(stderr, "cannot read %s / %s with the given shape\n", argv[1], argv[2]);
        return 2;
    }

    bpgl_ctx* ctx = NULL;
    CHECK_BPGL(bpgl_create(&ctx, 0, BPGL_F32, m, n, nblock, NULL));
    const int64_t w = n / nblock, wp = bpgl_block_width_padded(ctx), scratch_bytes = bpgl_scratch_bytes(ctx);

    /* A in the layout bpgl_bind documents: block k at k * block_stride, rows lda apart (here the
     * reference's np.hsplit stack (nblock, m, wp), gpu_calculation.py:172-173, rows padded to wp) */
    const size_t a_elems = (size_t)nblock * (size_t)m * (size_t)wp;
    float* Ah = (float*)calloc(a_elems, sizeof(float));
    if (!Ah) { fprintf(stderr, "out of host memory\n"); return 1; }
    for (int64_t k = 0; k < nblock; ++k)
        for (int64_t i = 0; i < m; ++i)
            memcpy(Ah + ((size_t)k * m + i) * wp, A + (size_t)i * n + k * w, (size_t)w * sizeof(float));

    void *dA = NULL, *scratch = NULL;
    double *db = NULL, *dx = NULL, *derr = NULL, *ddiag = NULL;
    HIP_OK(hipMalloc(&dA, a_elems * sizeof(float)));
    HIP_OK(hipMalloc(&scratch, (size_t)scratch_bytes));   /* hipMalloc: 256-byte aligned */
    HIP_OK(hipMalloc((void**)&db, (size_t)m * sizeof(double)));
    HIP_OK(hipMalloc((void**)&dx, (size_t)nblock * wp * sizeof(double)));
    HIP_OK(hipMalloc((void**)&derr, (size_t)iters * sizeof(double)));
    HIP_OK(hipMalloc((void**)&ddiag, (size_t)nblock * wp * sizeof(double)));
    HIP_OK(hipMemcpy(dA, Ah, a_elems * sizeof(float), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(db, b, (size_t)m * sizeof(double), hipMemcpyHostToDevice));
    HIP_OK(hipMemset(dx, 0, (size_t)nblock * wp * sizeof(double)));   /* x0 = 0, lasso.py:89 */

    CHECK_BPGL(bpgl_bind(ctx, dA, wp, m * wp, scratch, scratch_bytes));
    CHECK_BPGL(bpgl_diag_ata(ctx, ddiag));
    int64_t done = 0;
    CHECK_BPGL(bpgl_iterate(ctx, iters, NULL, mu, db, dx, derr, NULL, err_bound, &done));
    int64_t t_last = 0;
    int stopped = 0;
    CHECK_BPGL(bpgl_solver_status(ctx, NULL, &stopped, &t_last, NULL, NULL));

    double* xp = (double*)malloc((size_t)nblock * wp * sizeof(double));
    double* x = (double*)malloc((size_t)n * sizeof(double));
    double* err = (double*)malloc((size_t)iters * sizeof(double));
    if (!xp || !x || !err) { fprintf(stderr, "out of host memory\n"); return 1; }
    HIP_OK(hipMemcpy(xp, dx, (size_t)nblock * wp * sizeof(double), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(err, derr, (size_t)iters * sizeof(double), hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < nblock; ++k) memcpy(x + k * w, xp + k * wp, (size_t)w * sizeof(double));
    if (write_file(argv[9], x, (size_t)n * sizeof(double)) || write_file(argv[10], err, (size_t)iters * sizeof(double))) {
        fprintf(stderr, "cannot write the outputs\n");
        return 1;
    }
    printf("%lld %d %lld\n", (long long)done, stopped, (long long)t_last);

    bpgl_destroy(ctx);
    hipFree(dA); hipFree(scratch); hipFree(db); hipFree(dx); hipFree(derr); hipFree(ddiag);
    free(A); free(b); free(Ah); free(xp); free(x); free(err);
    return 0;
}
