/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * A Gaussian-recipe lasso instance that the build container and the GPU box generate bit for bit
 * identically, for the long-horizon full-size parity fixtures (tests/golden/make_gauss.py,
 * tests/test_fullsize.py).  The recipe is the reference's (parameters.py:17-33): A with N(0, 1)
 * entries and every row scaled to unit l2 norm, x_true sparse with density `den` and N(0, 1)
 * values, e ~ N(0, 1e-4).  Bit-reproducibility across CPUs rules out libm's transcendental
 * functions (glibc selects implementations per CPU), so every N(0, 1) draw is the Irwin-Hall
 * approximant: the sum of 12 independent 16-bit uniforms minus 6 (mean 0, variance 1 up to
 * 2^-32, support +-6), from a counter-based hash (splitmix64's finaliser) of (seed, stream,
 * index).  Only integer operations, exact scalings and the IEEE-exact double operations
 * (+, *, /, sqrt) are used, in a fixed order per row (-ffp-contract=off): the result is
 * independent of the CPU and of the thread count.
 */
#include <math.h>
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static uint64_t gi_mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* N(0, 1) approximant number `idx` of stream `stream`: 12 uniforms of 16 bits from 3 hashes */
static double gi_normal(uint64_t seed, uint64_t stream, uint64_t idx) {
    const uint64_t base = gi_mix(seed ^ gi_mix(stream * 0x100000001b3ull));
    int64_t s = 0;
    for (uint64_t k = 0; k < 3; ++k) {
        const uint64_t h = gi_mix(base + 3u * idx + k);
        s += (int64_t)(h & 0xffff) + (int64_t)((h >> 16) & 0xffff) + (int64_t)((h >> 32) & 0xffff) +
             (int64_t)(h >> 48);
    }
    /* each uniform is (u + 1/2) / 2^16, u in [0, 65535]: sum - 6 = (s + 6) / 2^16 - 6, exact */
    return ((double)s + 6.0) * 0x1.0p-16 - 6.0;
}

/* a uniform in [0, 1) of stream `stream` (53 bits) */
static double gi_uniform(uint64_t seed, uint64_t stream, uint64_t idx) {
    const uint64_t h = gi_mix(gi_mix(seed ^ gi_mix(stream * 0x100000001b3ull)) + idx);
    return (double)(h >> 11) * 0x1.0p-53;
}

/* row i of A (fp32, unit l2 norm) into row[0..n) */
static void gi_row(uint64_t seed, int64_t i, int64_t n, float* row) {
    double ss = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        const double z = gi_normal(seed, 1, (uint64_t)(i * n + j));
        ss += z * z;
    }
    const double nrm = sqrt(ss);
    for (int64_t j = 0; j < n; ++j) row[j] = (float)(gi_normal(seed, 1, (uint64_t)(i * n + j)) / nrm);
}

/* rows row0 .. row0 + nrows - 1 of the instance's A (a [nrows][n] fp32 slice) */
int oracle_gauss_rows(uint64_t seed, int64_t row0, int64_t nrows, int64_t n, float* out) {
    if (row0 < 0 || nrows < 0 || n <= 0) return -1;
    for (int64_t i = 0; i < nrows; ++i) gi_row(seed, row0 + i, n, out + i * n);
    return 0;
}

/*
 * A [m][n] fp32 (rows N(0, 1), unit l2 norm, each row normalised in fp64 before the one rounding
 * to fp32), x_true [n] (density den, N(0, 1) values), e [m] (N(0, 1e-4)).  Any output may be NULL.
 */
int oracle_gauss_instance(uint64_t seed, int64_t m, int64_t n, double den, float* A, double* x_true,
                          double* e, int nthreads) {
    if (m <= 0 || n <= 0) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    if (A) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < m; ++i) gi_row(seed, i, n, A + i * n);
    }
    if (x_true)
        for (int64_t j = 0; j < n; ++j)
            x_true[j] = gi_uniform(seed, 2, (uint64_t)j) < den ? gi_normal(seed, 3, (uint64_t)j) : 0.0;
    if (e)
        for (int64_t i = 0; i < m; ++i) e[i] = 0.01 * gi_normal(seed, 4, (uint64_t)i);
    return 0;
}
