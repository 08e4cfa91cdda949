// One-HBM-pass probe (diagnostics only, not part of the product): can one launch stream
// A from HBM once and produce both S = A D and U = A^T S (the two products of one
// iteration when the gradient is carried by G += gamma U)?
//
// 256 persistent blocks (one per CU), 5 waves each.  Group g = blockIdx % 8 owns row
// chunks c = g, g + 8, ... (H rows each); block j = blockIdx / 8 of the group owns
// columns [j SW, (j+1) SW).  Waves 0-3 stream their 512-column slice of each chunk into
// an NB-slot LDS ring (LDS-DMA), compute the chunk's row partials of A D (phase 1) and,
// L steps later, U += A^T S for that chunk from the same LDS copy (phase 2).  Wave 4
// exchanges the partials with the group's other blocks: it publishes each row partial as
// two tagged 8-byte granules (fp32 hi, fp32 lo, 32-bit launch tag) with sc1 stores and
// gathers the 32 blocks' granules of a chunk published L - 2 steps earlier (sc1 loads,
// bounded re-polls).  One raw barrier per step.  Every spin is bounded: on timeout the
// error word is set and the kernel still finishes.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((address_space(3))) void* lds_ptr;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kGroups = 8;
constexpr int kSW = 2048;       // columns per block (fp32: 8 KiB per row)
constexpr int kWaveCols = 512;  // columns per compute wave

// H rows per chunk, kP tiles loaded ahead, phase-2 lag kL (publish -> gather distance kL - 2),
// NOWAIT (diagnostic): gather without checking tags (wrong S; bounds the exchange cost)
template <int H, int kP, int kL, int NOWAIT>
__global__ __launch_bounds__(320) void onepass(const float* __restrict__ A, long long lda, long long m,
                                               const double* __restrict__ D, double* __restrict__ S,
                                               double* __restrict__ Ug, unsigned long long* gran,
                                               unsigned tag, unsigned* err) {
    constexpr int kNB = kP + kL + 1;                  // LDS ring slots
    constexpr int TILE = H * kSW * 4;                 // bytes per slot
    __shared__ __attribute__((aligned(16))) char ring[kNB * TILE];
    __shared__ double part[2][H][4];                   // per step parity: row partial of each compute wave
    __shared__ double sbuf[2][H];                      // gathered S of a chunk, by parity
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = blockIdx.x % kGroups, j = blockIdx.x / kGroups;
    const int nb = gridDim.x / kGroups;               // blocks per group (32)
    const long long nchunk = m / H;
    const long long K = (nchunk - g + kGroups - 1) / kGroups;   // chunks of this group
    const long long col0 = (long long)j * kSW;

    // compute-wave state
    double d[8] = {0, 0, 0, 0, 0, 0, 0, 0}, u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int wcol = wave * kWaveCols;                // this wave's slice inside the segment
    if (wave < 4) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < 4; ++e) d[4 * h + e] = D[col0 + wcol + h * 256 + lane * 4 + e];
    }
    // LDS-DMA of tile k (chunk g + 8k) by compute wave `wave`: H rows x 2 KiB slice = 2H pieces
    auto issue_tile = [&](long long k) {
        const long long kk = k < K ? k : K - 1;       // clamped tail: reload into an unread slot
        const long long row0 = (g + kGroups * kk) * H;
        char* slot = ring + (int)(k % kNB) * TILE + wave * (H * kWaveCols * 4);
#pragma unroll
        for (int p = 0; p < 2 * H; ++p) {
            const float* src = A + (row0 + p / 2) * lda + col0 + wcol + (p & 1) * 256 + lane * 4;
            __builtin_amdgcn_global_load_lds(src, (lds_ptr)(slot + p * 1024), 16, 0, 0);
        }
    };
    if (wave < 4) for (int k = 0; k < kP; ++k) issue_tile(k);

    unsigned long long* mygran = gran;
    unsigned polls_left = 1u << 16;   // per launch and wave: a failed exchange ends in ~65 ms, flagged
    for (long long step = 0; step < K + kL; ++step) {
        // tile `step` landed (this wave's pieces), then everyone
        if (wave < 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kP - 1) * 2 * H) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (wave < 4) {
            if (step < K) {   // phase 1: row partials of tile `step`
                const char* t = ring + (int)(step % kNB) * TILE + wave * (H * kWaveCols * 4);
#pragma unroll
                for (int r = 0; r < H; ++r) {
                    const float4 a0 = *reinterpret_cast<const float4*>(t + r * 2048 + lane * 16);
                    const float4 a1 = *reinterpret_cast<const float4*>(t + r * 2048 + 1024 + lane * 16);
                    double s = 0.0;
                    s = fma((double)a0.x, d[0], s); s = fma((double)a0.y, d[1], s);
                    s = fma((double)a0.z, d[2], s); s = fma((double)a0.w, d[3], s);
                    s = fma((double)a1.x, d[4], s); s = fma((double)a1.y, d[5], s);
                    s = fma((double)a1.z, d[6], s); s = fma((double)a1.w, d[7], s);
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                    if (lane == 0) part[step & 1][r][wave] = s;
                }
            }
            const long long k2 = step - kL;
            if (k2 >= 0) {    // phase 2: U += A^T S for tile k2 (its S gathered last step)
                const char* t = ring + (int)(k2 % kNB) * TILE + wave * (H * kWaveCols * 4);
#pragma unroll
                for (int r = 0; r < H; ++r) {
                    const double sr = sbuf[k2 & 1][r];
                    const float4 a0 = *reinterpret_cast<const float4*>(t + r * 2048 + lane * 16);
                    const float4 a1 = *reinterpret_cast<const float4*>(t + r * 2048 + 1024 + lane * 16);
                    u[0] = fma((double)a0.x, sr, u[0]); u[1] = fma((double)a0.y, sr, u[1]);
                    u[2] = fma((double)a0.z, sr, u[2]); u[3] = fma((double)a0.w, sr, u[3]);
                    u[4] = fma((double)a1.x, sr, u[4]); u[5] = fma((double)a1.y, sr, u[5]);
                    u[6] = fma((double)a1.z, sr, u[6]); u[7] = fma((double)a1.w, sr, u[7]);
                }
            }
            issue_tile(step + kP);   // slot of tile step+kP-kNB = step-kL-1: phase 2 done last step
        } else if (NOWAIT != 2) {   // NOWAIT == 2 (diagnostic): no exchange at all
            // exchange wave: publish chunk step-1, gather chunk step-kL+1
            const long long kp = step - 1;
            if (kp >= 0 && kp < K && lane < H) {
                const int r = lane;
                const double p = ((part[kp & 1][r][0] + part[kp & 1][r][1]) + part[kp & 1][r][2]) + part[kp & 1][r][3];
                const float hi = (float)p;
                const float lo = (float)(p - (double)hi);
                const long long row = (g + kGroups * kp) * H + r;
                const unsigned long long g0 = ((unsigned long long)(2 * tag) << 32) | __float_as_uint(hi);
                const unsigned long long g1 = ((unsigned long long)(2 * tag + 1) << 32) | __float_as_uint(lo);
                unsigned long long* dst = mygran + (row * nb + j) * 2;
                __hip_atomic_store(dst, g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(dst + 1, g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const long long kg = step - kL + 1;
            if (kg >= 0 && kg < K) {
                // lane -> (row r, block jj): H * nb pairs (<= 64)
                const int r = lane / nb, jj = lane % nb;
                const bool act = r < H;
                const long long row = (g + kGroups * kg) * H + (act ? r : 0);
                const unsigned long long* src = mygran + (row * nb + (act ? jj : 0)) * 2;
                double v = 0.0;
                bool ok = false;
                while (true) {
                    const unsigned long long a = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long b = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = NOWAIT || !act || ((unsigned)(a >> 32) == 2 * tag && (unsigned)(b >> 32) == 2 * tag + 1);
                    if (act && ok) v = (double)__uint_as_float((unsigned)a) + (double)__uint_as_float((unsigned)b);
                    if (__all(ok)) break;
                    if (polls_left == 0) { if (lane == 0) atomicOr(err, 1u); break; }
                    --polls_left;
                    __builtin_amdgcn_s_sleep(1);
                }
                // fixed-order sum over the nb blocks of each row (lanes r*nb .. r*nb+nb-1)
                for (int o = 1; o < nb; o <<= 1) {
                    const double w = __shfl_down(v, o);
                    if ((lane % nb) + o < nb && (lane % (2 * o)) == 0) v += w;
                }
                if (act && jj == 0) {
                    sbuf[kg & 1][r] = v;
                    if (j == 0) S[row] = v;
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave < 4) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < 4; ++e) Ug[(long long)g * (nb * kSW) + col0 + wcol + h * 256 + lane * 4 + e] = u[4 * h + e];
    }
}

extern "C" double onepass_run(const void* A, long long lda, long long m, const void* D, void* S, void* Ug,
                              void* gran, unsigned* err, int iters, unsigned tag0, int variant) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = (cus / kGroups) * kGroups;
    unsigned tag = tag0;
    auto run = [&]() {
#define OP(H, P, LG, NW)                                                                                     \
    hipLaunchKernelGGL((onepass<H, P, LG, NW>), dim3(blocks), dim3(320), 0, 0, (const float*)A, lda, m,           \
                       (const double*)D, (double*)S, (double*)Ug, (unsigned long long*)gran, tag, err)
        switch (variant) {
            case 0: OP(2, 2, 6, 0); break;
            case 1: OP(2, 4, 4, 0); break;
            case 2: OP(2, 4, 4, 2); break;
            case 3: OP(2, 2, 6, 2); break;
            case 4: OP(1, 8, 8, 2); break;
            case 5: OP(1, 10, 6, 2); break;
            default: OP(2, 6, 2, 2); break;
        }
#undef OP
        ++tag;
    };
    run();
    (void)hipEventRecord(e0, 0);
    for (int k = 0; k < iters; ++k) run();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (double)ms / iters;
}
