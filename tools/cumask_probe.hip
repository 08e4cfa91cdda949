// Where do the blocks of a kernel launched on a CU-masked stream run?  
//
// For each of the masks distributed.xcd_symmetric_cu_mask builds (1, 2, 4 and 8 partitions
// of the 256 CUs) this launches a grid of short spinning blocks on a stream created with
// hipExtStreamCreateWithCUMask and records, per block, the XCC id and the HW_ID register
// (SE / SH / CU of the block), then prints the number of distinct CUs each XCD ran blocks on.
// A mask that left an XCD without CUs would leave that XCD's blocks undispatched, so the masks
// used here give every XCD CUs under either bit-to-XCD mapping (interleaved or contiguous);
// the probe shows which one the driver uses.
//
// build: hipcc --offload-arch=gfx950 -O2 -o tools/_cumask_probe tools/cumask_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

__global__ void k_where(unsigned* out, long long spin) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int words = cus / 32, G = 4 * cus;
    unsigned* d = nullptr;
    CHECK(hipMalloc(&d, 8 * G));
    std::vector<unsigned> h(2 * G);
    printf("device CUs %d\n", cus);
    for (int nranks : {1, 2, 4, 8}) {
        for (int rank = 0; rank < nranks; ++rank) {
            unsigned word = 0;
            std::vector<uint32_t> mask(words, 0u);
            if (nranks == 8) {   // word j: the four bits of residue (rank + j) mod 8
                for (int j = 0; j < words; ++j)
                    for (int q = 0; q < 4; ++q) mask[j] |= 1u << (8 * q + (rank + j) % 8);
                word = mask[0];
            } else {
                for (int k = 0; k < 4 / nranks; ++k) word |= 0xFFu << (8 * (rank + k * nranks));
                for (auto& v : mask) v = word;
            }
            hipStream_t s;
            CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask.data()));
            uint32_t back[32] = {};
            CHECK(hipExtStreamGetCUMask(s, 32, back));
            int nb = 0;
            for (int i = 0; i < words; ++i) nb += __builtin_popcount(back[i]);
            CHECK(hipMemsetAsync(d, 0xff, 8 * G, s));
            hipLaunchKernelGGL(k_where, dim3(G), dim3(256), 0, s, d, 2000LL);   // 2000 ticks of 100 MHz = 20 us
            CHECK(hipGetLastError());
            CHECK(hipStreamSynchronize(s));
            CHECK(hipMemcpy(h.data(), d, 8 * G, hipMemcpyDeviceToHost));
            std::set<unsigned> per[16];
            int bad = 0;
            for (int b = 0; b < G; ++b) {
                const unsigned x = h[2 * b], hw = h[2 * b + 1];
                if (x >= 16) { ++bad; continue; }
                per[x].insert(hw & 0xff00u);   // SE / SH / CU fields, without wave / SIMD
            }
            int xcc_of_b[8] = {};
            for (int b = 0; b < 8; ++b) xcc_of_b[b] = (int)h[2 * b];
            printf("partitions %d rank %d mask word[0] 0x%08x (stream reports %d CUs):", nranks, rank, word, nb);
            for (int x = 0; x < 8; ++x) printf(" xcd%d=%zu", x, per[x].size());
            printf("  blocks 0-7 on xcd");
            for (int b = 0; b < 8; ++b) printf(" %d", xcc_of_b[b]);
            printf("%s\n", bad ? "  (missing blocks!)" : "");
            CHECK(hipStreamDestroy(s));
        }
    }
    {   // an ordinary stream for comparison
        uint32_t back[32] = {};
        hipStream_t s;
        CHECK(hipStreamCreate(&s));
        CHECK(hipExtStreamGetCUMask(s, 32, back));
        int nb = 0;
        for (int i = 0; i < 32; ++i) nb += __builtin_popcount(back[i]);
        printf("ordinary stream reports %d CUs\n", nb);
        CHECK(hipStreamDestroy(s));
    }
    CHECK(hipFree(d));
    return 0;
}
