// Host-side helpers shared by the two C-ABI translation units of libbpgl.so
// (bpgl.hip: single right-hand side; bpgl_panel_abi.hip: k right-hand sides).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/bpgl.h"

namespace bpgl_host {
// thread-local message behind bpgl_last_error(); returns `code`
int fail(int code, const char* fmt, ...);

inline int64_t up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// bump allocator over the caller's scratch buffer (256-byte aligned pieces)
struct Carve {
    int64_t off = 0;
    int64_t take(int64_t bytes) {
        int64_t o = off;
        off = up(off + bytes, 256);
        return o;
    }
};

constexpr int kGraphIters = 8;   // iterations captured per replayed hipGraph (panel; RCCL contexts' cap)
// single-RHS solver: hipGraphs of 1, 2, 4, ..., kGraphMaxIters iterations, so a run of n iterations
// costs about log2(n) replays instead of n / 8
constexpr int kGraphLevels = 7;
constexpr int kGraphMaxIters = 1 << (kGraphLevels - 1);

constexpr int kMaskWords = 32;   // CU mask words queried (1024 CUs)

inline int popcount_mask(const uint32_t* mask, int words, int cus) {
    int n = 0;
    for (int i = 0; i < words; ++i) {
        uint32_t v = mask[i];
        if (32 * i >= cus) break;
        if (32 * (i + 1) > cus) v &= (1u << (cus - 32 * i)) - 1u;
        n += __builtin_popcount(v);
    }
    return n;
}

// CUs a stream may use (its CU mask, hipExtStreamGetCUMask), 0 if unknown
inline int stream_cus(hipStream_t s, int dev_cus) {
    uint32_t mask[kMaskWords] = {};
    if (hipExtStreamGetCUMask(s, kMaskWords, mask) != hipSuccess) {
        (void)hipGetLastError();   // the query's own error only: not sticky, later launch checks read it
        return 0;
    }
    return popcount_mask(mask, kMaskWords, dev_cus);
}

// CUs a kernel launched on stream s can occupy: the stream's CU mask when it has one, else the device's
inline int usable_cus(hipStream_t s, int device) {
    int dev = 0;
    if (hipDeviceGetAttribute(&dev, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || dev <= 0) {
        (void)hipGetLastError();
        return 0;
    }
    const int n = stream_cus(s, dev);
    return (n > 0 && n < dev) ? n : dev;
}
}  // namespace bpgl_host

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return bpgl_host::fail(BPGL_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

#define LAUNCH_CHECK(what)                                                                   \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ != hipSuccess) return bpgl_host::fail(BPGL_E_HIP, "launch %s: %s", what, hipGetErrorString(e_)); \
    } while (0)
