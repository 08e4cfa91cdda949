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
