// Device helpers shared by the single-RHS kernels (bpgl_kernels.h) and the panel
// kernels (bpgl_panel.h): block shape, fixed-order wave reductions, and the
// reference's scalar operators (cpu_calculation.py:5-11).
#pragma once
#include <hip/hip_runtime.h>

namespace bpgl {

constexpr int kThreads = 256;   // 4 waves of 64
constexpr int kWaves = 4;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
// max that propagates NaN (as numpy's max does)
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { double u = __shfl_xor(v, o); v = (u > v || u != u) ? u : v; }
    return v;
}

__device__ __forceinline__ double soft_thr(double t, double tau) {   // cpu_calculation.py:5-6
    const double mag = fabs(t) - tau;
    const double sg = t > 0.0 ? 1.0 : (t < 0.0 ? -1.0 : 0.0);
    return sg * (mag > 0.0 ? mag : 0.0);
}
__device__ __forceinline__ double proj(double v, double lo, double hi) {  // cpu_calculation.py:10-11
    const double a = v < hi ? v : hi;
    return a > lo ? a : lo;
}

}  // namespace bpgl
