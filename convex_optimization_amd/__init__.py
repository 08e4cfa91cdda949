"""convex_optimization_amd -- MI355X-native block best-response lasso hot path.

Drop-in modules for the reference's call surface:
  ``cpu_calculation``  host helpers (numpy), same names and shapes
  ``gpu_calculation``  ``GPU_Calculation`` over hand-written gfx950 HIP kernels
                       (``_lib/libbpgl.so``, C ABI in ``include/bpgl.h``)
  ``lasso``            drivers: ClassLasso / ClassLassoR / ClassLassoDevice
  ``parameters``       problem instances (reference recipe + in-HBM generator)
  ``distributed``      column-sharded multi-GPU path (RCCL all-reduce)
"""
__version__ = "0.1.0"

__all__ = ["cpu_calculation", "gpu_calculation", "lasso", "parameters", "distributed"]
