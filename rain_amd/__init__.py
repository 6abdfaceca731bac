"""rain_amd — MI355X-native (gfx950/HIP) differentiable Gaussian-splat rasterizer with the
operator surface of sharonal10/rain's diff_gaussian_rasterization, plus the training-step
harness (GaussianModel counterpart, view-sharded multi-GPU step) around it.

Product path: rain_amd.diff_gaussian_rasterization -> rain_amd._native (ctypes) ->
rain_amd/lib/librain_raster.so (C ABI: include/rain_raster.h).
"""
__version__ = "0.1.0"
