"""``submodules.diff_gaussian_rasterization.diff_gaussian_rasterization`` — the import path of
gaussian_renderer/__init__.py:5 — re-exporting the MI355X operator surface unchanged."""
from rain_amd.diff_gaussian_rasterization import (  # noqa: F401
    GaussianRasterizationSettings, GaussianRasterizer, _C, _RasterizeGaussians, rasterize_gaussians)
