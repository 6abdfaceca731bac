"""Import shim: ``from diff_gaussian_rasterization import GaussianRasterizer, ...`` (the name the
reference's environment.yml installs) resolves to the MI355X implementation in rain_amd."""
from rain_amd.diff_gaussian_rasterization import (  # noqa: F401
    GaussianRasterizationSettings, GaussianRasterizer, _C, _RasterizeGaussians, rasterize_gaussians)
