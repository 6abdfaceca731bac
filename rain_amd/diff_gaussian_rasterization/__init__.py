"""Operator surface of the reference rasterizer over the MI355X ``_C``.

Interface only (the computation is in ``_C`` -> include/rain_raster.h -> rain_amd/csrc): the public
names, field order, argument meaning, error messages, debug-snapshot behaviour and autograd
contract are those of the reference's
submodules/diff_gaussian_rasterization/diff_gaussian_rasterization/__init__.py (Inria
Gaussian-Splatting licence, LICENSE.md there) — ``rasterize_gaussians`` (:10-31),
``_RasterizeGaussians`` (:33-146), ``GaussianRasterizationSettings`` (:148-161),
``GaussianRasterizer`` (:163-212) — so ``gaussian_renderer.render`` (gaussian_renderer/__init__.py:
9-79) runs against it unchanged.  The code is organised differently: argument packing and the
debug snapshot are shared helpers.
"""
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

_MSG_COLOR = 'Please provide excatly one of either SHs or precomputed colors!'  # reference text, typo included
_MSG_COV = 'Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!'


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    low_pass: float


def _host_copy(values):
    """CPU clones of every tensor argument (what the reference dumps when a debug call fails)."""
    return tuple(v.cpu().clone() if isinstance(v, torch.Tensor) else v for v in values)


def _invoke(fn, args, debug: bool, dump: str, message: str):
    """Call a ``_C`` entry point; in debug mode a failing call leaves ``dump`` (torch.save of the
    arguments on the CPU) in the working directory before the exception propagates
    (__init__.py:73-80,123-130)."""
    if not debug:
        return fn(*args)
    snapshot = _host_copy(args)
    try:
        return fn(*args)
    except Exception:
        torch.save(snapshot, dump)
        print(message)
        raise


def _forward_args(s: GaussianRasterizationSettings, means3D, colors, opacities, scales, rotations, cov3D, sh):
    """Argument tuple of _C.rasterize_gaussians (rasterize_points.cu:24-44)."""
    return (s.bg, means3D, colors, opacities, scales, rotations, s.scale_modifier, cov3D, s.viewmatrix,
            s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree, s.campos,
            s.prefiltered, s.debug, s.low_pass)


def _backward_args(s: GaussianRasterizationSettings, saved, num_rendered, grad_color):
    """Argument tuple of _C.rasterize_gaussians_backward (rasterize_points.cu:110-133)."""
    colors, means3D, scales, rotations, cov3D, radii, sh, geom, binning, img = saved
    return (s.bg, means3D, radii, colors, scales, rotations, s.scale_modifier, cov3D, s.viewmatrix, s.projmatrix,
            s.tanfovx, s.tanfovy, grad_color, sh, s.sh_degree, s.campos, geom, num_rendered, binning, img, s.debug,
            s.low_pass)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        s = raster_settings
        args = _forward_args(s, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh)
        num_rendered, color, radii, depth, geom, binning, img = _invoke(
            _C.rasterize_gaussians, args, s.debug, "snapshot_fw.dump",
            "\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom, binning,
                              img)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_out_color, grad_radii, grad_depth):
        # depth receives no gradient: grad_depth is accepted and dropped (__init__.py:91-120)
        s = ctx.raster_settings
        args = _backward_args(s, ctx.saved_tensors, ctx.num_rendered, grad_out_color)
        d_means2D, d_colors, d_opacities, d_means3D, d_cov3D, d_sh, d_scales, d_rotations = _invoke(
            _C.rasterize_gaussians_backward, args, s.debug, "snapshot_bw.dump",
            "\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
        # order of forward()'s inputs; raster_settings gets None
        return d_means3D, d_means2D, d_sh, d_colors, d_opacities, d_scales, d_rotations, d_cov3D, None


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def _absent_as_empty(*tensors):
    """None -> torch.Tensor([]) (a CPU numel-0 tensor, which _C reads as 'absent', __init__.py:189-199)."""
    return tuple(torch.Tensor([]) if t is None else t for t in tensors)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        s = self.raster_settings
        with torch.no_grad():
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        if (shs is None) == (colors_precomp is None):
            raise Exception(_MSG_COLOR)
        have_pair = scales is not None and rotations is not None
        have_any = scales is not None or rotations is not None
        if (cov3D_precomp is None and not have_pair) or (cov3D_precomp is not None and have_any):
            raise Exception(_MSG_COV)
        shs, colors_precomp, scales, rotations, cov3D_precomp = _absent_as_empty(shs, colors_precomp, scales,
                                                                                 rotations, cov3D_precomp)
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, self.raster_settings)

    @torch.no_grad()
    def render_depth_normal(self, means3D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None):
        """Forward only, with the auxiliary outputs of BASELINE configs[4]: returns (color [3,H,W],
        radii [P], depth [1,H,W], normal [3,H,W]).  The normal map (no reference counterpart) blends
        each Gaussian's view-space smallest-scale axis, facing the camera, like depth: sum of
        alpha*T*n, no background (include/rain_raster.h RR_FLAG_AUX_NORMAL).  Needs scales/rotations."""
        if (shs is None) == (colors_precomp is None):
            raise Exception(_MSG_COLOR)
        if scales is None or rotations is None:
            raise Exception('render_depth_normal needs the scale/rotation pair (normals come from the scale axes)')
        shs, colors_precomp, cov3D = _absent_as_empty(shs, colors_precomp, None)
        args = _forward_args(self.raster_settings, means3D, colors_precomp, opacities, scales, rotations, cov3D, shs)
        out = _C.rasterize_gaussians_aux(*args)
        return out[1], out[2], out[3], out[4]


__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
           "_C"]
