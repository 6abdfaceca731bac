"""render() counterpart (gaussian_renderer/__init__.py:9-79).

Identical contract: builds GaussianRasterizationSettings from the camera, creates the
``means2D`` gradient sink (its .grad receives the NDC-space screen gradient), picks the SH /
precomputed-colour and scale-rotation / precomputed-covariance inputs from the pipeline flags,
and returns {render, viewspace_points, visibility_filter, radii, depth}.  When the model's getters
are GaussianModel's own and the pipeline flags are the defaults, the rasterizer takes the raw
parameters and applies the getters in-kernel (rain_amd.fused.RasterizeRawParams): the same
outputs and leaf gradients without the getters' elementwise autograd chain and the get_features
concatenation (RAIN_RENDER_RAW=0 disables it).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch

from .diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
from .sh_utils import eval_sh


# render()'s raw-parameter fast path (rain_amd.fused.RasterizeRawParams): RAIN_RENDER_RAW=0 keeps every
# call on the getters + GaussianRasterizer route.
RAW_RENDER = os.environ.get("RAIN_RENDER_RAW", "1") != "0"


def _raw_path_ok(pc, pipe, override_color) -> bool:
    """The getters of `pc` are GaussianModel's own (exp / normalize / sigmoid / concatenation,
    gaussian_model.py:85-105) on contiguous fp32 device tensors, and the pipeline asks for the
    default SH and scale/rotation inputs: the rasterizer may then take the raw parameters and
    apply the getters in-kernel (identical arithmetic, one autograd node)."""
    from .gaussian_model import GaussianModel

    if not RAW_RENDER or override_color is not None or pipe.convert_SHs_python or pipe.compute_cov3D_python \
            or pipe.debug or not isinstance(pc, GaussianModel):
        return False
    cls = type(pc)
    if any(getattr(cls, n) is not getattr(GaussianModel, n)
           for n in ("get_xyz", "get_features", "get_scaling", "get_rotation", "get_opacity")):
        return False
    if pc.scaling_activation is not torch.exp or pc.opacity_activation is not torch.sigmoid \
            or pc.rotation_activation is not torch.nn.functional.normalize:
        return False
    ts = (pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation)
    return all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ts) \
        and pc._features_rest.shape[1] + 1 <= 16


_ZERO_SINKS: dict = {}  # device -> [P, 3] fp32 zeros (render()'s means2D sink on the raw path)


def _zero_sink(xyz: torch.Tensor) -> torch.Tensor:
    z = _ZERO_SINKS.get(xyz.device)
    if z is None or z.shape != xyz.shape or z.dtype != xyz.dtype:
        z = _ZERO_SINKS[xyz.device] = torch.zeros_like(xyz, memory_format=torch.contiguous_format)
    return z


@dataclass
class PipelineParams:
    """arguments/__init__.py:54-59."""
    convert_SHs_python: bool = False
    compute_cov3D_python: bool = False
    debug: bool = False


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, scaling_modifier=1.0, override_color=None,
           low_pass=0.3):
    xyz = pc.get_xyz
    raw = _raw_path_ok(pc, pipe, override_color)
    if raw:
        # the means2D gradient sink as a fresh leaf over a cached zero buffer (the rasterizer never
        # reads its values): autograd hands it the backward's own gradient tensor, where the
        # reference's `zeros_like + 0` with retain_grad() costs a fill, an add and a gradient clone
        screenspace_points = _zero_sink(xyz).detach().requires_grad_()
    else:
        screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device) + 0
        try:
            screenspace_points.retain_grad()
        except Exception:
            pass

    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree, campos=viewpoint_camera.camera_center, prefiltered=False, debug=pipe.debug,
        low_pass=low_pass)
    if raw:
        from .fused import RasterizeRawParams

        rendered_image, radii, depth = RasterizeRawParams.apply(
            pc._xyz, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation, screenspace_points,
            pc.active_sh_degree, raster_settings.image_width, raster_settings.image_height, tanfovx, tanfovy,
            raster_settings.viewmatrix, raster_settings.projmatrix, raster_settings.campos, bg_color, low_pass,
            scaling_modifier)
        return {"render": rendered_image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
                "radii": radii, "depth": depth}
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)

    means3D = xyz
    means2D = screenspace_points
    opacity = pc.get_opacity
    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales = pc.get_scaling
        rotations = pc.get_rotation
    shs = colors_precomp = None
    if override_color is None:
        if pipe.convert_SHs_python:
            shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = (pc.get_xyz - viewpoint_camera.camera_center.repeat(pc.get_features.shape[0], 1))
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            sh2rgb = eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized)
            colors_precomp = torch.clamp_min(sh2rgb + 0.5, 0.0)
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color

    rendered_image, radii, depth = rasterizer(means3D=means3D, means2D=means2D, shs=shs,
                                              colors_precomp=colors_precomp, opacities=opacity, scales=scales,
                                              rotations=rotations, cov3D_precomp=cov3D_precomp)
    return {"render": rendered_image, "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
            "radii": radii, "depth": depth}


@torch.no_grad()
def render_depth_normal(viewpoint_camera, pc, bg_color: torch.Tensor, scaling_modifier=1.0, low_pass=0.3):
    """Evaluation-time render with the auxiliary outputs of BASELINE configs[4] (depth + normal):
    {render [3,H,W], depth [1,H,W], normal [3,H,W], radii, visibility_filter}.  No autograd graph."""
    settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5), bg=bg_color,
        scale_modifier=scaling_modifier, viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform, sh_degree=pc.active_sh_degree,
        campos=viewpoint_camera.camera_center, prefiltered=False, debug=False, low_pass=low_pass)
    color, radii, depth, normal = GaussianRasterizer(settings).render_depth_normal(
        pc.get_xyz, pc.get_opacity, shs=pc.get_features, scales=pc.get_scaling, rotations=pc.get_rotation)
    return {"render": color, "depth": depth, "normal": normal, "radii": radii, "visibility_filter": radii > 0}
