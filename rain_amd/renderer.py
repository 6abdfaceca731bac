"""render() counterpart (gaussian_renderer/__init__.py:9-79).

Identical contract: builds GaussianRasterizationSettings from the camera, creates the
``means2D`` gradient sink (its .grad receives the NDC-space screen gradient), picks the SH /
precomputed-colour and scale-rotation / precomputed-covariance inputs from the pipeline flags,
and returns {render, viewspace_points, visibility_filter, radii, depth}.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
from .sh_utils import eval_sh


@dataclass
class PipelineParams:
    """arguments/__init__.py:54-59."""
    convert_SHs_python: bool = False
    compute_cov3D_python: bool = False
    debug: bool = False


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, scaling_modifier=1.0, override_color=None,
           low_pass=0.3):
    xyz = pc.get_xyz
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
