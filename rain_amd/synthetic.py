"""Seeded synthetic scenes of SURVEY §8(d) (no datasets or checkpoints exist offline).

Gaussians follow the reference's NeRF-synthetic random init (scene/dataset_readers.py:283-287,
scene/gaussian_model.py:114-137): means uniform in [-1.3, 1.3]^3, f_dc = RGB2SH(SH2RGB(U/255)),
scales = log(sqrt(mean squared 3-NN distance)), identity rotations, opacity logit(0.1).
The "bench" variant randomises what training would have moved: unit quaternions,
opacity U(0.05, 0.95), f_rest ~ N(0, 0.05^2).
"""
from __future__ import annotations

import math

import numpy as np
import torch

SH_C0 = 0.28209479177387814


def RGB2SH(rgb):
    return (rgb - 0.5) / SH_C0


def SH2RGB(sh):
    return sh * SH_C0 + 0.5


def inverse_sigmoid(x):
    return torch.log(x / (1 - x))


def knn3_mean_sq_dist_cpu(points: np.ndarray) -> np.ndarray:
    """Exact mean squared distance to the 3 nearest other points (what simple_knn's distCUDA2
    computes, simple_knn.cu:136-172) — CPU path used only when the HIP knn is unavailable."""
    from scipy.spatial import cKDTree

    pts = np.asarray(points, dtype=np.float32)
    tree = cKDTree(pts)
    d, _ = tree.query(pts, k=4)
    d = d[:, 1:].astype(np.float32)
    return (d * d).mean(axis=1).astype(np.float32)


def init_scales(points: torch.Tensor) -> torch.Tensor:
    """scales = log(sqrt(clamp_min(distCUDA2(points), 1e-7))) repeated x3 (gaussian_model.py:124-125)."""
    if points.is_cuda:  # the HIP simple-knn (include/rain_knn.h); raises if the library is missing
        from .simple_knn import distCUDA2

        d2 = distCUDA2(points)
    else:  # CPU-only test scenes
        d2 = torch.from_numpy(knn3_mean_sq_dist_cpu(points.detach().cpu().numpy()))
    d2 = torch.clamp_min(d2, 0.0000001)
    return torch.log(torch.sqrt(d2))[..., None].repeat(1, 3)


def random_gaussians(P: int, sh_degree: int = 3, seed: int = 0, bench: bool = True, device="cpu",
                     extent: float = 1.3):
    """Pre-activation Gaussian parameters in the GaussianModel layout (gaussian_model.py:131-136):
    xyz [P,3], f_dc [P,1,3], f_rest [P,(D+1)^2-1,3], scaling [P,3] (log), rotation [P,4] (raw),
    opacity [P,1] (logit)."""
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    xyz = torch.from_numpy((rng.random((P, 3)) * 2 * extent - extent).astype(np.float32))
    shs = rng.random((P, 3)) / 255.0
    f_dc = RGB2SH(torch.from_numpy(SH2RGB(shs)).float()).reshape(P, 1, 3)
    K = (sh_degree + 1) ** 2
    if bench:
        f_rest = torch.randn((P, K - 1, 3), generator=g) * 0.05
        q = torch.randn((P, 4), generator=g)
        rot = q / q.norm(dim=1, keepdim=True)
        opac = inverse_sigmoid(torch.rand((P, 1), generator=g) * 0.9 + 0.05)
    else:
        f_rest = torch.zeros((P, K - 1, 3))
        rot = torch.zeros((P, 4))
        rot[:, 0] = 1
        opac = inverse_sigmoid(0.1 * torch.ones((P, 1)))
    xyz_dev = xyz.to(device)
    scaling = init_scales(xyz_dev).float()
    return dict(xyz=xyz_dev, f_dc=f_dc.to(device), f_rest=f_rest.float().to(device), scaling=scaling.to(device),
                rotation=rot.float().to(device), opacity=opac.float().to(device))


def activated(params: dict, sh_degree: int | None = None):
    """GaussianModel getters (gaussian_model.py:85-105): exp scales, normalised rotations,
    sigmoid opacity, concatenated SH."""
    return dict(
        means3D=params["xyz"],
        scales=torch.exp(params["scaling"]),
        rotations=torch.nn.functional.normalize(params["rotation"]),
        opacities=torch.sigmoid(params["opacity"]),
        shs=torch.cat((params["f_dc"], params["f_rest"]), dim=1),
    )


def settings_for(cam, sh_degree: int, bg=None, low_pass: float = 0.3, scale_modifier: float = 1.0,
                 debug: bool = False):
    """GaussianRasterizationSettings exactly as render() builds them (gaussian_renderer/__init__.py:17-34)."""
    from .diff_gaussian_rasterization import GaussianRasterizationSettings

    dev = cam.world_view_transform.device
    if bg is None:
        bg = torch.zeros(3, dtype=torch.float32, device=dev)
    return GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg, scale_modifier=scale_modifier,
        viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, sh_degree=sh_degree,
        campos=cam.camera_center, prefiltered=False, debug=debug, low_pass=low_pass)
