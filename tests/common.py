"""Shared scene construction and comparison helpers for the parity tests."""
from __future__ import annotations

import math

import numpy as np
import torch

from rain_amd import cameras, synthetic


def rel_l1(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.abs(b).sum()
    if den == 0:
        return float(np.abs(a).sum())
    return float(np.abs(a - b).sum() / den)


def make_scene(P=2000, W=128, H=96, sh_degree=3, active_degree=None, seed=0, bench=True, cam_index=0, n_cams=8,
               low_pass=0.3, bg=(0.0, 0.0, 0.0), precomp_colors=False, precomp_cov=False, scale_modifier=1.0,
               extent=1.3, radius=4.0, scale_mult=1.0):
    """CPU float32 inputs for one rasterizer call + the settings fields (numpy)."""
    if active_degree is None:
        active_degree = sh_degree
    params = synthetic.random_gaussians(P, sh_degree=sh_degree, seed=seed, bench=bench, extent=extent)
    if scale_mult != 1.0:
        params["scaling"] = params["scaling"] + math.log(scale_mult)
    act = synthetic.activated(params)
    cam = cameras.fibonacci_cameras(n_cams, W, H, radius=radius)[cam_index]
    inp = dict(means3D=act["means3D"].float().contiguous(), opacities=act["opacities"].float().contiguous())
    if precomp_colors:
        g = torch.Generator().manual_seed(seed + 1)
        inp["colors_precomp"] = torch.rand((P, 3), generator=g)
    else:
        inp["shs"] = act["shs"].float().contiguous()
    if precomp_cov:
        L = build_scaling_rotation(act["scales"] * scale_modifier, act["rotations"])
        S = L @ L.transpose(1, 2)
        inp["cov3D_precomp"] = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]],
                                           dim=1).contiguous()
    else:
        inp["scales"] = act["scales"].float().contiguous()
        inp["rotations"] = act["rotations"].float().contiguous()
    st = dict(image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
              bg=torch.tensor(bg, dtype=torch.float32), scale_modifier=float(scale_modifier),
              viewmatrix=cam.world_view_transform.float().contiguous(),
              projmatrix=cam.full_proj_transform.float().contiguous(), sh_degree=active_degree,
              campos=cam.camera_center.float().contiguous(), prefiltered=False, debug=False, low_pass=float(low_pass))
    return inp, st


def build_scaling_rotation(s, r):
    """utils/general_utils.py:75-84 (restated on CPU; the reference hard-codes device='cuda')."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), dtype=s.dtype)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    L = torch.zeros((s.shape[0], 3, 3), dtype=s.dtype)
    L[:, 0, 0] = s[:, 0]
    L[:, 1, 1] = s[:, 1]
    L[:, 2, 2] = s[:, 2]
    return R @ L


def oracle_settings(O, st):
    return O.Settings(**{k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in st.items()})


def oracle_run(O, inp, st, dL_dpix=None, nthreads=0):
    s = oracle_settings(O, st)
    n = {k: v.numpy() for k, v in inp.items()}
    nr, color, radii, depth, state = O.forward(s, n["means3D"], n["opacities"], shs=n.get("shs"),
                                               colors_precomp=n.get("colors_precomp"), scales=n.get("scales"),
                                               rotations=n.get("rotations"), cov3D_precomp=n.get("cov3D_precomp"),
                                               nthreads=nthreads)
    out = dict(num_rendered=nr, color=color, radii=radii, depth=depth, state=state)
    if dL_dpix is not None:
        g = O.backward(state, s, n["means3D"], radii, dL_dpix, shs=n.get("shs"), colors_precomp=n.get("colors_precomp"),
                       scales=n.get("scales"), rotations=n.get("rotations"), cov3D_precomp=n.get("cov3D_precomp"),
                       nthreads=nthreads)
        out["grads"] = dict(zip(GRAD_NAMES + ["dL_dconic"], g))
    return out


GRAD_NAMES = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations"]


def gpu_run(inp, st, device, dL_dpix=None):
    """Call the MI355X _C directly (the reference's pybind-level entry points)."""
    from rain_amd.diff_gaussian_rasterization import _C

    d = {k: v.to(device) for k, v in inp.items()}
    e = torch.Tensor([])
    s = {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in st.items()}
    sh = d.get("shs", e)
    args = (s["bg"], d["means3D"], d.get("colors_precomp", e), d["opacities"], d.get("scales", e),
            d.get("rotations", e), s["scale_modifier"], d.get("cov3D_precomp", e), s["viewmatrix"], s["projmatrix"],
            s["tanfovx"], s["tanfovy"], s["image_height"], s["image_width"], sh, s["sh_degree"], s["campos"],
            s["prefiltered"], s["debug"], s["low_pass"])
    nr, color, radii, depth, geom, binning, img = _C.rasterize_gaussians(*args)
    out = dict(num_rendered=nr, color=color.cpu().numpy(), radii=radii.cpu().numpy(), depth=depth.cpu().numpy(),
               buffers=(geom, binning, img))
    if dL_dpix is not None:
        g = _C.rasterize_gaussians_backward(
            s["bg"], d["means3D"], radii, d.get("colors_precomp", e), d.get("scales", e), d.get("rotations", e),
            s["scale_modifier"], d.get("cov3D_precomp", e), s["viewmatrix"], s["projmatrix"], s["tanfovx"],
            s["tanfovy"], torch.from_numpy(dL_dpix).to(device), sh, s["sh_degree"], s["campos"], geom, nr, binning,
            img, s["debug"], s["low_pass"])
        torch.cuda.synchronize()
        out["grads"] = {k: v.cpu().numpy() for k, v in zip(GRAD_NAMES, g)}
    return out
