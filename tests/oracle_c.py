"""`_C`-shaped wrapper of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Same three functions and tuples as the reference's pybind module (rasterize_points.cu:24-212),
computed by oracle/raster_oracle.c on CPU tensors.  CPU tests monkeypatch it in place of the MI355X
``_C`` to exercise the autograd plumbing, the render() contract and the multi-process training
step on machines without a GPU (BASELINE.json configs[0]: the reference's CPU-runnable case).
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from oracle import oracle as O

_states = {}
_ids = itertools.count(1)


def _np(t):
    if t is None or t.numel() == 0:
        return None
    return t.detach().cpu().float().contiguous().numpy()


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug, low_pass):
    out = _forward(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                   viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                   prefiltered, debug, low_pass, False)
    return out[:4] + out[5:]


def rasterize_gaussians_aux(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                            viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                            prefiltered, debug, low_pass):
    return _forward(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                    viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                    prefiltered, debug, low_pass, True)


def _forward(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
             viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
             prefiltered, debug, low_pass, normal):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    s = O.Settings(image_height=int(image_height), image_width=int(image_width), tanfovx=float(tan_fovx),
                   tanfovy=float(tan_fovy), bg=_np(background), scale_modifier=float(scale_modifier),
                   viewmatrix=_np(viewmatrix), projmatrix=_np(projmatrix), sh_degree=int(degree), campos=_np(campos),
                   prefiltered=bool(prefiltered), low_pass=float(low_pass))
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    if P == 0:
        z = torch.zeros((0,), dtype=torch.uint8)
        return (0, torch.zeros((3, H, W)), torch.zeros((0,), dtype=torch.int32), torch.zeros((1, H, W)),
                torch.zeros((3, H, W)) if normal else None, z, z, z)
    res = O.forward(s, _np(means3D), _np(opacity), shs=_np(sh), colors_precomp=_np(colors), scales=_np(scales),
                    rotations=_np(rotations), cov3D_precomp=_np(cov3D_precomp), nthreads=1, normal=normal)
    nr, color, radii, depth, st = res[:5]
    nmap = torch.from_numpy(res[5]) if normal else None
    key = next(_ids)
    _states[key] = (st, s)
    geom = torch.tensor([key], dtype=torch.int64)
    empty = torch.zeros((0,), dtype=torch.uint8)
    return nr, torch.from_numpy(color), torch.from_numpy(radii), torch.from_numpy(depth), nmap, geom, empty, empty


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree,
                                 campos, geomBuffer, R, binningBuffer, imageBuffer, debug, low_pass):
    P = means3D.size(0)
    M = sh.size(1) if sh.size(0) != 0 else 0
    if P == 0:
        z = lambda *sh_: torch.zeros(sh_)  # noqa: E731
        return z(0, 3), z(0, 3), z(0, 1), z(0, 3), z(0, 6), z(0, M, 3), z(0, 3), z(0, 4)
    st, s = _states.pop(int(geomBuffer[0]))
    g = O.backward(st, s, _np(means3D), radii.cpu().numpy(), _np(dL_dout_color), shs=_np(sh),
                   colors_precomp=_np(colors), scales=_np(scales), rotations=_np(rotations),
                   cov3D_precomp=_np(cov3D_precomp), nthreads=1)
    return tuple(torch.from_numpy(np.ascontiguousarray(x)) for x in g[:8])


def mark_visible(means3D, viewmatrix, projmatrix):
    return torch.from_numpy(O.mark_visible(_np(means3D), _np(viewmatrix), _np(projmatrix)))
