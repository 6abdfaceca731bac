"""Differentiable float64 torch restatement of the rasterizer forward — TEST INFRASTRUCTURE ONLY.

Used to validate the oracle's hand-written backward (raster_oracle.c, restating backward.cu)
by autograd: given the oracle forward's discrete decisions (which Gaussians are visible, and per
pixel the ordered list of Gaussians actually blended), the image is a smooth function of the
inputs, and autograd of it must equal the reference backward up to the documented deviations,
which this restatement reproduces on purpose:

 1. no gradient mask for the 0.99 alpha clamp (backward.cu:528: dL/dG = o·dL/dalpha always);
 2. the EWA clamp of t.x/t.z to ±1.3·tanfov: the clamped coordinate is a constant for the
    gradient (backward.cu:165-166,252-254);
 3. depth receives no gradient (only the colour image is differentiated);
 4. dL/dmeans2D is the gradient w.r.t. the NDC position (backward.cu:450-451,535-536);
 5. dL/dscales is the gradient w.r.t. the MODIFIED scale scale_modifier·s — the chain-rule factor
    scale_modifier is missing in backward.cu:285-315 (it only matters when scale_modifier != 1);
 and differs by design in the 1e-7 regulariser of backward.cu:193 (denom² + 1e-7), which this
 exact restatement does not have (relative effect <= 1e-7/det², ~1e-5 for the smallest splats).

Follows forward.cu:107-141 (cov3D), :63-102 (cov2D), :144-246 (preprocess), :251-369 (blend),
auxiliary.h:30-33 (ndc2Pix), utils/sh_utils.py (SH).
"""
from __future__ import annotations

import numpy as np
import torch

C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
      1.445305721320277, -0.5900435899266435]


def _sh(deg, sh, d):
    """sh: [n, M, 3]; d: [n, 3] unit."""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = C0 * sh[:, 0]
    if deg > 0:
        r = r - C1 * y * sh[:, 1] + C1 * z * sh[:, 2] - C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            r = (r + C2[0] * xy * sh[:, 4] + C2[1] * yz * sh[:, 5] + C2[2] * (2 * zz - xx - yy) * sh[:, 6] +
                 C2[3] * xz * sh[:, 7] + C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                r = (r + C3[0] * y * (3 * xx - yy) * sh[:, 9] + C3[1] * xy * z * sh[:, 10] +
                     C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12] +
                     C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + C3[5] * z * (xx - yy) * sh[:, 14] +
                     C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r + 0.5


def _rot(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], 1)
    return R


def render_autograd(st, inputs: dict, blend_lists, visible: np.ndarray, dL_dpix: np.ndarray):
    """Returns a dict of float64 gradients (same names as the reference backward's outputs)."""
    dt = torch.float64
    H, W = int(st["image_height"]), int(st["image_width"])
    view = torch.as_tensor(np.asarray(st["viewmatrix"]), dtype=dt).reshape(4, 4)  # column-major memory
    proj = torch.as_tensor(np.asarray(st["projmatrix"]), dtype=dt).reshape(4, 4)
    campos = torch.as_tensor(np.asarray(st["campos"]), dtype=dt)
    bg = torch.as_tensor(np.asarray(st["bg"]), dtype=dt)
    tanfovx, tanfovy = float(st["tanfovx"]), float(st["tanfovy"])
    fx, fy = W / (2.0 * tanfovx), H / (2.0 * tanfovy)
    mod, low_pass, D = float(st["scale_modifier"]), float(st["low_pass"]), int(st["sh_degree"])

    leaf = {k: torch.as_tensor(np.asarray(v), dtype=dt).clone().requires_grad_(True) for k, v in inputs.items()}
    m = leaf["means3D"]
    P = m.shape[0]
    ones = torch.ones((P, 1), dtype=dt)
    mh = torch.cat([m, ones], 1)
    # memory m[0..15] column-major: x' = m0 x + m4 y + m8 z + m12 -> row-vector form mh @ M
    p_hom = mh @ proj
    p_w = 1.0 / (p_hom[:, 3:4] + 1e-7)
    ndc = (p_hom[:, :2] * p_w)
    ndc.retain_grad()
    pix = torch.stack([((ndc[:, 0] + 1.0) * W - 1.0) * 0.5, ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5], 1)
    t = (mh @ view)[:, :3]

    if "cov3D_precomp" in leaf:
        cov6 = leaf["cov3D_precomp"]
    else:
        R = _rot(leaf["rotations"])
        sc = leaf["scales"]
        s = sc + (mod - 1.0) * sc.detach()  # value mod*s, gradient w.r.t. mod*s (deviation 5)
        Mm = s[:, :, None] * R.transpose(1, 2)  # M[i][j] = s_i R[j][i]
        Sg = Mm.transpose(1, 2) @ Mm
        cov6 = torch.stack([Sg[:, 0, 0], Sg[:, 0, 1], Sg[:, 0, 2], Sg[:, 1, 1], Sg[:, 1, 2], Sg[:, 2, 2]], 1)
        cov6.retain_grad()
    V = torch.stack([torch.stack([cov6[:, 0], cov6[:, 1], cov6[:, 2]], -1),
                     torch.stack([cov6[:, 1], cov6[:, 3], cov6[:, 4]], -1),
                     torch.stack([cov6[:, 2], cov6[:, 4], cov6[:, 5]], -1)], 1)
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    tz = t[:, 2]
    txtz, tytz = t[:, 0] / tz, t[:, 1] / tz
    cx = (txtz < -limx) | (txtz > limx)
    cy = (tytz < -limy) | (tytz > limy)
    tx = torch.where(cx, (txtz.clamp(-limx, limx) * tz).detach(), t[:, 0])
    ty = torch.where(cy, (tytz.clamp(-limy, limy) * tz).detach(), t[:, 1])
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -(fx * tx) / (tz * tz)], -1),
                     torch.stack([zero, fy / tz, -(fy * ty) / (tz * tz)], -1)], 1)  # [P,2,3]
    Wr = view[:3, :3].T  # R_w2c[i][j] = view_mem[4j+i]
    A = J @ Wr
    cov2 = A @ V @ A.transpose(1, 2)
    a = cov2[:, 0, 0] + low_pass
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + low_pass
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], 1)
    opac = leaf["opacities"].reshape(-1)

    if "colors_precomp" in leaf:
        colors = leaf["colors_precomp"]
    else:
        d = m - campos
        d = d / d.norm(dim=1, keepdim=True)
        colors = torch.clamp_min(_sh(D, leaf["shs"], d), 0.0)
        colors.retain_grad()

    vis = torch.as_tensor(visible)
    img = bg[:, None, None].repeat(1, H, W).clone()
    out = torch.zeros((3, H * W), dtype=dt)
    Kmax = max((len(l) for l in blend_lists), default=0)
    if Kmax > 0:
        ids = torch.full((H * W, Kmax), -1, dtype=torch.long)
        for i, l in enumerate(blend_lists):
            if len(l):
                ids[i, :len(l)] = torch.as_tensor(l.astype(np.int64))
        valid = ids >= 0
        g = ids.clamp(min=0)
        pyx = torch.stack(torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt), indexing="ij"),
                          -1).reshape(-1, 1, 2)
        dxy = pix[g] - pyx.flip(-1)  # (x, y)
        co = conic[g]
        power = -0.5 * (co[..., 0] * dxy[..., 0] ** 2 + co[..., 2] * dxy[..., 1] ** 2) - co[..., 1] * dxy[..., 0] * dxy[..., 1]
        oG = opac[g] * torch.exp(power)
        alpha = oG - (oG - 0.99).clamp(min=0).detach()  # value min(0.99, oG), gradient of oG (deviation 1)
        alpha = torch.where(valid, alpha, torch.zeros_like(alpha))
        one_m = 1.0 - alpha
        Tpre = torch.cumprod(torch.cat([torch.ones((H * W, 1), dtype=dt), one_m[:, :-1]], 1), 1)
        wgt = alpha * Tpre
        out = (wgt[..., None] * colors[g]).sum(1).T  # [3, HW]
        Tfin = torch.prod(one_m, 1)
        img = out.reshape(3, H, W) + Tfin.reshape(1, H, W) * bg[:, None, None]
    L = (img * torch.as_tensor(dL_dpix, dtype=dt)).sum()
    L.backward()

    def g_(x, shape=None):
        return np.zeros(shape) if x.grad is None else x.grad.detach().numpy()

    res = dict(
        dL_dmeans3D=g_(m), dL_dopacity=g_(leaf["opacities"]),
        dL_dmeans2D=np.concatenate([g_(ndc, (P, 2)), np.zeros((P, 1))], 1),
    )
    if "shs" in leaf:
        res["dL_dsh"] = g_(leaf["shs"])
        res["dL_dcolors"] = g_(colors, (P, 3))
    else:
        res["dL_dcolors"] = g_(leaf["colors_precomp"])
    if "scales" in leaf:
        res["dL_dscales"] = g_(leaf["scales"])
        res["dL_drotations"] = g_(leaf["rotations"])
        res["dL_dcov3D"] = g_(cov6, (P, 6))
    else:
        res["dL_dcov3D"] = g_(leaf["cov3D_precomp"])
    res["image"] = img.detach().numpy()
    return res
