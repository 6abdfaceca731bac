"""Training loss (utils/loss_utils.py:6-53): loss = (1-λ)·L1 + λ·(1-SSIM), 11x11 Gaussian window σ=1.5.

The reference's own ``ssim`` (depthwise 11x11 conv2d) is restated as test infrastructure in
oracle/loss_ref.py.  ``fused_l1_ssim_loss`` is what the train step uses: the whole loss and its gradient in two HIP
kernels (rain_amd/csrc/loss.hip) — the window is an outer product of the 1-D Gaussian
(loss_utils.py:15-19), so it is applied as two 11-tap passes over an LDS tile.  ``ssim_separable``
is the same factorisation in torch (a CPU-testable statement of what the kernel computes).  All are
pinned to the reference's ssim values by tests/golden/loss.npz.
"""
from __future__ import annotations

import ctypes
from functools import lru_cache
from math import exp

import torch
import torch.nn.functional as F


def window_1d(window_size: int = 11, sigma: float = 1.5) -> torch.Tensor:
    """The loss's 1-D Gaussian window (utils/loss_utils.py:15-17): exp(-(x - size//2)² / 2σ²)
    evaluated in double, stored as fp32 and normalised by its fp32 sum — the same fp32 weights the
    reference convolves with (pinned by tests/golden/loss.npz)."""
    c = window_size // 2
    w = torch.tensor([exp(-((i - c) ** 2) / (2.0 * sigma * sigma)) for i in range(window_size)],
                     dtype=torch.float32)
    return w / w.sum()


_WINDOW = None


def _window_host():
    """The reference's 1-D window gaussian(11, 1.5) (fp32 exp values normalised in fp32)."""
    global _WINDOW
    if _WINDOW is None:
        g = window_1d(11, 1.5)
        _WINDOW = (ctypes.c_float * 11)(*[float(v) for v in g])
    return _WINDOW


_ONES = {}


def _ones(device):
    """A cached device scalar 1.0 (the default grad_loss; read-only for the kernels)."""
    t = _ONES.get(device)
    if t is None:
        t = _ONES[device] = torch.ones((1,), dtype=torch.float32, device=device)
    return t


def l1_ssim_forward(img, gt, lambda_dssim):
    """Fused forward (include/rain_loss.h).  Returns (loss scalar, parts [3], workspace); the
    workspace carries the per-pixel SSIM derivative maps the backward needs."""
    from . import _native as N

    L = N.loss_lib()
    img = img.contiguous()
    gt = gt.contiguous()
    C, H, W = img.shape[-3:]
    ws = torch.empty((L.rl_workspace_bytes(C, H, W),), dtype=torch.uint8, device=img.device)
    loss = torch.empty((), dtype=torch.float32, device=img.device)
    parts = torch.empty((3,), dtype=torch.float32, device=img.device)
    rc = L.rl_l1_ssim_forward(img.data_ptr(), gt.data_ptr(), C, H, W, float(lambda_dssim), _window_host(),
                              ws.data_ptr(), ws.numel(), loss.data_ptr(), parts.data_ptr(), N.stream_of(img))
    if rc:
        raise RuntimeError(L.rl_last_error().decode())
    return loss, parts, ws


def l1_ssim_backward(img, gt, lambda_dssim, ws, grad_loss=None):
    """dLoss/dimg scaled by grad_loss (a device scalar; None = 1)."""
    from . import _native as N

    L = N.loss_lib()
    img = img.contiguous()
    gt = gt.contiguous()
    C, H, W = img.shape[-3:]
    dimg = torch.empty_like(img)
    if grad_loss is None:
        grad_loss = _ones(img.device)
    g = grad_loss.reshape(1).contiguous().float()
    rc = L.rl_l1_ssim_backward(img.data_ptr(), gt.data_ptr(), C, H, W, float(lambda_dssim), _window_host(),
                               ws.data_ptr(), g.data_ptr(), dimg.data_ptr(), N.stream_of(img))
    if rc:
        raise RuntimeError(L.rl_last_error().decode())
    return dimg


def l1_ssim_forward_backward(img, gt, lambda_dssim, grad_loss=None):
    """Forward and backward at once (the training step's form): (loss, parts, dimg), bitwise
    l1_ssim_forward's loss / parts and l1_ssim_backward's dimg, in two launches instead of three."""
    from . import _native as N

    L = N.loss_lib()
    img = img.contiguous()
    gt = gt.contiguous()
    C, H, W = img.shape[-3:]
    ws = torch.empty((L.rl_workspace_bytes(C, H, W),), dtype=torch.uint8, device=img.device)
    loss = torch.empty((), dtype=torch.float32, device=img.device)
    parts = torch.empty((3,), dtype=torch.float32, device=img.device)
    dimg = torch.empty_like(img)
    if grad_loss is None:
        grad_loss = _ones(img.device)
    g = grad_loss.reshape(1).contiguous().float()
    rc = L.rl_l1_ssim_forward_backward(img.data_ptr(), gt.data_ptr(), C, H, W, float(lambda_dssim), _window_host(),
                                       ws.data_ptr(), ws.numel(), loss.data_ptr(), parts.data_ptr(), g.data_ptr(),
                                       dimg.data_ptr(), N.stream_of(img))
    if rc:
        raise RuntimeError(L.rl_last_error().decode())
    return loss, parts, dimg


class _FusedL1SSIM(torch.autograd.Function):
    """(1-λ)·L1 + λ·(1-SSIM) in two HIP kernels (rain_amd/csrc/loss.hip, include/rain_loss.h)."""

    @staticmethod
    def forward(ctx, img, gt, lambda_dssim):
        img = img.contiguous()
        gt = gt.contiguous()
        loss, parts, ws = l1_ssim_forward(img, gt, lambda_dssim)
        ctx.save_for_backward(img, gt, ws)
        ctx.lam = float(lambda_dssim)
        ctx.mark_non_differentiable(parts)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for `parts` (a fill per step)
        return loss, parts

    @staticmethod
    def backward(ctx, grad_loss, _grad_parts):
        if grad_loss is None:  # the loss itself not in the differentiated graph: zero gradient
            return None, None, None
        img, gt, ws = ctx.saved_tensors
        return l1_ssim_backward(img, gt, ctx.lam, ws, grad_loss), None, None


def fused_l1_ssim_loss(img, gt, lambda_dssim=0.2):
    """Returns (loss, parts) where parts = [loss, L1, SSIM] (device, no sync)."""
    if img.dim() != 3 or img.device.type != "cuda":
        raise RuntimeError("fused_l1_ssim_loss expects a [C,H,W] tensor on a HIP device")
    return _FusedL1SSIM.apply(img, gt, lambda_dssim)


@lru_cache(maxsize=8)
def _sep_windows(window_size, channels, device, dtype):
    g = window_1d(window_size, 1.5).to(device=device, dtype=dtype)
    return (g.view(1, 1, 1, window_size).expand(channels, 1, 1, window_size).contiguous(),
            g.view(1, 1, window_size, 1).expand(channels, 1, window_size, 1).contiguous())


def ssim_separable(img1, img2, window_size=11):
    """Mean SSIM with the separable form of the same window; all five filtered maps in one batch."""
    C = img1.size(-3)
    x = torch.stack([img1, img2, img1 * img1, img2 * img2, img1 * img2], 0).reshape(1, 5 * C, *img1.shape[-2:])
    wh, wv = _sep_windows(window_size, 5 * C, img1.device, img1.dtype)
    p = window_size // 2
    y = F.conv2d(F.conv2d(x, wh, padding=(0, p), groups=5 * C), wv, padding=(p, 0), groups=5 * C)
    mu1, mu2, e11, e22, e12 = y.view(5, C, *img1.shape[-2:]).unbind(0)
    mu1_sq, mu2_sq, mu1_mu2 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    sigma1_sq, sigma2_sq, sigma12 = e11 - mu1_sq, e22 - mu2_sq, e12 - mu1_mu2
    C1 = 0.01 ** 2
    C2 = 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    return ssim_map.mean()
