"""CPU/torch restatement of the reference training loss — TEST INFRASTRUCTURE ONLY (the checker the
fused HIP loss kernels are compared with; never imported by the product package ``rain_amd``).

Follows utils/loss_utils.py: ``l1_loss`` (:6-7), the 11x11 Gaussian window with sigma 1.5
(:15-23) applied as a depthwise 2-D convolution with zero padding, and the SSIM map of
``_ssim`` (:32-53) with C1 = 0.01², C2 = 0.03², averaged over every element.  Pinned to values
produced by the reference itself (tests/golden/loss.npz, tests/test_golden.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from rain_amd.loss import window_1d

_C1 = 0.01 ** 2
_C2 = 0.03 ** 2


def l1_loss(pred, gt):
    """Mean absolute error over every element."""
    return (pred - gt).abs().mean()


def window_2d(size: int, channels: int, like: torch.Tensor) -> torch.Tensor:
    """Outer product of the 1-D window, one copy per channel: [C, 1, size, size]."""
    g = window_1d(size, 1.5).unsqueeze(1)
    w = (g @ g.t()).float()
    return w.expand(channels, 1, size, size).contiguous().to(device=like.device, dtype=like.dtype)


def ssim(img1, img2, window_size: int = 11, size_average: bool = True):
    """Structural similarity of two [C,H,W] (or [N,C,H,W]) images."""
    C = img1.size(-3)
    w = window_2d(window_size, C, img1)

    def blur(x):
        return F.conv2d(x, w, padding=window_size // 2, groups=C)

    m1, m2 = blur(img1), blur(img2)
    m1s, m2s, m12 = m1.pow(2), m2.pow(2), m1 * m2
    v1 = blur(img1 * img1) - m1s
    v2 = blur(img2 * img2) - m2s
    cov = blur(img1 * img2) - m12
    num = (2 * m12 + _C1) * (2 * cov + _C2)
    den = (m1s + m2s + _C1) * (v1 + v2 + _C2)
    smap = num / den
    return smap.mean() if size_average else smap.mean(1).mean(1).mean(1)
