"""Training loss (utils/loss_utils.py:6-53): loss = (1-λ)·L1 + λ·(1-SSIM), 11x11 Gaussian window σ=1.5.

``ssim`` follows the reference exactly (depthwise 11x11 conv2d).  ``ssim_separable`` computes the
same quantity with the window factored into 1x11 and 11x1 passes (the window is an outer product
of the 1-D Gaussian, loss_utils.py:15-19); it is what the train step uses (5 filtered maps, 2 cheap
1-D passes each instead of one 121-tap pass).  Both are pinned to the reference's ssim values by
tests/golden/loss.npz.
"""
from __future__ import annotations

from functools import lru_cache
from math import exp

import torch
import torch.nn.functional as F


def l1_loss(network_output, gt):
    return torch.abs((network_output - gt)).mean()


def l2_loss(network_output, gt):
    return ((network_output - gt) ** 2).mean()


def gaussian(window_size, sigma):
    gauss = torch.Tensor([exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)])
    return gauss / gauss.sum()


def create_window(window_size, channel):
    _1D_window = gaussian(window_size, 1.5).unsqueeze(1)
    _2D_window = _1D_window.mm(_1D_window.t()).float().unsqueeze(0).unsqueeze(0)
    return _2D_window.expand(channel, 1, window_size, window_size).contiguous()


def ssim(img1, img2, window_size=11, size_average=True):
    channel = img1.size(-3)
    window = create_window(window_size, channel).to(img1.device).type_as(img1)
    return _ssim(img1, img2, window, window_size, channel, size_average)


def _ssim(img1, img2, window, window_size, channel, size_average=True):
    mu1 = F.conv2d(img1, window, padding=window_size // 2, groups=channel)
    mu2 = F.conv2d(img2, window, padding=window_size // 2, groups=channel)
    mu1_sq = mu1.pow(2)
    mu2_sq = mu2.pow(2)
    mu1_mu2 = mu1 * mu2
    sigma1_sq = F.conv2d(img1 * img1, window, padding=window_size // 2, groups=channel) - mu1_sq
    sigma2_sq = F.conv2d(img2 * img2, window, padding=window_size // 2, groups=channel) - mu2_sq
    sigma12 = F.conv2d(img1 * img2, window, padding=window_size // 2, groups=channel) - mu1_mu2
    C1 = 0.01 ** 2
    C2 = 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    if size_average:
        return ssim_map.mean()
    return ssim_map.mean(1).mean(1).mean(1)


@lru_cache(maxsize=8)
def _sep_windows(window_size, channels, device, dtype):
    g = gaussian(window_size, 1.5).to(device=device, dtype=dtype)
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
