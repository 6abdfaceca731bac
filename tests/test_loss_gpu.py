"""Fused L1+SSIM HIP loss vs the reference formulation (utils/loss_utils.py) in torch fp32/fp64."""
import pytest
import torch

from oracle.loss_ref import l1_loss, ssim
from rain_amd.loss import fused_l1_ssim_loss

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,W", [(96, 128), (75, 100), (9, 200), (540, 960), (1080, 1920)])
def test_fused_loss_matches_reference(gpu, H, W):
    g = torch.Generator().manual_seed(H * W)
    img = torch.rand((3, H, W), generator=g).to(gpu)
    gt = (img.cpu() * 0.7 + 0.3 * torch.rand((3, H, W), generator=g)).to(gpu)
    lam = 0.2
    x = img.clone().requires_grad_(True)
    loss, parts = fused_l1_ssim_loss(x, gt, lam)
    loss.backward()
    # reference in float64 (conv2d of the exact 2-D window)
    xr = img.double().cpu().clone().requires_grad_(True)
    gtr = gt.double().cpu()
    ref = (1 - lam) * l1_loss(xr, gtr) + lam * (1 - ssim(xr, gtr))
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 2e-6 * abs(float(ref)) + 1e-7
    assert abs(float(parts[2]) - float(ssim(img.double().cpu(), gtr))) < 2e-6
    gref = xr.grad.float().to(gpu)
    rel = float((x.grad - gref).abs().sum() / gref.abs().sum())
    assert rel < 1e-4, rel


def test_fused_loss_grad_scale(gpu):
    img = torch.rand((3, 64, 48), device=gpu)
    gt = torch.rand((3, 64, 48), device=gpu)
    x1 = img.clone().requires_grad_(True)
    l1, _ = fused_l1_ssim_loss(x1, gt)
    (3.0 * l1).backward()
    x2 = img.clone().requires_grad_(True)
    l2, _ = fused_l1_ssim_loss(x2, gt)
    l2.backward()
    torch.testing.assert_close(x1.grad, 3.0 * x2.grad, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("H,W", [(75, 100), (9, 200), (1080, 1920)])
def test_forward_backward_in_one_call_is_bitwise_the_two_calls(gpu, H, W):
    """rl_l1_ssim_forward_backward (the loss finalize rides on the backward launch) gives bitwise
    the loss / parts of rl_l1_ssim_forward and the dimg of rl_l1_ssim_backward, also with a
    grad_loss scale."""
    from rain_amd.loss import l1_ssim_backward, l1_ssim_forward, l1_ssim_forward_backward

    g = torch.Generator().manual_seed(7 * H + W)
    img = torch.rand((3, H, W), generator=g).to(gpu)
    gt = (img.cpu() * 0.6 + 0.4 * torch.rand((3, H, W), generator=g)).to(gpu)
    for scale in (None, 2.5):
        gl = None if scale is None else torch.tensor([scale], device=gpu)
        loss, parts, ws = l1_ssim_forward(img, gt, 0.2)
        dimg = l1_ssim_backward(img, gt, 0.2, ws, gl)
        loss2, parts2, dimg2 = l1_ssim_forward_backward(img, gt, 0.2, gl)
        assert torch.equal(loss, loss2) and torch.equal(parts, parts2)
        assert torch.equal(dimg, dimg2)


