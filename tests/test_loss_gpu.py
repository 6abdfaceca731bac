"""Fused L1+SSIM HIP loss vs the reference formulation (utils/loss_utils.py) in torch fp32/fp64."""
import numpy as np
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


@pytest.fixture
def two_pass():
    """rl_l1_ssim_forward_backward as the two passes over stored maps (rl_set_fused_band(0), the
    default)."""
    from rain_amd import _native as N

    N.loss_lib().rl_set_fused_band(0)
    yield


@pytest.fixture(params=[16, 32, 64])
def band_walk(request):
    from rain_amd import _native as N

    assert N.loss_lib().rl_set_fused_band(request.param) == 0
    yield request.param
    N.loss_lib().rl_set_fused_band(0)


@pytest.mark.parametrize("H,W", [(75, 100), (9, 200), (1080, 1920)])
def test_forward_backward_in_one_call_is_bitwise_the_two_calls(gpu, two_pass, H, W):
    """rl_l1_ssim_forward_backward in its two-pass form (the loss finalize rides on the backward
    launch) gives bitwise the loss / parts of rl_l1_ssim_forward and the dimg of
    rl_l1_ssim_backward, also with a grad_loss scale."""
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


@pytest.mark.parametrize("H,W", [(75, 100), (9, 200), (33, 55), (96, 54), (540, 960), (1080, 1920)])
def test_one_band_walk_matches_the_two_passes(gpu, band_walk, H, W):
    """rl_l1_ssim_forward_backward's one-band-walk form (rl_set_fused_band: the derivative maps
    formed and blurred on chip, 54-column blocks) against the separate forward + backward passes: dimg to float
    contraction (1e-6 of its scale), loss and parts to float rounding (a different block partition
    of the sums), also with a grad_loss scale; and against the float64 reference like the two-pass
    loss."""
    from rain_amd.loss import l1_ssim_backward, l1_ssim_forward, l1_ssim_forward_backward

    g = torch.Generator().manual_seed(11 * H + W)
    img = torch.rand((3, H, W), generator=g).to(gpu)
    gt = (img.cpu() * 0.6 + 0.4 * torch.rand((3, H, W), generator=g)).to(gpu)
    for scale in (None, 2.5):
        gl = None if scale is None else torch.tensor([scale], device=gpu)
        loss, parts, ws = l1_ssim_forward(img, gt, 0.2)
        dimg = l1_ssim_backward(img, gt, 0.2, ws, gl)
        loss2, parts2, dimg2 = l1_ssim_forward_backward(img, gt, 0.2, gl)
        assert torch.isfinite(dimg2).all()
        assert float((dimg2 - dimg).abs().max()) <= 1e-6 * float(dimg.abs().max()), (H, W, scale)
        torch.testing.assert_close(loss2, loss, rtol=2e-6, atol=0)
        torch.testing.assert_close(parts2, parts, rtol=2e-6, atol=1e-9)
    xr = img.double().cpu()
    ref = 0.8 * l1_loss(xr, gt.double().cpu()) + 0.2 * (1 - ssim(xr, gt.double().cpu()))
    assert abs(float(loss2) - float(ref)) <= 2e-6 * abs(float(ref)) + 1e-7


def _open_bits(pattern, H, W, gen):
    """An open-tile mask (16 x 16-px tiles, bit ty * tx_n + tx) of the given shape."""
    tx, ty = (W + 15) // 16, (H + 15) // 16
    o = torch.zeros((ty, tx), dtype=torch.bool)
    if pattern == "all":
        o[:] = True
    elif pattern == "bottom":
        o[ty - max(1, ty // 3):, :] = True
    elif pattern == "corner":
        o[ty - 1, tx - 1] = True
    elif pattern == "random":
        o = torch.rand((ty, tx), generator=gen) < 0.1
    flat = o.flatten()
    words = [0] * ((flat.numel() + 31) // 32)
    for i in torch.nonzero(flat).flatten().tolist():
        words[i // 32] |= 1 << (i % 32)
    return words, tx, ty


@pytest.mark.parametrize("pattern", ["none", "all", "bottom", "corner", "random"])
@pytest.mark.parametrize("H,W", [(75, 100), (9, 200), (540, 960), (1080, 1920)])
def test_split_loss_is_bitwise_the_one_call(gpu, two_pass, pattern, H, W):
    """rl_l1_ssim_forward_backward_part: part 1 (bands whose rows hold no open tile) then part 2 (the
    rest + the finalize) write bitwise the loss, parts and dimg of rl_l1_ssim_forward_backward, for
    any open-tile mask; the parts overlap nothing (each writes only its bands: the other part's
    rows of dimg keep a sentinel until it runs)."""
    import ctypes

    from rain_amd import _native as N
    from rain_amd.loss import _window_host, l1_ssim_forward_backward

    g = torch.Generator().manual_seed(13 * H + W)
    img = torch.rand((3, H, W), generator=g).to(gpu)
    gt = (img.cpu() * 0.6 + 0.4 * torch.rand((3, H, W), generator=g)).to(gpu)
    words, tx, ty = _open_bits(pattern, H, W, g)
    bits32 = torch.from_numpy(np.array(words, dtype=np.uint32).view(np.int32)).to(gpu)
    L = N.loss_lib()
    loss, parts, dimg = l1_ssim_forward_backward(img, gt, 0.2)
    ws = torch.empty((L.rl_workspace_bytes(3, H, W),), dtype=torch.uint8, device=gpu)
    loss2 = torch.empty((), dtype=torch.float32, device=gpu)
    parts2 = torch.empty((3,), dtype=torch.float32, device=gpu)
    dimg2 = torch.full_like(img, float("nan"))
    one = torch.ones((1,), dtype=torch.float32, device=gpu)
    args = (img.data_ptr(), gt.data_ptr(), 3, H, W, 0.2, _window_host(), ws.data_ptr(), ws.numel(), loss2.data_ptr(),
            parts2.data_ptr(), one.data_ptr(), dimg2.data_ptr(), bits32.data_ptr(), tx, ty)
    st = N.stream_of(img)
    assert L.rl_l1_ssim_forward_backward_part(*args, 1, None, st) == 0, L.rl_last_error()
    torch.cuda.synchronize()
    done1 = ~torch.isnan(dimg2)
    if pattern == "none":
        assert bool(done1.all())
    if pattern == "all":
        assert not bool(done1.any())
    assert torch.equal(dimg2[done1], dimg[done1])
    assert L.rl_l1_ssim_forward_backward_part(*args, 2, None, st) == 0, L.rl_last_error()
    torch.cuda.synchronize()
    assert torch.equal(loss2, loss) and torch.equal(parts2, parts)
    assert torch.equal(dimg2, dimg)
    # argument checks
    bad = list(args)
    bad[14] = tx + 1
    assert L.rl_l1_ssim_forward_backward_part(*bad, 1, None, st) == 1
    assert L.rl_l1_ssim_forward_backward_part(*args, 3, None, st) == 1
