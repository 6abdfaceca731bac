"""Native densification (include/rain_train.h rt_densify_*) against the torch
restatement of densify_and_prune (GaussianModel.native_densify = False: gaussian_model.py:339-415 op
for op): the same survivors in the same order, the same values (split children's xyz within the
rounding of the reference's bmm; split children's log-scales within an ulp: expf/logf of the device
library here, ATen's exp/log kernels there) and the same optimizer-state surgery."""
import math

import pytest
import torch

from rain_amd import synthetic
from rain_amd.gaussian_model import PARAM_NAMES, GaussianModel, OptimizationParams

pytestmark = pytest.mark.gpu
EXTENT = 4.4


def _model(P, seed):
    g = GaussianModel(3, divide_ratio=0.8, device="cuda")
    p = synthetic.random_gaussians(P, sh_degree=3, seed=seed, bench=True, device="cuda")
    gen = torch.Generator().manual_seed(seed + 1)
    # scales across the clone/split boundary (percent_dense * extent = 0.044), 1% past the
    # world-size prune (0.1 * extent); 5% of the opacities below min_opacity
    s = torch.empty((P, 3)).uniform_(math.log(0.005), math.log(0.2), generator=gen)
    s[: P // 100] = math.log(0.6)
    p["scaling"] = s.to("cuda")
    o = p["opacity"].clone()
    o[P // 100: P // 100 + P // 20] = -6.0
    p["opacity"] = o
    g.set_params(p)
    g.active_sh_degree = 3
    g.spatial_lr_scale = EXTENT
    g.training_setup(OptimizationParams())
    return g


def _prime(g, seed):
    """Non-trivial Adam moments and densification statistics (identical for identical seeds)."""
    gen = torch.Generator(device="cuda").manual_seed(seed)
    for p in g.params():
        p.grad = torch.randn(p.shape, device="cuda", generator=gen) * 1e-3
    g.optimizer.step()
    g.optimizer.zero_grad(set_to_none=True)
    P = g.get_xyz.shape[0]
    g.denom = torch.randint(0, 4, (P, 1), device="cuda", generator=gen).float()
    g.xyz_gradient_accum = torch.rand((P, 1), device="cuda", generator=gen) * 6e-4 * g.denom
    g.max_radii2D = torch.rand((P,), device="cuda", generator=gen) * 40


@pytest.mark.parametrize("max_screen_size,abe_split", [(None, False), (20, False), (None, True), (20, True)])
def test_native_densify_matches_torch(max_screen_size, abe_split):
    """abe_split: the RAIN-GS warm-up split (train.py:138-140, gaussian_model.py:342-364) — the
    split Gaussians' copies at xyz * 0.3 * extent after the clones, and the reference's unused
    normals drawn before the split's (the children match only if both sides draw them)."""
    P = 40_000
    a, b = _model(P, 3), _model(P, 3)
    _prime(a, 5)
    _prime(b, 5)
    a.native_densify = False
    a.densify_and_prune(0.0002, 0.005, EXTENT, max_screen_size, abe_split=abe_split,
                        generator=torch.Generator(device="cuda").manual_seed(11))
    b.densify_and_prune(0.0002, 0.005, EXTENT, max_screen_size, abe_split=abe_split,
                        generator=torch.Generator(device="cuda").manual_seed(11))
    Pn = a.get_xyz.shape[0]
    assert b.get_xyz.shape[0] == Pn and Pn != P
    for name, pa, pb in zip(PARAM_NAMES, a.params(), b.params()):
        assert pa.shape == pb.shape, name
        if name == "xyz":
            torch.testing.assert_close(pb.detach(), pa.detach(), rtol=1e-6, atol=1e-6)
        elif name == "scaling":
            torch.testing.assert_close(pb.detach(), pa.detach(), rtol=1e-6, atol=1e-7)
            n_orig_clone = int((pa.detach() == pb.detach()).all(dim=1).sum())
            assert n_orig_clone > 0
        else:
            assert torch.equal(pa.detach(), pb.detach()), name
        sa, sb = a.optimizer.state[pa], b.optimizer.state[pb]
        assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"]), name
        assert float(sa["step"]) == float(sb["step"])
        assert any(pb is grp["params"][0] for grp in b.optimizer.param_groups)
    for t in (b.xyz_gradient_accum, b.denom, b.max_radii2D):
        assert t.shape[0] == Pn and float(t.abs().sum()) == 0.0


def test_abe_split_rows_follow_the_reference_layout():
    """Native abe_split: the rows after the clones are the split Gaussians' copies (xyz scaled by
    0.3 * extent, the other raw parameters unchanged, zero moments), then the split children."""
    P = 20_000
    g = _model(P, 4)
    _prime(g, 6)
    raw = {n: p.detach().clone() for n, p in zip(PARAM_NAMES, g.params())}
    grads = g.xyz_gradient_accum / g.denom
    grads[grads.isnan()] = 0.0
    smax = torch.exp(raw["scaling"]).max(dim=1).values
    split = (grads.squeeze(1) >= 0.0002) & (smax > g.percent_dense * EXTENT)
    clone = (torch.norm(grads, dim=-1) >= 0.0002) & (smax <= g.percent_dense * EXTENT)
    op = torch.sigmoid(raw["opacity"]).squeeze(1)
    keep_orig = ~split & (op >= 0.005)
    keep_clone = clone & (op >= 0.005)
    keep_abe = split & (op >= 0.005)  # max_screen_size None: opacity is the only prune
    g.densify_and_prune(0.0002, 0.005, EXTENT, None, abe_split=True,
                        generator=torch.Generator(device="cuda").manual_seed(2))
    A, B, E = int(keep_orig.sum()), int(keep_clone.sum()), int(keep_abe.sum())
    assert E > 0
    new = {n: p.detach() for n, p in zip(PARAM_NAMES, g.params())}
    abe = slice(A + B, A + B + E)
    torch.testing.assert_close(new["xyz"][abe], raw["xyz"][keep_abe] * 0.3 * EXTENT, rtol=0, atol=0)
    for n in ("f_dc", "f_rest", "opacity", "rotation"):
        assert torch.equal(new[n][abe], raw[n][keep_abe]), n
    torch.testing.assert_close(new["scaling"][abe], raw["scaling"][keep_abe], rtol=1e-6, atol=1e-7)
    st = g.optimizer.state[g.params()[0]]
    assert float(st["exp_avg"][abe].abs().sum()) == 0.0
    assert new["xyz"].shape[0] == A + B + E + 2 * E  # children: the same opacity prune


def test_native_densify_without_optimizer_state():
    """Groups with no Adam state yet (no step taken): only the parameters are rebuilt."""
    a, b = _model(5000, 7), _model(5000, 7)
    for g in (a, b):
        P = g.get_xyz.shape[0]
        g.denom = torch.ones((P, 1), device="cuda")
        g.xyz_gradient_accum = torch.full((P, 1), 1e-3, device="cuda")
    a.native_densify = False
    a.densify_and_prune(0.0002, 0.005, EXTENT, None, generator=torch.Generator(device="cuda").manual_seed(1))
    b.densify_and_prune(0.0002, 0.005, EXTENT, None, generator=torch.Generator(device="cuda").manual_seed(1))
    for name, pa, pb in zip(PARAM_NAMES, a.params(), b.params()):
        assert pa.shape == pb.shape, name
        if name in ("xyz", "scaling"):
            torch.testing.assert_close(pb.detach(), pa.detach(), rtol=1e-6, atol=1e-6)
        else:
            assert torch.equal(pa.detach(), pb.detach()), name
        assert len(b.optimizer.state.get(pb, {})) == len(a.optimizer.state.get(pa, {}))


def test_native_densification_stats_equal_torch(gpu):
    """GaussianModel.add_densification_stats / update_max_radii on HIP tensors (rain_train.h
    rt_densify_stats / rt_max_radii, one launch each) give the torch expressions' values
    (gaussian_model.py:419-421, train.py:133): counts and radii bitwise, the norm sums to the last
    ulp (torch's reduction may contract x*x + y*y into an fma)."""
    P = 50_000
    gen = torch.Generator(device="cuda").manual_seed(3)
    g = GaussianModel(3, device="cuda")
    g.set_params(synthetic.random_gaussians(P, sh_degree=3, seed=2, bench=True, device="cuda"))
    g.xyz_gradient_accum = torch.rand((P, 1), device="cuda", generator=gen)
    g.denom = torch.randint(0, 5, (P, 1), device="cuda", generator=gen).float()
    g.max_radii2D = torch.randint(0, 40, (P,), device="cuda", generator=gen).float()
    vsp = torch.zeros((P, 3), device="cuda", requires_grad=True)
    vsp.grad = torch.randn((P, 3), device="cuda", generator=gen) * 1e-3
    vis = torch.rand((P,), device="cuda", generator=gen) > 0.3
    radii = torch.randint(0, 60, (P,), device="cuda", generator=gen, dtype=torch.int32)
    m = vis.reshape(-1, 1)
    want_acc = g.xyz_gradient_accum + torch.where(m, torch.norm(vsp.grad[:, :2], dim=-1, keepdim=True), 0.0)
    want_den = g.denom + m.float()
    want_rad = torch.where(vis, torch.maximum(g.max_radii2D, radii.float()), g.max_radii2D)
    g.add_densification_stats(vsp, vis)
    g.update_max_radii(radii, vis)
    assert float(((g.xyz_gradient_accum - want_acc).abs() / want_acc.abs().clamp_min(1e-30)).max()) <= 2.5e-7
    assert torch.equal(g.denom, want_den)
    assert torch.equal(g.max_radii2D, want_rad)
