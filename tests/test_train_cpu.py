"""CPU tests of the host side around the rasterizer: the render() contract, the autograd plumbing
(BASELINE.json configs[0]: 10k Gaussians, 256x256, SH 0, forward+backward on CPU), densification,
and the view-sharded multi-process training step over gloo (world size 2).  The rasterizer itself is
the CPU oracle here (tests/oracle_c.py, monkeypatched in for the HIP `_C`)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import rain_amd.diff_gaussian_rasterization as dgr
from rain_amd import cameras, synthetic
from rain_amd.gaussian_model import GaussianModel, OptimizationParams
from oracle.loss_ref import l1_loss, ssim
from rain_amd.renderer import PipelineParams, render
from rain_amd.train import TrainConfig, Trainer
from tests import oracle_c


def _ref_loss(img, gt, lam):
    return (1.0 - lam) * l1_loss(img, gt) + lam * (1.0 - ssim(img, gt))


def _model(P, sh_degree, seed=0, bench=True):
    g = GaussianModel(sh_degree, divide_ratio=0.8, device="cpu")
    g.set_params(synthetic.random_gaussians(P, sh_degree=sh_degree, seed=seed, bench=bench))
    g.active_sh_degree = sh_degree
    g.spatial_lr_scale = 4.4
    return g


@pytest.fixture
def cpu_rasterizer(monkeypatch, oracle):
    monkeypatch.setattr(dgr, "_C", oracle_c)
    return oracle_c


def test_render_contract_cfg1(cpu_rasterizer):
    g = _model(10_000, 0)
    g.training_setup(OptimizationParams())
    cam = cameras.fibonacci_cameras(4, 256, 256)[0]
    out = render(cam, g, PipelineParams(), torch.zeros(3))
    assert set(out) == {"render", "viewspace_points", "visibility_filter", "radii", "depth"}
    assert out["render"].shape == (3, 256, 256) and out["depth"].shape == (1, 256, 256)
    assert out["radii"].dtype == torch.int32 and out["radii"].shape == (10_000,)
    assert torch.equal(out["visibility_filter"], out["radii"] > 0)
    gt = torch.rand(3, 256, 256, generator=torch.Generator().manual_seed(1))
    _ref_loss(out["render"], gt, 0.2).backward()
    vsp = out["viewspace_points"].grad
    assert vsp.shape == (10_000, 3) and float(vsp[:, 2].abs().sum()) == 0.0
    vis = out["visibility_filter"]
    for p in g.params():
        assert p.grad is not None and torch.isfinite(p.grad).all()
    assert float(g._xyz.grad[vis].abs().sum()) > 0 and float(g._xyz.grad[~vis].abs().sum()) == 0
    assert float(g._opacity.grad.abs().sum()) > 0 and float(g._features_dc.grad.abs().sum()) > 0


def test_python_paths_match_kernel_paths(cpu_rasterizer):
    """convert_SHs_python / compute_cov3D_python (gaussian_renderer/__init__.py:44-58) give the same
    image as the in-kernel SH and covariance paths."""
    g = _model(3000, 3)
    cam = cameras.fibonacci_cameras(4, 96, 80)[1]
    with torch.no_grad():
        a = render(cam, g, PipelineParams(), torch.zeros(3))["render"]
        b = render(cam, g, PipelineParams(convert_SHs_python=True, compute_cov3D_python=True), torch.zeros(3))["render"]
    assert float((a - b).abs().sum() / a.abs().sum()) < 1e-5


def test_debug_snapshot_on_error(cpu_rasterizer, monkeypatch, tmp_path):
    monkeypatch.chdir(tmp_path)

    def boom(*args):
        raise RuntimeError("kernel failure")

    monkeypatch.setattr(cpu_rasterizer, "rasterize_gaussians", boom)
    g = _model(100, 0)
    cam = cameras.fibonacci_cameras(4, 32, 32)[0]
    with pytest.raises(RuntimeError, match="kernel failure"):
        render(cam, g, PipelineParams(debug=True), torch.zeros(3))
    args = torch.load(tmp_path / "snapshot_fw.dump", weights_only=True)
    assert len(args) == 20 and args[13] == 32


def test_densify_and_prune_bookkeeping(cpu_rasterizer):
    g = _model(2000, 1)
    opt = OptimizationParams()
    g.training_setup(opt)
    cams = cameras.fibonacci_cameras(8, 64, 48)
    gts = [torch.rand(3, 48, 64, generator=torch.Generator().manual_seed(i)) for i in range(8)]
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(c2f=False), scene_extent=4.4, loss_fn=_ref_loss)
    opt.densify_grad_threshold = 1e-6  # force clones/splits on a tiny run
    for it in range(595, 601):
        info = tr.step(it)
    assert info.densified
    P = g.get_xyz.shape[0]
    assert P != 2000
    for grp in g.optimizer.param_groups:
        p = grp["params"][0]
        assert p.shape[0] == P
        st = g.optimizer.state.get(p)
        if st:
            assert st["exp_avg"].shape == p.shape
    assert g.xyz_gradient_accum.shape == (P, 1) and g.max_radii2D.shape == (P,)


def test_ours_new_warmup_abe_split_and_lr_shift(cpu_rasterizer):
    """--ours_new (train.py:73-77, 138-140): during the warm-up the densify adds the abe copies of
    the split Gaussians and the learning-rate schedule has not started; after it, the schedule runs
    on iteration - warmup_iter."""
    cams = cameras.fibonacci_cameras(8, 64, 48)
    gts = [torch.rand(3, 48, 64, generator=torch.Generator().manual_seed(i)) for i in range(8)]
    sizes = {}
    for mode in ("plain", "ours_new"):
        g = _model(2000, 1)
        opt = OptimizationParams()
        g.training_setup(opt)
        lr0 = next(grp["lr"] for grp in g.optimizer.param_groups if grp["name"] == "xyz")
        cfg = TrainConfig(c2f=False, ours_new=True, warmup_iter=700) if mode == "ours_new" else TrainConfig(c2f=False)
        tr = Trainer(g, cams, gts, opt, PipelineParams(), cfg, scene_extent=4.4, loss_fn=_ref_loss)
        opt.densify_grad_threshold = 1e-6  # force clones/splits on a tiny run
        for it in range(595, 601):
            info = tr.step(it)
        assert info.densified
        sizes[mode] = g.get_xyz.shape[0]
        lr = next(grp["lr"] for grp in g.optimizer.param_groups if grp["name"] == "xyz")
        if mode == "ours_new":
            assert lr == lr0  # warm-up: update_learning_rate not called yet
            tr.step(702)
            lr = next(grp["lr"] for grp in g.optimizer.param_groups if grp["name"] == "xyz")
            assert lr == g.xyz_scheduler_args(2)
        else:
            assert lr == g.xyz_scheduler_args(600)
    assert sizes["ours_new"] > sizes["plain"]  # the abe copies (N - 1 = 1 per kept split Gaussian)


# ---- view-sharded data parallel over gloo ------------------------------------------------

def _scene():
    torch.manual_seed(0)
    cams = cameras.fibonacci_cameras(6, 48, 40)
    gts = [torch.rand(3, 40, 48, generator=torch.Generator().manual_seed(10 + i)) for i in range(6)]
    return cams, gts


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    dgr._C = oracle_c
    cams, gts = _scene()
    g = _model(800, 1, seed=3)
    opt = OptimizationParams()
    g.training_setup(opt)
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(c2f=False, seed=5), scene_extent=4.4,
                 loss_fn=_ref_loss)
    for it in (1, 2, 3):
        tr.step(it)
    tr.sync_densify_stats()  # statistics stay per rank until densify consumes them
    torch.save({n: p.detach().clone() for n, p in zip(("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"),
                                                     g.params())} | {"accum": g.xyz_gradient_accum.clone(),
                                                                    "denom": g.denom.clone(),
                                                                    "maxr": g.max_radii2D.clone()},
               f"{out_path}.{rank}")
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_view_sharded_step_gloo(oracle, tmp_path, monkeypatch, world):
    """N ranks x 1 view per step == 1 process accumulating the same N views' gradients (mean),
    summing their densification statistics, then one Adam step; replicas stay identical.  World 4
    also covers a flat layout padded to 4 slices (the driver's N = 4 / 8 runs shard the same way)."""
    out = str(tmp_path / "r")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    r0 = rs[0]
    for r1 in rs[1:]:
        for k in r0:
            assert torch.equal(r0[k], r1[k]), f"replicas diverged on {k}"

    # single-process reference with the same view schedule
    monkeypatch.setattr(dgr, "_C", oracle_c)
    from rain_amd.train import ViewSampler

    cams, gts = _scene()
    g = _model(800, 1, seed=3)
    opt = OptimizationParams()
    g.training_setup(opt)
    sampler = ViewSampler(len(cams), world, seed=5)
    bg = torch.zeros(3)
    for it in (1, 2, 3):
        g.update_learning_rate(it)
        views = sampler.next_group()
        grads = [torch.zeros_like(p) for p in g.params()]
        for v in views:
            for p in g.params():
                p.grad = None
            pkg = render(cams[v], g, PipelineParams(), bg)
            _ref_loss(pkg["render"], gts[v], opt.lambda_dssim).backward()
            for acc, p in zip(grads, g.params()):
                acc += p.grad
            with torch.no_grad():
                vis = pkg["visibility_filter"]
                g.max_radii2D[vis] = torch.max(g.max_radii2D[vis], pkg["radii"][vis].float())
                g.add_densification_stats(pkg["viewspace_points"], vis)
        with torch.no_grad():
            for acc, p in zip(grads, g.params()):
                p.grad = acc / float(world)
            g.optimizer.step()
            g.optimizer.zero_grad(set_to_none=True)
    ref = dict(zip(("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"), g.params()))
    for k, v in ref.items():
        # the gloo exchange adds the ranks' gradients in rank order (Trainer.Exchange), the order in
        # which the reference accumulates the same views
        torch.testing.assert_close(r0[k], v.detach(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(r0["accum"], g.xyz_gradient_accum, rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(r0["denom"], g.denom)
    torch.testing.assert_close(r0["maxr"], g.max_radii2D)


def _event_opt():
    opt = OptimizationParams()
    opt.densify_from_iter, opt.densification_interval, opt.opacity_reset_interval = 1, 2, 3
    return opt


def _worker_events(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    dgr._C = oracle_c
    cams, gts = _scene()
    g = _model(800, 1, seed=3)
    opt = _event_opt()
    g.training_setup(opt)
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(c2f=False, seed=5), scene_extent=4.4,
                 loss_fn=_ref_loss)
    flags = [tr.step(it).densified for it in range(1, 8)]
    tr.sync_optimizer_state()  # iteration 7 (ordinary) advanced only this rank's moment slice
    out = {n: p.detach().clone() for n, p in zip(("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"),
                                                  g.params())}
    for n, p in zip(("xyz", "opacity", "f_rest"), (g._xyz, g._opacity, g._features_rest)):
        out["m_" + n] = g.optimizer.state[p]["exp_avg"].clone()
        out["v_" + n] = g.optimizer.state[p]["exp_avg_sq"].clone()
    out["densified"] = torch.tensor(flags)
    torch.save(out, f"{out_path}.{rank}")
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_view_sharded_densify_and_reset_gloo(oracle, tmp_path, monkeypatch, world):
    """Iterations with densify/prune (2, 4, 6) and opacity reset (3, 6) in the sharded step: Adam
    moments gathered, statistics merged, the replaced opacity skipped; replicas stay identical and
    equal one process running the reference schedule on the mean of the same views' gradients."""
    out = str(tmp_path / "e")
    mp.start_processes(_worker_events, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    r0 = rs[0]
    for r1 in rs[1:]:
        for k in r0:
            assert torch.equal(r0[k], r1[k]), f"replicas diverged on {k}"
    assert r0["densified"].tolist() == [False, True, False, True, False, True, False]

    monkeypatch.setattr(dgr, "_C", oracle_c)
    from rain_amd.train import ViewSampler

    cams, gts = _scene()
    g = _model(800, 1, seed=3)
    opt = _event_opt()
    g.training_setup(opt)
    tr1 = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(c2f=False, seed=5), scene_extent=4.4,
                  loss_fn=_ref_loss)
    sampler = ViewSampler(len(cams), world, seed=5)
    bg = torch.zeros(3)
    slots = None
    for it in range(1, 8):
        g.update_learning_rate(it)
        grads = [torch.zeros_like(p) for p in g.params()]
        P = g.get_xyz.shape[0]
        if slots is None:  # per-rank statistics, merged in rank order where the sharded step merges them
            slots = [(torch.zeros(P, 1), torch.zeros(P, 1), torch.zeros(P)) for _ in range(world)]
        for r, v in enumerate(sampler.next_group()):
            for p in g.params():
                p.grad = None
            pkg = render(cams[v], g, PipelineParams(), bg)
            _ref_loss(pkg["render"], gts[v], opt.lambda_dssim).backward()
            for acc, p in zip(grads, g.params()):
                acc += p.grad
            with torch.no_grad():
                vis = pkg["visibility_filter"]
                a, d, m = slots[r]
                m[vis] = torch.max(m[vis], pkg["radii"][vis].float())
                a[vis] += torch.norm(pkg["viewspace_points"].grad[vis, :2], dim=-1, keepdim=True)
                d[vis] += 1
        with torch.no_grad():
            for acc, p in zip(grads, g.params()):
                p.grad = acc / float(world)
            if tr1._events(it)[0]:
                g.xyz_gradient_accum = slots[0][0].clone()
                g.denom = slots[0][1].clone()
                g.max_radii2D = slots[0][2].clone()
                for a, d, m in slots[1:]:
                    g.xyz_gradient_accum += a
                    g.denom += d
                    torch.maximum(g.max_radii2D, m, out=g.max_radii2D)
                slots = None
            tr1._densify_and_adam(it)
            g.optimizer.zero_grad(set_to_none=True)
    ref = dict(zip(("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"), g.params()))
    for k, v in ref.items():
        assert r0[k].shape == v.shape, k
        torch.testing.assert_close(r0[k], v.detach(), rtol=1e-5, atol=1e-7)
    for n, p in zip(("xyz", "opacity", "f_rest"), (g._xyz, g._opacity, g._features_rest)):
        torch.testing.assert_close(r0["m_" + n], g.optimizer.state[p]["exp_avg"], rtol=1e-5, atol=1e-9)
        torch.testing.assert_close(r0["v_" + n], g.optimizer.state[p]["exp_avg_sq"], rtol=1e-5, atol=1e-12)
