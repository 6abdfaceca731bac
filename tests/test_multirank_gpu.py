"""The view-sharded FUSED training step (the path `bench.py --gpus N` takes: train.py:87-147 with the
raw-parameter rasterizer, Trainer._finish and optim.sharded_adam_step) run by 2 real ranks.

Both ranks share cuda:0 and talk over gloo (RCCL refuses two ranks on one device; the driver's
8-GPU run uses RCCL through the same Trainer code, Trainer.Exchange only changes where the bytes
are staged).  The ranks are spawned before this process touches the GPU (conftest orders this
module first).  Iterations 1..7 cover ordinary steps (1, 5, 7), densify/prune (2, 4, 6) and opacity
reset (3, 6).  Bar: replicas bit-identical, and equal to one process accumulating
the same two views' gradients (mean) and statistics (sum) and stepping once.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
P, W, H, V = 20_000, 160, 120, 6
ITERS = range(1, 8)


def _opt():
    from rain_amd.gaussian_model import OptimizationParams

    return OptimizationParams(densify_from_iter=1, densification_interval=2, opacity_reset_interval=3)


def _scene(dev):
    from rain_amd import cameras, synthetic
    from rain_amd.gaussian_model import GaussianModel

    cams = [c.to(dev) for c in cameras.fibonacci_cameras(V, W, H)]
    gts = [torch.rand(3, H, W, generator=torch.Generator().manual_seed(20 + i)).to(dev) for i in range(V)]
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    p = synthetic.random_gaussians(P, sh_degree=3, seed=6, bench=True)
    p["scaling"] = p["scaling"] + 0.3 * torch.randn(p["scaling"].shape, generator=torch.Generator().manual_seed(1))
    g.set_params(p)
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    opt = _opt()
    opt.densify_grad_threshold = 2e-5  # some clones / splits at this tiny scale
    g.training_setup(opt)
    return g, opt, cams, gts


def _snapshot(g, flags):
    out = {n: p.detach().cpu().clone() for n, p in zip(NAMES, g.params())}
    for n, p in zip(NAMES, g.params()):
        out["m_" + n] = g.optimizer.state[p]["exp_avg"].detach().cpu().clone()
        out["v_" + n] = g.optimizer.state[p]["exp_avg_sq"].detach().cpu().clone()
    out["accum"] = g.xyz_gradient_accum.cpu().clone()
    out["denom"] = g.denom.cpu().clone()
    out["maxr"] = g.max_radii2D.cpu().clone()
    out["densified"] = torch.tensor(flags)
    return out


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    g, opt, cams, gts = _scene(dev)
    tr = Trainer(g, cams, gts, opt, cfg=TrainConfig(c2f=False, seed=5), scene_extent=4.4)
    assert tr.fused and tr.world == world
    flags = [tr.step(it).densified for it in ITERS]
    tr.sync_densify_stats()  # merge what accumulated since the last densify
    tr.sync_optimizer_state()  # iteration 7 advanced only this rank's slice of the moments
    torch.cuda.synchronize()
    torch.save(_snapshot(g, flags), f"{out_path}.{rank}")
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _reference(dev, world=2):
    """One process: the world's views of each step through the fused forward/backward, gradients
    summed then divided by the world size, statistics accumulated view after view, then the world-1 densify/Adam logic."""
    from rain_amd import fused
    from rain_amd.loss import l1_ssim_backward, l1_ssim_forward
    from rain_amd.train import TrainConfig, Trainer, ViewSampler

    g, opt, cams, gts = _scene(dev)
    tr = Trainer(g, cams, gts, opt, cfg=TrainConfig(c2f=False, seed=5), scene_extent=4.4)
    sampler = ViewSampler(V, world, seed=5)
    bg = torch.zeros(3, device=dev)
    flags = []
    for it in ITERS:
        g.update_learning_rate(it)
        views = sampler.next_group()
        acc = [torch.zeros_like(p) for p in g.params()]
        for v in views:
            color, radii, depth, st = fused.forward(g, cams[v], bg, 0.3)
            _, _, ws = l1_ssim_forward(color, gts[v], opt.lambda_dssim)
            dimg = l1_ssim_backward(color, gts[v], opt.lambda_dssim, ws)
            grads = {n: torch.empty_like(p) for n, p in zip(NAMES, g.params())}
            fused.backward(st, dimg, grads, (g.xyz_gradient_accum, g.denom, g.max_radii2D))
            for a, n in zip(acc, NAMES):
                a += grads[n]
        g.bind_flat_grad()
        for a, p in zip(acc, g.params()):
            p.grad.copy_(a / float(world))
        flags.append(tr._densify_and_adam(it))
    torch.cuda.synchronize()
    return _snapshot(g, flags)


def _close(x, y, rel, floor=1.0):
    scale = max(floor, float(y.abs().max())) if y.numel() else 1.0
    return x.shape == y.shape and (y.numel() == 0 or float((x - y).abs().max()) <= rel * scale)


def test_view_sharded_fused_step_two_ranks(tmp_path):
    if torch.cuda.device_count() < 1:  # does not initialise the GPU in this process
        pytest.skip("no HIP device")
    out = str(tmp_path / "rank")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    r0, r1 = torch.load(out + ".0", weights_only=True), torch.load(out + ".1", weights_only=True)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), f"replicas diverged on {k}"
    assert r0["densified"].tolist() == [False, True, False, True, False, True, False]

    ref = _reference(torch.device("cuda:0"))
    assert ref["densified"].tolist() == r0["densified"].tolist()
    assert r0["xyz"].shape == ref["xyz"].shape, "densify made different decisions"
    # the backward accumulates per-Gaussian gradients with float atomics in a run-dependent order;
    # Adam's division by sqrt(v) turns last-bit differences into ~1e-6 relative parameter
    # differences (tests/test_fused_gpu.py::test_adam_fused_into_backward_matches_separate_step)
    for n in NAMES:
        assert _close(r0[n], ref[n], 1e-5), (n, float((r0[n] - ref[n]).abs().max()))
        assert _close(r0["m_" + n], ref["m_" + n], 1e-4, floor=1e-30), "m_" + n
        assert _close(r0["v_" + n], ref["v_" + n], 1e-4, floor=1e-30), "v_" + n
    assert torch.equal(r0["denom"], ref["denom"])
    assert torch.equal(r0["maxr"], ref["maxr"])
    assert _close(r0["accum"], ref["accum"], 1e-5, floor=1e-30)


def test_view_sharded_fused_step_four_ranks(tmp_path):
    """World 4 (the flat buffers padded to 4 slices, as in the driver's N = 4 / 8 runs), 4 ranks on
    cuda:0 over gloo.  Replicas must stay bit-identical.  Against one process summing the same 4
    views: the collective adds in its own order, so a gradient that cancels to ~0 across the views
    can change sign and Adam's early ~lr*sign(g) steps move that element the other way; those
    elements must be few and each within a few lr of the reference."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no HIP device")
    world = 4
    out = str(tmp_path / "rank")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    for r in rs[1:]:
        for k in rs[0]:
            assert torch.equal(rs[0][k], r[k]), f"replicas diverged on {k}"
    r0 = rs[0]
    assert r0["densified"].tolist() == [False, True, False, True, False, True, False]
    ref = _reference(torch.device("cuda:0"), world)
    assert ref["densified"].tolist() == r0["densified"].tolist()
    assert r0["xyz"].shape == ref["xyz"].shape, "densify made different decisions"
    for n in NAMES:
        x, y = r0[n], ref[n]
        scale = max(1.0, float(y.abs().max()))
        off = (x - y).abs() > 1e-5 * scale
        assert off.float().mean().item() <= 0.05, (n, int(off.sum()))
        assert float((x - y).abs().max()) <= 0.2 * scale, (n, float((x - y).abs().max()))
    assert torch.equal(r0["denom"], ref["denom"])
    assert torch.equal(r0["maxr"], ref["maxr"])
    assert _close(r0["accum"], ref["accum"], 1e-3, floor=1e-30)
