"""The view-sharded FUSED training step (the path `bench.py --gpus N` takes: train.py:87-147 with the
raw-parameter rasterizer, Trainer._finish and optim.sharded_adam_step) run by 2 and 4 real ranks.

The ranks share cuda:0 and talk over gloo (RCCL refuses two ranks on one device; the driver's
8-GPU run uses RCCL through the same Trainer code, Trainer.Exchange only changes where the bytes
are staged and in which order a sum of more than two terms is added).  The ranks are spawned
before this process touches the GPU (conftest orders this module first).

Scenes:
* "small": 20k Gaussians @ 160x120, iterations 1..7 = ordinary steps (1, 5, 7), densify/prune
  (2, 4, 6) and opacity reset (3, 6);
* "cfg4": BASELINE.json configs[3]'s workload on one GPU — 1M Gaussians, 200 cameras, 1920x1080,
  SH 3 — iterations 1..4 with a densify at 2 that clones every small and splits every large
  Gaussian (1M -> 2M), then two ordinary sharded steps at 2M.  Its decisions are made
  insensitive to last-bit differences (gradient threshold 0, scales bimodal far from the
  clone/split boundary, opacities far from the prune threshold), so the comparison below is of
  values, not of a coin flip at a threshold.

The fused step on N ranks is the Gaussian-sharded one (rain_amd/sharded.py): each rank renders its
view from geometry the row owners preprocessed, and the owners run every view's per-Gaussian
backward, the sum over views in view order, and Adam on their rows.

Bars: replicas bit-identical after Trainer.sync_state (every parameter, Adam
moment and statistic), and equal to one process that renders the same views, sums their
raw-parameter gradients in view order, divides by N and steps, to <= 1e-4 relative L1 per tensor
for parameters and both moments.  What remains between the two is the blend backward's float
atomics (run-dependent order) and Adam turning a last-bit change of a cancelling gradient into a
full lr step.
"""
import hashlib
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
REL_L1 = 1e-4


class _LazyGT:
    """Seeded random ground-truth images, made on first use (200 views x 25 MB at 1080p)."""

    def __init__(self, n, W, H, dev):
        self.n, self.W, self.H, self.dev = n, W, H, dev
        self.cache = {}

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if i not in self.cache:
            g = torch.Generator().manual_seed(1000 + i)
            self.cache[i] = torch.rand(3, self.H, self.W, generator=g).to(self.dev)
        return self.cache[i]


SCENES = {
    "small": dict(P=20_000, W=160, H=120, V=6, iters=range(1, 8), expect=[False, True, False, True, False, True, False]),
    # world 8: the same scene with 16 cameras (a step takes 8 distinct views)
    "small8": dict(P=20_000, W=160, H=120, V=16, iters=range(1, 8),
                   expect=[False, True, False, True, False, True, False]),
    # c2f on, cameras of two image sizes: the low-pass value of a step must be the same
    # on every rank; 1000 Gaussians so that the schedule's H*W / N / 9pi exceeds its 0.3 floor
    # (160x120: 0.68, 128x96: 0.43)
    "mixed": dict(P=1_000, W=160, H=120, V=6, iters=range(1, 6), expect=[False, True, False, True, False], c2f=True),
    "cfg4": dict(P=1_000_000, W=1920, H=1080, V=200, iters=range(1, 5), expect=[False, True, False, False]),
}


# "mixed": image size per camera index; the first view groups of the tests' seed (5) mix both sizes
MIXED_SIZES = [(160, 120), (128, 96), (128, 96), (160, 120), (160, 120), (128, 96)]


def _c2f(name):
    return bool(SCENES[name].get("c2f", False))


def _opt(name):
    from rain_amd.gaussian_model import OptimizationParams

    if name in ("small", "small8", "mixed"):
        o = OptimizationParams(densify_from_iter=1, densification_interval=2, opacity_reset_interval=3)
        o.densify_grad_threshold = 2e-5  # some clones / splits at this tiny scale
        return o
    o = OptimizationParams(densify_from_iter=1, densification_interval=2, densify_until_iter=3)
    o.densify_grad_threshold = 0.0  # every Gaussian is selected: clone (small) or split (large)
    return o


def _scene(dev, name):
    from rain_amd import cameras, synthetic
    from rain_amd.gaussian_model import GaussianModel

    s = SCENES[name]
    P, W, H, V = s["P"], s["W"], s["H"], s["V"]
    if name == "mixed":
        cams = [cameras.fibonacci_cameras(V, w, h)[i].to(dev) for i, (w, h) in enumerate(MIXED_SIZES)]
    else:
        cams = [c.to(dev) for c in cameras.fibonacci_cameras(V, W, H)]
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    p = synthetic.random_gaussians(P, sh_degree=3, seed=6, bench=True)
    gen = torch.Generator().manual_seed(1)
    if name in ("small", "small8", "mixed"):
        gts = [torch.rand(3, int(c.image_height), int(c.image_width), generator=torch.Generator().manual_seed(20 + i))
               .to(dev) for i, c in enumerate(cams)]
        p["scaling"] = p["scaling"] + 0.3 * torch.randn(p["scaling"].shape, generator=gen)
    else:
        gts = _LazyGT(V, W, H, dev)
        # bimodal world scales, far on both sides of percent_dense * extent = 0.044: 90 % at
        # ~0.004 (cloned), 10 % at ~0.06 (split; their children 0.0375, pruned never)
        big = torch.rand(P, generator=gen) < 0.1
        base = torch.where(big, torch.tensor(0.06), torch.tensor(0.004)).log()
        p["scaling"] = base[:, None] + 0.1 * (2 * torch.rand((P, 3), generator=gen) - 1)
    g.set_params(p)
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    opt = _opt(name)
    g.training_setup(opt)
    return g, opt, cams, gts


def _snapshot(g):
    out = {n: p.detach() for n, p in zip(NAMES, g.params())}
    for n, p in zip(NAMES, g.params()):
        out["m_" + n] = g.optimizer.state[p]["exp_avg"].detach()
        out["v_" + n] = g.optimizer.state[p]["exp_avg_sq"].detach()
    out["accum"] = g.xyz_gradient_accum
    out["denom"] = g.denom
    out["maxr"] = g.max_radii2D
    return out


def _digest(t):
    return hashlib.blake2b(t.detach().contiguous().cpu().view(torch.uint8).numpy().tobytes(), digest_size=16).hexdigest()


def _worker(rank, world, port, out_path, name, chunk_rows=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    g, opt, cams, gts = _scene(dev, name)
    tr = Trainer(g, cams, gts, opt, cfg=TrainConfig(c2f=_c2f(name), seed=5), scene_extent=4.4)
    assert tr.fused and tr.world == world and not tr.exchange.direct and tr._owner is not None
    tr._owner.rec_chunk_rows = chunk_rows
    flags = [tr.step(it).densified for it in SCENES[name]["iters"]]
    tr.sync_state()  # parameters, moments and statistics are current only on their owner's rows
    torch.cuda.synchronize()
    snap = _snapshot(g)
    digests = {k: _digest(v) for k, v in snap.items()}
    if rank == 0:
        torch.save({"snap": {k: v.cpu() for k, v in snap.items()}, "digests": digests, "flags": flags},
                   f"{out_path}.{rank}")
    else:
        torch.save({"digests": digests, "flags": flags}, f"{out_path}.{rank}")
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _reference(dev, world, name):
    """One process: the world's views of each step through the fused forward/backward, raw-parameter
    gradients summed in view order then divided by the world size, statistics accumulated view
    after view, then the world-1 densify/Adam logic."""
    from rain_amd import fused
    from rain_amd.gaussian_model import low_pass_schedule
    from rain_amd.loss import l1_ssim_backward, l1_ssim_forward
    from rain_amd.train import TrainConfig, Trainer, ViewSampler

    g, opt, cams, gts = _scene(dev, name)
    tr = Trainer(g, cams, gts, opt, cfg=TrainConfig(c2f=_c2f(name), seed=5), scene_extent=4.4)
    sampler = ViewSampler(len(cams), world, seed=5)
    bg = torch.zeros(3, device=dev)
    flags = []
    lp = 0.3
    for it in SCENES[name]["iters"]:
        g.update_learning_rate(it)
        views = sampler.next_group()
        if _c2f(name) and it == 1:  # train.py:95-107 on the step's first view, as one process would
            c0 = cams[views[0]]
            lp = low_pass_schedule(c0.image_height, c0.image_width, g.get_xyz.shape[0], 300.0)
            assert lp > 0.3 and len({(int(cams[v].image_width), int(cams[v].image_height)) for v in views}) > 1
        acc = None
        for v in views:
            color, radii, depth, st = fused.forward(g, cams[v], bg, lp)
            _, _, ws = l1_ssim_forward(color, gts[v], opt.lambda_dssim)
            dimg = l1_ssim_backward(color, gts[v], opt.lambda_dssim, ws)
            grads = {n: torch.empty_like(p) for n, p in zip(NAMES, g.params())}
            stats = (g.xyz_gradient_accum, g.denom, g.max_radii2D) if it < opt.densify_until_iter else None
            fused.backward(st, dimg, grads, stats)
            if acc is None:
                acc = [grads[n].clone() for n in NAMES]
            else:
                for a, n in zip(acc, NAMES):
                    a += grads[n]
        g.bind_flat_grad()
        for a, p in zip(acc, g.params()):
            p.grad.copy_(a * (1.0 / world))
        flags.append(tr._densify_and_adam(it))
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in _snapshot(g).items()}, flags


def _rel_l1(x, y):
    x, y = x.double(), y.double()
    den = float(y.abs().sum())
    return float((x - y).abs().sum()) / den if den > 0 else float((x - y).abs().sum())


def _run(tmp_path, world, name, chunk_rows=None):
    if torch.cuda.device_count() < 1:  # does not initialise the GPU in this process
        pytest.skip("no HIP device")
    out = str(tmp_path / "rank")
    mp.start_processes(_worker, args=(world, _free_port(), out, name, chunk_rows), nprocs=world, join=True,
                       start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    for r in rs[1:]:
        assert r["digests"] == rs[0]["digests"], [k for k in r["digests"] if r["digests"][k] != rs[0]["digests"][k]]
    assert rs[0]["flags"] == SCENES[name]["expect"]
    r0 = rs[0]["snap"]
    ref, flags = _reference(torch.device("cuda:0"), world, name)
    assert flags == rs[0]["flags"]
    assert r0["xyz"].shape == ref["xyz"].shape, "densify made different decisions"
    errs = {}
    for n in NAMES:
        for k in (n, "m_" + n, "v_" + n):
            errs[k] = _rel_l1(r0[k], ref[k])
    print(f"\n[{name} world {world}] P = {r0['xyz'].shape[0]}, rel L1: " +
          ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    bad = {k: v for k, v in errs.items() if not v <= REL_L1}
    assert not bad, bad
    # statistics: visibility / radius can flip for a Gaussian whose projection changed by an ulp
    assert (r0["denom"] != ref["denom"]).float().mean().item() <= 1e-4
    dm = (r0["maxr"] - ref["maxr"]).abs()
    assert (dm > 0).float().mean().item() <= 1e-4 and dm.max().item() <= 1.0
    assert _rel_l1(r0["accum"], ref["accum"]) <= REL_L1
    return r0


def test_view_sharded_fused_step_two_ranks(tmp_path):
    _run(tmp_path, 2, "small")


def test_view_sharded_fused_step_two_ranks_chunked_exchange(tmp_path):
    """The record exchange in row chunks of 256 (40 chunks per owner; rr_backward_records' chunked
    layout, one all-to-all and one owner launch per chunk) against the same bars."""
    _run(tmp_path, 2, "small", chunk_rows=256)


@pytest.mark.parametrize("world", [2, 4])
def test_view_sharded_fused_step_c2f_mixed_image_sizes(tmp_path, world):
    """c2f low-pass on and views of two image sizes in one step: every rank must render and run its
    owner backward with the step's one low-pass value (from the first view of the group), equal to
    one process rendering the same views (ranks used their own view's size)."""
    _run(tmp_path, world, "mixed")


def test_view_sharded_fused_step_four_ranks(tmp_path):
    """World 4: the flat buffers padded to 4 slices, as in the driver's N = 4 / 8 runs."""
    _run(tmp_path, 4, "small")


def test_view_sharded_fused_step_eight_ranks(tmp_path):
    """World 8, the node size of BASELINE configs[3] / [4]: eight gloo processes on one GPU, Q = 2560
    owned rows per rank, 7 peers in every all-to-all; replicas bit-identical and equal to one
    process summing the same 8 views."""
    _run(tmp_path, 8, "small8")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_view_sharded_fused_step_cfg4_size(tmp_path, world):
    """BASELINE configs[3]'s workload (1M Gaussians, 200 cameras, 1080p) through the sharded step,
    including a densify at size (1M -> 2M) and ordinary steps after it; at world 8 the partition
    the driver's 8-GPU run uses (Q = 125,184 rows per rank before the densify)."""
    r0 = _run(tmp_path, world, "cfg4")
    assert r0["xyz"].shape[0] == 2_000_000


def _worker_rccl(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)  # bench.py's init
    from rain_amd.train import TrainConfig, Trainer

    g, opt, cams, gts = _scene(dev, "small")
    tr = Trainer(g, cams, gts, opt, cfg=TrainConfig(c2f=False, seed=5), scene_extent=4.4, exchange=True)
    assert tr.fused and tr.sharded and tr.exchange.direct and tr._owner is not None
    flags = [tr.step(it).densified for it in SCENES["small"]["iters"]]
    tr.sync_state()
    torch.cuda.synchronize()
    torch.save({"snap": {k: v.cpu() for k, v in _snapshot(g).items()}, "flags": flags}, f"{out_path}.{rank}")
    torch.distributed.destroy_process_group()


def test_rccl_exchange_path_one_rank(tmp_path):
    """The RCCL branch of Trainer.Exchange (all_to_all_single / all_gather_into_tensor on device
    tensors) and bench.py's init_process_group("nccl", device_id=...) on a one-rank group (the box
    has one GPU): the Gaussian-sharded step (rain_amd/sharded.py), forced at world 1, must equal the
    plain single-GPU step (Adam fused into the backward) through ordinary, densify and reset
    iterations."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no HIP device")
    out = str(tmp_path / "rccl")
    mp.start_processes(_worker_rccl, args=(1, _free_port(), out), nprocs=1, join=True, start_method="spawn")
    got = torch.load(out + ".0", weights_only=True)
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    g, opt, cams, gts = _scene(dev, "small")
    tr = Trainer(g, cams, gts, opt, cfg=TrainConfig(c2f=False, seed=5), scene_extent=4.4)
    assert tr.fused and not tr.sharded
    flags = [tr.step(it).densified for it in SCENES["small"]["iters"]]
    torch.cuda.synchronize()
    ref = {k: v.cpu() for k, v in _snapshot(g).items()}
    assert flags == got["flags"] == SCENES["small"]["expect"]
    for k in ref:
        assert got["snap"][k].shape == ref[k].shape, k
        e = _rel_l1(got["snap"][k], ref[k])
        assert e <= REL_L1, (k, e)
