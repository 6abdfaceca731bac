"""Training step around the rasterizer.

One call of ``Trainer.step`` is one iteration of train.py:71-147 — learning-rate update, SH-degree
ramp, RAIN-GS low-pass schedule, render, L1+SSIM loss, backward, densification statistics,
periodic densify/prune and opacity reset, Adam — executed on every rank of a view-sharded
data-parallel group:

* every rank holds the full Gaussian set and Adam state (replicas);
* at step s rank r renders view ``perm[s*N + r]`` of a permutation shared by all ranks (the
  reference's pop-random-without-replacement, train.py:87-89, done globally);
* after backward ONE all-reduce (SUM) covers every parameter gradient (they are views into one
  flat buffer) plus the per-view densification increments; gradients are then averaged, the
  increments summed (N views add their norms exactly like N sequential iterations would); a second,
  small all-reduce (MAX) merges max_radii2D;
* Adam / densify then run identically on every rank (same RNG seed), so replicas stay equal.

With world_size 1 there is no collective and the step is the reference's iteration.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .gaussian_model import GaussianModel, OptimizationParams, low_pass_schedule
from .loss import fused_l1_ssim_loss
from .renderer import PipelineParams, render


@dataclass
class TrainConfig:
    c2f: bool = True                 # RAIN-GS coarse-to-fine low-pass (train.py:95-107)
    c2f_every_step: int = 1000
    c2f_max_lowpass: float = 300.0
    warmup_iter: int = 0             # abe_split warm-up (train.py:38-39,138)
    ours: bool = False               # SH ramp from 5000 (train.py:79-85)
    white_background: bool = False
    seed: int = 0
    densify: bool = True


class ViewSampler:
    """Shared permutation of camera indices; rank r takes the r-th of each group of N."""

    def __init__(self, n_views: int, world: int, seed: int = 0):
        self.n, self.world = n_views, world
        self.rng = random.Random(seed)
        self.perm: list[int] = []

    def next_group(self):
        out = []
        for _ in range(self.world):
            if not self.perm:
                self.perm = list(range(self.n))
                self.rng.shuffle(self.perm)
            out.append(self.perm.pop())
        return out


@dataclass
class StepInfo:
    loss: float | None
    num_gaussians: int
    view: int
    low_pass: float
    densified: bool = False


class Trainer:
    def __init__(self, gaussians: GaussianModel, cameras, gt_images, opt: OptimizationParams | None = None,
                 pipe: PipelineParams | None = None, cfg: TrainConfig | None = None, scene_extent: float = 1.0,
                 group=None, loss_fn=None, fused: bool | None = None):
        self.g = gaussians
        self.cams = cameras
        self.gt = gt_images
        self.opt = opt or OptimizationParams()
        self.pipe = pipe or PipelineParams()
        self.cfg = cfg or TrainConfig()
        self.extent = scene_extent
        self.group = group
        # loss_fn(image, gt, lambda_dssim) -> scalar; default: the fused HIP L1+SSIM kernels
        self.loss_fn = loss_fn or (lambda img, gt, lam: fused_l1_ssim_loss(img, gt, lam)[0])
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.sampler = ViewSampler(len(cameras), self.world, self.cfg.seed)
        dev = gaussians.device
        self.background = torch.tensor([1, 1, 1] if self.cfg.white_background else [0, 0, 0], dtype=torch.float32,
                                       device=dev)
        self.low_pass = 0.3
        self.densify_gen = torch.Generator(device=dev).manual_seed(self.cfg.seed + 12345)
        if self.cfg.warmup_iter > 0:
            self.opt.densify_until_iter += self.cfg.warmup_iter
        # Fused step (rain_amd.fused): getters + their backward inside the rasterizer, gradients
        # written straight into the flat buffer, densification statistics folded into the backward
        # kernel, no autograd graph.  Needs the default loss and the SH / scale-rotation path.
        plain_pipe = not (self.pipe.convert_SHs_python or self.pipe.compute_cov3D_python)
        auto = dev.type == "cuda" and loss_fn is None and plain_pipe
        self.fused = auto if fused is None else bool(fused)
        if self.fused and not (dev.type == "cuda" and loss_fn is None and plain_pipe):
            raise ValueError("fused step needs a HIP device, the default loss and the default pipeline")

    def _low_pass_and_view(self, iteration):
        g, opt, cfg = self.g, self.opt, self.cfg
        g.update_learning_rate(iteration)
        if cfg.ours:
            if iteration >= 5000 and iteration % 1000 == 0:
                g.oneupSHdegree()
        elif iteration % 1000 == 0:
            g.oneupSHdegree()
        views = self.sampler.next_group()
        vidx = views[self.rank]
        cam = self.cams[vidx]
        if cfg.c2f:
            if iteration == 1 or (iteration % cfg.c2f_every_step == 0 and iteration < opt.densify_until_iter):
                self.low_pass = low_pass_schedule(cam.image_height, cam.image_width, g.get_xyz.shape[0],
                                                  cfg.c2f_max_lowpass)
        else:
            self.low_pass = 0.3
        return vidx, cam

    def _events(self, iteration):
        """(densify/prune now, opacity reset now) — train.py:136-143."""
        opt, cfg = self.opt, self.cfg
        if iteration >= opt.densify_until_iter:
            return False, False
        densify = cfg.densify and iteration > opt.densify_from_iter and iteration % opt.densification_interval == 0
        reset = iteration % opt.opacity_reset_interval == 0 or (cfg.white_background and
                                                                 iteration == opt.densify_from_iter)
        return densify, reset

    def _densify_and_adam(self, iteration, adam_done=False):
        g, opt, cfg = self.g, self.opt, self.cfg
        densified = False
        if iteration < opt.densify_until_iter:
            if cfg.densify and iteration > opt.densify_from_iter and iteration % opt.densification_interval == 0:
                size_threshold = 20 if iteration > opt.opacity_reset_interval else None
                abe_split = iteration <= cfg.warmup_iter
                g.densify_and_prune(opt.densify_grad_threshold, 0.005, self.extent, size_threshold, N=2,
                                    abe_split=abe_split, generator=self.densify_gen)
                densified = True
            if iteration % opt.opacity_reset_interval == 0 or (cfg.white_background and
                                                               iteration == opt.densify_from_iter):
                g.reset_opacity()
        if iteration < opt.iterations and not adam_done:
            # after densify_and_prune the parameters are new tensors with grad None, so this step
            # skips them, exactly as the reference's optimizer.step() does (train.py:145-147)
            g.optimizer.step()
            g.optimizer.zero_grad(set_to_none=True)
        return densified

    def step(self, iteration: int, sync_loss: bool = False) -> StepInfo:
        if self.fused:
            return self._step_fused(iteration, sync_loss)
        return self._step_autograd(iteration, sync_loss)

    def _step_fused(self, iteration: int, sync_loss: bool) -> StepInfo:
        from . import fused
        from .loss import l1_ssim_backward, l1_ssim_forward

        g, opt = self.g, self.opt
        vidx, cam = self._low_pass_and_view(iteration)
        P = g.get_xyz.shape[0]
        densify_phase = iteration < opt.densify_until_iter
        # Single GPU, and no densify/prune or opacity reset this iteration (they replace parameter
        # tensors before the reference's optimizer.step()): the Adam step runs inside the backward
        # kernel and the gradients never exist in HBM.
        densify_now, reset_now = self._events(iteration)
        fuse_adam = (self.world == 1 and iteration < opt.iterations and not densify_now and not reset_now
                     and hasattr(g.optimizer, "fused_step"))
        extra = 2 * P if (self.world > 1 and densify_phase) else 0
        flat = None if fuse_adam else g.bind_flat_grad(extra=extra, zero=False)  # backward overwrites all grads
        with torch.no_grad():
            image, radii, _depth, st = fused.forward(g, cam, self.background, self.low_pass)
            gt = self.gt[vidx]
            loss, _parts, lws = l1_ssim_forward(image, gt, opt.lambda_dssim)
            dimg = l1_ssim_backward(image, gt, opt.lambda_dssim, lws)
            grads = None if fuse_adam else dict(
                xyz=g._xyz.grad, f_dc=g._features_dc.grad, f_rest=g._features_rest.grad, opacity=g._opacity.grad,
                scaling=g._scaling.grad, rotation=g._rotation.grad)
            nparam = None if flat is None else flat.numel() - extra
            stats = None
            local_max = None
            if densify_phase:
                if self.world > 1:
                    local_max = g.max_radii2D.clone()
                    stats = (flat[nparam:nparam + P], flat[nparam + P:], local_max)
                else:
                    stats = (g.xyz_gradient_accum, g.denom, g.max_radii2D)
            fused.backward(st, dimg, grads, stats, adam=g.optimizer.fused_step(g) if fuse_adam else None)
            if self.world > 1:
                dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
                flat[:nparam].mul_(1.0 / self.world)
                if densify_phase:
                    dist.all_reduce(local_max, op=dist.ReduceOp.MAX, group=self.group)
                    g.max_radii2D = local_max
                    g.xyz_gradient_accum += flat[nparam:nparam + P].unsqueeze(1)
                    g.denom += flat[nparam + P:].unsqueeze(1)
            densified = self._densify_and_adam(iteration, adam_done=fuse_adam)
        return StepInfo(loss=float(loss.item()) if sync_loss else None, num_gaussians=g.get_xyz.shape[0],
                        view=vidx, low_pass=self.low_pass, densified=densified)

    def _step_autograd(self, iteration: int, sync_loss: bool = False) -> StepInfo:
        """The reference-API step: render() through GaussianRasterizer + autograd (train.py:109-147)."""
        g, opt = self.g, self.opt
        vidx, cam = self._low_pass_and_view(iteration)
        P = g.get_xyz.shape[0]
        densify_phase = iteration < opt.densify_until_iter
        flat = g.bind_flat_grad(extra=2 * P if (self.world > 1 and densify_phase) else 0)

        pkg = render(cam, g, self.pipe, self.background, low_pass=self.low_pass)
        image, vsp, vis, radii = pkg["render"], pkg["viewspace_points"], pkg["visibility_filter"], pkg["radii"]
        gt = self.gt[vidx]
        # (1-λ)·L1 + λ·(1-SSIM) (train.py:113-114), by default one fused HIP forward/backward
        loss = self.loss_fn(image, gt, opt.lambda_dssim)
        loss.backward()

        with torch.no_grad():
            nparam = flat.numel() - (2 * P if (self.world > 1 and densify_phase) else 0)
            if self.world > 1:
                if densify_phase:
                    acc = flat[nparam:nparam + P]
                    den = flat[nparam + P:]
                    acc[vis] = torch.norm(vsp.grad[vis, :2], dim=-1)
                    den[vis] = 1.0
                dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
                flat[:nparam].mul_(1.0 / self.world)
            if densify_phase:
                if self.world > 1:
                    local = g.max_radii2D.clone()
                    local[vis] = torch.max(local[vis], radii[vis].float())
                    dist.all_reduce(local, op=dist.ReduceOp.MAX, group=self.group)
                    g.max_radii2D = local
                    g.xyz_gradient_accum += flat[nparam:nparam + P].unsqueeze(1)
                    g.denom += flat[nparam + P:].unsqueeze(1)
                else:
                    g.max_radii2D[vis] = torch.max(g.max_radii2D[vis], radii[vis].float())
                    g.add_densification_stats(vsp, vis)
            densified = self._densify_and_adam(iteration)
        return StepInfo(loss=float(loss.item()) if sync_loss else None, num_gaussians=g.get_xyz.shape[0],
                        view=vidx, low_pass=self.low_pass, densified=densified)
