"""Training step around the rasterizer.

One call of ``Trainer.step`` is one iteration of train.py:71-147 — learning-rate update, SH-degree
ramp, RAIN-GS low-pass schedule, render, L1+SSIM loss, backward, densification statistics,
periodic densify/prune and opacity reset, Adam — executed on every rank of a view-sharded
data-parallel group:

* every rank holds the full Gaussian set and Adam state (replicas);
* at step s rank r renders view ``perm[s*N + r]`` of a permutation shared by all ranks (the
  reference's pop-random-without-replacement, train.py:87-89, done globally);
* after backward the gradients (views into one flat buffer) are reduce-scattered (SUM); each rank
  applies Adam, scaled by 1/N, to its 1/N slice of the flat parameter / moment buffers and the
  parameter buffer is all-gathered — the bytes of one all-reduce, 1/N of the optimizer work
  (Trainer._finish);
* densification statistics accumulate per rank and are merged (SUM, and MAX for max_radii2D) only
  on densify iterations, where the Adam moments are all-gathered too; densify / prune / opacity
  reset then run identically on every rank (same RNG seed), so replicas stay equal (N views add
  their norms exactly like N sequential iterations would).

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
from .optim import sharded_adam_step
from .renderer import PipelineParams, render


@dataclass
class TrainConfig:
    c2f: bool = True                 # RAIN-GS coarse-to-fine low-pass (train.py:95-107)
    c2f_every_step: int = 1000
    c2f_max_lowpass: float = 300.0
    warmup_iter: int = 0             # abe_split warm-up (train.py:38-39,138)
    ours: bool = False               # SH ramp from 5000 (train.py:79-85)
    ours_new: bool = False           # --ours_new: SH ramp from 5000, learning-rate schedule shifted by
                                     # warmup_iter (train.py:73-77; the reference's flag also sets
                                     # warmup_iter = 10000, train.py:279-280)
    white_background: bool = False
    seed: int = 0
    densify: bool = True


def _serves_cuda_with_nccl(group) -> bool:
    """True when the group's collectives on HIP tensors go through RCCL: backend "nccl", or a
    mixed backend string that maps cuda to nccl (e.g. "cuda:nccl,cpu:gloo")."""
    b = str(dist.get_backend(group)).lower()
    if ":" not in b:
        return b == "nccl"
    return any(part.strip() == "cuda:nccl" for part in b.split(","))


class Exchange:
    """The step's collectives over `group`.

    RCCL (the group serves HIP tensors with "nccl") runs them on the device tensors directly, in
    RCCL's own reduction order.  Otherwise (gloo: the multi-process CPU tests and the multi-rank
    tests on one GPU) the tensors are staged through host memory and every SUM is formed by
    gathering all ranks' contributions and adding them in rank order, ((x_0 + x_1) + x_2) + ...:
    deterministic, independent of how the buffer is split into collectives (the chunked exchange
    equals the serial one bitwise), and the order in which one process accumulating the same
    views adds them.  The two backends can therefore differ in the last bits of a sum of more
    than two terms."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.direct = _serves_cuda_with_nccl(group)

    def _gather_host(self, t: torch.Tensor):
        h = t.detach().to("cpu", copy=True).contiguous()
        parts = [torch.empty_like(h) for _ in range(self.world)]
        dist.all_gather(parts, h, group=self.group)
        return parts

    def reduce_scatter_sum(self, out: torch.Tensor, inp: torch.Tensor):
        """out <- slice `rank` of the elementwise SUM over ranks of inp (inp.numel() = world * out.numel())."""
        if self.direct:
            dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group)
            return
        S = out.numel()
        parts = self._gather_host(inp)
        acc = parts[0][self.rank * S:(self.rank + 1) * S].clone()
        for p in parts[1:]:
            acc += p[self.rank * S:(self.rank + 1) * S]
        out.copy_(acc)

    def all_gather_inplace(self, buf: torch.Tensor, lo: int, S: int):
        """Every rank contributes buf[lo:lo+S] (lo = rank*S within buf); afterwards buf holds all slices."""
        if self.direct:
            dist.all_gather_into_tensor(buf, buf[lo:lo + S], group=self.group)
            return
        out = torch.empty(buf.numel(), dtype=buf.dtype)
        dist.all_gather_into_tensor(out, buf[lo:lo + S].to("cpu", copy=True), group=self.group)
        buf.copy_(out)

    def all_to_all(self, recv: torch.Tensor, send: torch.Tensor, async_op: bool = False):
        """Chunk j of `send` (N equal chunks) goes to rank j; chunk i of `recv` comes from rank i.
        async_op (RCCL only): returns the collective's work handle; its wait() makes the current
        stream wait for it.  Otherwise the exchange is complete on return (None)."""
        if self.direct:
            return dist.all_to_all_single(recv, send, group=self.group, async_op=async_op)
        h = send.detach().to("cpu", copy=True).contiguous()
        out = torch.empty_like(h)
        dist.all_to_all_single(out, h, group=self.group)
        recv.copy_(out)
        return None

    def all_gather_rows(self, t: torch.Tensor, Q: int, lo: int):
        """Rank r contributes rows [r*Q, r*Q + Q) of t (rows past t's end as padding); afterwards
        every rank's t holds every rank's rows."""
        P = t.shape[0]
        flat = t.view(P, -1)
        n = max(0, min(Q, P - lo))
        send = torch.zeros((Q, flat.shape[1]), dtype=t.dtype, device=t.device)
        if n:
            send[:n].copy_(flat[lo:lo + n])
        if self.direct:
            out = torch.empty((self.world * Q, flat.shape[1]), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, send, group=self.group)
        else:
            out = torch.empty((self.world * Q, flat.shape[1]), dtype=t.dtype)
            dist.all_gather_into_tensor(out, send.cpu(), group=self.group)
        flat.copy_(out[:P])

    def all_reduce(self, t: torch.Tensor, op):
        if self.direct:
            dist.all_reduce(t, op=op, group=self.group)
            return
        if op != dist.ReduceOp.SUM:  # MAX / MIN: order-free
            h = t.to("cpu", copy=True)
            dist.all_reduce(h, op=op, group=self.group)
            t.copy_(h)
            return
        parts = self._gather_host(t)
        acc = parts[0].clone()
        for p in parts[1:]:
            acc += p
        t.copy_(acc)


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
                 group=None, loss_fn=None, fused: bool | None = None, exchange: bool | None = None):
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
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        # the sharded exchange path runs whenever world > 1; exchange=True forces it at world 1
        # too (a one-rank group: exercises the collectives, e.g. RCCL, on a single GPU)
        self.sharded = self.world > 1 or (bool(exchange) and dist_on)
        self.exchange = Exchange(group) if self.sharded else None
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
        self._bin_cache = None
        self.reuse_binning = True  # fused step: one native forward call over a reused binning buffer
        # fused step, single GPU: the backward of step s also preprocesses step s+1's frame on the
        # parameters it has just stepped (rain_amd.fused.prepare_next / include/rain_raster.h
        # rr_next_frame); step s+1 then renders from that geometry.  Step s+1's view, learning rate,
        # SH degree and low-pass are decided at step s (after s's optimizer block is built), in the
        # order the unfused step would decide them.  So with fuse_next the Trainer's own state (the
        # view sampler's position, the next step's learning rate and low-pass) is one step ahead of
        # the last completed step: a checkpoint taken between steps records step s+1's decisions.
        # The precomputed geometry itself is dropped if the parameters change between the steps
        # (replaced tensors, or in-place edits such as a manual reset or a checkpoint restore: the
        # tensors' version counters), and step s+1 then preprocesses normally.
        self.fuse_next = True
        self._pending = None  # (iteration, view index, camera, low_pass, NextFrame or None, params signature)
        self._shard = None
        # the fused step on N > 1 ranks (or a forced exchange): Gaussian-sharded, view-parallel
        # (rain_amd/sharded.py); the autograd step keeps the replicated gradient exchange
        self._owner = None
        if self.sharded and self.fused:
            from .sharded import ShardedStep

            self._owner = ShardedStep(self.exchange, self.rank, self.world)
        if self.fused and not (dev.type == "cuda" and loss_fn is None and plain_pipe):
            raise ValueError("fused step needs a HIP device, the default loss and the default pipeline")

    def _low_pass_and_view(self, iteration):
        g, opt, cfg = self.g, self.opt, self.cfg
        if cfg.ours_new:  # train.py:73-75: the schedule starts after the warm-up
            if iteration >= cfg.warmup_iter:
                g.update_learning_rate(iteration - cfg.warmup_iter)
        else:
            g.update_learning_rate(iteration)
        if cfg.ours or cfg.ours_new:
            if iteration >= 5000 and iteration % 1000 == 0:
                g.oneupSHdegree()
        elif iteration % 1000 == 0:
            g.oneupSHdegree()
        views = self.sampler.next_group()
        self._views = views
        vidx = views[self.rank]
        cam = self.cams[vidx]
        if cfg.c2f:
            if iteration == 1 or (iteration % cfg.c2f_every_step == 0 and iteration < opt.densify_until_iter):
                # one value per step on every rank: the schedule reads the image size of the step's
                # FIRST view (views[0], the one a single process would render first), so ranks whose
                # own views differ in size still blur every Gaussian alike
                c0 = self.cams[views[0]]
                self.low_pass = low_pass_schedule(c0.image_height, c0.image_width, g.get_xyz.shape[0],
                                                  cfg.c2f_max_lowpass)
        else:
            self.low_pass = 0.3
        return vidx, cam

    def _sh_steps_up(self, iteration) -> bool:
        """Whether _low_pass_and_view(iteration) raises the active SH degree (train.py:79-85)."""
        g, cfg = self.g, self.cfg
        if g.active_sh_degree >= g.max_sh_degree:
            return False
        if cfg.ours or cfg.ours_new:
            return iteration >= 5000 and iteration % 1000 == 0
        return iteration % 1000 == 0

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

    def _step_owner(self, iteration: int, sync_loss: bool) -> StepInfo:
        """The fused step on the Gaussian-sharded ranks (rain_amd/sharded.py): one view per rank, Adam
        of the owned rows inside the per-Gaussian backward.  Densify / prune and opacity reset
        (train.py:136-143) gather full replicas first and run identically on every rank; on a
        densify iteration the reference's optimizer.step() finds only replaced parameters (no step),
        on a reset-only iteration it steps every group but the replaced opacity."""
        from .diff_gaussian_rasterization import _C
        from .loss import l1_ssim_forward_backward

        g, opt = self.g, self.opt
        if not hasattr(g.optimizer, "fused_step"):  # before any collective of the step starts
            raise ValueError("the Gaussian-sharded fused step applies Adam inside its owner kernel: the model's "
                             "optimizer must be rain_amd.optim.FusedAdam (GaussianModel.training_setup builds one); "
                             "use Trainer(fused=False) for another optimizer")
        vidx, _cam = self._low_pass_and_view(iteration)
        cams = [self.cams[v] for v in self._views]
        densify_phase = iteration < opt.densify_until_iter
        densify_now, reset_now = self._events(iteration)
        adam = None
        if iteration < opt.iterations and not densify_now:
            adam = g.optimizer.fused_step(g, skip=("opacity",) if reset_now else ())
        stats = (g.xyz_gradient_accum, g.denom, g.max_radii2D) if densify_phase else None
        gt = self.gt[vidx]
        lam = opt.lambda_dssim

        def loss_fn(image):
            loss, _parts, dimg = l1_ssim_forward_backward(image, gt, lam)
            return dimg, loss

        with torch.no_grad():
            _image, loss = self._owner.step(g, cams, self.background, self.low_pass, _C.frame_flags(), loss_fn, adam,
                                            stats)
            densified = False
            if densify_now or reset_now:
                self._owner.sync_replicas(g)
                densified = self._densify_and_adam(iteration, adam_done=True)
        return StepInfo(loss=float(loss.item()) if sync_loss else None, num_gaussians=g.get_xyz.shape[0],
                        view=vidx, low_pass=self.low_pass, densified=densified)

    def sync_state(self):
        """Make every rank's GaussianModel a full, current replica (parameters, Adam moments,
        densification statistics), e.g. before a checkpoint, an evaluation render or the end of
        training.  Gaussian-sharded fused step: all-gather the row blocks.  Replicated (autograd)
        step: merge the statistics (SUM / MAX: consumes them, like densify) and gather the moments."""
        if self._owner is not None:
            self._owner.sync_replicas(self.g)
        elif self.sharded:
            self.sync_densify_stats()
            self.sync_optimizer_state()

    def _params_signature(self):
        """Identity and in-place version of every parameter tensor (the fused backward's own
        in-place Adam writes go through raw pointers and leave the versions unchanged)."""
        return tuple((p.data_ptr(), p._version) for p in self.g.params())

    def _step_fused(self, iteration: int, sync_loss: bool) -> StepInfo:
        from . import fused
        from .loss import l1_ssim_forward_backward

        if self._owner is not None:
            return self._step_owner(iteration, sync_loss)

        if self._bin_cache is None:
            self._bin_cache = fused.BinningCache()
        g, opt = self.g, self.opt
        pend, self._pending = self._pending, None
        if pend is not None and pend[0] == iteration:  # decided (and maybe preprocessed) by step s-1
            _it, vidx, cam, self.low_pass, nxt, sig = pend
            if nxt is not None and (nxt.P != g.get_xyz.shape[0] or nxt.frame.D != g.active_sh_degree
                                    or sig != self._params_signature()):
                nxt = None  # the parameters changed since step s-1's backward preprocessed this frame
        else:
            vidx, cam = self._low_pass_and_view(iteration)
            nxt = None
        densify_phase = iteration < opt.densify_until_iter
        densify_now, reset_now = self._events(iteration)
        # Single GPU, and no densify/prune or opacity reset this iteration (they replace parameter
        # tensors before the reference's optimizer.step()): the Adam step runs inside the backward
        # kernel and the gradients never exist in HBM.
        fuse_adam = (not self.sharded and iteration < opt.iterations and not densify_now and not reset_now
                     and hasattr(g.optimizer, "fused_step"))
        if self.sharded:
            g.pack_flat_state(self.world)
        flat = None if fuse_adam else g.bind_flat_grad(zero=False, pad_to=self.world)  # backward overwrites all
        # Everything the backward needs from Python is prepared BEFORE the forward: the forward's one
        # host wait (the pair-count read-back, rasterizer_impl.cu:273) returns when the device is at
        # this frame's depth sort, and from there the host must enqueue the binning, the blends, the
        # loss and the backward faster than the device runs them (~0.45 ms of kernels); the Adam
        # block (step counts, bias corrections) does not depend on the frame.
        adam = g.optimizer.fused_step(g) if fuse_adam else None
        grads = None if fuse_adam else dict(
            xyz=g._xyz.grad, f_dc=g._features_dc.grad, f_rest=g._features_rest.grad, opacity=g._opacity.grad,
            scaling=g._scaling.grad, rotation=g._rotation.grad)
        # densification statistics accumulate per rank; ranks merge them only when densify consumes
        # them (_finish)
        stats = (g.xyz_gradient_accum, g.denom, g.max_radii2D) if densify_phase else None
        gt = self.gt[vidx]
        # the next step's frame, preprocessed by this step's backward: only when this step's Adam runs
        # inside that backward (no densify / reset replacing parameters) and the SH degree stays
        next_frame = None
        if (fuse_adam and self.fuse_next and not self.sharded and iteration + 1 < opt.iterations
                and not self._sh_steps_up(iteration + 1)):
            low_pass_now = self.low_pass
            vidx1, cam1 = self._low_pass_and_view(iteration + 1)
            next_frame = fused.prepare_next(g, cam1, self.background, self.low_pass)
            self._pending = [iteration + 1, vidx1, cam1, self.low_pass, next_frame, None]
            self.low_pass = low_pass_now
        with torch.no_grad():
            cache = self._bin_cache if self.reuse_binning else None
            if nxt is not None:
                image, radii, _depth, st = fused.forward_next(nxt, g, cache=cache)
            else:
                image, radii, _depth, st = fused.forward(g, cam, self.background, self.low_pass, cache=cache)
            # loss and dL/dimage in one call (bitwise the separate forward / backward)
            loss, _parts, dimg = l1_ssim_forward_backward(image, gt, opt.lambda_dssim)
            fused.backward(st, dimg, grads, stats, adam=adam, next_frame=next_frame)
            densified = self._finish(iteration, flat, densify_now, reset_now, adam_done=fuse_adam)
        if self._pending is not None:  # the parameters the pending geometry was computed from
            self._pending[5] = self._params_signature()
        return StepInfo(loss=float(loss.item()) if sync_loss else None, num_gaussians=g.get_xyz.shape[0],
                        view=vidx, low_pass=self.low_pass, densified=densified)

    def _finish(self, iteration, flat, densify_now, reset_now, adam_done=False):
        """Gradient exchange + optimizer step + densification (train.py:132-147) after the backward.

        N = 1: densify / reset, then Adam (unless the backward kernel already applied it).
        N > 1, ordinary iteration (no densify / reset): reduce-scatter the flat gradient SUM, each
        rank runs Adam (scaled by 1/N) on its 1/N slice of the flat parameter / moment buffers, then
        all-gathers the parameter buffer — the bytes of one all-reduce, 1/N of the optimizer work.
        N > 1, densify / reset iteration (1 in 100): all-gather the Adam moments (each rank kept only
        its slice current), merge the per-rank densification statistics (SUM / MAX) when densify
        runs, all-reduce the gradients if an optimizer step follows (reset only: the reference
        steps every group but the replaced opacity), then the N = 1 logic on identical replicas."""
        g, opt = self.g, self.opt
        if not self.sharded:
            return self._densify_and_adam(iteration, adam_done=adam_done)
        fp, fm, fv, _offs, n = g.pack_flat_state(self.world)
        S = n // self.world
        lo = self.rank * S
        if not (densify_now or reset_now):
            if iteration < opt.iterations:
                if self._shard is None or self._shard.numel() != S or self._shard.device != flat.device:
                    self._shard = torch.empty(S, dtype=flat.dtype, device=flat.device)
                self.exchange.reduce_scatter_sum(self._shard, flat[:n])
                sharded_adam_step(g.optimizer, g.params(), _offs, self._shard, lo, 1.0 / self.world)
                self.exchange.all_gather_inplace(fp, lo, S)
                for p in g.params():
                    p.grad = None
            return False
        self.exchange.all_gather_inplace(fm, lo, S)
        self.exchange.all_gather_inplace(fv, lo, S)
        if densify_now:
            self.sync_densify_stats()
        elif iteration < opt.iterations:
            self.exchange.all_reduce(flat[:n], dist.ReduceOp.SUM)
            flat[:n].mul_(1.0 / self.world)
        return self._densify_and_adam(iteration)

    def sync_densify_stats(self):
        """Merge the per-rank densification statistics in place: gradient-norm sums and view
        counts add (SUM), max_radii2D takes the MAX — what N sequential views would have left.
        Ranks then hold the merged values, so call it only where they are consumed and reset
        (densify), or on copies."""
        g = self.g
        if self.sharded:
            self.exchange.all_reduce(g.xyz_gradient_accum, dist.ReduceOp.SUM)
            self.exchange.all_reduce(g.denom, dist.ReduceOp.SUM)
            self.exchange.all_reduce(g.max_radii2D, dist.ReduceOp.MAX)

    def sync_optimizer_state(self):
        """All-gather the Adam moments: on ordinary sharded iterations each rank advances only its
        1/N slice of exp_avg / exp_avg_sq, so call this before reading or checkpointing the full
        optimizer state (GaussianModel.capture, train.py:148-150).  Parameters are always full."""
        if self.sharded:
            _fp, fm, fv, _offs, n = self.g.pack_flat_state(self.world)
            S = n // self.world
            self.exchange.all_gather_inplace(fm, self.rank * S, S)
            self.exchange.all_gather_inplace(fv, self.rank * S, S)

    def _step_autograd(self, iteration: int, sync_loss: bool = False) -> StepInfo:
        """The reference-API step: render() through GaussianRasterizer + autograd (train.py:109-147)."""
        g, opt = self.g, self.opt
        vidx, cam = self._low_pass_and_view(iteration)
        densify_phase = iteration < opt.densify_until_iter
        densify_now, reset_now = self._events(iteration)
        if self.sharded:  # gradients accumulate into the flat buffer the exchange reduces
            g.pack_flat_state(self.world)
            flat = g.bind_flat_grad(pad_to=self.world)
        else:  # the reference's zero_grad(set_to_none=True): autograd allocates fresh gradients
            flat = None
            for p in g.params():
                p.grad = None

        pkg = render(cam, g, self.pipe, self.background, low_pass=self.low_pass)
        image, vsp, vis, radii = pkg["render"], pkg["viewspace_points"], pkg["visibility_filter"], pkg["radii"]
        gt = self.gt[vidx]
        # (1-λ)·L1 + λ·(1-SSIM) (train.py:113-114), by default one fused HIP forward/backward
        loss = self.loss_fn(image, gt, opt.lambda_dssim)
        loss.backward()

        with torch.no_grad():
            if densify_phase:  # train.py:132-134, per rank (merged by _finish when densify runs)
                g.update_max_radii(radii, vis)
                g.add_densification_stats(vsp, vis)
            densified = self._finish(iteration, flat, densify_now, reset_now)
        return StepInfo(loss=float(loss.item()) if sync_loss else None, num_gaussians=g.get_xyz.shape[0],
                        view=vidx, low_pass=self.low_pass, densified=densified)
