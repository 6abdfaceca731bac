"""Fused Adam for the Gaussian parameter groups (include/rain_train.h).

Drop-in for the reference's ``torch.optim.Adam(l, lr=0.0, eps=1e-15)``
(scene/gaussian_model.py:153): same constructor, param_groups (with their "name" keys, which the
densification surgery relies on, gaussian_model.py:200-291), per-parameter state
{"step", "exp_avg", "exp_avg_sq"} and state_dict layout — but every group is updated by ONE HIP
launch per step instead of torch's per-group multi-tensor launches.  Arithmetic follows torch's
default foreach Adam in fp32 (see rain_train.h; tests/test_fused_gpu.py checks it against both
torch implementations).  Parameters whose .grad is None are skipped, as in torch.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _native as N


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        if weight_decay != 0.0:
            raise ValueError("rain_amd FusedAdam: weight_decay is not supported (the reference uses none)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0, amsgrad=False, maximize=False)
        super().__init__(params, defaults)
        N.train_lib()  # fail loudly now if the native library is missing

    def _param_group(self, p):
        for g in self.param_groups:
            for q in g["params"]:
                if q is p:
                    return g
        raise KeyError("parameter is not managed by this optimizer")

    @torch.no_grad()
    def fused_step(self, model, skip=()):
        """Book-keeping of one Adam step over the six GaussianModel groups done by the backward
        kernel itself (include/rain_raster.h rr_adam): advances each parameter's step count exactly
        as step() would and returns the rr_adam block (lrs, bias corrections, moment buffers).
        Groups named in `skip` are not stepped: their step count stays and their rr_adam entry is
        left empty (param NULL), as torch's step() leaves a parameter whose .grad is None."""
        names = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
        params = (model._xyz, model._features_dc, model._features_rest, model._opacity, model._scaling,
                  model._rotation)
        ad = N.RRAdam()
        betas = None
        for name, p in zip(names, params):
            if name in skip:
                continue
            group = self._param_group(p)
            b1, b2 = group["betas"]
            if betas is None:
                betas = (float(b1), float(b2), float(group["eps"]))
            elif betas != (float(b1), float(b2), float(group["eps"])):
                raise RuntimeError("rain_amd FusedAdam.fused_step: all groups must share betas and eps")
            state = self.state[p]
            if len(state) == 0:
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            stp = state["step"]
            if stp.device.type != "cpu":
                stp = state["step"] = stp.detach().to("cpu", torch.float32)
            stp += 1.0
            k = float(stp.item())
            g = getattr(ad, name)
            g.param = p.data_ptr()
            g.exp_avg = state["exp_avg"].data_ptr()
            g.exp_avg_sq = state["exp_avg_sq"].data_ptr()
            g.lr = float(group["lr"])
            g.bias_correction1 = 1.0 - math.pow(b1, k)
            g.bias_correction2_sqrt = math.sqrt(1.0 - math.pow(b2, k))
        ad.beta1, ad.beta2, ad.eps = betas
        return ad

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches = {}  # (beta1, beta2, eps, device) -> [RTAdamGroup]
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.device.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("rain_amd FusedAdam: parameters must be contiguous float32 HIP tensors")
                g = p.grad
                if g.is_sparse or not g.is_contiguous() or g.dtype != torch.float32:
                    raise RuntimeError("rain_amd FusedAdam: gradients must be dense contiguous float32")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                stp = state["step"]
                if stp.device.type != "cpu":  # e.g. loaded from a torch fused/capturable Adam
                    stp = state["step"] = stp.detach().to("cpu", torch.float32)
                stp += 1.0
                k = float(stp.item())
                bc1 = 1.0 - math.pow(b1, k)
                bc2s = math.sqrt(1.0 - math.pow(b2, k))
                m, v = state["exp_avg"], state["exp_avg_sq"]
                batches.setdefault((float(b1), float(b2), float(group["eps"]), p.device), []).append(
                    (N.RTAdamGroup(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                                   float(group["lr"]), bc1, bc2s), p))
        L = N.train_lib()
        for (b1, b2, eps, dev), items in batches.items():
            stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            for i in range(0, len(items), N.RT_MAX_GROUPS):
                chunk = items[i:i + N.RT_MAX_GROUPS]
                arr = (N.RTAdamGroup * len(chunk))(*[c[0] for c in chunk])
                rc = L.rt_adam_step(arr, len(chunk), b1, b2, eps, stream)
                if rc != 0:
                    raise RuntimeError(f"rt_adam_step: {L.rt_last_error().decode(errors='replace')}")
        return loss


@torch.no_grad()
def sharded_adam_step(optimizer, params, offsets, shard_grad: torch.Tensor, lo: int, grad_scale: float):
    """One Adam step restricted to the slice [lo, lo + S) of the flat parameter / moment buffers
    (GaussianModel.pack_flat_state), S = shard_grad.numel(), with shard_grad = that slice of the
    gradient SUM over ranks (reduce-scatter output).  Every element is updated exactly as
    optimizer.step() after grad.mul_(grad_scale) would update it; every group's step count advances
    on every rank (also when its segment misses the slice), so all ranks keep identical counts.
    FusedAdam: one launch (rt_adam_step_scaled); torch.optim.Adam (CPU replicas in the gloo tests):
    torch's own single-tensor Adam on the slices."""
    hi = lo + shard_grad.numel()
    items = []
    for p, off in zip(params, offsets):
        group = next(g for g in optimizer.param_groups if any(q is p for q in g["params"]))
        st = optimizer.state[p]
        if len(st) == 0:
            raise RuntimeError("sharded_adam_step: pack the optimizer state first (GaussianModel.pack_flat_state)")
        st["step"] += 1.0
        a, b = max(off, lo), min(off + p.numel(), hi)
        if a < b:
            items.append((group, p, st, a - off, a - lo, b - a))
    if isinstance(optimizer, FusedAdam):
        if not items:
            return
        groups = []
        b1 = b2 = eps = None
        for group, p, st, po, go, n in items:
            gb1, gb2 = group["betas"]
            b1, b2, eps = float(gb1), float(gb2), float(group["eps"])
            k = float(st["step"].item())
            groups.append(N.RTAdamGroup(p.data_ptr() + 4 * po, shard_grad.data_ptr() + 4 * go,
                                        st["exp_avg"].data_ptr() + 4 * po, st["exp_avg_sq"].data_ptr() + 4 * po, n,
                                        float(group["lr"]), 1.0 - math.pow(gb1, k), math.sqrt(1.0 - math.pow(gb2, k))))
        arr = (N.RTAdamGroup * len(groups))(*groups)
        stream = ctypes.c_void_p(torch.cuda.current_stream(shard_grad.device).cuda_stream)
        rc = N.train_lib().rt_adam_step_scaled(arr, len(groups), b1, b2, eps, float(grad_scale), stream)
        if rc != 0:
            raise RuntimeError(f"rt_adam_step_scaled: {N.train_lib().rt_last_error().decode(errors='replace')}")
        return
    from torch.optim.adam import adam as adam_functional

    for group, p, st, po, go, n in items:
        b1, b2 = group["betas"]
        g = shard_grad[go:go + n] * grad_scale
        step = (st["step"] - 1.0).clone()  # the functional form advances its own copy
        adam_functional([p.data.view(-1)[po:po + n]], [g], [st["exp_avg"].view(-1)[po:po + n]],
                        [st["exp_avg_sq"].view(-1)[po:po + n]], [], [step], foreach=False, amsgrad=False,
                        beta1=b1, beta2=b2, lr=group["lr"], weight_decay=0.0, eps=group["eps"], maximize=False)
