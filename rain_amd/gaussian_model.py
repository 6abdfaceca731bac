"""GaussianModel counterpart (§8(f) #3).

Same attributes, getters, optimizer groups, learning-rate schedule, densification statistics and
densify/clone/split/prune semantics as scene/gaussian_model.py:13-421 (RAIN-GS fork: `divide_ratio`,
`abe_split`), with the device made explicit (the reference hard-codes "cuda") and one extra layout
choice for the view-sharded multi-GPU step: every parameter's gradient is a view into ONE flat fp32
buffer (`flat_grad`) so a single all-reduce covers all of them (rain_amd/train.py).

Attribution: the optimizer-state surgery (replace_tensor_to_optimizer, _prune_optimizer,
cat_tensors_to_optimizer, densification_postfix) and the torch densify/clone/split restatement
follow the reference's scene/gaussian_model.py (Inria 3D Gaussian Splatting, GRAPHDECO research
group, Inria Gaussian-Splatting licence — LICENSE.md in the reference; RAIN-GS modifications by its
authors) closely, because train.py's loop depends on their exact behaviour.  The HIP densify path
(rain_amd/csrc/densify.hip) is an independent design.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch import nn

from . import synthetic


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:18-36."""

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        log_lerp = np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
        return delay_rate * log_lerp

    return helper


def inverse_sigmoid(x):
    return torch.log(x / (1 - x))


def build_rotation(r):
    """utils/general_utils.py:52-73 (device follows the input)."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def build_scaling_rotation(s, r):
    """utils/general_utils.py:75-84."""
    L = torch.zeros((s.shape[0], 3, 3), dtype=torch.float, device=s.device)
    R = build_rotation(r)
    L[:, 0, 0] = s[:, 0]
    L[:, 1, 1] = s[:, 1]
    L[:, 2, 2] = s[:, 2]
    return R @ L


def strip_symmetric(L):
    """utils/general_utils.py:38-50."""
    return torch.stack([L[:, 0, 0], L[:, 0, 1], L[:, 0, 2], L[:, 1, 1], L[:, 1, 2], L[:, 2, 2]], dim=1)


class OptimizationParams:
    """arguments/__init__.py:61-80 defaults."""

    def __init__(self, **kw):
        self.iterations = 30_000
        self.position_lr_init = 0.00016
        self.position_lr_final = 0.0000016
        self.position_lr_delay_mult = 0.01
        self.position_lr_max_steps = 30_000
        self.feature_lr = 0.0025
        self.opacity_lr = 0.05
        self.scaling_lr = 0.005
        self.rotation_lr = 0.001
        self.percent_dense = 0.01
        self.lambda_dssim = 0.2
        self.densification_interval = 100
        self.opacity_reset_interval = 3000
        self.densify_from_iter = 500
        self.densify_until_iter = 15_000
        self.densify_grad_threshold = 0.0002
        self.random_background = False
        for k, v in kw.items():
            setattr(self, k, v)


PARAM_NAMES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


class GaussianModel:
    def __init__(self, sh_degree: int, divide_ratio: float = 0.8, device="cuda"):
        self.active_sh_degree = 0
        self.max_sh_degree = sh_degree
        self.device = torch.device(device)
        e = torch.empty(0, device=self.device)
        self._xyz = self._features_dc = self._features_rest = e
        self._scaling = self._rotation = self._opacity = e
        self.max_radii2D = e
        self.xyz_gradient_accum = e
        self.denom = e
        self.optimizer = None
        self.percent_dense = 0
        self.spatial_lr_scale = 0
        self.divide_ratio = divide_ratio
        self.flat_grad = None
        self._packed = None
        self.scaling_activation = torch.exp
        self.scaling_inverse_activation = torch.log
        self.opacity_activation = torch.sigmoid
        self.inverse_opacity_activation = inverse_sigmoid
        self.rotation_activation = torch.nn.functional.normalize

    # ---- checkpoint tuple (gaussian_model.py:51-83) ----
    def capture(self):
        return (self.active_sh_degree, self._xyz, self._features_dc, self._features_rest, self._scaling,
                self._rotation, self._opacity, self.max_radii2D, self.xyz_gradient_accum, self.denom,
                self.optimizer.state_dict(), self.spatial_lr_scale)

    def restore(self, model_args, training_args):
        (self.active_sh_degree, self._xyz, self._features_dc, self._features_rest, self._scaling, self._rotation,
         self._opacity, self.max_radii2D, xyz_gradient_accum, denom, opt_dict, self.spatial_lr_scale) = model_args
        self.training_setup(training_args)
        self.xyz_gradient_accum = xyz_gradient_accum
        self.denom = denom
        self.optimizer.load_state_dict(opt_dict)

    # ---- PLY (gaussian_model.py:167-246), via rain_amd.ply instead of plyfile ----
    def construct_list_of_attributes(self):
        names = ["x", "y", "z", "nx", "ny", "nz"]
        names += [f"f_dc_{i}" for i in range(self._features_dc.shape[1] * self._features_dc.shape[2])]
        names += [f"f_rest_{i}" for i in range(self._features_rest.shape[1] * self._features_rest.shape[2])]
        names.append("opacity")
        names += [f"scale_{i}" for i in range(self._scaling.shape[1])]
        names += [f"rot_{i}" for i in range(self._rotation.shape[1])]
        return names

    def save_ply(self, path):
        """Pre-activation values; SH stored channel-major ([P,3,K] flattened, gaussian_model.py:184-185)."""
        from .ply import write_vertices

        xyz = self._xyz.detach().cpu().numpy()
        f_dc = self._features_dc.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
        f_rest = self._features_rest.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
        cols = np.concatenate((xyz, np.zeros_like(xyz), f_dc, f_rest, self._opacity.detach().cpu().numpy(),
                               self._scaling.detach().cpu().numpy(), self._rotation.detach().cpu().numpy()), axis=1)
        names = self.construct_list_of_attributes()
        write_vertices(path, {n: cols[:, i] for i, n in enumerate(names)})

    def load_ply(self, path):
        from .ply import read_elements

        v = read_elements(path)["vertex"]
        names = v.dtype.names

        def group(prefix):
            ks = sorted((n for n in names if n.startswith(prefix)), key=lambda x: int(x.split("_")[-1]))
            return np.stack([np.asarray(v[k], dtype=np.float64) for k in ks], axis=1) if ks else \
                np.zeros((len(v), 0))

        xyz = np.stack([np.asarray(v[k], dtype=np.float64) for k in ("x", "y", "z")], axis=1)
        opacities = np.asarray(v["opacity"], dtype=np.float64)[..., None]
        f_dc = np.stack([np.asarray(v[f"f_dc_{i}"], dtype=np.float64) for i in range(3)], axis=1)[..., None]
        extra = group("f_rest_")
        K1 = (self.max_sh_degree + 1) ** 2 - 1
        assert extra.shape[1] == 3 * K1, f"{path}: {extra.shape[1]} f_rest columns, expected {3 * K1}"
        extra = extra.reshape(len(v), 3, K1)
        dev = self.device
        t = lambda a: torch.tensor(a, dtype=torch.float, device=dev)  # noqa: E731
        self._xyz = nn.Parameter(t(xyz).requires_grad_(True))
        self._features_dc = nn.Parameter(t(f_dc).transpose(1, 2).contiguous().requires_grad_(True))
        self._features_rest = nn.Parameter(t(extra).transpose(1, 2).contiguous().requires_grad_(True))
        self._opacity = nn.Parameter(t(opacities).requires_grad_(True))
        self._scaling = nn.Parameter(t(group("scale_")).requires_grad_(True))
        self._rotation = nn.Parameter(t(group("rot")).requires_grad_(True))
        self.max_radii2D = torch.zeros((self._xyz.shape[0]), device=dev)
        self.active_sh_degree = self.max_sh_degree

    # ---- getters (gaussian_model.py:85-108) ----
    @property
    def get_scaling(self):
        return self.scaling_activation(self._scaling)

    @property
    def get_rotation(self):
        return self.rotation_activation(self._rotation)

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_opacity(self):
        return self.opacity_activation(self._opacity)

    def get_covariance(self, scaling_modifier=1):
        L = build_scaling_rotation(scaling_modifier * self.get_scaling, self._rotation)
        return strip_symmetric(L @ L.transpose(1, 2))

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # ---- init (gaussian_model.py:114-137) ----
    def create_from_pcd(self, points: np.ndarray, colors: np.ndarray, spatial_lr_scale: float):
        self.spatial_lr_scale = spatial_lr_scale
        dev = self.device
        fused_point_cloud = torch.tensor(np.asarray(points)).float().to(dev)
        fused_color = synthetic.RGB2SH(torch.tensor(np.asarray(colors)).float().to(dev))
        features = torch.zeros((fused_color.shape[0], 3, (self.max_sh_degree + 1) ** 2), device=dev)
        features[:, :3, 0] = fused_color
        scales = synthetic.init_scales(fused_point_cloud)
        rots = torch.zeros((fused_point_cloud.shape[0], 4), device=dev)
        rots[:, 0] = 1
        opacities = inverse_sigmoid(0.1 * torch.ones((fused_point_cloud.shape[0], 1), dtype=torch.float, device=dev))
        self.set_params(dict(xyz=fused_point_cloud, f_dc=features[:, :, 0:1].transpose(1, 2).contiguous(),
                             f_rest=features[:, :, 1:].transpose(1, 2).contiguous(), scaling=scales,
                             rotation=rots, opacity=opacities))

    def set_params(self, p: dict):
        dev = self.device
        self._xyz = nn.Parameter(p["xyz"].to(dev).float().contiguous().requires_grad_(True))
        self._features_dc = nn.Parameter(p["f_dc"].to(dev).float().contiguous().requires_grad_(True))
        self._features_rest = nn.Parameter(p["f_rest"].to(dev).float().contiguous().requires_grad_(True))
        self._scaling = nn.Parameter(p["scaling"].to(dev).float().contiguous().requires_grad_(True))
        self._rotation = nn.Parameter(p["rotation"].to(dev).float().contiguous().requires_grad_(True))
        self._opacity = nn.Parameter(p["opacity"].to(dev).float().contiguous().requires_grad_(True))
        self.max_radii2D = torch.zeros((self._xyz.shape[0]), device=dev)

    # ---- optimizer (gaussian_model.py:139-165) ----
    def training_setup(self, training_args):
        self.percent_dense = training_args.percent_dense
        dev = self.device
        self.xyz_gradient_accum = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.denom = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        groups = [
            {'params': [self._xyz], 'lr': training_args.position_lr_init * self.spatial_lr_scale, "name": "xyz"},
            {'params': [self._features_dc], 'lr': training_args.feature_lr, "name": "f_dc"},
            {'params': [self._features_rest], 'lr': training_args.feature_lr / 20.0, "name": "f_rest"},
            {'params': [self._opacity], 'lr': training_args.opacity_lr, "name": "opacity"},
            {'params': [self._scaling], 'lr': training_args.scaling_lr, "name": "scaling"},
            {'params': [self._rotation], 'lr': training_args.rotation_lr, "name": "rotation"},
        ]
        if self.device.type == "cuda":
            # one HIP launch for all six groups (include/rain_train.h); same state layout as torch Adam
            from .optim import FusedAdam
            self.optimizer = FusedAdam(groups, lr=0.0, eps=1e-15)
        else:
            self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        self.xyz_scheduler_args = get_expon_lr_func(
            lr_init=training_args.position_lr_init * self.spatial_lr_scale,
            lr_final=training_args.position_lr_final * self.spatial_lr_scale,
            lr_delay_mult=training_args.position_lr_delay_mult, max_steps=training_args.position_lr_max_steps)
        self.flat_grad = None
        self._packed = None

    def update_learning_rate(self, iteration):
        for param_group in self.optimizer.param_groups:
            if param_group["name"] == "xyz":
                lr = self.xyz_scheduler_args(iteration)
                param_group['lr'] = lr
                return lr

    # ---- flat gradient buffer (one all-reduce per step) ----
    def params(self):
        return [self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling, self._rotation]

    FLAT_ALIGN = 64  # floats: every parameter's gradient view starts on a 256-B boundary

    def flat_layout(self, pad_to: int = 1):
        """Segment offsets of the six parameters in the flat buffers (each padded to FLAT_ALIGN
        floats) and the total length, padded to a multiple of FLAT_ALIGN * pad_to so that it splits
        into pad_to equal, 256-B aligned shards."""
        a = self.FLAT_ALIGN
        offs, off = [], 0
        for p in self.params():
            offs.append(off)
            off += (p.numel() + a - 1) // a * a
        unit = a * max(int(pad_to), 1)
        return offs, (off + unit - 1) // unit * unit

    def bind_flat_grad(self, extra: int = 0, zero: bool = True, pad_to: int = 1):
        """Make every parameter's .grad a view into one fp32 buffer (flat_layout(pad_to), plus
        `extra` trailing floats) and return the buffer.  The whole buffer is zeroed if `zero`,
        otherwise only the trailing `extra` floats (for writers that overwrite every gradient, e.g.
        the fused raw-parameter backward)."""
        ps = self.params()
        offs, n = self.flat_layout(pad_to)
        if self.flat_grad is None or self.flat_grad.numel() != n + extra:
            self.flat_grad = torch.zeros(n + extra, device=self.device)
        elif zero:
            self.flat_grad.zero_()
        elif extra:
            self.flat_grad[n:].zero_()
        for p, off in zip(ps, offs):
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
        return self.flat_grad

    def pack_flat_state(self, pad_to: int = 1):
        """Move the six parameters and their Adam moments into three flat fp32 buffers with the
        flat-gradient layout (flat_layout(pad_to)); parameters keep their identity (only .data is
        re-pointed), so param_groups and optimizer.state stay valid.  Used by the view-sharded step:
        a rank updates the slice [r*n/N, (r+1)*n/N) of all three buffers, then all-gathers the
        parameter buffer.  Re-packs only after densification / opacity reset replaced tensors.
        Returns (params, exp_avg, exp_avg_sq, offsets, n)."""
        ps = self.params()
        key = (pad_to,) + tuple(id(p) for p in ps) + tuple(p.data_ptr() for p in ps)
        if self._packed is not None and self._packed[0] == key:
            return self._packed[1]
        offs, n = self.flat_layout(pad_to)
        fp, fm, fv = (torch.zeros(n, device=self.device) for _ in range(3))
        for p, off in zip(ps, offs):
            k = p.numel()
            fp[off:off + k].copy_(p.data.reshape(-1))
            st = self.optimizer.state[p]
            if len(st) == 0:  # the state torch's Adam creates on its first step
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
            else:
                fm[off:off + k].copy_(st["exp_avg"].reshape(-1))
                fv[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
            p.data = fp[off:off + k].view_as(p)
            st["exp_avg"] = fm[off:off + k].view_as(p)
            st["exp_avg_sq"] = fv[off:off + k].view_as(p)
        out = (fp, fm, fv, offs, n)
        self._packed = ((pad_to,) + tuple(id(p) for p in ps) + tuple(p.data_ptr() for p in ps), out)
        return out

    # ---- densification (gaussian_model.py:200-421) ----
    def reset_opacity(self):
        opacities_new = inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01))
        optimizable_tensors = self.replace_tensor_to_optimizer(opacities_new, "opacity")
        self._opacity = optimizable_tensors["opacity"]

    def replace_tensor_to_optimizer(self, tensor, name):
        optimizable_tensors = {}
        for group in self.optimizer.param_groups:
            if group["name"] == name:
                stored_state = self.optimizer.state.get(group['params'][0], None)
                stored_state["exp_avg"] = torch.zeros_like(tensor)
                stored_state["exp_avg_sq"] = torch.zeros_like(tensor)
                del self.optimizer.state[group['params'][0]]
                group["params"][0] = nn.Parameter(tensor.requires_grad_(True))
                self.optimizer.state[group['params'][0]] = stored_state
                optimizable_tensors[group["name"]] = group["params"][0]
        self.flat_grad = None
        return optimizable_tensors

    def _prune_optimizer(self, mask):
        optimizable_tensors = {}
        for group in self.optimizer.param_groups:
            stored_state = self.optimizer.state.get(group['params'][0], None)
            if stored_state is not None:
                stored_state["exp_avg"] = stored_state["exp_avg"][mask]
                stored_state["exp_avg_sq"] = stored_state["exp_avg_sq"][mask]
                del self.optimizer.state[group['params'][0]]
                group["params"][0] = nn.Parameter((group["params"][0][mask].requires_grad_(True)))
                self.optimizer.state[group['params'][0]] = stored_state
                optimizable_tensors[group["name"]] = group["params"][0]
            else:
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
                optimizable_tensors[group["name"]] = group["params"][0]
        self.flat_grad = None
        return optimizable_tensors

    def prune_points(self, mask):
        valid_points_mask = ~mask
        t = self._prune_optimizer(valid_points_mask)
        self._xyz, self._features_dc, self._features_rest = t["xyz"], t["f_dc"], t["f_rest"]
        self._opacity, self._scaling, self._rotation = t["opacity"], t["scaling"], t["rotation"]
        self.xyz_gradient_accum = self.xyz_gradient_accum[valid_points_mask]
        self.denom = self.denom[valid_points_mask]
        self.max_radii2D = self.max_radii2D[valid_points_mask]

    def cat_tensors_to_optimizer(self, tensors_dict):
        optimizable_tensors = {}
        for group in self.optimizer.param_groups:
            assert len(group["params"]) == 1
            extension_tensor = tensors_dict[group["name"]]
            stored_state = self.optimizer.state.get(group['params'][0], None)
            if stored_state is not None:
                stored_state["exp_avg"] = torch.cat((stored_state["exp_avg"], torch.zeros_like(extension_tensor)), 0)
                stored_state["exp_avg_sq"] = torch.cat((stored_state["exp_avg_sq"],
                                                        torch.zeros_like(extension_tensor)), 0)
                del self.optimizer.state[group['params'][0]]
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], extension_tensor), 0)
                                                  .requires_grad_(True))
                self.optimizer.state[group['params'][0]] = stored_state
                optimizable_tensors[group["name"]] = group["params"][0]
            else:
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], extension_tensor), 0)
                                                  .requires_grad_(True))
                optimizable_tensors[group["name"]] = group["params"][0]
        self.flat_grad = None
        return optimizable_tensors

    def densification_postfix(self, new_xyz, new_features_dc, new_features_rest, new_opacities, new_scaling,
                              new_rotation):
        d = {"xyz": new_xyz, "f_dc": new_features_dc, "f_rest": new_features_rest, "opacity": new_opacities,
             "scaling": new_scaling, "rotation": new_rotation}
        t = self.cat_tensors_to_optimizer(d)
        self._xyz, self._features_dc, self._features_rest = t["xyz"], t["f_dc"], t["f_rest"]
        self._opacity, self._scaling, self._rotation = t["opacity"], t["scaling"], t["rotation"]
        dev = self.device
        self.xyz_gradient_accum = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.denom = torch.zeros((self.get_xyz.shape[0], 1), device=dev)
        self.max_radii2D = torch.zeros((self.get_xyz.shape[0]), device=dev)

    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2, abe_split=False, generator=None):
        dev = self.device
        n_init_points = self.get_xyz.shape[0]
        if abe_split:  # RAIN-GS warm-up split (gaussian_model.py:342-364)
            BACK_N = N - 1
            padded_grad = torch.zeros((n_init_points), device=dev)
            padded_grad[:grads.shape[0]] = grads.squeeze()
            selected_pts_mask = torch.where(padded_grad >= grad_threshold, True, False)
            selected_pts_mask = torch.logical_and(
                selected_pts_mask, torch.max(self.get_scaling, dim=1).values > self.percent_dense * scene_extent)
            new_xyz = self.get_xyz[selected_pts_mask].repeat(BACK_N, 1)
            new_scaling = self.scaling_inverse_activation(self.get_scaling[selected_pts_mask].repeat(BACK_N, 1))
            new_rotation = self._rotation[selected_pts_mask].repeat(BACK_N, 1)
            new_features_dc = self._features_dc[selected_pts_mask].repeat(BACK_N, 1, 1)
            new_features_rest = self._features_rest[selected_pts_mask].repeat(BACK_N, 1, 1)
            new_opacity = self._opacity[selected_pts_mask].repeat(BACK_N, 1)
            # the reference draws (and never uses) BACK_N rows of normals per selected Gaussian here
            # (gaussian_model.py:349-351): drawn too, so the split below sees the same random stream
            stds = self.get_scaling[selected_pts_mask].repeat(BACK_N, 1)
            torch.normal(mean=torch.zeros((stds.size(0), 3), device=dev), std=stds, generator=generator)
            new_xyz = new_xyz * 0.3 * scene_extent
            self.densification_postfix(new_xyz, new_features_dc, new_features_rest, new_opacity, new_scaling,
                                       new_rotation)
            n_init_points = self.get_xyz.shape[0]

        padded_grad = torch.zeros((n_init_points), device=dev)
        padded_grad[:grads.shape[0]] = grads.squeeze()
        selected_pts_mask = torch.where(padded_grad >= grad_threshold, True, False)
        selected_pts_mask = torch.logical_and(
            selected_pts_mask, torch.max(self.get_scaling, dim=1).values > self.percent_dense * scene_extent)
        stds = self.get_scaling[selected_pts_mask].repeat(N, 1)
        means = torch.zeros((stds.size(0), 3), device=dev)
        samples = torch.normal(mean=means, std=stds, generator=generator)
        rots = build_rotation(self._rotation[selected_pts_mask]).repeat(N, 1, 1)
        new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self.get_xyz[selected_pts_mask].repeat(N, 1)
        new_scaling = self.scaling_inverse_activation(
            self.get_scaling[selected_pts_mask].repeat(N, 1) / (self.divide_ratio * N))
        new_rotation = self._rotation[selected_pts_mask].repeat(N, 1)
        new_features_dc = self._features_dc[selected_pts_mask].repeat(N, 1, 1)
        new_features_rest = self._features_rest[selected_pts_mask].repeat(N, 1, 1)
        new_opacity = self._opacity[selected_pts_mask].repeat(N, 1)
        self.densification_postfix(new_xyz, new_features_dc, new_features_rest, new_opacity, new_scaling,
                                   new_rotation)
        prune_filter = torch.cat((selected_pts_mask,
                                  torch.zeros(N * selected_pts_mask.sum(), device=dev, dtype=bool)))
        self.prune_points(prune_filter)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        selected_pts_mask = torch.where(torch.norm(grads, dim=-1) >= grad_threshold, True, False)
        selected_pts_mask = torch.logical_and(
            selected_pts_mask, torch.max(self.get_scaling, dim=1).values <= self.percent_dense * scene_extent)
        self.densification_postfix(self._xyz[selected_pts_mask], self._features_dc[selected_pts_mask],
                                   self._features_rest[selected_pts_mask], self._opacity[selected_pts_mask],
                                   self._scaling[selected_pts_mask], self._rotation[selected_pts_mask])

    # HIP devices densify with the stream-compaction kernels (include/rain_train.h rt_densify_*);
    # False selects the torch restatement below (tests compare the two)
    native_densify = True

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, N=2, abe_split=False,
                          generator=None):
        # (abe_split with max_grad <= 0 would also select the abe copies for the split: torch path)
        if (self.native_densify and self.device.type == "cuda" and self._xyz.shape[0] > 0
                and not (abe_split and max_grad <= 0)):
            return self._densify_and_prune_native(max_grad, min_opacity, extent, max_screen_size, N, generator,
                                                  abe_split)
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent, N=N, abe_split=abe_split, generator=generator)
        prune_mask = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            big_points_vs = self.max_radii2D > max_screen_size
            big_points_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
            prune_mask = torch.logical_or(torch.logical_or(prune_mask, big_points_vs), big_points_ws)
        self.prune_points(prune_mask)

    def _densify_and_prune_native(self, max_grad, min_opacity, extent, max_screen_size, N, generator,
                                  abe_split=False):
        """densify_and_clone + densify_and_split (with the RAIN-GS abe copies when abe_split) + prune
        (gaussian_model.py:339-415) as one stream compaction on the device: the same decisions, the
        survivors in the same order, the same values (the split children's xyz up to the rounding of
        the reference's bmm) and the same optimizer-state surgery (new Parameters, zero moments for
        the new Gaussians)."""
        import ctypes

        from . import _native as NV

        L = NV.train_lib()
        dev = self.device
        P = self._xyz.shape[0]

        def ptr(t):
            return None if t is None or t.numel() == 0 else ctypes.c_void_p(t.data_ptr())

        def check(rc, what):
            if rc != 0:
                raise RuntimeError(f"{what}: {L.rt_last_error().decode(errors='replace')}")

        prm = NV.RTDensifyParams(P, int(N), float(max_grad), float(self.percent_dense * extent), float(min_opacity),
                                 float(0.1 * extent), int(bool(max_screen_size)), float(self.divide_ratio * N),
                                 int(bool(abe_split)), 0.3, float(extent))
        ws = torch.empty((L.rt_densify_workspace_bytes(P),), dtype=torch.uint8, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        acc, den = self.xyz_gradient_accum.contiguous(), self.denom.contiguous()
        sc, op, rot = (t.detach().contiguous() for t in (self._scaling, self._opacity, self._rotation))
        counts = (ctypes.c_int64 * 5)()
        check(L.rt_densify_plan(ctypes.byref(prm), ptr(acc), ptr(den), ptr(sc), ptr(op), ptr(ws), ws.numel(), counts,
                                stream), "rt_densify_plan")
        A, B, C, S, E = (int(c) for c in counts)
        # torch.normal(mean=0, std) draws normal_(0, 1) into its output first: same draws, same
        # generator; with abe_split the reference's unused (N - 1) * S rows come first
        if abe_split and S and N > 1:
            torch.empty(((N - 1) * S, 3), device=dev).normal_(0.0, 1.0, generator=generator)
        z = torch.empty((N * S, 3), device=dev).normal_(0.0, 1.0, generator=generator) if S else None
        Pn = A + B + (N - 1) * E + N * C
        kinds = {"xyz": NV.RT_GROUP_XYZ, "scaling": NV.RT_GROUP_SCALING}
        plans, structs = [], []
        for group in self.optimizer.param_groups:
            p = group["params"][0]
            st = self.optimizer.state.get(p, None)
            has = st is not None and "exp_avg" in st
            width = math.prod(p.shape[1:])
            out = torch.empty((Pn,) + tuple(p.shape[1:]), device=dev)
            om = torch.empty_like(out) if has else None
            ov = torch.empty_like(out) if has else None
            src = p.detach().contiguous()
            m = st["exp_avg"].contiguous() if has else None
            v = st["exp_avg_sq"].contiguous() if has else None
            if width > 0:
                structs.append(NV.RTDensifyGroup(ptr(src), ptr(m), ptr(v), ptr(out), ptr(om), ptr(ov), width,
                                                 kinds.get(group["name"], NV.RT_GROUP_OTHER)))
            plans.append((group, p, st, out, om, ov, (src, m, v)))
        arr = (NV.RTDensifyGroup * max(len(structs), 1))(*structs)
        check(L.rt_densify_apply(ctypes.byref(prm), ptr(sc), ptr(rot), ptr(z), ptr(ws), arr, len(structs), counts,
                                 stream), "rt_densify_apply")
        new = {}
        for group, p, st, out, om, ov, _keep in plans:
            param = nn.Parameter(out.requires_grad_(True))
            if st is not None:
                del self.optimizer.state[p]
                if om is not None:
                    st["exp_avg"], st["exp_avg_sq"] = om, ov
                self.optimizer.state[param] = st
            group["params"][0] = param
            new[group["name"]] = param
        self._xyz, self._features_dc, self._features_rest = new["xyz"], new["f_dc"], new["f_rest"]
        self._opacity, self._scaling, self._rotation = new["opacity"], new["scaling"], new["rotation"]
        self.xyz_gradient_accum = torch.zeros((Pn, 1), device=dev)
        self.denom = torch.zeros((Pn, 1), device=dev)
        self.max_radii2D = torch.zeros((Pn,), device=dev)
        self.flat_grad = None

    def add_densification_stats(self, viewspace_point_tensor, update_filter):
        """gaussian_model.py:419-421 (consumes the NDC-space dL/dmeans2D the rasterizer returns).
        The reference's boolean-mask indexing makes the host wait for the device (the mask's count
        sizes the gather); the same update as a select keeps the step free of host syncs: masked
        rows gain exactly the reference's norm, the others exactly 0."""
        g = viewspace_point_tensor.grad
        if g.is_cuda and self._stats_native(g, update_filter):  # one launch (rain_train.h rt_densify_stats)
            from . import _native
            _native.check_rt(_native.train_lib().rt_densify_stats(
                g.shape[0], g.data_ptr(), g.stride(0), update_filter.data_ptr(), self.xyz_gradient_accum.data_ptr(),
                self.denom.data_ptr(), _native.stream_of(g)), "densify stats")
            return
        m = update_filter.reshape(-1, 1)
        self.xyz_gradient_accum += torch.where(m, torch.norm(g[:, :2], dim=-1, keepdim=True), 0.0)
        self.denom += m.to(self.denom.dtype)

    def _stats_native(self, g, mask):
        """The statistics arrays and inputs in the layout the native kernels take."""
        P = g.shape[0]
        return (g.dtype == torch.float32 and g.dim() == 2 and g.shape[1] >= 2 and g.stride(1) == 1
                and g.stride(0) >= 2 and mask.dtype == torch.bool and mask.is_contiguous() and mask.numel() == P
                and mask.device == g.device
                and all(t.device == g.device and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == P
                        for t in (self.xyz_gradient_accum, self.denom, self.max_radii2D)))

    def update_max_radii(self, radii, visibility_filter):
        """train.py:133, max_radii2D[vis] = max(max_radii2D[vis], radii[vis]), without the host sync of
        boolean-mask indexing (the same values)."""
        P = radii.numel()
        if radii.is_cuda and radii.dtype == torch.int32 and radii.is_contiguous() \
                and visibility_filter.dtype == torch.bool and visibility_filter.is_contiguous() \
                and visibility_filter.numel() == P and visibility_filter.device == radii.device \
                and self.max_radii2D.device == radii.device \
                and self.max_radii2D.dtype == torch.float32 and self.max_radii2D.is_contiguous() \
                and self.max_radii2D.numel() == P:
            from . import _native
            _native.check_rt(_native.train_lib().rt_max_radii(
                radii.numel(), radii.data_ptr(), visibility_filter.data_ptr(), self.max_radii2D.data_ptr(),
                _native.stream_of(radii)), "max radii")
            return
        self.max_radii2D = torch.where(visibility_filter, torch.maximum(self.max_radii2D, radii.float()),
                                       self.max_radii2D)


def low_pass_schedule(H, W, N, c2f_max_lowpass=300.0):
    """RAIN-GS coarse-to-fine low-pass filter (train.py:95-107)."""
    lp = max(H * W / N / (9 * math.pi), 0.3)
    if c2f_max_lowpass > 0:
        lp = min(lp, c2f_max_lowpass)
    return lp
