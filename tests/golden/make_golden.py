"""Generate the golden fixtures under tests/golden/ by calling the REFERENCE's own importable
Python helpers (dev container only; /root/reference does not exist on the GPU box).

Pins the pieces of the hot path whose reference implementation runs on CPU:
  sh_eval.npz      utils/sh_utils.py:34-77 eval_sh (+0.5, clamp_min 0: gaussian_renderer/__init__.py:57-58)
                   for degrees 0..3 — the SH polynomial the forward/backward kernels implement
                   (forward.cu:9-60 is the same polynomial)
  camera.npz       utils/graphics_utils.py getWorld2View2 / getProjectionMatrix / fov2focal / focal2fov and
                   scene/cameras.py:108-111 matrix assembly for synthetic cameras (the kernels' inputs)
  loss.npz         utils/loss_utils.py l1_loss / ssim values and gradients (train.py:113-114)
  lr.npz           utils/general_utils.py get_expon_lr_func (train-step xyz LR schedule)
  cov3d.npz        utils/general_utils.py build_rotation / build_scaling_rotation / strip_symmetric composed
                   as scene/gaussian_model.py:16-20 (build_covariance_from_scaling_rotation): Sigma3D, the
                   compute_cov3D_python path (gaussian_renderer/__init__.py:44-48) and the quantity
                   computeCov3D (forward.cu:107-141, F4 step 4) builds in-kernel; plus inverse_sigmoid (:7-8)
                   and the getters' activations (torch.exp, F.normalize, torch.sigmoid) on the same inputs.
                   Those helpers hard-code device="cuda", so they run with a module-scoped CPU view of
                   `torch` (CpuTorch below) — the reference's arithmetic, on the CPU.

The fixtures are data (inputs + outputs); no reference source is copied.
Run:  python tests/golden/make_golden.py
"""
import math
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = os.environ.get("RAIN_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


class CpuTorch:
    """Stand-in for the `torch` global of ONE reference module: every attribute is torch's own,
    except that tensor factories ignore `device` (the reference asks for "cuda"; none exists here)."""

    def __getattr__(self, name):
        return getattr(torch, name)

    @staticmethod
    def zeros(*shape, device=None, **kw):
        return torch.zeros(*shape, **kw)


def main():
    sys.path.insert(0, REF)
    from utils import general_utils, graphics_utils, loss_utils, sh_utils  # reference modules

    rng = np.random.default_rng(1234)
    torch.manual_seed(1234)

    # ---- SH ----
    out = {}
    for deg in range(4):
        n = 257
        sh = torch.from_numpy(rng.standard_normal((n, 3, 16)).astype(np.float32) * 0.5)
        d = torch.from_numpy(rng.standard_normal((n, 3)).astype(np.float32))
        d = d / d.norm(dim=1, keepdim=True)
        val = sh_utils.eval_sh(deg, sh, d)
        out[f"sh_{deg}"] = sh.numpy()
        out[f"dirs_{deg}"] = d.numpy()
        out[f"eval_{deg}"] = val.numpy()
        out[f"rgb_{deg}"] = torch.clamp_min(val + 0.5, 0.0).numpy()
    rgb = torch.rand(64, 3)
    out["rgb2sh_in"] = rgb.numpy()
    out["rgb2sh_out"] = sh_utils.RGB2SH(rgb).numpy()
    np.savez_compressed(os.path.join(HERE, "sh_eval.npz"), **out)

    # ---- cameras ----
    out = {}
    W, H, fovx = 800, 600, 0.6911112
    fovy = graphics_utils.focal2fov(graphics_utils.fov2focal(fovx, W), H)
    out["fovy"] = np.array([fovy])
    out["focal"] = np.array([graphics_utils.fov2focal(fovx, W)])
    for i in range(6):
        # a random look-at rig in the reference's (R = c2w rotation, T = w2c translation) convention
        eye = rng.standard_normal(3)
        eye = 4.0 * eye / np.linalg.norm(eye)
        fwd = -eye / np.linalg.norm(eye)
        up = np.array([0.0, 0.0, 1.0])
        right = np.cross(fwd, up)
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        c2w = np.eye(4)
        c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, down, fwd, eye
        w2c = np.linalg.inv(c2w)
        R, T = np.transpose(w2c[:3, :3]), w2c[:3, 3]
        wv = torch.tensor(graphics_utils.getWorld2View2(R, T)).transpose(0, 1)
        pm = graphics_utils.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pm.unsqueeze(0)).squeeze(0)
        out[f"R_{i}"], out[f"T_{i}"] = R, T
        out[f"view_{i}"] = wv.numpy()
        out[f"proj_{i}"] = pm.numpy()
        out[f"full_{i}"] = full.numpy()
        out[f"campos_{i}"] = wv.inverse()[3, :3].numpy()
    np.savez_compressed(os.path.join(HERE, "camera.npz"), **out)

    # ---- loss ----
    out = {}
    for i, (h, w) in enumerate([(40, 56), (33, 47)]):
        a = torch.rand(3, h, w, dtype=torch.float32)
        b = (0.6 * a + 0.4 * torch.rand(3, h, w)).float()
        x = a.clone().requires_grad_(True)
        l1 = loss_utils.l1_loss(x, b)
        s = loss_utils.ssim(x, b)
        loss = 0.8 * l1 + 0.2 * (1.0 - s)
        loss.backward()
        out[f"img_{i}"], out[f"gt_{i}"] = a.numpy(), b.numpy()
        out[f"l1_{i}"] = np.array([float(l1)])
        out[f"ssim_{i}"] = np.array([float(s)])
        out[f"loss_{i}"] = np.array([float(loss)])
        out[f"grad_{i}"] = x.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "loss.npz"), **out)

    # ---- Sigma3D / activations ----
    general_utils.torch = CpuTorch()  # module-scoped: only general_utils sees the CPU view
    out = {}
    n = 1024
    raw_scaling = torch.from_numpy(rng.normal(-3.0, 0.8, (n, 3)).astype(np.float32))
    raw_rotation = torch.from_numpy(rng.standard_normal((n, 4)).astype(np.float32) * 1.7)
    raw_opacity = torch.from_numpy(rng.normal(0.0, 2.0, (n, 1)).astype(np.float32))
    scales = torch.exp(raw_scaling)                            # scaling_activation
    rot_unit = torch.nn.functional.normalize(raw_rotation)     # rotation_activation
    out["raw_scaling"], out["raw_rotation"], out["raw_opacity"] = (raw_scaling.numpy(), raw_rotation.numpy(),
                                                                    raw_opacity.numpy())
    out["scales"], out["rot_unit"] = scales.numpy(), rot_unit.numpy()
    out["opacity"] = torch.sigmoid(raw_opacity).numpy()
    out["inverse_sigmoid"] = general_utils.inverse_sigmoid(torch.sigmoid(raw_opacity)).numpy()
    out["rotation_matrix"] = general_utils.build_rotation(raw_rotation).numpy()
    for tag, mod in (("m1", 1.0), ("m07", 0.7)):
        for rtag, rot in (("raw", raw_rotation), ("unit", rot_unit)):
            L = general_utils.build_scaling_rotation(mod * scales, rot)
            out[f"cov_{tag}_{rtag}"] = general_utils.strip_symmetric(L @ L.transpose(1, 2)).numpy()
    np.savez_compressed(os.path.join(HERE, "cov3d.npz"), **out)

    # ---- lr schedule ----
    f = general_utils.get_expon_lr_func(lr_init=0.00016 * 4.4, lr_final=0.0000016 * 4.4, lr_delay_mult=0.01,
                                        max_steps=30000)
    steps = np.array([0, 1, 10, 100, 999, 1000, 5000, 15000, 29999, 30000, 40000])
    np.savez_compressed(os.path.join(HERE, "lr.npz"), steps=steps, lr=np.array([f(int(s)) for s in steps]))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
