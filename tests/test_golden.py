"""Pin the oracle and the host-side restatements against fixtures produced by the REFERENCE's own
Python code (tests/golden/make_golden.py): SH evaluation, camera matrices, loss, LR schedule."""
import os

import numpy as np
import torch

from oracle import loss_ref
from rain_amd import cameras, gaussian_model, loss, sh_utils

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(G, name))


def test_oracle_sh_matches_reference_eval_sh(oracle):
    """forward.cu:9-60 (restated in raster_oracle.c) == utils/sh_utils.py eval_sh + 0.5, clamp 0."""
    d = _load("sh_eval.npz")
    for deg in range(4):
        sh_ref_layout = d[f"sh_{deg}"]                    # [n, 3, 16] (reference eval_sh layout)
        shs = np.ascontiguousarray(np.transpose(sh_ref_layout, (0, 2, 1)))  # kernel layout [n, 16, 3]
        rgb, clamped = oracle.sh_eval(deg, shs, d[f"dirs_{deg}"])
        np.testing.assert_allclose(rgb, d[f"rgb_{deg}"], rtol=0, atol=2e-6)
        pre = d[f"eval_{deg}"] + 0.5
        sure = np.abs(pre) > 1e-5
        np.testing.assert_array_equal(clamped[sure], (pre < 0)[sure])


def test_host_eval_sh_bitwise(oracle):
    d = _load("sh_eval.npz")
    for deg in range(4):
        v = sh_utils.eval_sh(deg, torch.from_numpy(d[f"sh_{deg}"]), torch.from_numpy(d[f"dirs_{deg}"]))
        np.testing.assert_array_equal(v.numpy(), d[f"eval_{deg}"])
    np.testing.assert_array_equal(sh_utils.RGB2SH(torch.from_numpy(d["rgb2sh_in"])).numpy(), d["rgb2sh_out"])


def test_camera_matrices_match_reference():
    d = _load("camera.npz")
    W, H, fovx = 800, 600, 0.6911112
    fovy = cameras.focal2fov(cameras.fov2focal(fovx, W), H)
    assert fovy == float(d["fovy"][0])
    for i in range(6):
        cam = cameras.Camera(d[f"R_{i}"], d[f"T_{i}"], fovx, fovy, W, H)
        np.testing.assert_array_equal(cam.world_view_transform.numpy(), d[f"view_{i}"])
        np.testing.assert_array_equal(cam.projection_matrix.numpy(), d[f"proj_{i}"])
        np.testing.assert_array_equal(cam.full_proj_transform.numpy(), d[f"full_{i}"])
        np.testing.assert_allclose(cam.camera_center.numpy(), d[f"campos_{i}"], rtol=0, atol=1e-6)


def test_loss_matches_reference():
    d = _load("loss.npz")
    for i in range(2):
        a = torch.from_numpy(d[f"img_{i}"])
        b = torch.from_numpy(d[f"gt_{i}"])
        x = a.clone().requires_grad_(True)
        l1 = loss_ref.l1_loss(x, b)
        s = loss_ref.ssim(x, b)
        total = 0.8 * l1 + 0.2 * (1.0 - s)
        total.backward()
        assert float(l1) == float(d[f"l1_{i}"][0])
        assert abs(float(s) - float(d[f"ssim_{i}"][0])) < 1e-7
        np.testing.assert_allclose(x.grad.numpy(), d[f"grad_{i}"], rtol=1e-5, atol=1e-9)
        # the separable factorisation the fused HIP kernel implements
        s2 = loss.ssim_separable(a, b)
        assert abs(float(s2) - float(d[f"ssim_{i}"][0])) < 2e-6


def test_lr_schedule_matches_reference():
    d = _load("lr.npz")
    f = gaussian_model.get_expon_lr_func(lr_init=0.00016 * 4.4, lr_final=0.0000016 * 4.4, lr_delay_mult=0.01,
                                         max_steps=30000)
    np.testing.assert_array_equal(np.array([f(int(s)) for s in d["steps"]]), d["lr"])


def _cov_close(got, want, rel=4e-6):
    """Sigma3D entries within `rel` of each Gaussian's largest variance (float32 rounding of a
    different but equivalent evaluation order: glm's M^T M vs torch's (R S)(R S)^T)."""
    scale = np.abs(want[:, [0, 3, 5]]).max(axis=1, keepdims=True)
    err = np.abs(got.astype(np.float64) - want) / scale
    assert err.max() <= rel, err.max()


def test_oracle_cov3d_matches_reference(oracle):
    """computeCov3D as restated in raster_oracle.c (forward.cu:107-141, fed the getters' unit
    quaternions as render() does) == the reference's build_scaling_rotation / strip_symmetric
    composition (gaussian_model.py:16-20) on the same scales, rotations and scale modifiers."""
    d = _load("cov3d.npz")
    for tag, mod in (("m1", 1.0), ("m07", 0.7)):
        _cov_close(oracle.cov3d(d["scales"], mod, d["rot_unit"]), d[f"cov_{tag}_unit"])
        # the Python path normalises raw quaternions itself: same Sigma as the unit ones
        _cov_close(d[f"cov_{tag}_raw"].astype(np.float32), d[f"cov_{tag}_unit"])


def test_host_getters_and_covariance_match_reference():
    """rain_amd.gaussian_model's restatements (the compute_cov3D_python path and the getters)."""
    d = _load("cov3d.npz")
    s, r = torch.from_numpy(d["scales"]), torch.from_numpy(d["raw_rotation"])
    np.testing.assert_array_equal(gaussian_model.build_rotation(r).numpy(), d["rotation_matrix"])
    for tag, mod in (("m1", 1.0), ("m07", 0.7)):
        L = gaussian_model.build_scaling_rotation(mod * s, r)
        np.testing.assert_array_equal(gaussian_model.strip_symmetric(L @ L.transpose(1, 2)).numpy(),
                                      d[f"cov_{tag}_raw"])
    op = torch.from_numpy(d["raw_opacity"])
    np.testing.assert_array_equal(torch.sigmoid(op).numpy(), d["opacity"])
    np.testing.assert_array_equal(gaussian_model.inverse_sigmoid(torch.sigmoid(op)).numpy(), d["inverse_sigmoid"])
    np.testing.assert_array_equal(torch.nn.functional.normalize(r).numpy(), d["rot_unit"])
    np.testing.assert_array_equal(torch.exp(torch.from_numpy(d["raw_scaling"])).numpy(), d["scales"])
