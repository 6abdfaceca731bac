"""CPU known-answer test of the oracle's aux normal map (the checker for tests/test_aux_normal_gpu.py):
one flat Gaussian (smallest scale along world z) seen by a synthetic camera.  At the pixel under its
centre the map is alpha * n with n = +-(R_w2c e_z), signed to face the camera."""
import math

import numpy as np
import torch

from rain_amd.cameras import fibonacci_cameras


def test_single_flat_gaussian(oracle):
    W = H = 64
    cam = fibonacci_cameras(5, W, H)[2]
    view = cam.world_view_transform.float().numpy()  # column-major: view.reshape(16)[4j+i] = R_w2c[i][j]
    st = oracle.Settings(image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx * 0.5),
                         tanfovy=math.tan(cam.FoVy * 0.5), bg=np.zeros(3, np.float32), scale_modifier=1.0,
                         viewmatrix=view, projmatrix=cam.full_proj_transform.float().numpy(), sh_degree=0,
                         campos=cam.camera_center.float().numpy(), low_pass=0.3)
    means = np.zeros((1, 3), np.float32)
    nr, color, radii, depth, state, nmap = oracle.forward(
        st, means, np.array([[0.8]], np.float32), colors_precomp=np.ones((1, 3), np.float32),
        scales=np.array([[0.3, 0.25, 0.001]], np.float32), rotations=np.array([[1, 0, 0, 0]], np.float32),
        normal=True)
    assert radii[0] > 0
    m = view.reshape(16)
    n_view = np.array([m[8], m[9], m[10]], np.float64)  # R_w2c e_z
    p_view = np.array([m[12], m[13], m[14]], np.float64)  # origin in view space
    if n_view @ p_view > 0:
        n_view = -n_view
    # brightest pixel = the centre: there T = 1 and the map is alpha * n
    a = color[0]
    y, x = np.unravel_index(np.argmax(a), a.shape)
    v = nmap[:, y, x].astype(np.float64)
    alpha = float(a[y, x])
    np.testing.assert_allclose(v, alpha * n_view, rtol=1e-4, atol=1e-6)
    assert np.allclose(np.linalg.norm(nmap, axis=0), color[0], atol=1e-6)  # |N| = alpha everywhere (one Gaussian)
