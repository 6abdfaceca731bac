"""Camera matrices in the reference's conventions.

Restates, in numpy/torch, the helpers the reference uses to build the rasterizer's
``viewmatrix`` / ``projmatrix`` / ``campos`` inputs:

* ``getWorld2View2``      utils/graphics_utils.py:27-38
* ``getProjectionMatrix`` utils/graphics_utils.py:40-60
* ``fov2focal/focal2fov`` utils/graphics_utils.py:62-66
* ``Camera`` matrices     scene/cameras.py:102-111  (world_view_transform is W2C^T, i.e. the
  column-major memory layout the kernels read; full_proj_transform = (P·W2C)^T)

plus the synthetic camera rig of SURVEY §8(d): N views on a Fibonacci sphere looking at the
origin (up = +z), NeRF-synthetic FoV.  Pinned against the reference's own functions by
tests/golden (make_golden.py imports them in the dev container).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


def getWorld2View2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = (C2W[:3, 3] + translate) * scale
    C2W[:3, 3] = cam_center
    return np.float32(np.linalg.inv(C2W))


def getProjectionMatrix(znear, zfar, fovX, fovY):
    tan_half_y = math.tan(fovY / 2)
    tan_half_x = math.tan(fovX / 2)
    top = tan_half_y * znear
    bottom = -top
    right = tan_half_x * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def fov2focal(fov, pixels):
    return pixels / (2 * math.tan(fov / 2))


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


@dataclass
class Camera:
    """Matrix part of scene/cameras.py:Camera (no image).  All tensors on ``device``."""
    R: np.ndarray
    T: np.ndarray
    FoVx: float
    FoVy: float
    image_width: int
    image_height: int
    uid: int = 0
    znear: float = 0.01
    zfar: float = 100.0
    device: str = "cpu"

    def __post_init__(self):
        # transposed then made contiguous once: the kernels read the column-major W2C, and a strided
        # view would cost a copy kernel in every render
        self.world_view_transform = torch.tensor(getWorld2View2(self.R, self.T)).transpose(0, 1).contiguous().to(
            self.device)
        self.projection_matrix = getProjectionMatrix(self.znear, self.zfar, self.FoVx, self.FoVy).transpose(0, 1).to(
            self.device)
        self.full_proj_transform = (self.world_view_transform.unsqueeze(0).bmm(
            self.projection_matrix.unsqueeze(0))).squeeze(0)
        self.camera_center = self.world_view_transform.inverse()[3, :3].contiguous()

    def to(self, device):
        return Camera(self.R, self.T, self.FoVx, self.FoVy, self.image_width, self.image_height, self.uid,
                      self.znear, self.zfar, str(device))


def look_at_R_T(eye: np.ndarray, target=np.zeros(3), up=np.array([0.0, 0.0, 1.0])):
    """COLMAP-style (R, T) for a camera at ``eye`` looking at ``target``: x right, y down, z forward.

    The reference stores R as camera-to-world rotation and T as the world-to-camera translation
    (scene/dataset_readers.py:246-252: R = transpose(w2c[:3,:3]), T = w2c[:3,3])."""
    fwd = target - eye
    fwd = fwd / np.linalg.norm(fwd)
    right = np.cross(fwd, up)
    if np.linalg.norm(right) < 1e-6:
        right = np.cross(fwd, np.array([0.0, 1.0, 0.0]))
    right = right / np.linalg.norm(right)
    down = np.cross(fwd, right)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, down, fwd, eye
    w2c = np.linalg.inv(c2w)
    return np.transpose(w2c[:3, :3]), w2c[:3, 3]


def fibonacci_cameras(n: int, width: int, height: int, radius: float = 4.0, fovx: float = 0.6911112,
                      device: str = "cpu"):
    """``n`` views on a Fibonacci sphere of ``radius`` looking at the origin."""
    fovy = focal2fov(fov2focal(fovx, width), height)
    cams = []
    golden = math.pi * (3.0 - math.sqrt(5.0))
    for i in range(n):
        z = 1.0 - 2.0 * (i + 0.5) / n
        r = math.sqrt(max(0.0, 1.0 - z * z))
        th = golden * i
        eye = radius * np.array([r * math.cos(th), r * math.sin(th), z])
        R, T = look_at_R_T(eye)
        cams.append(Camera(R, T, fovx, fovy, width, height, uid=i, device=device))
    return cams
