"""``simple_knn._C`` over the C ABI in include/rain_knn.h (librain_knn.so).

distCUDA2(points [P,3] float32 on a HIP device) -> [P] float32: mean squared distance to the 3
nearest other points (spatial.cu:4-13, simple_knn.cu:164-207), exact, with the reference's edge
behaviour (origin-including Morton bbox; FLT_MAX for missing neighbours when P < 4).  The result is
allocated on ``points.device`` and computed on its current stream; there is no CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native as N


def distCUDA2(points: torch.Tensor) -> torch.Tensor:
    if points.dim() != 2 or points.size(1) != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    if points.device.type != "cuda":
        raise RuntimeError("rain_amd simple_knn: points must be on a HIP device (no CPU fallback)")
    pts = points.contiguous().float()
    P = pts.size(0)
    out = torch.zeros((P,), dtype=torch.float32, device=pts.device)
    if P == 0:
        return out
    L = N.knn()
    ws = torch.empty((L.sk_workspace_bytes(P),), dtype=torch.uint8, device=pts.device)
    rc = L.sk_dist_cuda2(P, ctypes.c_void_p(pts.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                         ctypes.c_void_p(ws.data_ptr()), ws.numel(), N.stream_of(pts))
    if rc != 0:
        raise RuntimeError(f"distCUDA2: {L.sk_last_error().decode(errors='replace')}")
    return out
