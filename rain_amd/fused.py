"""Training-step rasterizer over GaussianModel's raw parameters (include/rain_raster.h
RR_FLAG_RAW_PARAMS).

The reference's iteration (train.py:109-134) goes: getters (exp / normalize / sigmoid / cat,
gaussian_model.py:85-105) -> render() -> rasterizer -> autograd back through the getters into six
leaf gradients, plus masked scatters for the densification statistics.  Here the getters run
inside the rasterizer's preprocess, the chain rule through them runs inside its per-Gaussian
backward kernel, which writes the six raw-parameter gradients straight into their (flat) .grad
buffers and folds in the densification statistics — no SH concatenation, no autograd graph, no
[P,3] means2D tensor.  The arithmetic is the same as the reference-API path (rain_amd.renderer /
diff_gaussian_rasterization) on the activated tensors; tests/test_fused_gpu.py compares the two.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import torch

from . import _native as N
from .diff_gaussian_rasterization import _C


def _p(t):
    return None if t is None or t.numel() == 0 else ctypes.c_void_p(t.data_ptr())


@dataclass
class RawFrame:
    """State a forward hands to its backward (the reference's saved tensors, __init__.py:85-87)."""
    frame: N.RRFrame
    cam: N.RRCamera
    gs: N.RRGaussians
    keep: tuple
    radii: torch.Tensor
    geom: torch.Tensor
    img: torch.Tensor
    binning: torch.Tensor
    num_rendered: int
    P: int
    M: int


class BinningCache:
    """A grow-only binning buffer reused frame after frame (the training loop renders one frame,
    runs its backward, then renders the next, all on one stream, so frame s+1's binning never
    overwrites a list frame s's backward still reads).  With it the forward is one native call
    (rr_forward): the device waits only for the pair-count read-back, not for a return to Python."""

    def __init__(self, headroom: float = 1.25):
        self.buf = None
        self.headroom = headroom

    def get(self, nbytes: int, dev) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != dev:
            self.buf = torch.empty((int(nbytes * self.headroom) + 4096,), dtype=torch.uint8, device=dev)
        return self.buf


def forward(model, camera, bg: torch.Tensor, low_pass: float, scale_modifier: float = 1.0,
            cache: BinningCache | None = None):
    """Render `camera` from `model` (a GaussianModel) in raw-parameter mode.
    Returns (color [3,H,W], radii [P] int32, depth [1,H,W], RawFrame).  With `cache` the binning
    buffer is reused (see BinningCache) and must not be needed by an earlier frame's pending
    backward."""
    xyz = model._xyz
    dev = xyz.device
    if dev.type != "cuda":
        raise RuntimeError("rain_amd.fused: tensors must be on a HIP device (no CPU fallback)")
    P = xyz.shape[0]
    H, W = int(camera.image_height), int(camera.image_width)
    f_dc, f_rest = model._features_dc, model._features_rest
    M = 1 + f_rest.shape[1]
    D = model.active_sh_degree
    L = N.raster()
    flags = N.RR_FLAG_RAW_PARAMS | _C.frame_flags()
    frame = N.RRFrame(P, D, M, W, H, math.tan(camera.FoVx * 0.5), math.tan(camera.FoVy * 0.5),
                      float(scale_modifier), float(low_pass), 0, 0, flags)
    keep = (bg.contiguous(), camera.world_view_transform.contiguous(), camera.full_proj_transform.contiguous(),
            camera.camera_center.contiguous())
    cam = N.RRCamera(*[_p(t) for t in keep])
    params = tuple(t.detach() for t in (xyz, f_dc, model._opacity, model._scaling, model._rotation, f_rest))
    for t in params:
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError("rain_amd.fused: parameters must be contiguous float32")
    gs = N.RRGaussians(_p(params[0]), _p(params[1]), None, _p(params[2]), _p(params[3]), _p(params[4]), None,
                       _p(params[5]))
    fo = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    color = torch.empty((3, H, W), **fo)
    depth = torch.empty((1, H, W), **fo)
    radii = torch.empty((P,), dtype=torch.int32, device=dev)
    geom = torch.empty((L.rr_geometry_bytes(P),), **u8)
    img = torch.empty((L.rr_image_bytes(W, H),), **u8)
    stream = N.stream_of(xyz)
    nr, npairs = ctypes.c_int(0), ctypes.c_int(0)
    if P > 0 and cache is not None:
        binning = cache.buf if cache.buf is not None and cache.buf.device == dev else torch.empty((0,), **u8)
        need = ctypes.c_size_t(0)
        rc = L.rr_forward(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _p(radii), _p(geom), geom.numel(),
                          _p(img), img.numel(), _p(binning), binning.numel(), ctypes.byref(nr), ctypes.byref(npairs),
                          ctypes.byref(need), _p(color), _p(depth), stream)
        if rc == N.RR_INCOMPLETE:  # the pairs outgrew the buffer: grow it and run stage 2
            binning = cache.get(need.value, dev)
            rc = L.rr_forward_render(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _p(radii), _p(geom),
                                     _p(img), _p(binning), binning.numel(), npairs.value, _p(color), _p(depth),
                                     stream)
        N.check(rc, "fused forward")
        st = RawFrame(frame, cam, gs, (keep, params), radii, geom, img, binning, nr.value, P, M)
        return color, radii, depth, st
    if P > 0:
        N.check(L.rr_forward_geometry(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _p(radii), _p(geom),
                                      geom.numel(), _p(img), img.numel(), ctypes.byref(nr), ctypes.byref(npairs),
                                      stream), "fused forward")
    binning = torch.empty((L.rr_binning_bytes(npairs.value, W, H) if npairs.value > 0 else 0,), **u8)
    if P > 0:
        N.check(L.rr_forward_render(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _p(radii), _p(geom),
                                    _p(img), _p(binning), binning.numel(), npairs.value, _p(color), _p(depth),
                                    stream), "fused forward")
    else:
        color.copy_(bg.view(3, 1, 1).expand(3, H, W))
        depth.zero_()
    st = RawFrame(frame, cam, gs, (keep, params), radii, geom, img, binning, nr.value, P, M)
    return color, radii, depth, st


def backward(st: RawFrame, dL_dpix: torch.Tensor, grads: dict | None, stats: tuple | None = None,
             adam: "N.RRAdam | None" = None):
    """Write dLoss/d(raw parameter) into grads['xyz'|'f_dc'|'f_rest'|'opacity'|'scaling'|'rotation']
    (contiguous fp32 tensors of the parameter shapes, fully overwritten) and, if `stats` =
    (grad_accum [P,1], denom [P,1], max_radii2D [P]) is given, update the densification statistics
    in place for every Gaussian with radii > 0.  With `adam` (rain_amd.optim.FusedAdam.fused_step)
    the optimizer step is applied to the parameters in the same pass and `grads` may be None."""
    if st.P == 0:
        return
    L = N.raster()
    dpix = dL_dpix.contiguous()
    names = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")
    if grads is None:
        if adam is None:
            raise RuntimeError("rain_amd.fused.backward: nothing to do (no gradients requested, no optimizer step)")
        grads = dict.fromkeys(names)
    for k in names:
        if grads[k] is not None and not grads[k].is_contiguous():
            raise RuntimeError(f"rain_amd.fused: grads[{k!r}] must be contiguous")
    acc, den, mr = stats if stats is not None else (None, None, None)
    out = N.RRGrads(None, None, _p(grads["opacity"]), _p(grads["xyz"]), None, _p(grads["f_dc"]),
                    _p(grads["scaling"]), _p(grads["rotation"]), _p(grads["f_rest"]), _p(acc), _p(den), _p(mr),
                    ctypes.pointer(adam) if adam is not None else None)
    dev = dpix.device
    ws = torch.empty((L.rr_backward_workspace_bytes(st.P),), dtype=torch.uint8, device=dev)
    N.check(L.rr_backward(ctypes.byref(st.frame), ctypes.byref(st.cam), ctypes.byref(st.gs), _p(st.radii),
                          _p(st.geom), _p(st.img), _p(st.binning), st.num_rendered, _p(dpix), _p(ws), ws.numel(),
                          ctypes.byref(out), N.stream_of(dpix)), "fused backward")
