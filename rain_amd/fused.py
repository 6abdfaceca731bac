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
    # the backward's accumulator workspace, zero-filled by the forward render
    # (rr_set_forward_workspace); the first backward uses it, a second one allocates its own
    ws: torch.Tensor | None = None


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
    params = (model._xyz, model._features_dc, model._features_rest, model._opacity, model._scaling,
              model._rotation)
    return forward_params(params, model.active_sh_degree, int(camera.image_width), int(camera.image_height),
                          math.tan(camera.FoVx * 0.5), math.tan(camera.FoVy * 0.5), camera.world_view_transform,
                          camera.full_proj_transform, camera.camera_center, bg, low_pass, scale_modifier, cache)


def forward_params(params, sh_degree: int, W: int, H: int, tanfovx: float, tanfovy: float, viewmatrix, projmatrix,
                   campos, bg: torch.Tensor, low_pass: float, scale_modifier: float = 1.0,
                   cache: BinningCache | None = None):
    """forward() on explicit raw parameters (xyz, f_dc, f_rest, opacity, scaling, rotation) — the
    GaussianModel attributes before activation — and camera values as render() puts them in
    GaussianRasterizationSettings."""
    xyz = params[0]
    dev = xyz.device
    if dev.type != "cuda":
        raise RuntimeError("rain_amd.fused: tensors must be on a HIP device (no CPU fallback)")
    P = xyz.shape[0]
    H, W = int(H), int(W)
    f_dc, f_rest = params[1], params[2]
    M = 1 + f_rest.shape[1]
    D = int(sh_degree)
    L = N.raster()
    flags = N.RR_FLAG_RAW_PARAMS | _C.frame_flags()
    frame = N.RRFrame(P, D, M, W, H, float(tanfovx), float(tanfovy), float(scale_modifier), float(low_pass), 0, 0,
                      flags)
    keep = (bg.contiguous(), viewmatrix.contiguous(), projmatrix.contiguous(), campos.contiguous())
    cam = N.RRCamera(*[_p(t) for t in keep])
    # kernel argument order: xyz, f_dc, opacity, scaling, rotation, f_rest
    params = tuple(t.detach() for t in (xyz, f_dc, params[3], params[4], params[5], f_rest))
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
    ws = _register_workspace(L, P, dev)
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
        _check_render(L, rc, "fused forward")
        st = RawFrame(frame, cam, gs, (keep, params), radii, geom, img, binning, nr.value, P, M, ws)
        return color, radii, depth, st
    if P > 0:
        _check_render(L, L.rr_forward_geometry(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _p(radii),
                                               _p(geom), geom.numel(), _p(img), img.numel(), ctypes.byref(nr),
                                               ctypes.byref(npairs), stream), "fused forward")
    binning = torch.empty((L.rr_binning_bytes(npairs.value, W, H) if npairs.value > 0 else 0,), **u8)
    if P > 0:
        _check_render(L, L.rr_forward_render(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _p(radii),
                                             _p(geom), _p(img), _p(binning), binning.numel(), npairs.value, _p(color),
                                             _p(depth), stream), "fused forward")
    else:
        color.copy_(bg.view(3, 1, 1).expand(3, H, W))
        depth.zero_()
    st = RawFrame(frame, cam, gs, (keep, params), radii, geom, img, binning, nr.value, P, M, ws)
    return color, radii, depth, st


def _register_workspace(L, P: int, dev) -> torch.Tensor | None:
    """The backward's accumulator workspace, registered for the coming render to zero-fill
    (rr_set_forward_workspace: the backward then skips its clear)."""
    if P <= 0:
        return None
    ws = torch.empty((L.rr_backward_workspace_bytes(P),), dtype=torch.uint8, device=dev)
    N.check(L.rr_set_forward_workspace(_p(ws), ws.numel()), "register workspace")
    return ws


def _check_render(L, rc: int, what: str):
    """N.check, dropping a workspace registration a failed call left pending (it must not outlive
    its buffer)."""
    if rc not in (0, N.RR_INCOMPLETE):
        L.rr_set_forward_workspace(None, 0)
    N.check(rc, what)


@dataclass
class NextFrame:
    """A frame whose preprocess the previous step's backward runs on the parameters it has just
    stepped (include/rain_raster.h rr_next_frame); forward_next() then renders it from the filled
    geometry buffer.  Built by prepare_next() before that backward."""
    frame: N.RRFrame
    cam: N.RRCamera
    keep: tuple
    radii: torch.Tensor
    geom: torch.Tensor
    P: int
    M: int
    W: int
    H: int
    desc: N.RRNextFrame = None

    def __post_init__(self):
        self.desc = N.RRNextFrame(ctypes.pointer(self.frame), ctypes.pointer(self.cam), _p(self.radii), _p(self.geom),
                                  self.geom.numel())


def prepare_next(model, camera, bg: torch.Tensor, low_pass: float, scale_modifier: float = 1.0) -> NextFrame:
    """The next frame's descriptor and output buffers (geometry buffer, radii) for `camera` at the
    model's current P, M and SH degree."""
    xyz = model._xyz
    dev = xyz.device
    P = xyz.shape[0]
    H, W = int(camera.image_height), int(camera.image_width)
    M = 1 + model._features_rest.shape[1]
    L = N.raster()
    frame = N.RRFrame(P, int(model.active_sh_degree), M, W, H, math.tan(camera.FoVx * 0.5),
                      math.tan(camera.FoVy * 0.5), float(scale_modifier), float(low_pass), 0, 0,
                      N.RR_FLAG_RAW_PARAMS | _C.frame_flags())
    keep = (bg.contiguous(), camera.world_view_transform.contiguous(), camera.full_proj_transform.contiguous(),
            camera.camera_center.contiguous())
    cam = N.RRCamera(*[_p(t) for t in keep])
    radii = torch.empty((P,), dtype=torch.int32, device=dev)
    geom = torch.empty((L.rr_geometry_bytes(P),), dtype=torch.uint8, device=dev)
    return NextFrame(frame, cam, keep, radii, geom, P, M, W, H)


def forward_next(nxt: NextFrame, model, cache: BinningCache | None = None):
    """forward() of a frame whose geometry the previous backward filled (rr_forward_from_geometry):
    the same outputs and RawFrame, without the preprocess launch."""
    L = N.raster()
    dev = nxt.geom.device
    P, W, H = nxt.P, nxt.W, nxt.H
    params = tuple(t.detach() for t in (model._xyz, model._features_dc, model._opacity, model._scaling,
                                        model._rotation, model._features_rest))
    gs = N.RRGaussians(_p(params[0]), _p(params[1]), None, _p(params[2]), _p(params[3]), _p(params[4]), None,
                       _p(params[5]))
    fo = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    color = torch.empty((3, H, W), **fo)
    depth = torch.empty((1, H, W), **fo)
    img = torch.empty((L.rr_image_bytes(W, H),), **u8)
    stream = N.stream_of(nxt.geom)
    nr, npairs = ctypes.c_int(0), ctypes.c_int(0)
    need = ctypes.c_size_t(0)
    ws = _register_workspace(L, P, dev)
    binning = cache.buf if cache is not None and cache.buf is not None and cache.buf.device == dev \
        else torch.empty((0,), **u8)
    rc = L.rr_forward_from_geometry(ctypes.byref(nxt.frame), ctypes.byref(nxt.cam), _p(nxt.radii), _p(nxt.geom),
                                    nxt.geom.numel(), _p(img), img.numel(), _p(binning), binning.numel(),
                                    ctypes.byref(nr), ctypes.byref(npairs), ctypes.byref(need), _p(color), _p(depth),
                                    stream)
    if rc == N.RR_INCOMPLETE:  # the pairs outgrew the buffer: grow it and run the second stage
        binning = cache.get(need.value, dev) if cache is not None else torch.empty((need.value,), **u8)
        rc = L.rr_forward_render_geometry(ctypes.byref(nxt.frame), ctypes.byref(nxt.cam), _p(nxt.radii),
                                          _p(nxt.geom), _p(img), _p(binning), binning.numel(), npairs.value,
                                          _p(color), _p(depth), stream)
    _check_render(L, rc, "fused forward (precomputed geometry)")
    st = RawFrame(nxt.frame, nxt.cam, gs, (nxt.keep, params), nxt.radii, nxt.geom, img, binning, nr.value, P, nxt.M,
                  ws)
    return color, nxt.radii, depth, st


def backward(st: RawFrame, dL_dpix: torch.Tensor, grads: dict | None, stats: tuple | None = None,
             adam: "N.RRAdam | None" = None, dmeans2D: torch.Tensor | None = None, next_frame: NextFrame | None = None):
    """Write dLoss/d(raw parameter) into grads['xyz'|'f_dc'|'f_rest'|'opacity'|'scaling'|'rotation']
    (contiguous fp32 tensors of the parameter shapes, fully overwritten) and, if `stats` =
    (grad_accum [P,1], denom [P,1], max_radii2D [P]) is given, update the densification statistics
    in place for every Gaussian with radii > 0.  With `adam` (rain_amd.optim.FusedAdam.fused_step)
    the optimizer step is applied to the parameters in the same pass and `grads` may be None; with
    `next_frame` (prepare_next, needs `adam`) the same pass runs that frame's preprocess on the
    stepped parameters.
    `dmeans2D` ([P,3] contiguous fp32, optional) receives the screen-space (NDC) mean gradient —
    what the reference leaves in viewspace_points.grad — with z = 0."""
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
    if dmeans2D is not None and (not dmeans2D.is_contiguous() or tuple(dmeans2D.shape) != (st.P, 3)):
        raise RuntimeError("rain_amd.fused: dmeans2D must be a contiguous [P, 3] tensor")
    out = N.RRGrads(_p(dmeans2D), None, _p(grads["opacity"]), _p(grads["xyz"]), None, _p(grads["f_dc"]),
                    _p(grads["scaling"]), _p(grads["rotation"]), _p(grads["f_rest"]), _p(acc), _p(den), _p(mr),
                    ctypes.pointer(adam) if adam is not None else None,
                    ctypes.pointer(next_frame.desc) if next_frame is not None else None)
    dev = dpix.device
    frame = st.frame
    if st.ws is not None:  # zero-filled by the forward render: the backward skips its clear
        ws, st.ws = st.ws, None
        frame = N.RRFrame.from_buffer_copy(st.frame)
        frame.flags |= N.RR_FLAG_WORKSPACE_REGISTERED
    else:
        ws = torch.empty((L.rr_backward_workspace_bytes(st.P),), dtype=torch.uint8, device=dev)
    N.check(L.rr_backward(ctypes.byref(frame), ctypes.byref(st.cam), ctypes.byref(st.gs), _p(st.radii),
                          _p(st.geom), _p(st.img), _p(st.binning), st.num_rendered, _p(dpix), _p(ws), ws.numel(),
                          ctypes.byref(out), N.stream_of(dpix)), "fused backward")


class RasterizeRawParams(torch.autograd.Function):
    """The rasterizer as an autograd function of GaussianModel's RAW parameters (render()'s fast
    path, rain_amd/renderer.py): the getters' activations (exp, normalize, sigmoid, the f_dc /
    f_rest concatenation — gaussian_model.py:85-105) run inside the preprocess and their chain rule
    inside the per-Gaussian backward, so autograd sees one node instead of the getters' elementwise
    kernels and the [P,16,3] feature copy.  Gradients: the six raw parameters and means2D (the
    NDC-space screen gradient the reference leaves in viewspace_points.grad); the same arithmetic
    as GaussianRasterizer over the activated tensors (tests/test_fused_gpu.py)."""

    @staticmethod
    def forward(ctx, xyz, f_dc, f_rest, opacity, scaling, rotation, means2D, sh_degree, W, H, tanfovx, tanfovy,
                viewmatrix, projmatrix, campos, bg, low_pass, scale_modifier):
        color, radii, depth, st = forward_params((xyz, f_dc, f_rest, opacity, scaling, rotation), sh_degree, W, H,
                                                 tanfovx, tanfovy, viewmatrix, projmatrix, campos, bg, low_pass,
                                                 scale_modifier)
        # the parameters as saved tensors (the reference saves its inputs, __init__.py:85-87): autograd's
        # version check then rejects a backward after they were modified in place.  The scratch
        # buffers and camera tensors are saved too, so that autograd frees them after a backward
        # that does not retain the graph; ctx keeps only the descriptors (plain structs).
        keep, _p6 = st.keep
        ctx.save_for_backward(xyz, f_dc, f_rest, opacity, scaling, rotation, st.radii, st.geom, st.img, st.binning,
                              st.ws, *keep)
        ctx.desc = (st.frame, st.cam, st.gs, st.num_rendered, st.P, st.M)
        ctx.mark_non_differentiable(radii, depth)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for radii / depth (two fills)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_color, _grad_radii, _grad_depth):
        # (raises if a parameter changed in place since the forward)
        xyz, f_dc, f_rest, opacity, scaling, rotation, radii, geom, img, binning, ws, *keep = ctx.saved_tensors
        frame, cam, gs, num_rendered, P, M = ctx.desc
        p = (xyz, f_dc, opacity, scaling, rotation, f_rest)  # kernel order
        # the zero-filled workspace serves the first backward only (a retained graph's second one
        # allocates and clears its own)
        ws_first = ws if not getattr(ctx, "ws_used", False) else None
        ctx.ws_used = True
        st = RawFrame(frame, cam, gs, (tuple(keep), p), radii, geom, img, binning, num_rendered, P, M, ws_first)
        if grad_color is None:  # the image unused by the loss (materialize_grads off)
            grad_color = torch.zeros((3, frame.height, frame.width), dtype=torch.float32, device=xyz.device)
        grads = dict(xyz=torch.empty_like(p[0]), f_dc=torch.empty_like(p[1]), opacity=torch.empty_like(p[2]),
                     scaling=torch.empty_like(p[3]), rotation=torch.empty_like(p[4]), f_rest=torch.empty_like(p[5]))
        d2 = torch.empty((st.P, 3), dtype=torch.float32, device=p[0].device)
        backward(st, grad_color, grads, dmeans2D=d2)
        return (grads["xyz"], grads["f_dc"], grads["f_rest"], grads["opacity"], grads["scaling"], grads["rotation"], d2,
                None, None, None, None, None, None, None, None, None, None, None)
