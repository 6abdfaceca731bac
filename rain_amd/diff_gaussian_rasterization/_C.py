"""MI355X ``_C`` module: same functions, argument orders and return tuples as the reference's
pybind extension (submodules/diff_gaussian_rasterization/ext.cpp:4-7, rasterize_points.cu:24-212),
implemented over the C ABI in include/rain_raster.h.

* ``rasterize_gaussians``           ≙ RasterizeGaussiansCUDA          (rasterize_points.cu:24-108)
* ``rasterize_gaussians_backward``  ≙ RasterizeGaussiansBackwardCUDA  (rasterize_points.cu:110-191)
* ``mark_visible``                  ≙ markVisible                     (rasterize_points.cu:193-212)

Differences that are deliberate and invisible to callers: scratch buffers are sized by the C
ABI's *_bytes() queries instead of grown through std::function callbacks; outputs the kernels
write completely are allocated with torch.empty (the reference zero-fills them first); scratch and
outputs live on ``means3D.device`` and kernels run on torch's current stream of that device (the
reference uses the current device and the legacy default stream).
"""
from __future__ import annotations

import ctypes
import os

import torch

from .. import _native as N

NUM_CHANNELS = 3

# Exact tile culling (include/rain_raster.h RR_FLAG_NO_TILE_CULLING): identical outputs, fewer
# (tile, Gaussian) pairs.  RAIN_TILE_CULLING=0 restores the reference's bounding-square binning.
TILE_CULLING = os.environ.get("RAIN_TILE_CULLING", "1") != "0"
# Early-stop binning (include/rain_raster.h RR_FLAG_FULL_BINNING): identical outputs, tile lists
# cut past saturation.  False (or RAIN_EARLY_STOP=0) bins every pair (full per-tile lists).
EARLY_STOP = os.environ.get("RAIN_EARLY_STOP", "1") != "0"


def frame_flags():
    return (0 if TILE_CULLING else N.RR_FLAG_NO_TILE_CULLING) | (0 if EARLY_STOP else N.RR_FLAG_FULL_BINNING)


def _ptr(t):
    """Device pointer of a tensor, or None for an empty ("absent") tensor (nullptr in the reference)."""
    if t is None or t.numel() == 0:
        return None
    return ctypes.c_void_p(t.data_ptr())


def _dev_f32(t, device, name):
    if t is None or t.numel() == 0:
        return None
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be a float32 tensor (got {t.dtype})")
    if t.device != device:
        raise RuntimeError(f"{name} must be on {device} (got {t.device})")
    return t.contiguous()


def _require_device(means3D):
    if means3D.device.type != "cuda":
        raise RuntimeError("rain_amd rasterizer: tensors must be on a HIP device (no CPU fallback)")
    return means3D.device


def _frame(P, degree, M, W, H, tan_fovx, tan_fovy, scale_modifier, low_pass, prefiltered, debug):
    flags = frame_flags()
    return N.RRFrame(int(P), int(degree), int(M), int(W), int(H), float(tan_fovx), float(tan_fovy),
                     float(scale_modifier), float(low_pass), int(bool(prefiltered)), int(bool(debug)), flags)


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug, low_pass):
    out = _rasterize(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                     viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                     prefiltered, debug, low_pass, False)
    return out[:4] + out[5:]


def rasterize_gaussians_aux(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                            viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                            prefiltered, debug, low_pass):
    """rasterize_gaussians plus the aux normal map (include/rain_raster.h RR_FLAG_AUX_NORMAL; no
    reference counterpart): returns (num_rendered, color, radii, depth, normal [3,H,W], geomBuffer,
    binningBuffer, imgBuffer).  The buffers are valid for rasterize_gaussians_backward."""
    return _rasterize(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                      viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                      prefiltered, debug, low_pass, True)


def _rasterize(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
               viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
               prefiltered, debug, low_pass, normal):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    device = _require_device(means3D)
    fopts = dict(dtype=torch.float32, device=device)
    u8 = dict(dtype=torch.uint8, device=device)
    if P == 0:
        return (0, torch.zeros((NUM_CHANNELS, H, W), **fopts), torch.zeros((0,), dtype=torch.int32, device=device),
                torch.zeros((1, H, W), **fopts), torch.zeros((3, H, W), **fopts) if normal else None,
                torch.empty((0,), **u8), torch.empty((0,), **u8), torch.empty((0,), **u8))
    L = N.raster()
    M = sh.size(1) if sh.size(0) != 0 else 0
    keep = dict(
        bg=_dev_f32(background, device, "bg"), means3D=_dev_f32(means3D, device, "means3D"),
        colors=_dev_f32(colors, device, "colors_precomp"), opacity=_dev_f32(opacity, device, "opacities"),
        scales=_dev_f32(scales, device, "scales"), rotations=_dev_f32(rotations, device, "rotations"),
        cov3D=_dev_f32(cov3D_precomp, device, "cov3D_precomp"), view=_dev_f32(viewmatrix, device, "viewmatrix"),
        proj=_dev_f32(projmatrix, device, "projmatrix"), sh=_dev_f32(sh, device, "sh"),
        campos=_dev_f32(campos, device, "campos"))
    frame = _frame(P, degree, M, W, H, tan_fovx, tan_fovy, scale_modifier, low_pass, prefiltered, debug)
    if normal:
        frame.flags |= N.RR_FLAG_AUX_NORMAL
    cam = N.RRCamera(_ptr(keep["bg"]), _ptr(keep["view"]), _ptr(keep["proj"]), _ptr(keep["campos"]))
    gs = N.RRGaussians(_ptr(keep["means3D"]), _ptr(keep["sh"]), _ptr(keep["colors"]), _ptr(keep["opacity"]),
                       _ptr(keep["scales"]), _ptr(keep["rotations"]), _ptr(keep["cov3D"]))
    out_color = torch.empty((NUM_CHANNELS, H, W), **fopts)
    out_depth = torch.empty((1, H, W), **fopts)
    out_normal = torch.empty((3, H, W), **fopts) if normal else None
    radii = torch.empty((P,), dtype=torch.int32, device=device)
    geom = torch.empty((L.rr_geometry_bytes(P),), **u8)
    img = torch.empty((L.rr_image_bytes(W, H),), **u8)
    stream = N.stream_of(means3D)
    nr = ctypes.c_int(0)
    npairs = ctypes.c_int(0)
    N.check(L.rr_forward_geometry(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _ptr(radii),
                                  _ptr(geom), geom.numel(), _ptr(img), img.numel(), ctypes.byref(nr),
                                  ctypes.byref(npairs), stream),
            "rasterize_gaussians")
    num_rendered, num_pairs = nr.value, npairs.value
    binning = torch.empty((L.rr_binning_bytes(num_pairs, W, H) if num_pairs > 0 else 0,), **u8)
    N.check(L.rr_forward_render_aux(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _ptr(radii),
                                    _ptr(geom), _ptr(img), _ptr(binning), binning.numel(), num_pairs,
                                    _ptr(out_color), _ptr(out_depth), _ptr(out_normal), stream),
            "rasterize_gaussians")
    # num_rendered is the reference's value (sum of bounding-square tile counts)
    return num_rendered, out_color, radii, out_depth, out_normal, geom, binning, img


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree,
                                 campos, geomBuffer, R, binningBuffer, imageBuffer, debug, low_pass):
    P = means3D.size(0)
    H, W = dL_dout_color.size(1), dL_dout_color.size(2)
    M = sh.size(1) if sh.size(0) != 0 else 0
    device = _require_device(means3D)
    fopts = dict(dtype=torch.float32, device=device)
    if P == 0:
        z = lambda *s: torch.zeros(s, **fopts)  # noqa: E731
        return (z(0, 3), z(0, NUM_CHANNELS), z(0, 1), z(0, 3), z(0, 6), z(0, M, 3), z(0, 3), z(0, 4))
    L = N.raster()
    keep = dict(
        bg=_dev_f32(background, device, "bg"), means3D=_dev_f32(means3D, device, "means3D"),
        colors=_dev_f32(colors, device, "colors_precomp"), scales=_dev_f32(scales, device, "scales"),
        rotations=_dev_f32(rotations, device, "rotations"), cov3D=_dev_f32(cov3D_precomp, device, "cov3D_precomp"),
        view=_dev_f32(viewmatrix, device, "viewmatrix"), proj=_dev_f32(projmatrix, device, "projmatrix"),
        sh=_dev_f32(sh, device, "sh"), campos=_dev_f32(campos, device, "campos"),
        dpix=_dev_f32(dL_dout_color, device, "dL_dout_color"), radii=radii.contiguous())
    # opacities are not needed by the backward (the reference does not pass them either)
    frame = _frame(P, degree, M, W, H, tan_fovx, tan_fovy, scale_modifier, low_pass, False, debug)
    cam = N.RRCamera(_ptr(keep["bg"]), _ptr(keep["view"]), _ptr(keep["proj"]), _ptr(keep["campos"]))
    gs = N.RRGaussians(_ptr(keep["means3D"]), _ptr(keep["sh"]), _ptr(keep["colors"]), None,
                       _ptr(keep["scales"]), _ptr(keep["rotations"]), _ptr(keep["cov3D"]))
    out = dict(dL_dmeans2D=torch.empty((P, 3), **fopts), dL_dcolors=torch.empty((P, NUM_CHANNELS), **fopts),
               dL_dopacity=torch.empty((P, 1), **fopts), dL_dmeans3D=torch.empty((P, 3), **fopts),
               dL_dcov3D=torch.empty((P, 6), **fopts), dL_dsh=torch.empty((P, M, 3), **fopts),
               dL_dscales=torch.empty((P, 3), **fopts), dL_drotations=torch.empty((P, 4), **fopts))
    grads = N.RRGrads(*[_ptr(out[k]) for k in ("dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D",
                                               "dL_dcov3D", "dL_dsh", "dL_dscales", "dL_drotations")])
    ws = torch.empty((L.rr_backward_workspace_bytes(P),), dtype=torch.uint8, device=device)
    stream = N.stream_of(means3D)
    N.check(L.rr_backward(ctypes.byref(frame), ctypes.byref(cam), ctypes.byref(gs), _ptr(keep["radii"]),
                          _ptr(geomBuffer), _ptr(imageBuffer), _ptr(binningBuffer), int(R), _ptr(keep["dpix"]),
                          _ptr(ws), ws.numel(), ctypes.byref(grads), stream),
            "rasterize_gaussians_backward")
    return (out["dL_dmeans2D"], out["dL_dcolors"], out["dL_dopacity"], out["dL_dmeans3D"], out["dL_dcov3D"],
            out["dL_dsh"], out["dL_dscales"], out["dL_drotations"])


def mark_visible(means3D, viewmatrix, projmatrix):
    P = means3D.size(0)
    device = _require_device(means3D)
    present = torch.zeros((P,), dtype=torch.bool, device=device)
    if P != 0:
        m = _dev_f32(means3D, device, "means3D")
        v = _dev_f32(viewmatrix, device, "viewmatrix")
        p = _dev_f32(projmatrix, device, "projmatrix")
        N.check(N.raster().rr_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), N.stream_of(means3D)),
                "mark_visible")
    return present


def debug_views(geomBuffer, binningBuffer, imageBuffer, num_rendered, P, W, H):
    """Copies of the forward's private binning/image state (tests only): point_list [8 num_pairs]
    (4 slots per pair in the phase-A region [0, 4L) and the phase-B region [4L, 8L); tile t's list
    is point_list[ranges[t, 0]:ranges[t, 1]]),
    ranges [T,2], tile_max [T], final_T [H,W], n_contrib [H,W], splats [P,12]."""
    f = _frame(P, 0, 0, W, H, 1.0, 1.0, 1.0, 0.3, False, False)
    num_rendered = frame_stats(geomBuffer, imageBuffer, P, W, H)["num_pairs"]
    v = N.RRDebugViews()
    N.check(N.raster().rr_debug_get_views(ctypes.byref(f), _ptr(geomBuffer), _ptr(imageBuffer), _ptr(binningBuffer),
                                          int(num_rendered), ctypes.byref(v)), "debug_views")
    dev = geomBuffer.device
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy

    def grab(ptr, n, dtype, src):
        out = torch.empty((n,), dtype=dtype, device=dev)
        if n:
            base = src.data_ptr()
            off = ptr - base
            nbytes = n * out.element_size()
            assert 0 <= off and off + nbytes <= src.numel(), "debug view outside its buffer"
            out.view(torch.uint8).copy_(src[off:off + nbytes])
        return out

    return dict(
        # per-tile lists live at the ranges' absolute positions: 4 slots per (bin, Gaussian) pair
        # (phase A's region [0, 4L) and phase B's [4L, 8L); clamped to the buffer)
        point_list=grab(v.point_list, min(8 * num_rendered, (binningBuffer.numel() - (v.point_list -
                                          binningBuffer.data_ptr())) // 4), torch.int32, binningBuffer)
        if num_rendered else torch.empty((0,), dtype=torch.int32, device=dev),
        ranges=grab(v.ranges, 2 * T, torch.int32, imageBuffer).view(T, 2),
        tile_max=grab(v.tile_max, T, torch.int32, imageBuffer),
        final_T=grab(v.final_T, H * W, torch.float32, imageBuffer).view(H, W),
        n_contrib=grab(v.n_contrib, H * W, torch.int32, imageBuffer).view(H, W),
        splats=grab(v.splats, 12 * P, torch.float32, geomBuffer).view(P, 12))


def frame_stats(geomBuffer, imageBuffer, P, W, H):
    """(L, visible count V, L_eff = sum of per-tile max n_contrib, T) of the last forward — bench/tests."""
    f = _frame(P, 0, 0, W, H, 1.0, 1.0, 1.0, 0.3, False, False)
    st = N.RRFrameStats()
    N.check(N.raster().rr_read_frame_stats(ctypes.byref(f), _ptr(geomBuffer), _ptr(imageBuffer), ctypes.byref(st),
                                           N.stream_of(geomBuffer)), "frame_stats")
    return dict(num_rendered=st.num_rendered, num_visible=st.num_visible, l_eff=st.l_eff, tiles=st.tiles,
                num_pairs=st.num_pairs, num_binned=st.num_binned, phase_b_pairs=st.phase_b_pairs,
                phase_b_slots=st.phase_b_slots)
