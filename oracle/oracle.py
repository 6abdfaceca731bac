"""ctypes front-end of the CPU oracle (oracle/raster_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package ``rain_amd``.

The functions mirror the reference's ``_C`` entry points
(submodules/diff_gaussian_rasterization/rasterize_points.cu:24-212) on numpy float32
arrays: ``forward`` ≙ RasterizeGaussiansCUDA, ``backward`` ≙ RasterizeGaussiansBackwardCUDA,
``mark_visible`` ≙ markVisible.  Parity status: see raster_oracle.c header ("parity
unpinned" against the reference binary, SH/camera pieces pinned by tests/golden).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (Makefile next to this file)."""
    src = [os.path.join(_HERE, f) for f in ("raster_oracle.c", "knn_oracle.c")]
    if force or not os.path.exists(_LIB_PATH) or any(os.path.getmtime(s) > os.path.getmtime(_LIB_PATH) for s in src):
        subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_forward.restype = ctypes.c_void_p
        L.orc_forward.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int, _f32p,
            _f32p, _f32p, _f32p, _f32p, ctypes.c_float, _f32p, _f32p,
            _f32p, _f32p, _f32p, ctypes.c_float, ctypes.c_float,
            ctypes.c_int, ctypes.c_float, _f32p, _f32p, _i32p, _i32p, ctypes.c_int, _f32p]
        L.orc_backward.restype = ctypes.c_int
        L.orc_backward.argtypes = [
            ctypes.c_void_p, _f32p, _f32p, _i32p, _f32p, _f32p, ctypes.c_float, _f32p, _f32p,
            _f32p, _f32p, _f32p, ctypes.c_float, ctypes.c_float, _f32p, _f32p, ctypes.c_float,
            _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, ctypes.c_int]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_mark_visible.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _u8p]
        L.orc_get_higher_msb.restype = ctypes.c_uint32
        L.orc_get_higher_msb.argtypes = [ctypes.c_uint32]
        for name, rt in (("orc_point_list", _u32p), ("orc_ranges", _u32p), ("orc_final_T", _f32p),
                         ("orc_n_contrib", _u32p), ("orc_xy", _f32p), ("orc_depths", _f32p),
                         ("orc_conic_opacity", _f32p), ("orc_rgb", _f32p), ("orc_cov3D", _f32p),
                         ("orc_clamped", _u8p), ("orc_tiles_touched", _u32p)):
            fn = getattr(L, name)
            fn.restype = rt
            fn.argtypes = [ctypes.c_void_p]
        L.orc_num_rendered.restype = ctypes.c_int
        L.orc_num_rendered.argtypes = [ctypes.c_void_p]
        L.orc_threads.restype = ctypes.c_int
        L.orc_sh_eval.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _f32p, _f32p, _u8p]
        L.orc_pixel_blend_list.restype = ctypes.c_int
        L.orc_pixel_blend_list.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _u32p, ctypes.c_int]
        L.orc_cov3d.restype = None
        L.orc_cov3d.argtypes = [ctypes.c_int, _f32p, ctypes.c_float, _f32p, _f32p]
        L.orc_dist_knn3.restype = None
        L.orc_dist_knn3.argtypes = [ctypes.c_int, _f32p, _f32p, ctypes.POINTER(ctypes.c_uint32), _f32p]
        _lib = L
    return _lib


def _p(a, typ=_f32p):
    if a is None:
        return None
    return a.ctypes.data_as(typ)


def _f32(a):
    if a is None:
        return None
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return a if a.size > 0 else None


@dataclass
class Settings:
    """Same fields as GaussianRasterizationSettings (diff_gaussian_rasterization/__init__.py:148-161)."""
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: np.ndarray
    scale_modifier: float
    viewmatrix: np.ndarray
    projmatrix: np.ndarray
    sh_degree: int
    campos: np.ndarray
    prefiltered: bool = False
    debug: bool = False
    low_pass: float = 0.3


class State:
    """Owns the C-side forward state (geometry, binning, image) until backward."""

    def __init__(self, handle, P, W, H):
        self.handle = handle
        self.P, self.W, self.H = P, W, H

    def __del__(self):
        try:
            if self.handle and _lib is not None:
                _lib.orc_free(self.handle)
        except Exception:  # interpreter shutdown
            pass
        self.handle = None

    def _arr(self, name, n, dtype):
        ptr = getattr(lib(), name)(self.handle)
        if n == 0:
            return np.zeros(0, dtype=dtype)
        return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)

    def blend_lists(self, cap: int = 4096):
        """Per pixel (row-major), the ordered Gaussian ids the forward blended."""
        L = lib()
        buf = np.zeros(cap, np.uint32)
        out = []
        for py in range(self.H):
            for px in range(self.W):
                n = L.orc_pixel_blend_list(self.handle, px, py, _p(buf, _u32p), cap)
                out.append(buf[:min(n, cap)].copy())
        return out

    @property
    def num_rendered(self):
        return lib().orc_num_rendered(self.handle)

    def internals(self):
        P, N = self.P, self.W * self.H
        gx, gy = (self.W + 15) // 16, (self.H + 15) // 16
        L = self.num_rendered
        return {
            "point_list": self._arr("orc_point_list", L, np.uint32),
            "ranges": self._arr("orc_ranges", 2 * gx * gy, np.uint32).reshape(-1, 2),
            "final_T": self._arr("orc_final_T", N, np.float32).reshape(self.H, self.W),
            "n_contrib": self._arr("orc_n_contrib", N, np.uint32).reshape(self.H, self.W),
            "xy": self._arr("orc_xy", 2 * P, np.float32).reshape(P, 2),
            "depths": self._arr("orc_depths", P, np.float32),
            "conic_opacity": self._arr("orc_conic_opacity", 4 * P, np.float32).reshape(P, 4),
            "rgb": self._arr("orc_rgb", 3 * P, np.float32).reshape(P, 3),
            "cov3D": self._arr("orc_cov3D", 6 * P, np.float32).reshape(P, 6),
            "clamped": self._arr("orc_clamped", 3 * P, np.uint8).reshape(P, 3),
            "tiles_touched": self._arr("orc_tiles_touched", P, np.uint32),
        }


def forward(s: Settings, means3D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
            cov3D_precomp=None, nthreads: int = 0, normal: bool = False):
    """≙ _C.rasterize_gaussians: returns (num_rendered, color[3,H,W], radii[P], depth[1,H,W], State),
    plus the aux normal map [3,H,W] as a 6th element when `normal` (include/rain_raster.h
    RR_FLAG_AUX_NORMAL; no reference counterpart)."""
    L = lib()
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    H, W = int(s.image_height), int(s.image_width)
    shs, colors_precomp = _f32(shs), _f32(colors_precomp)
    scales, rotations, cov3D_precomp = _f32(scales), _f32(rotations), _f32(cov3D_precomp)
    opac = _f32(opacities)
    M = shs.reshape(P, -1, 3).shape[1] if shs is not None else 0
    bg = _f32(s.bg)
    view, proj, campos = _f32(s.viewmatrix).reshape(16), _f32(s.projmatrix).reshape(16), _f32(s.campos)
    color = np.zeros((3, H, W), np.float32)
    depth = np.zeros((1, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    if normal and (scales is None or rotations is None):
        raise ValueError("the aux normal map needs scales/rotations")
    nmap = np.zeros((3, H, W), np.float32) if normal else None
    nr = ctypes.c_int(0)
    h = L.orc_forward(P, int(s.sh_degree), M, _p(bg), W, H, _p(means3D), _p(shs), _p(colors_precomp), _p(opac),
                      _p(scales), float(s.scale_modifier), _p(rotations), _p(cov3D_precomp), _p(view), _p(proj),
                      _p(campos), float(s.tanfovx), float(s.tanfovy), int(bool(s.prefiltered)), float(s.low_pass),
                      _p(color), _p(depth), _p(radii, _i32p), ctypes.byref(nr), int(nthreads), _p(nmap))
    st = State(h, P, W, H)
    if normal:
        return nr.value, color, radii, depth, st, nmap
    return nr.value, color, radii, depth, st


def backward(st: State, s: Settings, means3D, radii, dL_dout_color, shs=None, colors_precomp=None, scales=None,
             rotations=None, cov3D_precomp=None, nthreads: int = 0):
    """≙ _C.rasterize_gaussians_backward: returns the 8-tuple
    (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)
    plus dL_dconic[P,4] as a 9th element (not part of the reference's return)."""
    L = lib()
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    shs, colors_precomp = _f32(shs), _f32(colors_precomp)
    scales, rotations, cov3D_precomp = _f32(scales), _f32(rotations), _f32(cov3D_precomp)
    M = shs.reshape(P, -1, 3).shape[1] if shs is not None else 0
    bg = _f32(s.bg)
    view, proj, campos = _f32(s.viewmatrix).reshape(16), _f32(s.projmatrix).reshape(16), _f32(s.campos)
    dpix = _f32(dL_dout_color)
    radii = np.ascontiguousarray(radii, dtype=np.int32)
    out = dict(
        dL_dmeans2D=np.zeros((P, 3), np.float32), dL_dcolors=np.zeros((P, 3), np.float32),
        dL_dopacity=np.zeros((P, 1), np.float32), dL_dmeans3D=np.zeros((P, 3), np.float32),
        dL_dcov3D=np.zeros((P, 6), np.float32), dL_dsh=np.zeros((P, M, 3), np.float32),
        dL_dscales=np.zeros((P, 3), np.float32), dL_drotations=np.zeros((P, 4), np.float32),
        dL_dconic=np.zeros((P, 4), np.float32))
    if P > 0:
        rc = L.orc_backward(st.handle, _p(bg), _p(means3D), _p(radii, _i32p), _p(colors_precomp), _p(scales),
                            float(s.scale_modifier), _p(rotations), _p(cov3D_precomp), _p(view), _p(proj),
                            _p(campos), float(s.tanfovx), float(s.tanfovy), _p(shs), _p(dpix), float(s.low_pass),
                            _p(out["dL_dmeans2D"]), _p(out["dL_dcolors"]), _p(out["dL_dopacity"]),
                            _p(out["dL_dmeans3D"]), _p(out["dL_dcov3D"]), _p(out["dL_dsh"]),
                            _p(out["dL_dscales"]), _p(out["dL_drotations"]), _p(out["dL_dconic"]), int(nthreads))
        if rc != 0:
            raise RuntimeError("oracle backward failed")
    return (out["dL_dmeans2D"], out["dL_dcolors"], out["dL_dopacity"], out["dL_dmeans3D"], out["dL_dcov3D"],
            out["dL_dsh"], out["dL_dscales"], out["dL_drotations"], out["dL_dconic"])


def mark_visible(means3D, viewmatrix, projmatrix):
    means3D = _f32(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    out = np.zeros(P, np.uint8)
    if P:
        lib().orc_mark_visible(P, _p(means3D), _p(_f32(viewmatrix).reshape(16)), _p(_f32(projmatrix).reshape(16)),
                               _p(out, _u8p))
    return out.astype(bool)


def sh_eval(deg, shs, dirs):
    """forward.cu:9-60 on unit directions: returns (rgb = max(SH+0.5, 0) [n,3], clamped [n,3] bool).
    shs is [n, M, 3] (kernel layout, coefficient-major)."""
    shs = _f32(shs)
    n, M = shs.shape[0], shs.shape[1]
    d = _f32(dirs).reshape(n, 3)
    out = np.zeros((n, 3), np.float32)
    cl = np.zeros((n, 3), np.uint8)
    lib().orc_sh_eval(int(deg), M, n, _p(d), _p(shs), _p(out), _p(cl, _u8p))
    return out, cl.astype(bool)


def cov3d(scales, scale_modifier, rotations):
    """Sigma3D (xx, xy, xz, yy, yz, zz) per Gaussian, computeCov3D (forward.cu:107-141)."""
    s = _f32(scales)
    r = _f32(rotations)
    out = np.zeros((s.shape[0], 6), np.float32)
    lib().orc_cov3d(s.shape[0], _p(s), float(scale_modifier), _p(r), _p(out))
    return out


def get_higher_msb(n: int) -> int:
    return int(lib().orc_get_higher_msb(n))


def dist_knn3(points, details=False):
    """≙ simple_knn distCUDA2 (simple_knn.cu:164-207): mean squared distance to the 3 nearest
    neighbours.  With details=True also returns the Morton-sorted order and the bbox (origin
    included, simple_knn.cu:172-181)."""
    pts = _f32(points)
    pts = np.zeros((0, 3), np.float32) if pts is None else pts.reshape(-1, 3)
    P = pts.shape[0]
    out = np.zeros(P, np.float32)
    order = np.zeros(P, np.uint32)
    bbox = np.zeros(6, np.float32)
    if P:
        lib().orc_dist_knn3(P, _p(pts), _p(out), order.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _p(bbox))
    return (out, order, bbox) if details else out
