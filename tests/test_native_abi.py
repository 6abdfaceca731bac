"""CPU checks of the drop-in boundary: the C-ABI libraries load, export every symbol their headers
declare, size queries behave, argument validation mirrors the reference's errors, and the product
path refuses CPU tensors (there is no CPU fallback)."""
import ctypes
import os
import re

import pytest
import torch

from rain_amd import _native as N
from rain_amd.diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer, _C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:int|size_t|char\s*\*|char|void\s*\*)\s*\*?\s*(r[rlt]_\w+|sk_\w+)\s*\(", src,
                                 flags=re.M)))


@pytest.mark.parametrize("header,lib,listed", [("rain_raster.h", N.RASTER_LIB, N.RASTER_SYMBOLS),
                                               ("rain_loss.h", N.LOSS_LIB, N.LOSS_SYMBOLS),
                                               ("rain_train.h", N.TRAIN_LIB, N.TRAIN_SYMBOLS),
                                               ("rain_knn.h", N.KNN_LIB, N.KNN_SYMBOLS)])
def test_library_exports_every_declared_symbol(header, lib, listed):
    names = _declared(header)
    assert names, header
    so = ctypes.CDLL(lib)
    for n in names:
        assert hasattr(so, n), f"{os.path.basename(lib)} does not export {n}"
    assert sorted(listed) == names


def test_size_queries():
    L = N.raster()
    assert L.rr_geometry_bytes(0) > 0
    assert L.rr_geometry_bytes(1000) < L.rr_geometry_bytes(100000) < L.rr_geometry_bytes(1000000)
    assert L.rr_image_bytes(1920, 1080) >= 1920 * 1080 * 8
    assert L.rr_binning_bytes(1000, 256, 256) < L.rr_binning_bytes(10_000_000, 1920, 1080)
    assert L.rr_backward_workspace_bytes(1000) >= 1000 * 64
    assert N.loss_lib().rl_workspace_bytes(3, 1080, 1920) >= 3 * 3 * 1080 * 1920 * 4
    assert L.rr_version().decode().startswith("rain_amd")


def test_geometry_layout_and_sharded_step_validation():
    """rr_geometry_layout: the preprocess arrays' offsets inside a geometry buffer (the sharded
    step's all-to-all writes there): distinct, ordered, 256-B aligned, inside rr_geometry_bytes.
    The sharded entry points refuse bad row blocks / views before touching a device."""
    L = N.raster()
    for P in (256, 20480, 1000192):
        o = (ctypes.c_size_t * 5)()
        assert L.rr_geometry_layout(P, o) == 0
        offs = list(o)
        assert offs == sorted(offs) and len(set(offs)) == 5 and all(x % 256 == 0 for x in offs)
        assert offs[1] - offs[0] >= 48 * P and offs[2] - offs[1] >= 8 * P and offs[3] - offs[2] >= 4 * P
        assert offs[4] + 4 * (P // 256) <= L.rr_geometry_bytes(P)
    assert L.rr_geometry_layout(-1, (ctypes.c_size_t * 5)()) == 1
    f = N.RRFrame(300, 3, 16, 64, 48, 0.5, 0.4, 1.0, 0.3, 0, 0, N.RR_FLAG_RAW_PARAMS)
    cam = N.RRCamera(1, 1, 1, 1)
    g = N.RRGaussians(1, 1, None, 1, 1, 1, None, 1)
    rc = L.rr_preprocess_rows(ctypes.byref(f), ctypes.byref(cam), ctypes.byref(g), 300, 1, 1, 1, 1, 1, 1, None)
    assert rc == 1 and b"multiple of 256" in L.rr_last_error()
    views = (N.RRView * 17)()
    offs6 = (ctypes.c_size_t * 6)()
    rc = L.rr_preprocess_rows_views(ctypes.byref(f), views, 17, ctypes.byref(g), 512, None, 0, offs6, 1, None)
    assert rc == 1 and b"num_views" in L.rr_last_error()
    rc = L.rr_preprocess_rows_views(ctypes.byref(f), views, 2, ctypes.byref(g), 300, None, 0, offs6, 1, None)
    assert rc == 1 and b"multiple of 256" in L.rr_last_error()
    rc = L.rr_preprocess_rows_views(ctypes.byref(f), views, 2, ctypes.byref(g), 512, None, 0, offs6, 1, None)
    assert rc == 1 and b"bad view" in L.rr_last_error()  # null matrices
    offs5 = (ctypes.c_size_t * 5)()
    rc = L.rr_unpack_rows(2, 300, None, 0, offs5, None, 0, None, None)
    assert rc == 1 and b"multiple of 256" in L.rr_last_error()
    rc = L.rr_unpack_rows(2, 256, 1, 12, offs5, 1, 1 << 30, 1, None)
    assert rc == 1 and b"alignment" in L.rr_last_error()
    out = N.RRGrads()
    rc = L.rr_gauss_backward_views(ctypes.byref(f), views, 17, ctypes.byref(g), None, 300, 1.0, ctypes.byref(out), None)
    assert rc == 1 and b"num_views" in L.rr_last_error()
    nr, npairs, need = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_size_t(0)
    rc = L.rr_forward_from_geometry(ctypes.byref(f), ctypes.byref(cam), None, None, 0, None, 0, None, 0,
                                    ctypes.byref(nr), ctypes.byref(npairs), ctypes.byref(need), None, None, None)
    # any P is accepted (the geometry kernels take a ragged last block); a null buffer is not
    assert rc == 1 and b"null buffer" in L.rr_last_error()


def test_validation_errors_without_gpu():
    L = N.raster()
    f = N.RRFrame(10, 3, 16, 64, 48, 0.5, 0.4, 1.0, 0.3, 0, 0)
    cam = N.RRCamera(None, None, None, None)
    g = N.RRGaussians(None, None, None, None, None, None, None)
    nr = ctypes.c_int(-1)
    rc = L.rr_forward_geometry(ctypes.byref(f), ctypes.byref(cam), ctypes.byref(g), None, None, 0, None, 0,
                               ctypes.byref(nr), ctypes.byref(nr), None)
    assert rc == 1 and b"required" in L.rr_last_error()
    # both SH and colours given -> the reference's message
    g = N.RRGaussians(1, 1, 1, 1, 1, 1, None)
    cam = N.RRCamera(1, 1, 1, 1)
    rc = L.rr_forward_geometry(ctypes.byref(f), ctypes.byref(cam), ctypes.byref(g), None, None, 0, None, 0,
                               ctypes.byref(nr), ctypes.byref(nr), None)
    assert rc == 1 and b"exactly one of either SHs" in L.rr_last_error().replace(b"excatly", b"exactly")
    # P == 0 is a no-op success (rasterize_points.cu:72)
    f0 = N.RRFrame(0, 0, 0, 64, 48, 0.5, 0.4, 1.0, 0.3, 0, 0)
    assert L.rr_forward_geometry(ctypes.byref(f0), ctypes.byref(cam), ctypes.byref(g), None, None, 0, None, 0,
                                 ctypes.byref(nr), ctypes.byref(nr), None) == 0 and nr.value == 0


def test_forward_workspace_registration_validation():
    """rr_set_forward_workspace (no device call): 16-B alignment and size, NULL drops it; the
    tuning keys exist, and a removed A/B key is refused."""
    L = N.raster()
    assert L.rr_set_forward_workspace(8, 64) == 1 and b"16-byte" in L.rr_last_error()
    assert L.rr_set_forward_workspace(16, 40) == 1
    assert L.rr_set_forward_workspace(None, 0) == 0
    for key, dflt in (("sx_lds_cap", 0), ("phase_b_gather", 1), ("dup_b_rows", 1), ("dup_big_bins", 32),
                      ("sx_bucket", 1), ("wide_bin_keys", 0), ("pair_scan_direct_blocks", -1),
                      ("sort_min_units", 0), ("sort_min_units_tile", 0), ("sort_max_rounds", 0), ("early_den", 0)):
        assert L.rr_set_tuning(key.encode(), dflt) == 0, key
    for key in ("phase_a_gather", "cut_in_scan", "forward_clear", "bwd_waves"):
        assert L.rr_set_tuning(key.encode(), 0) == 1 and b"unknown tuning key" in L.rr_last_error()
    assert N.RR_FLAG_WORKSPACE_REGISTERED == 16


def _settings(device="cpu"):
    return GaussianRasterizationSettings(
        image_height=48, image_width=64, tanfovx=0.5, tanfovy=0.4, bg=torch.zeros(3, device=device),
        scale_modifier=1.0, viewmatrix=torch.eye(4, device=device), projmatrix=torch.eye(4, device=device),
        sh_degree=0, campos=torch.zeros(3, device=device), prefiltered=False, debug=False, low_pass=0.3)


def test_python_surface_validation_messages():
    r = GaussianRasterizer(_settings())
    m = torch.zeros(5, 3)
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(means3D=m, means2D=m, opacities=torch.zeros(5, 1), scales=m, rotations=torch.zeros(5, 4))
    with pytest.raises(Exception, match="exactly one of either scale/rotation pair or precomputed 3D covariance"):
        r(means3D=m, means2D=m, opacities=torch.zeros(5, 1), shs=torch.zeros(5, 1, 3))
    with pytest.raises(Exception, match="exactly one of either scale/rotation pair"):
        r(means3D=m, means2D=m, opacities=torch.zeros(5, 1), shs=torch.zeros(5, 1, 3), scales=m,
          rotations=torch.zeros(5, 4), cov3D_precomp=torch.zeros(5, 6))


def test_no_cpu_fallback():
    s = _settings()
    e = torch.Tensor([])
    m = torch.zeros(5, 3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _C.rasterize_gaussians(s.bg, m, e, torch.zeros(5, 1), m, torch.zeros(5, 4), 1.0, e, s.viewmatrix,
                               s.projmatrix, 0.5, 0.4, 48, 64, e, 0, s.campos, False, False, 0.3)
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        _C.rasterize_gaussians(s.bg, torch.zeros(5, 2), e, torch.zeros(5, 1), m, torch.zeros(5, 4), 1.0, e,
                               s.viewmatrix, s.projmatrix, 0.5, 0.4, 48, 64, e, 0, s.campos, False, False, 0.3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _C.mark_visible(m, s.viewmatrix, s.projmatrix)


def test_import_shim_is_the_product():
    import diff_gaussian_rasterization as shim

    assert shim.GaussianRasterizer is GaussianRasterizer
    assert shim._C is _C


def test_reference_import_path_resolves_to_the_product():
    """gaussian_renderer/__init__.py:5 imports exactly this dotted path; the reference package's
    `from ..setup import _C` (diff_gaussian_rasterization/__init__.py:4) resolves too."""
    import importlib

    m = importlib.import_module("submodules.diff_gaussian_rasterization.diff_gaussian_rasterization")
    from submodules.diff_gaussian_rasterization.diff_gaussian_rasterization import (
        GaussianRasterizationSettings as S, GaussianRasterizer as R)
    from submodules.diff_gaussian_rasterization.setup import _C as setup_C

    from rain_amd.diff_gaussian_rasterization import GaussianRasterizationSettings, rasterize_gaussians

    assert R is GaussianRasterizer and S is GaussianRasterizationSettings
    assert m.rasterize_gaussians is rasterize_gaussians and m._C is _C and setup_C is _C
    assert S._fields == ("image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix",
                         "projmatrix", "sh_degree", "campos", "prefiltered", "debug", "low_pass")


def test_simple_knn_shim_and_no_cpu_fallback():
    import simple_knn
    from simple_knn._C import distCUDA2

    from rain_amd.simple_knn import distCUDA2 as native

    assert distCUDA2 is native and simple_knn.distCUDA2 is native
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        distCUDA2(torch.zeros(10, 3))
    with pytest.raises(RuntimeError, match="num_points, 3"):
        distCUDA2(torch.zeros(10, 2))
    L = N.knn()
    assert L.sk_workspace_bytes(1000) < L.sk_workspace_bytes(1_000_000)
    assert L.sk_dist_cuda2(-1, None, None, None, 0, None) != 0 and b"P" in L.sk_last_error()
    assert L.sk_dist_cuda2(0, None, None, None, 0, None) == 0
