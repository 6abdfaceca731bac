"""ctypes binding of the C-ABI rasterizer library (include/rain_raster.h).

This is the product path: it loads ``rain_amd/lib/librain_raster.so`` (built by
rain_amd/_build.py for gfx950) and raises if it is missing — there is no CPU fallback.
torch is imported first so that the HIP runtime torch ships (SONAME libamdhip64.so.7) is the
one the library binds to; torch tensors only provide device memory and the stream.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded before the HIP library; see module docstring)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_PKG, "lib")
# RAIN_RASTER_LIB: an alternative build of the same library (tools/build_variant.py A/B builds)
RASTER_LIB = os.environ.get("RAIN_RASTER_LIB") or os.path.join(LIB_DIR, "librain_raster.so")
KNN_LIB = os.path.join(LIB_DIR, "librain_knn.so")
KNN_SYMBOLS = ["sk_workspace_bytes", "sk_dist_cuda2", "sk_last_error"]

STAGES = ["preprocess", "depth_sort", "scan", "duplicate", "tile_sort", "ranges", "blend_fwd", "blend_bwd",
          "gauss_bwd", "memset"]


class RRFrame(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int), ("width", ctypes.c_int),
                ("height", ctypes.c_int), ("tan_fovx", ctypes.c_float), ("tan_fovy", ctypes.c_float),
                ("scale_modifier", ctypes.c_float), ("low_pass", ctypes.c_float), ("prefiltered", ctypes.c_int),
                ("debug", ctypes.c_int), ("flags", ctypes.c_int)]


RR_FLAG_NO_TILE_CULLING = 1
RR_FLAG_RAW_PARAMS = 2
RR_FLAG_FULL_BINNING = 4
RR_FLAG_AUX_NORMAL = 8
RR_FLAG_WORKSPACE_REGISTERED = 16
RR_INCOMPLETE = 4  # rr_forward: stage 1 done, binning buffer too small


class RRCamera(ctypes.Structure):
    _fields_ = [("background", ctypes.c_void_p), ("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p),
                ("campos", ctypes.c_void_p)]


class RRGaussians(ctypes.Structure):
    _fields_ = [("means3D", ctypes.c_void_p), ("shs", ctypes.c_void_p), ("colors_precomp", ctypes.c_void_p),
                ("opacities", ctypes.c_void_p), ("scales", ctypes.c_void_p), ("rotations", ctypes.c_void_p),
                ("cov3D_precomp", ctypes.c_void_p), ("shs_rest", ctypes.c_void_p)]


class RRAdamGroup(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("lr", ctypes.c_double), ("bias_correction1", ctypes.c_float),
                ("bias_correction2_sqrt", ctypes.c_float)]


class RRAdam(ctypes.Structure):
    _fields_ = [(n, RRAdamGroup) for n in ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")] + \
               [("beta1", ctypes.c_double), ("beta2", ctypes.c_double), ("eps", ctypes.c_double)]


class RRNextFrame(ctypes.Structure):
    """include/rain_raster.h rr_next_frame: the next frame's preprocess inside the backward."""
    _fields_ = [("frame", ctypes.POINTER(RRFrame)), ("cam", ctypes.POINTER(RRCamera)), ("radii", ctypes.c_void_p),
                ("geom_buffer", ctypes.c_void_p), ("geom_bytes", ctypes.c_size_t)]


class RRGrads(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D",
                                                "dL_dcov3D", "dL_dsh", "dL_dscales", "dL_drotations",
                                                "dL_dsh_rest", "grad_accum", "denom", "max_radii2D")] + \
               [("adam", ctypes.POINTER(RRAdam)), ("next", ctypes.POINTER(RRNextFrame))]


class RRView(ctypes.Structure):
    _fields_ = [("viewmatrix", ctypes.c_void_p), ("projmatrix", ctypes.c_void_p), ("campos", ctypes.c_void_p),
                ("tan_fovx", ctypes.c_float), ("tan_fovy", ctypes.c_float), ("low_pass", ctypes.c_float),
                ("width", ctypes.c_int), ("height", ctypes.c_int)]


RR_MAX_VIEWS = 16


class RRFrameStats(ctypes.Structure):
    _fields_ = [("num_rendered", ctypes.c_int64), ("num_visible", ctypes.c_int64), ("l_eff", ctypes.c_int64),
                ("tiles", ctypes.c_int64), ("num_pairs", ctypes.c_int64), ("num_binned", ctypes.c_int64),
                ("phase_b_pairs", ctypes.c_int64), ("phase_b_slots", ctypes.c_int64)]


class RRDebugViews(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("point_list", "ranges", "tile_max", "final_T", "n_contrib",
                                                "splats")]


# every symbol include/rain_raster.h declares (tests check the .so exports all of them)
RASTER_SYMBOLS = ["rr_geometry_bytes", "rr_image_bytes", "rr_binning_bytes", "rr_backward_workspace_bytes",
                  "rr_forward_geometry", "rr_forward_render", "rr_forward_render_aux", "rr_forward", "rr_backward", "rr_mark_visible", "rr_last_error",
                  "rr_version", "rr_read_frame_stats", "rr_debug_get_views", "rr_set_binning_config", "rr_set_tuning", "rr_debug_set_fwd_trace", "rr_profile_enable",
                  "rr_profile_select", "rr_profile_collect", "rr_stage_name", "rr_host_wait_stats", "rr_geometry_layout",
                  "rr_preprocess_rows", "rr_preprocess_rows_views", "rr_unpack_rows", "rr_forward_from_geometry",
                  "rr_forward_render_geometry",
                  "rr_backward_records", "rr_gauss_backward_views", "rr_set_forward_workspace"]

_raster = None
_knn = None


def _load(path):
    if not os.path.exists(path):
        raise ImportError(
            f"rain_amd: native library {path} is missing. Build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc, gfx950). There is no CPU fallback for the rasterizer.")
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def raster():
    """The loaded librain_raster.so with argtypes set."""
    global _raster
    if _raster is None:
        L = _load(RASTER_LIB)
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        for name in ("rr_geometry_bytes", "rr_backward_workspace_bytes"):
            getattr(L, name).restype = sz
            getattr(L, name).argtypes = [ci]
        L.rr_image_bytes.restype = sz
        L.rr_image_bytes.argtypes = [ci, ci]
        L.rr_binning_bytes.restype = sz
        L.rr_binning_bytes.argtypes = [ci, ci, ci]
        fp, cp, gp = ctypes.POINTER(RRFrame), ctypes.POINTER(RRCamera), ctypes.POINTER(RRGaussians)
        L.rr_forward_geometry.restype = ci
        L.rr_forward_geometry.argtypes = [fp, cp, gp, vp, vp, sz, vp, sz, ctypes.POINTER(ci), ctypes.POINTER(ci), vp]
        L.rr_forward_render.restype = ci
        L.rr_forward_render.argtypes = [fp, cp, gp, vp, vp, vp, vp, sz, ci, vp, vp, vp]
        L.rr_forward_render_aux.restype = ci
        L.rr_forward_render_aux.argtypes = [fp, cp, gp, vp, vp, vp, vp, sz, ci, vp, vp, vp, vp]
        L.rr_forward.restype = ci
        L.rr_forward.argtypes = [fp, cp, gp, vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(ci), ctypes.POINTER(ci),
                                 ctypes.POINTER(sz), vp, vp, vp]
        L.rr_backward.restype = ci
        L.rr_backward.argtypes = [fp, cp, gp, vp, vp, vp, vp, ci, vp, vp, sz, ctypes.POINTER(RRGrads), vp]
        L.rr_mark_visible.restype = ci
        L.rr_mark_visible.argtypes = [ci, vp, vp, vp, vp, vp]
        L.rr_last_error.restype = ctypes.c_char_p
        L.rr_version.restype = ctypes.c_char_p
        L.rr_read_frame_stats.restype = ci
        L.rr_read_frame_stats.argtypes = [fp, vp, vp, ctypes.POINTER(RRFrameStats), vp]
        L.rr_debug_get_views.restype = ci
        L.rr_debug_get_views.argtypes = [fp, vp, vp, vp, ci, ctypes.POINTER(RRDebugViews)]
        L.rr_host_wait_stats.restype = ci
        L.rr_host_wait_stats.argtypes = [ci, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        L.rr_profile_enable.restype = ci
        L.rr_profile_enable.argtypes = [ci]
        L.rr_set_forward_workspace.restype = ci
        L.rr_set_forward_workspace.argtypes = [vp, sz]
        L.rr_set_tuning.restype = ci
        L.rr_set_tuning.argtypes = [ctypes.c_char_p, ci]
        L.rr_debug_set_fwd_trace.restype = ci
        L.rr_debug_set_fwd_trace.argtypes = [ctypes.c_void_p]
        L.rr_set_binning_config.restype = ci
        L.rr_set_binning_config.argtypes = [ci, ci]
        L.rr_profile_select.restype = ci
        L.rr_profile_select.argtypes = [ctypes.c_uint]
        L.rr_profile_collect.restype = ci
        L.rr_profile_collect.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
        L.rr_stage_name.restype = ctypes.c_char_p
        L.rr_stage_name.argtypes = [ci]
        # Gaussian-sharded step (rain_amd/sharded.py)
        L.rr_geometry_layout.restype = ci
        L.rr_geometry_layout.argtypes = [ci, ctypes.POINTER(sz)]
        L.rr_preprocess_rows.restype = ci
        L.rr_preprocess_rows.argtypes = [fp, cp, gp, ci, vp, vp, vp, vp, vp, vp, vp]
        L.rr_preprocess_rows_views.restype = ci
        L.rr_preprocess_rows_views.argtypes = [fp, ctypes.POINTER(RRView), ci, gp, ci, vp, sz,
                                               ctypes.POINTER(ctypes.c_size_t), ci, vp]
        L.rr_unpack_rows.restype = ci
        L.rr_unpack_rows.argtypes = [ci, ci, vp, sz, ctypes.POINTER(ctypes.c_size_t), vp, sz, vp, vp]
        L.rr_forward_from_geometry.restype = ci
        L.rr_forward_from_geometry.argtypes = [fp, cp, vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(ci), ctypes.POINTER(ci),
                                               ctypes.POINTER(sz), vp, vp, vp]
        L.rr_forward_render_geometry.restype = ci
        L.rr_forward_render_geometry.argtypes = [fp, cp, vp, vp, vp, vp, sz, ci, vp, vp, vp]
        L.rr_backward_records.restype = ci
        L.rr_backward_records.argtypes = [fp, cp, vp, vp, vp, vp, ci, vp, vp, sz, ci, ci, vp, vp]
        L.rr_gauss_backward_views.restype = ci
        L.rr_gauss_backward_views.argtypes = [fp, ctypes.POINTER(RRView), ci, gp, vp, ci, ctypes.c_float,
                                              ctypes.POINTER(RRGrads), vp]
        _raster = L
    return _raster


LOSS_LIB = os.environ.get("RAIN_LOSS_LIB") or os.path.join(LIB_DIR, "librain_loss.so")
LOSS_SYMBOLS = ["rl_workspace_bytes", "rl_l1_ssim_forward", "rl_l1_ssim_backward", "rl_l1_ssim_forward_backward",
                "rl_last_error"]
_loss = None


def loss_lib():
    global _loss
    if _loss is None:
        L = _load(LOSS_LIB)
        vp, ci, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.rl_workspace_bytes.restype = ctypes.c_size_t
        L.rl_workspace_bytes.argtypes = [ci, ci, ci]
        L.rl_l1_ssim_forward.restype = ci
        L.rl_l1_ssim_forward.argtypes = [vp, vp, ci, ci, ci, cf, ctypes.POINTER(cf), vp, ctypes.c_size_t, vp, vp, vp]
        L.rl_l1_ssim_backward.restype = ci
        L.rl_l1_ssim_backward.argtypes = [vp, vp, ci, ci, ci, cf, ctypes.POINTER(cf), vp, vp, vp, vp]
        L.rl_l1_ssim_forward_backward.restype = ci
        L.rl_l1_ssim_forward_backward.argtypes = [vp, vp, ci, ci, ci, cf, ctypes.POINTER(cf), vp, ctypes.c_size_t, vp,
                                                  vp, vp, vp, vp]
        L.rl_last_error.restype = ctypes.c_char_p
        _loss = L
    return _loss


TRAIN_LIB = os.path.join(LIB_DIR, "librain_train.so")
TRAIN_SYMBOLS = ["rt_adam_step", "rt_adam_step_scaled", "rt_densify_workspace_bytes", "rt_densify_plan",
                 "rt_densify_apply", "rt_stream_copy", "rt_stream_rmw", "rt_trace_marker", "rt_densify_stats",
                 "rt_max_radii", "rt_last_error"]
RT_MAX_GROUPS = 8
_train = None


class RTDensifyParams(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int), ("n_split", ctypes.c_int), ("grad_threshold", ctypes.c_float),
                ("clone_split_scale", ctypes.c_float), ("min_opacity", ctypes.c_float),
                ("big_world_scale", ctypes.c_float), ("prune_big_world", ctypes.c_int),
                ("split_scale_div", ctypes.c_float), ("abe_split", ctypes.c_int), ("abe_xyz_scale0", ctypes.c_float),
                ("abe_xyz_scale1", ctypes.c_float)]


class RTDensifyGroup(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("param", "exp_avg", "exp_avg_sq", "out_param", "out_exp_avg",
                                                "out_exp_avg_sq")] + [("width", ctypes.c_int), ("kind", ctypes.c_int)]


RT_GROUP_OTHER, RT_GROUP_XYZ, RT_GROUP_SCALING = 0, 1, 2


class RTAdamGroup(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_int64), ("lr", ctypes.c_double),
                ("bias_correction1", ctypes.c_float), ("bias_correction2_sqrt", ctypes.c_float)]


def train_lib():
    global _train
    if _train is None:
        L = _load(TRAIN_LIB)
        L.rt_adam_step.restype = ctypes.c_int
        L.rt_adam_step.argtypes = [ctypes.POINTER(RTAdamGroup), ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_void_p]
        L.rt_adam_step_scaled.argtypes = [ctypes.POINTER(RTAdamGroup), ctypes.c_int, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_double, ctypes.c_float, ctypes.c_void_p]
        L.rt_adam_step_scaled.restype = ctypes.c_int
        vp = ctypes.c_void_p
        L.rt_densify_workspace_bytes.restype = ctypes.c_size_t
        L.rt_densify_workspace_bytes.argtypes = [ctypes.c_int]
        L.rt_densify_plan.restype = ctypes.c_int
        L.rt_densify_plan.argtypes = [ctypes.POINTER(RTDensifyParams), vp, vp, vp, vp, vp, ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_int64), vp]
        L.rt_densify_apply.restype = ctypes.c_int
        L.rt_densify_apply.argtypes = [ctypes.POINTER(RTDensifyParams), vp, vp, vp, vp,
                                       ctypes.POINTER(RTDensifyGroup), ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                       vp]
        L.rt_stream_copy.restype = ctypes.c_int
        L.rt_stream_copy.argtypes = [vp, vp, ctypes.c_size_t, vp]
        L.rt_stream_rmw.restype = ctypes.c_int
        L.rt_stream_rmw.argtypes = [vp, vp, vp, ctypes.c_size_t, vp]
        L.rt_trace_marker.restype = ctypes.c_int
        L.rt_trace_marker.argtypes = [ctypes.c_int, ctypes.c_int, vp]
        L.rt_densify_stats.restype = ctypes.c_int
        L.rt_densify_stats.argtypes = [ctypes.c_int, vp, ctypes.c_int, vp, vp, vp, vp]
        L.rt_max_radii.restype = ctypes.c_int
        L.rt_max_radii.argtypes = [ctypes.c_int, vp, vp, vp, vp]
        L.rt_last_error.restype = ctypes.c_char_p
        _train = L
    return _train


def knn():
    global _knn
    if _knn is None:
        L = _load(KNN_LIB)
        L.sk_dist_cuda2.restype = ctypes.c_int
        L.sk_dist_cuda2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.c_void_p]
        L.sk_workspace_bytes.restype = ctypes.c_size_t
        L.sk_workspace_bytes.argtypes = [ctypes.c_int]
        L.sk_last_error.restype = ctypes.c_char_p
        _knn = L
    return _knn


def check(rc: int, what: str):
    if rc != 0:
        msg = raster().rr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg}")


def check_rt(rc: int, what: str):
    """check() for librain_train.so calls (its own last-error slot)."""
    if rc != 0:
        msg = train_lib().rt_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg}")


def stream_of(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


class Profiler:
    """Per-stage kernel time via HIP events recorded by the library on the launch stream."""

    def __init__(self, stages=None):
        self.mask = 0xFFFFFFFF if stages is None else sum(1 << STAGES.index(s) for s in stages)

    def __enter__(self):
        raster().rr_profile_select(self.mask)
        raster().rr_profile_enable(1)
        return self

    def __exit__(self, *exc):
        raster().rr_profile_enable(0)
        raster().rr_profile_select(0xFFFFFFFF)

    @staticmethod
    def collect():
        n = len(STAGES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        check(raster().rr_profile_collect(ms, cnt), "profile collect")
        return {STAGES[i]: (ms[i], cnt[i]) for i in range(n)}
