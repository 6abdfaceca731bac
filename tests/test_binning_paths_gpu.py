"""Every binning path of the forward (rr_api.hip render_tiles) gives the reference's per-tile
lists: phase A by the windowed duplicate + bin sort; phase B by the gather path over its list
(default) or by the windowed path (frames of > 16384 bins); per-bin order by the bucket sort
(default) or by the LSD passes only; the phase-B gather's row masks or flat mask (frames over 128
tiles wide), its big-Gaussian workgroup path; windows of 2048 pairs with their starts marked by the
split scan; long runs depth-sorted in LDS or through their own output region (sx_lds_cap).  Each
path is forced onto a small frame by its tuning knob (include/rain_raster.h rr_set_tuning).

For each path: the exact (depth, index) lists of the reference's 64-bit-key sort with culling and
early stop off (tests/test_parity_gpu.py::_check_pair_order, against the oracle), the two-phase
frame bitwise equal to the single-phase one (same pairs in the same order per pixel), equal depths
(exact copies) in index order, and forward / backward parity with the oracle."""
import numpy as np
import pytest
import torch

from tests.common import gpu_run, make_scene, oracle_run
from tests.test_parity_gpu import _check_forward, _check_grads, _check_pair_order, _dpix

pytestmark = pytest.mark.gpu

# (tuning settings, their defaults to restore)
PATHS = {
    "default": {},
    "lsd_only": {"sx_bucket": (0, 1)},
    "windowed_b": {"phase_b_gather": (0, 1)},
    # units of kSplitWin (2048) pairs at these sizes: window starts from the split scan's marks
    "split_marks": {"sort_min_units_tile": (1, 1024), "sort_max_rounds": (8, 16)},
    "split_marks_windowed_b": {"sort_min_units_tile": (1, 1024), "sort_max_rounds": (8, 16),
                               "phase_b_gather": (0, 1)},
    # runs over 64 pairs through the global path (their own point_list region as scratch)
    "global_runs": {"sx_lds_cap": (64, 0)},
    "global_runs_windowed_b": {"sx_lds_cap": (64, 0), "phase_b_gather": (0, 1), "sx_bucket": (0, 1)},
    "dup_big_serial": {"dup_big_bins": (0, 32)},  # every phase-B Gaussian by its own thread
    "dup_b_flat_mask": {"dup_b_rows": (0, 1)},  # phase B tests the flat open-tile mask (wide frames' path)
    "dup_big_all": {"dup_big_bins": (1, 32)},  # every phase-B Gaussian of > 1 bin per workgroup
}

@pytest.fixture(params=list(PATHS))
def path(request):
    from rain_amd import _native as N

    L = N.raster()
    for k, (v, _d) in PATHS[request.param].items():
        N.check(L.rr_set_tuning(k.encode(), v), k)
    yield request.param
    for k, (_v, d) in PATHS[request.param].items():
        N.check(L.rr_set_tuning(k.encode(), d), k)
    N.check(L.rr_set_binning_config(0, 0), "binning config")


def test_pair_order(oracle, gpu, monkeypatch, path):
    inp, st = make_scene(P=3000, W=128, H=96, sh_degree=3)
    _check_pair_order(oracle, gpu, monkeypatch, inp, st)


def _split(den):
    from rain_amd import _native as N

    N.check(N.raster().rr_set_binning_config(den, 1), "binning config")


def test_two_phase_bitwise_and_oracle(oracle, gpu, monkeypatch, path):
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(P=6000, W=192, H=144, sh_degree=3)
    dpix = _dpix(st)
    monkeypatch.setattr(_C, "EARLY_STOP", False)
    full = gpu_run(inp, st, gpu, dL_dpix=dpix)
    monkeypatch.setattr(_C, "EARLY_STOP", True)
    _split(4)
    early = gpu_run(inp, st, gpu, dL_dpix=dpix)
    np.testing.assert_array_equal(early["radii"], full["radii"])
    np.testing.assert_array_equal(early["color"], full["color"])
    np.testing.assert_array_equal(early["depth"], full["depth"])
    ref = oracle_run(oracle, inp, st, dL_dpix=dpix)
    _check_forward(ref, early)
    _check_grads(ref, early)


def test_equal_depths_keep_index_order(gpu, monkeypatch, path):
    """Exact copies (densify clones) at one depth, in both phases: index order among them."""
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(P=1500, W=160, H=128, sh_degree=2, scale_mult=2.0)
    copies = 6
    n = 1500 // copies
    src = torch.randint(0, 1500, (n,), generator=torch.Generator().manual_seed(7))
    for k, v in inp.items():
        if isinstance(v, torch.Tensor) and v.dim() > 0 and v.shape[0] == 1500:
            rows = v[src.to(v.device)].repeat_interleave(copies, dim=0)
            v[: rows.shape[0]] = rows
    inp["opacities"] = inp["opacities"] * 0.2
    monkeypatch.setattr(_C, "EARLY_STOP", False)
    full = gpu_run(inp, st, gpu)
    monkeypatch.setattr(_C, "EARLY_STOP", True)
    _split(4)
    early = gpu_run(inp, st, gpu)
    np.testing.assert_array_equal(early["color"], full["color"])
    np.testing.assert_array_equal(early["depth"], full["depth"])
