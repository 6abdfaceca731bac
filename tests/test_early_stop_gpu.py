"""Early-stop binning (include/rain_raster.h RR_FLAG_FULL_BINNING, rr_set_binning_config): tile
lists built in two phases, cut past saturation.  The outputs must be those of full binning —
forward bitwise (every pixel blends the same pairs in the same order), gradients within the
atomics-order tolerance — and of the CPU oracle."""
import numpy as np
import pytest
import torch

from tests.common import gpu_run, make_scene, oracle_run, rel_l1
from tests.test_parity_gpu import _check_forward, _check_grads, _dpix

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["gather", "windows"])
def split(request, monkeypatch):
    """Force the two-phase path onto small frames: phase A = L/den pairs, any frame size; phase B
    binned by each of its two paths (rr_api.hip phase_b_gather: few pairs gathered per bin, or the
    windowed duplicate + bin sort)."""
    from rain_amd import _native as N
    from rain_amd.diff_gaussian_rasterization import _C

    def set_split(den):
        N.check(N.raster().rr_set_binning_config(den, 1), "binning config")

    N.check(N.raster().rr_set_tuning(b"phase_b_gather", 1 if request.param == "gather" else 0), "tuning")
    yield set_split
    N.check(N.raster().rr_set_tuning(b"phase_b_gather", 1), "tuning")  # the default
    N.check(N.raster().rr_set_binning_config(0, 0), "binning config")
    monkeypatch.setattr(_C, "EARLY_STOP", True)


def _stats(out, P, st):
    from rain_amd.diff_gaussian_rasterization import _C

    geom, binning, img = out["buffers"]
    return _C.frame_stats(geom, img, P, st["image_width"], st["image_height"])


@pytest.mark.parametrize("den", [2, 8, 64])
@pytest.mark.parametrize("scene", [dict(P=6000, W=192, H=144, sh_degree=3),
                                   dict(P=3000, W=200, H=120, sh_degree=2, scale_mult=3.0),
                                   dict(P=2500, W=128, H=96, sh_degree=3, bg=(1.0, 0.5, 0.25))])
def test_two_phase_equals_full_binning(gpu, split, monkeypatch, scene, den):
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(**scene)
    P = inp["means3D"].shape[0]
    dpix = _dpix(st)
    monkeypatch.setattr(_C, "EARLY_STOP", False)
    full = gpu_run(inp, st, gpu, dL_dpix=dpix)
    fs = _stats(full, P, st)
    monkeypatch.setattr(_C, "EARLY_STOP", True)
    split(den)
    early = gpu_run(inp, st, gpu, dL_dpix=dpix)
    es = _stats(early, P, st)
    assert es["num_pairs"] == fs["num_pairs"] and es["num_rendered"] == fs["num_rendered"]
    assert fs["num_binned"] == fs["num_pairs"]
    assert es["num_binned"] <= es["num_pairs"]
    np.testing.assert_array_equal(early["radii"], full["radii"])
    np.testing.assert_array_equal(early["color"], full["color"])  # same pairs, same order: bitwise
    np.testing.assert_array_equal(early["depth"], full["depth"])
    ev = _C.debug_views(early["buffers"][0], early["buffers"][1], early["buffers"][2], early["num_rendered"], P,
                        st["image_width"], st["image_height"])
    fv = _C.debug_views(full["buffers"][0], full["buffers"][1], full["buffers"][2], full["num_rendered"], P,
                        st["image_width"], st["image_height"])
    assert torch.equal(ev["n_contrib"], fv["n_contrib"])
    assert torch.equal(ev["final_T"], fv["final_T"])
    assert torch.equal(ev["tile_max"], fv["tile_max"])
    for k, a in early["grads"].items():
        b = full["grads"][k]
        if np.abs(b).sum() == 0:
            assert np.abs(a).max() < 1e-8, k
        else:
            assert rel_l1(a, b) <= 1e-5, (k, rel_l1(a, b))


def test_two_phase_cuts_saturated_tiles(gpu, split):
    """Opaque, large splats saturate every tile early: phase B must bin only a small remainder."""
    inp, st = make_scene(P=6000, W=192, H=144, sh_degree=1, scale_mult=3.0)
    inp["opacities"] = torch.full_like(inp["opacities"], 0.95)
    split(8)
    out = gpu_run(inp, st, gpu)
    s = _stats(out, inp["means3D"].shape[0], st)
    assert s["num_binned"] < 0.5 * s["num_pairs"], s


@pytest.mark.parametrize("case", [dict(P=3000, W=128, H=96, sh_degree=3),
                                  dict(P=2000, W=100, H=75, sh_degree=3),
                                  dict(P=1500, W=128, H=128, sh_degree=3, scale_mult=4.0)])
def test_two_phase_matches_oracle(oracle, gpu, split, case):
    inp, st = make_scene(**case)
    dpix = _dpix(st)
    ref = oracle_run(oracle, inp, st, dL_dpix=dpix)
    split(4)
    got = gpu_run(inp, st, gpu, dL_dpix=dpix)
    _check_forward(ref, got)
    _check_grads(ref, got)


def test_fused_raw_path_two_phase(gpu, split):
    """Training entry point (raw parameters, rain_amd.fused) under the two-phase path."""
    from rain_amd import cameras, fused, synthetic
    from rain_amd.gaussian_model import GaussianModel

    g = GaussianModel(3, device="cuda")
    g.set_params(synthetic.random_gaussians(20_000, sh_degree=3, seed=5, bench=True, device="cuda"))
    g.active_sh_degree = 3
    cam = cameras.fibonacci_cameras(8, 160, 120)[3].to("cuda")
    bg = torch.zeros(3, device="cuda")
    c_full, r_full, d_full, _ = fused.forward(g, cam, bg, 0.3)
    split(8)
    c, r, d, _ = fused.forward(g, cam, bg, 0.3)
    assert torch.equal(r, r_full)
    assert torch.equal(c, c_full)
    assert torch.equal(d, d_full)


@pytest.mark.parametrize("copies", [2, 48])
def test_two_phase_equal_depths(gpu, split, monkeypatch, copies):
    """Gaussians at one depth (densify clones: exact copies) must keep index order inside every tile
    list — the gather path's per-bin sort sees its phase-B pairs in no particular order and resolves
    equal depth keys by index (groups of up to 32 in place, longer ones by a full index-pass sort)."""
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(P=1500, W=160, H=128, sh_degree=2, scale_mult=2.0)
    n = 1500 // copies
    src = torch.randint(0, 1500, (n,), generator=torch.Generator().manual_seed(7))
    for k, v in inp.items():  # the first n * copies rows: `copies` copies of n source rows each
        if isinstance(v, torch.Tensor) and v.dim() > 0 and v.shape[0] == 1500:
            rows = v[src.to(v.device)].repeat_interleave(copies, dim=0)
            v[: rows.shape[0]] = rows
    # low opacity keeps tiles open, so that phase B holds the copies too
    inp["opacities"] = inp["opacities"] * 0.2
    dpix = _dpix(st)
    monkeypatch.setattr(_C, "EARLY_STOP", False)
    full = gpu_run(inp, st, gpu, dL_dpix=dpix)
    monkeypatch.setattr(_C, "EARLY_STOP", True)
    split(4)
    early = gpu_run(inp, st, gpu, dL_dpix=dpix)
    s = _stats(early, 1500, st)
    assert s["num_binned"] > s["num_pairs"] // 4, s  # phase B binned pairs
    np.testing.assert_array_equal(early["color"], full["color"])
    np.testing.assert_array_equal(early["depth"], full["depth"])


def test_phase_b_reservation_stays_in_its_region(gpu, split):
    """Phase B's gather duplicate reserves slots per Gaussian (rr_forward.hip k_dup_gather): on a
    frame where phase A closes no tile (faint Gaussians) and the Gaussians are elongated (their
    bounding rectangles hold many bins their ellipses never reach), the reservations must stay
    within the phase's pairs, the size of its region of the pair arrays — and the outputs equal
    full binning's."""
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(P=4000, W=256, H=192, sh_degree=1, scale_mult=1.0)
    P = inp["means3D"].shape[0]
    g = torch.Generator().manual_seed(11)
    sc = inp["scales"]
    sc[:, 0] = sc[:, 0] * 12.0  # long thin ellipses at random orientations
    sc[:, 1:] = sc[:, 1:] * 0.3
    inp["opacities"] = torch.full_like(inp["opacities"], 0.02)
    q = torch.randn(P, 4, generator=g)
    inp["rotations"] = (q / q.norm(dim=1, keepdim=True)).to(inp["rotations"].dtype)
    from unittest import mock

    with mock.patch.object(_C, "EARLY_STOP", False):
        full = gpu_run(inp, st, gpu)
    split(3)
    early = gpu_run(inp, st, gpu)
    s = _stats(early, P, st)
    assert s["phase_b_pairs"] > 0, s
    assert s["phase_b_slots"] <= s["phase_b_pairs"], s
    assert s["num_binned"] == s["num_pairs"], s  # nothing saturated: every pair binned
    np.testing.assert_array_equal(early["color"], full["color"])
    np.testing.assert_array_equal(early["depth"], full["depth"])


def test_second_render_without_a_pair_count_fails(gpu):
    """One render per pair count (rr_api.hip g_counted_img): rendering a frame again from the same
    geometry call would start the gather counters where the first render's ended."""
    import ctypes

    from rain_amd import _native as N
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(P=2000, W=128, H=96, sh_degree=3)
    out = gpu_run(inp, st, gpu)
    geom, binning, img = out["buffers"]
    L = N.raster()
    f = _C._frame(2000, 3, 16, st["image_width"], st["image_height"], 1.0, 1.0, 1.0, 0.3, False, False)
    # non-null stand-ins pass the argument checks; the render fails at the pair-count guard, before
    # any launch reads them
    x = geom.data_ptr()
    cam = N.RRCamera(x, x, x, x)
    g = N.RRGaussians(x, x, None, x, x, x, None, None)
    color = torch.empty(3, st["image_height"], st["image_width"], device=gpu)
    rc = L.rr_forward_render(ctypes.byref(f), ctypes.byref(cam), ctypes.byref(g), x, geom.data_ptr(),
                             img.data_ptr(), binning.data_ptr(), binning.numel(), out["num_rendered"],
                             color.data_ptr(), color.data_ptr(), None)
    assert rc == 1 and b"pair count" in L.rr_last_error()
