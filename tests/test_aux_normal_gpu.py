"""Auxiliary depth + normal outputs (BASELINE configs[4]; include/rain_raster.h RR_FLAG_AUX_NORMAL).

The reference renders no normals, so the normal map is parity-tested against the oracle's
restatement of the build's own definition (oracle/raster_oracle.c gaussian_normal) — parity
unpinned against the reference itself.  Colour / depth / gradients of the aux call must be those of
the plain call, bitwise (the aux channels ride along in the same blend loop)."""
import numpy as np
import pytest
import torch

from rain_amd import _native as N
from tests.common import GRAD_NAMES, make_scene, oracle_settings, rel_l1

pytestmark = pytest.mark.gpu


def _args(inp, st, dev):
    d = {k: v.to(dev) for k, v in inp.items()}
    s = {k: (v.to(dev) if isinstance(v, torch.Tensor) else v) for k, v in st.items()}
    e = torch.Tensor([])
    return (s["bg"], d["means3D"], d.get("colors_precomp", e), d["opacities"], d["scales"], d["rotations"],
            s["scale_modifier"], e, s["viewmatrix"], s["projmatrix"], s["tanfovx"], s["tanfovy"], s["image_height"],
            s["image_width"], d.get("shs", e), s["sh_degree"], s["campos"], s["prefiltered"], s["debug"],
            s["low_pass"]), d, s


@pytest.fixture(params=[0, 2], ids=["default_binning", "early_stop_split2"])
def binning(request):
    if request.param:
        N.check(N.raster().rr_set_binning_config(request.param, 1), "binning config")
    yield request.param
    N.check(N.raster().rr_set_binning_config(0, 0), "binning config")


@pytest.mark.parametrize("case", [dict(P=3000, W=128, H=96, sh_degree=3), dict(P=2000, W=100, H=75, sh_degree=1),
                                  dict(P=800, W=160, H=120, sh_degree=3, low_pass=300.0)],
                         ids=["sh3", "ragged", "low_pass_300"])
def test_normal_map_matches_oracle(oracle, gpu, binning, case):
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(**case)
    args, d, s = _args(inp, st, gpu)
    nr, color, radii, depth, normal, geom, binb, img = _C.rasterize_gaussians_aux(*args)
    nr0, color0, radii0, depth0, *_ = _C.rasterize_gaussians(*args)
    torch.cuda.synchronize()
    assert nr == nr0 and torch.equal(color, color0) and torch.equal(depth, depth0) and torch.equal(radii, radii0)
    n = {k: v.numpy() for k, v in inp.items()}
    ref = oracle.forward(oracle_settings(oracle, st), n["means3D"], n["opacities"], shs=n["shs"], scales=n["scales"],
                         rotations=n["rotations"], normal=True)
    nmap = ref[5]
    assert np.abs(nmap).sum() > 0
    e = rel_l1(normal.cpu().numpy(), nmap)
    assert e <= 1e-4, f"normal map rel L1 {e:.3e}"
    # per pixel |N| <= 1 - T_final (unit normals, weights alpha*T sum to 1 - T)
    nn = np.linalg.norm(normal.cpu().numpy(), axis=0)
    assert (nn <= 1.0 + 1e-5).all()


def test_aux_buffers_feed_the_backward(gpu):
    from rain_amd.diff_gaussian_rasterization import _C

    inp, st = make_scene(P=2000, W=96, H=80, sh_degree=3)
    args, d, s = _args(inp, st, gpu)
    dpix = torch.randn((3, 80, 96), generator=torch.Generator().manual_seed(3)).to(gpu)
    grads = []
    for aux in (False, True):
        out = _C.rasterize_gaussians_aux(*args) if aux else _C.rasterize_gaussians(*args)
        nr, radii = out[0], out[2]
        geom, binb, img = out[-3:]
        e = torch.Tensor([])
        g = _C.rasterize_gaussians_backward(s["bg"], d["means3D"], radii, e, d["scales"], d["rotations"],
                                            s["scale_modifier"], e, s["viewmatrix"], s["projmatrix"], s["tanfovx"],
                                            s["tanfovy"], dpix, d["shs"], s["sh_degree"], s["campos"], geom, nr, binb,
                                            img, False, s["low_pass"])
        grads.append([t.cpu() for t in g])
    for name, a, b in zip(GRAD_NAMES, *grads):  # float atomics: equal up to summation order
        assert rel_l1(a.numpy(), b.numpy()) <= 1e-5, name


def test_render_depth_normal_surface(gpu, monkeypatch):
    from rain_amd import renderer as renderer_mod
    from rain_amd import synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel
    from rain_amd.renderer import PipelineParams, render, render_depth_normal

    # render_depth_normal rasterizes the getters' outputs: compare with render() on the same route
    # (its raw-parameter fast path applies the getters in-kernel, an ulp away from torch's)
    monkeypatch.setattr(renderer_mod, "RAW_RENDER", False)

    g = GaussianModel(3, device=gpu)
    g.set_params(synthetic.random_gaussians(4000, sh_degree=3, seed=2, bench=True, device=gpu))
    g.active_sh_degree = 3
    cam = fibonacci_cameras(4, 160, 120)[1].to(gpu)
    bg = torch.zeros(3, device=gpu)
    out = render_depth_normal(cam, g, bg)
    with torch.no_grad():
        plain = render(cam, g, PipelineParams(), bg)
    assert set(out) == {"render", "depth", "normal", "radii", "visibility_filter"}
    assert out["normal"].shape == (3, 120, 160)
    assert torch.equal(out["render"], plain["render"]) and torch.equal(out["depth"], plain["depth"])
    n = out["normal"]
    assert float(n.abs().sum()) > 0 and float(torch.linalg.vector_norm(n, dim=0).max()) <= 1.0 + 1e-5
