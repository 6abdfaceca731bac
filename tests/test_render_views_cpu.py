"""render.py counterpart (rain_amd.render_views) on CPU with the oracle standing
in for the HIP `_C`: file layout and the depth / image encodings of render.py:19-43."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

import rain_amd.diff_gaussian_rasterization as dgr
from rain_amd import cameras, synthetic
from rain_amd.gaussian_model import GaussianModel
from rain_amd.render_views import depth_inferno, render_set
from rain_amd.renderer import PipelineParams, render, render_depth_normal
from tests import oracle_c


@pytest.fixture
def cpu_rasterizer(monkeypatch, oracle):
    monkeypatch.setattr(dgr, "_C", oracle_c)


def _model():
    g = GaussianModel(1, device="cpu")
    g.set_params(synthetic.random_gaussians(1500, sh_degree=1, seed=4))
    g.active_sh_degree = 1
    return g


def test_render_set_layout_and_encodings(cpu_rasterizer, tmp_path):
    g = _model()
    cams = cameras.fibonacci_cameras(2, 64, 48)
    bg = torch.zeros(3)
    bases = render_set(str(tmp_path), "test", 7000, cams, g, PipelineParams(), bg, normals=True)
    d = tmp_path / "test" / "ours_7000" / "renders"
    assert sorted(os.listdir(d)) == sorted(f"{i:05d}{s}.png" for i in range(2)
                                          for s in ("", "_depth", "_depth_inferno", "_normal"))
    assert (tmp_path / "test" / "ours_7000" / "gt").is_dir()
    with torch.no_grad():
        out = render(cams[0], g, PipelineParams(), bg)
    img = np.asarray(Image.open(bases[0] + ".png"))
    ref = (out["render"].mul(255).add(0.5).clamp(0, 255).permute(1, 2, 0).to(torch.uint8)).numpy()
    assert img.shape == (48, 64, 3) and np.array_equal(img, ref)
    dep = out["depth"]
    dn = (dep - dep.min()) / (dep.max() - dep.min() + 1e-6)
    dimg = np.asarray(Image.open(bases[0] + "_depth.png"))
    assert dimg.shape == (48, 64, 3) and np.array_equal(dimg[..., 0], dn.mul(255).add(0.5).clamp(0, 255).to(
        torch.uint8)[0].numpy())
    inf = np.asarray(Image.open(bases[0] + "_depth_inferno.png"))
    assert inf.shape == (48, 64, 4) and np.array_equal(inf, depth_inferno(dep[0].numpy()))


def test_render_depth_normal_cpu(cpu_rasterizer):
    g = _model()
    cam = cameras.fibonacci_cameras(3, 64, 48)[1]
    out = render_depth_normal(cam, g, torch.zeros(3))
    with torch.no_grad():
        plain = render(cam, g, PipelineParams(), torch.zeros(3))
    assert torch.equal(out["render"], plain["render"]) and torch.equal(out["depth"], plain["depth"])
    n = torch.linalg.vector_norm(out["normal"], dim=0)
    assert float(n.max()) <= 1 + 1e-5 and float(n.sum()) > 0
