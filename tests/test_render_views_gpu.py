"""render.py counterpart (rain_amd.render_views.render_set, SURVEY §8(f) #4, render.py:19-43) on the
HIP rasterizer: the PNGs it writes from the MI355X frame equal the encodings of the CPU oracle's
frame of the same model and camera.

Bar: the oracle and the GPU agree to ~1e-6 per pixel, so an 8-bit encoding can differ only where a
value sits within that of a rounding boundary: at most 1 level, on at most 0.1 % of the samples.
The inferno image may differ where depth crosses one of the colormap's 256 bins: by one LUT
step (a few levels per channel), on the same small share of samples."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from rain_amd import cameras, synthetic
from rain_amd.gaussian_model import GaussianModel
from rain_amd.render_views import depth_inferno, render_set
from rain_amd.renderer import PipelineParams
from tests.common import oracle_settings

pytestmark = pytest.mark.gpu


def _u8(x):
    """torchvision save_image's encoding of a [C,H,W] float array -> [H,W,C] uint8."""
    x = np.asarray(x, dtype=np.float32)
    if x.shape[0] == 1:
        x = np.repeat(x, 3, axis=0)
    return np.clip(x * 255.0 + 0.5, 0, 255).astype(np.uint8).transpose(1, 2, 0)


def _close_u8(a, b, what, max_level=1):
    a, b = np.asarray(a).astype(np.int32), np.asarray(b).astype(np.int32)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    d = np.abs(a - b)
    assert d.max() <= max_level, f"{what}: max level difference {d.max()}"
    assert (d > 0).mean() <= 1e-3, f"{what}: {(d > 0).mean():.2e} of samples differ"


def test_render_set_pngs_match_oracle_frames(oracle, gpu, tmp_path):
    P, W, H = 20_000, 320, 240
    raw = synthetic.random_gaussians(P, sh_degree=3, seed=9, bench=True, device=gpu)
    g = GaussianModel(3, device=gpu)
    g.set_params(raw)
    g.active_sh_degree = 3
    cams = [c.to(gpu) for c in cameras.fibonacci_cameras(3, W, H)]
    bg = torch.zeros(3, device=gpu)
    bases = render_set(str(tmp_path), "test", 30000, cams, g, PipelineParams(), bg, normals=True)
    d = tmp_path / "test" / "ours_30000" / "renders"
    assert sorted(os.listdir(d)) == sorted(f"{i:05d}{s}.png" for i in range(3)
                                          for s in ("", "_depth", "_depth_inferno", "_normal"))

    act = {k: v.detach().float().contiguous().cpu().numpy() for k, v in synthetic.activated(raw).items()}
    for base, cam in zip(bases, cameras.fibonacci_cameras(3, W, H)):
        st = synthetic.settings_for(cam, sh_degree=3)._asdict()
        s = oracle_settings(oracle, {k: (v.float().contiguous() if isinstance(v, torch.Tensor) else v)
                                     for k, v in st.items()})
        _nr, color, _radii, depth, _state, nmap = oracle.forward(
            s, act["means3D"], act["opacities"], shs=act["shs"], scales=act["scales"], rotations=act["rotations"],
            normal=True)
        _close_u8(np.asarray(Image.open(base + ".png")), _u8(color), "image")
        dep = depth.reshape(1, H, W).astype(np.float32)
        dn = (dep - dep.min()) / (dep.max() - dep.min() + np.float32(1e-6))
        _close_u8(np.asarray(Image.open(base + "_depth.png")), _u8(dn), "normalised depth")
        _close_u8(np.asarray(Image.open(base + "_depth_inferno.png")), depth_inferno(dep[0]), "inferno depth",
                  max_level=5)  # largest step between adjacent inferno LUT entries
        _close_u8(np.asarray(Image.open(base + "_normal.png")), _u8(nmap.reshape(3, H, W) * 0.5 + 0.5), "normal map")
