"""Offline rendering of a trained model (render.py:19-43 counterpart).

For every view: the image (``{idx:05d}.png``), the depth map min-max normalised to [0, 1]
(``{idx:05d}_depth.png``) and the depth through matplotlib's ``inferno`` colormap with
vmin = min and vmax = the 95th percentile (``{idx:05d}_depth_inferno.png``), written under
``<model_path>/<name>/ours_<iteration>/renders`` exactly as the reference lays them out.  PNG
encoding follows torchvision.utils.save_image (x*255 + 0.5, clamped, uint8; one-channel images
are written as RGB), which the reference uses and which is not installed here; the inferno image is
RGBA as imageio writes matplotlib's to_rgba output.  With ``normals=True`` the aux normal map
(include/rain_raster.h RR_FLAG_AUX_NORMAL) is written too (``{idx:05d}_normal.png``, n*0.5 + 0.5).

    python -m rain_amd.render_views --ply point_cloud.ply --model_path out --iteration 30000 \\
        --num_cams 10 --width 800 --height 800

Scene / COLMAP camera loading is out of scope; the CLI renders synthetic
Fibonacci-sphere cameras (rain_amd.cameras), the function API takes any camera list.
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from .renderer import PipelineParams, render, render_depth_normal


def _to_u8(img: torch.Tensor) -> np.ndarray:
    """torchvision.utils.save_image's conversion of a [C,H,W] float image (C = 1 or 3)."""
    x = img.detach().float().cpu()
    if x.shape[0] == 1:
        x = x.repeat(3, 1, 1)
    return x.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()


def save_image(img: torch.Tensor, path: str) -> None:
    from PIL import Image

    Image.fromarray(_to_u8(img)).save(path)


def depth_inferno(depth_hw: np.ndarray) -> np.ndarray:
    """render.py:33-37: Normalize(vmin=min, vmax=percentile(95)) -> inferno -> RGBA uint8."""
    import matplotlib as mpl
    import matplotlib.cm as cm

    norm = mpl.colors.Normalize(vmin=depth_hw.min(), vmax=np.percentile(depth_hw, 95))
    return (cm.ScalarMappable(norm=norm, cmap="inferno").to_rgba(depth_hw) * 255).astype("uint8")


def render_set(model_path, name, iteration, views, gaussians, pipeline, background, normals=False):
    """render.py:19-43 (the gt images are not written, as in the reference)."""
    from PIL import Image

    render_path = os.path.join(model_path, name, "ours_{}".format(iteration), "renders")
    os.makedirs(render_path, exist_ok=True)
    os.makedirs(os.path.join(model_path, name, "ours_{}".format(iteration), "gt"), exist_ok=True)
    written = []
    for idx, view in enumerate(views):
        with torch.no_grad():
            if normals:
                out = render_depth_normal(view, gaussians, background)
            else:
                out = render(view, gaussians, pipeline, background)
        image, depth = out["render"], out["depth"]
        depth_n = (depth - depth.min()) / (depth.max() - depth.min() + 1e-6)
        base = os.path.join(render_path, "{0:05d}".format(idx))
        Image.fromarray(depth_inferno(depth.permute(1, 2, 0).squeeze().cpu().numpy())).save(
            base + "_depth_inferno.png")
        save_image(image, base + ".png")
        save_image(depth_n, base + "_depth.png")
        if normals:
            save_image(out["normal"] * 0.5 + 0.5, base + "_normal.png")
        written.append(base)
    return written


def main(argv=None):
    from .cameras import fibonacci_cameras
    from .gaussian_model import GaussianModel

    ap = argparse.ArgumentParser(description="render a trained model (render.py counterpart)")
    ap.add_argument("--ply", required=True)
    ap.add_argument("--model_path", required=True)
    ap.add_argument("--iteration", type=int, default=30000)
    ap.add_argument("--sh_degree", type=int, default=3)
    ap.add_argument("--num_cams", type=int, default=10)
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--radius", type=float, default=4.0)
    ap.add_argument("--white_background", action="store_true")
    ap.add_argument("--normals", action="store_true")
    a = ap.parse_args(argv)
    dev = torch.device("cuda", torch.cuda.current_device())
    g = GaussianModel(a.sh_degree, device=dev)
    g.load_ply(a.ply)
    bg = torch.tensor([1.0, 1.0, 1.0] if a.white_background else [0.0, 0.0, 0.0], device=dev)
    cams = [c.to(dev) for c in fibonacci_cameras(a.num_cams, a.width, a.height, radius=a.radius)]
    render_set(a.model_path, "test", a.iteration, cams, g, PipelineParams(), bg, normals=a.normals)


if __name__ == "__main__":
    main()
