#!/usr/bin/env python3
"""Host-side cost of the fused training step at the bench configuration: cProfile over N steps
(sorted by own time), plus the wall time of each step phase measured without device syncs.
Used to find launch / Python overhead that leaves the GPU idle after the forward's one sync."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--binning-split", type=int, default=0)
    ap.add_argument("--no-cprofile", action="store_true")
    ap.add_argument("--raster-lib", default=None, help="alternative librain_raster.so (A/B of builds)")
    a = ap.parse_args()
    import torch

    from rain_amd import synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.renderer import PipelineParams, render
    from rain_amd.train import TrainConfig, Trainer

    from rain_amd import _native

    if a.raster_lib:
        _native.RASTER_LIB = os.path.abspath(a.raster_lib)
    dev = torch.device("cuda:0")
    if a.binning_split:
        _native.check(_native.raster().rr_set_binning_config(a.binning_split, 0), "binning config")
    W, H, D = 1920, 1080, 3
    cams = [c.to(dev) for c in fibonacci_cameras(50, W, H)]
    gm = GaussianModel(D, device=dev)
    gm.set_params(synthetic.random_gaussians(a.points, sh_degree=D, seed=1, bench=True, device=dev))
    gm.active_sh_degree = D
    bg = torch.zeros(3, device=dev)
    with torch.no_grad():
        gts = [render(c, gm, PipelineParams(), bg)["render"].clamp(0.0, 1.0).contiguous() for c in cams]
    del gm
    g = GaussianModel(D, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(a.points, sh_degree=D, seed=0, bench=True, device=dev))
    g.active_sh_degree = D
    g.spatial_lr_scale = 4.4
    opt = OptimizationParams()
    g.training_setup(opt)
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(seed=0), scene_extent=4.4)
    it = 901
    for _ in range(5):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    import ctypes
    wn, wc = ctypes.c_int64(0), ctypes.c_int64(0)
    _native.raster().rr_host_wait_stats(1, ctypes.byref(wn), ctypes.byref(wc))
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    if not a.no_cprofile:
        pr.enable()
    for _ in range(a.steps):
        tr.step(it)
        it += 1
    pr.disable()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    _native.raster().rr_host_wait_stats(1, ctypes.byref(wn), ctypes.byref(wc))
    print(f"lib {a.raster_lib} split {a.binning_split} ms/step {1e3 * (t1 - t0) / a.steps:.3f}  "
          f"host wait for the pair counts {wn.value / 1e3 / max(wc.value, 1):.1f} us per frame ({wc.value} waits)")
    if a.no_cprofile:
        return
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
