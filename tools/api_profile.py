#!/usr/bin/env python3
"""Host-side cost of the reference-API training step (what an unchanged train.py:109-147 runs:
render() -> GaussianRasterizer autograd -> GaussianModel getters autograd -> fused L1+SSIM ->
torch.optim.Adam) at the bench configuration: wall ms per step, and a cProfile of the Python side
sorted by own time, to find what keeps the GPU idle."""
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
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--points", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch

    from rain_amd import synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.renderer import PipelineParams, render
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    cams = [c.to(dev) for c in fibonacci_cameras(200, 1920, 1080)]
    gm = GaussianModel(3, device=dev)
    gm.set_params(synthetic.random_gaussians(a.points, sh_degree=3, seed=1, bench=True, device=dev))
    gm.active_sh_degree = 3
    with torch.no_grad():
        gts = [render(c, gm, PipelineParams(), torch.zeros(3, device=dev))["render"].clamp(0, 1).contiguous()
               for c in cams[:32]] * 7
    del gm
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(a.points, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    opt = OptimizationParams()
    g.training_setup(opt)
    groups = [{"params": q["params"], "lr": q["lr"], "name": q["name"]} for q in g.optimizer.param_groups]
    g.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(seed=1), scene_extent=4.4, fused=False)
    it = 1001
    for _ in range(5):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    ms = 1000.0 * (time.perf_counter() - t0) / a.steps
    print(f"api step: {ms:.3f} ms ({1000.0 / ms:.1f} it/s)", flush=True)
    # host time per step with the device out of the way (each step synced): Python + launch cost
    t_host = 0.0
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step(it)
        t_host += time.perf_counter() - t0
        it += 1
    print(f"host time to issue one step (device idle at start): {1000.0 * t_host / 10:.3f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
