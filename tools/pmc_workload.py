#!/usr/bin/env python3
"""Fixed workload for rocprofv3 counter passes: the bench's training step (1M Gaussians, SH 3,
1920x1080, rain_amd.train.Trainer on the fused raw-parameter path, Adam inside the backward)
for --steps iterations, so the counters describe the same kernels, in the same variants, as
bench.py's timed loop (densification is left out: it runs once per 100 iterations).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv \\
        -- python3 tools/pmc_workload.py
    (a second pass with --pmc WRITE_SIZE, ...), then tools/pmc_traffic.py turns the passes into
    profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    args = ap.parse_args()

    import torch

    from rain_amd import synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.renderer import PipelineParams, render
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    cams = [c.to(dev) for c in fibonacci_cameras(200, args.width, args.height)][: args.views]
    extent = 4.0 * 1.1  # as bench.py
    pipe = PipelineParams()
    bg = torch.zeros(3, device=dev)
    gt_model = GaussianModel(3, device=dev)
    gt_model.set_params(synthetic.random_gaussians(args.points, sh_degree=3, seed=1, bench=True, device=dev))
    gt_model.active_sh_degree = 3
    with torch.no_grad():
        gts = [render(c, gt_model, pipe, bg)["render"].clamp(0.0, 1.0).contiguous() for c in cams]
    del gt_model
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(args.points, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    g.spatial_lr_scale = extent
    opt = OptimizationParams()
    opt.densify_until_iter = 0
    g.training_setup(opt)
    tr = Trainer(g, cams, gts, opt, pipe, TrainConfig(seed=0), scene_extent=extent)
    for it in range(901, 901 + args.steps):
        tr.step(it)
    torch.cuda.synchronize()
    print("steps", args.steps, "ok")


if __name__ == "__main__":
    main()
