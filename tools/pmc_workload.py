#!/usr/bin/env python3
"""Fixed rasterizer workload for rocprofv3 counter passes: the bench model (1M Gaussians, SH 3,
1920x1080) rendered forward + backward on --frames views through the product path.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv \\
        -- python3 tools/pmc_workload.py
    (a second pass with --pmc WRITE_SIZE), then tools/pmc_traffic.py turns both into
    profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    args = ap.parse_args()

    import torch

    from rain_amd import synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.diff_gaussian_rasterization import GaussianRasterizer

    dev = torch.device("cuda:0")
    params = synthetic.random_gaussians(args.points, sh_degree=3, seed=0, bench=True, device=dev)
    act = synthetic.activated(params)
    cams = [c.to(dev) for c in fibonacci_cameras(200, args.width, args.height)]
    bg = torch.zeros(3, device=dev)
    for i in range(args.frames):
        lv = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
        means2D = torch.zeros_like(lv["means3D"], requires_grad=True)
        r = GaussianRasterizer(synthetic.settings_for(cams[i], 3, bg, low_pass=0.3))
        color, radii, depth = r(means2D=means2D, **lv)
        color.sum().backward()
    torch.cuda.synchronize()
    print("frames", args.frames, "ok")


if __name__ == "__main__":
    main()
