#!/usr/bin/env python3
"""The reference-API training step (Trainer(fused=False): render() -> GaussianRasterizer autograd ->
fused L1+SSIM -> the optimizer GaussianModel.training_setup builds) at the bench configuration,
with bench.py's trace markers around the timed steps, so that a rocprofv3 kernel trace of this
script is cut to those steps by tools/step_breakdown.py --window (--seq: the launch sequence with
the idle gaps the host leaves).  Prints the wall ms per step.

    rocprofv3 --kernel-trace -d gpurun_out/api -o run --output-format csv -- python3 tools/api_trace.py
"""
import argparse
import os
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

    from rain_amd import _native, synthetic
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
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(seed=1), scene_extent=4.4, fused=False)
    it = 1001
    for _ in range(5):
        tr.step(it)
        it += 1
    mark = _native.train_lib().rt_trace_marker
    _native.check_rt(mark(0, a.steps, _native.stream_of(tr.background)), "trace marker")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    ms = 1000.0 * (time.perf_counter() - t0) / a.steps
    _native.check_rt(mark(1, a.steps, _native.stream_of(tr.background)), "trace marker")
    torch.cuda.synchronize()
    print(f"api step (optimizer {type(g.optimizer).__name__}): {ms:.3f} ms ({1000.0 / ms:.1f} it/s)", flush=True)


if __name__ == "__main__":
    main()
