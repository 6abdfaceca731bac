#!/usr/bin/env python3
"""Host (Python + driver) time of the bench's training step, from cProfile over K steps: which
calls the host spends the step in, against the device's step time.  With --force-dist the
Gaussian-sharded step at world 1 (the N > 1 code path); needs RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT in the environment for that (tools/gpu_run.sh hostprobe sets them).

    python tools/host_probe.py [--force-dist] [--steps 40] [--top 35]
"""
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
    ap.add_argument("--force-dist", action="store_true")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--top", type=int, default=35)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from rain_amd import synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.renderer import PipelineParams, render
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    if a.force_dist:
        dist.init_process_group("nccl", device_id=dev)
    cams = [c.to(dev) for c in fibonacci_cameras(200, 1920, 1080)]
    gm = GaussianModel(3, device=dev)
    gm.set_params(synthetic.random_gaussians(a.points, sh_degree=3, seed=1, bench=True, device=dev))
    gm.active_sh_degree = 3
    with torch.no_grad():
        gts = [render(c, gm, PipelineParams(), torch.zeros(3, device=dev))["render"].clamp(0, 1).contiguous()
               for c in cams[:64]]
    del gm
    gts = gts * 4
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(a.points, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    opt = OptimizationParams()
    g.training_setup(opt)
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(seed=0), scene_extent=4.4,
                 exchange=True if a.force_dist else None)
    it = 1001
    for _ in range(10):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    # device-bound step time (no profiler)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    step_ms = 1000.0 * (time.perf_counter() - t0) / a.steps
    # host time of one step alone: enqueue everything, then wait (the device work overlaps only
    # the host's own waits inside the step)
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        tr.step(it)
        it += 1
    pr.disable()
    torch.cuda.synchronize()
    prof_ms = 1000.0 * (time.perf_counter() - t0) / a.steps
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    print(f"step {step_ms:.3f} ms (no profiler), {prof_ms:.3f} ms under cProfile; per-step host times below are "
          f"totals / {a.steps}")
    st.sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    if a.force_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
