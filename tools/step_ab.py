#!/usr/bin/env python3
"""In-process A/B of a training-step option at the bench configuration (1M Gaussians, 1080p,
SH 3): alternating blocks of steps with the option off / on, median ms per step of each.  Box-to-box
variance (a few %) hides small host-side wins; alternating blocks in one process does not.

    python tools/step_ab.py --option reuse_binning --blocks 6 --steps 50
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--option", default="reuse_binning", help="boolean Trainer attribute to toggle")
    ap.add_argument("--knob", default=None, help="native tuning key toggled 0/1 instead (rr_set_tuning)")
    ap.add_argument("--split", default=None,
                    help="comma-separated early-stop split denominators to compare (rr_set_binning_config)")
    ap.add_argument("--values", default=None, help="comma-separated integer values of --knob to compare (default 0,1)")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--stages", action="store_true", help="also report per-stage kernel time per arm")
    ap.add_argument("--steps", type=int, default=50)
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
               for c in cams]
    del gm
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(a.points, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    opt = OptimizationParams()
    opt.densify_until_iter = 0  # no densification: both arms see the same model size
    g.training_setup(opt)
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(seed=0, c2f=False), scene_extent=4.4)
    it = 1
    for _ in range(10):
        tr.step(it)
        it += 1
    arms = ([int(x) for x in a.split.split(",")] if a.split else
            [int(x) for x in a.values.split(",")] if a.values else [False, True])
    res = {v: [] for v in arms}
    stages = {v: {} for v in arms}
    for b in range(len(arms) * a.blocks):
        val = arms[b % len(arms)]
        if a.split:
            _native.check(_native.raster().rr_set_binning_config(val, 0), "binning config")
        elif a.knob:
            _native.check(_native.raster().rr_set_tuning(a.knob.encode(), int(val)), "tuning")
        else:
            setattr(tr, a.option, val)
        tr.step(it)
        it += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tr.step(it)
            it += 1
        torch.cuda.synchronize()
        res[val].append(1000 * (time.perf_counter() - t0) / a.steps)
        if a.stages:  # an extra profiled block: per-stage kernel time (HIP events) of this arm
            _native.Profiler.collect()
            with _native.Profiler():
                for _ in range(10):
                    tr.step(it)
                    it += 1
            for k, (ms, n) in _native.Profiler.collect().items():
                if n:
                    stages[val].setdefault(k, []).append(ms / 10)
    for v in arms:
        print(f"{'split' if a.split else (a.knob or a.option)}={v}: median {statistics.median(res[v]):.4f} ms/step  blocks {[round(x, 4) for x in res[v]]}")
        if a.stages:
            print("   stages ms/step:", {k: round(statistics.median(x), 4) for k, x in stages[v].items()})


if __name__ == "__main__":
    main()
