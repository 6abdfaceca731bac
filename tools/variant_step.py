#!/usr/bin/env python3
"""Per-stage kernel time and step time of the bench's training step for ONE build of
librain_raster.so (RAIN_RASTER_LIB selects a variant from tools/build_variant.py), as one JSON
line.  Run it once per variant in the same GPU call: same box, same clocks.

    RAIN_RASTER_LIB=gpurun_variants/x.so python tools/variant_step.py --tag x
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default=os.environ.get("RAIN_RASTER_LIB", "default"))
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--api", action="store_true", help="also time the reference-API step (Trainer(fused=False))")
    ap.add_argument("--pack", action="store_true", help="parameters and moments in three flat buffers (pack_flat_state)")
    ap.add_argument("--tune", action="append", default=[], help="rr_set_tuning key=value (repeatable)")
    ap.add_argument("--no-fuse-next", action="store_true",
                    help="the next frame's preprocess as its own launch (Trainer.fuse_next = False)")
    ap.add_argument("--skew-state", type=int, default=0,
                    help="re-place each Adam moment at an offset of this many KiB (+ 1/2 MiB steps) from "
                         "its parameter's alignment (HBM channel-placement probe)")
    a = ap.parse_args()
    import torch

    from rain_amd import _native, synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.renderer import PipelineParams, render
    from rain_amd.train import TrainConfig, Trainer

    for kv in a.tune:
        k, v = kv.split("=")
        _native.check(_native.raster().rr_set_tuning(k.encode(), int(v)), "rr_set_tuning " + kv)
    dev = torch.device("cuda:0")
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
    tr = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(seed=0), scene_extent=4.4)
    if a.no_fuse_next:
        tr.fuse_next = False
    if a.pack:
        g.optimizer.fused_step(g)  # creates the moment state the packing moves
        g.pack_flat_state(1)
    it = 1001
    for _ in range(10):
        tr.step(it)
        it += 1
    if a.skew_state:
        # each moment in a fresh buffer at a non-power-of-two offset, so that element i of a
        # parameter and of its two moments no longer share an address modulo the allocator's 2 MiB
        # alignment
        keep = []
        for k, p in enumerate(g.params()):
            st = g.optimizer.state[p]
            for j, name in enumerate(("exp_avg", "exp_avg_sq")):
                off = (j + 1) * (262144 + a.skew_state * 256)  # floats: (j+1) x (1 MiB + skew KiB)
                buf = torch.empty(p.numel() + off, device=dev)
                buf[off:].copy_(st[name].reshape(-1))
                st[name] = buf[off:].view_as(p)
                keep.append(buf)
        torch.cuda.synchronize()
        for _ in range(3):
            tr.step(it)
            it += 1
    _native.Profiler.collect()
    with _native.Profiler():
        for _ in range(20):
            tr.step(it)
            it += 1
    br = _native.Profiler.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.step(it)
        it += 1
    torch.cuda.synchronize()
    ms = 1000.0 * (time.perf_counter() - t0) / a.steps
    # a coarse sanity value of the trained state (float atomics make it differ in the last bits
    # between runs, so compare it approximately across variants)
    chk = float(sum(float(t.detach().double().abs().sum()) for t in g.params()))
    out = {"tag": a.tag, "ms_per_step": round(ms, 4), "state_abs_sum": chk,
           "stages_ms": {k: round(v[0] / 20, 4) for k, v in br.items() if v[1]}}
    if a.api:
        tr2 = Trainer(g, cams, gts, opt, PipelineParams(), TrainConfig(seed=1), scene_extent=4.4, fused=False)
        import torch.optim

        fused_opt = g.optimizer
        groups = [{"params": q["params"], "lr": q["lr"], "name": q["name"]} for q in fused_opt.param_groups]
        g.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        it = 2001
        for _ in range(5):
            tr2.step(it)
            it += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            tr2.step(it)
            it += 1
        torch.cuda.synchronize()
        out["api_ms_per_step"] = round(1000.0 * (time.perf_counter() - t0) / 20, 4)
        g.optimizer = fused_opt
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
