#!/usr/bin/env python3
"""Per-wave timeline of the forward blend at the bench workload (1M Gaussians, 1920x1080, SH 3).

Needs a build of librain_raster.so compiled with -DRR_FWD_TRACE=1 (tools/build_variant.py trace
-DRR_FWD_TRACE=1; RAIN_RASTER_LIB=gpurun_variants/trace.so).  Every wave of both blend phases
writes {start, end (s_memrealtime, 100 MHz), tile, pairs walked, list length, phase} into a
device buffer; this prints, per phase: kernel span, wave duration distribution, how many waves
are still running as the kernel drains, and the tiles of the last-finishing waves.

    RAIN_RASTER_LIB=$PWD/gpurun_variants/trace.so python tools/fwd_trace.py [--steps 5]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyse(rec, phase, tick_us=0.01):
    r = rec[(rec[:, 7] & 0xFF) == phase]
    r = r[(r[:, 0] | r[:, 1]) != 0]
    if len(r) == 0:
        print(f"phase {'SAB'[phase]}: no records")
        return
    start = (r[:, 1].astype(np.uint64) << np.uint64(32)) | r[:, 0].astype(np.uint64)
    end = (r[:, 3].astype(np.uint64) << np.uint64(32)) | r[:, 2].astype(np.uint64)
    t0 = start.min()
    s = (start - t0).astype(np.float64) * tick_us
    e = (end - t0).astype(np.float64) * tick_us
    d = e - s
    walked, n = r[:, 5].astype(np.int64), r[:, 6].astype(np.int64)
    span = e.max()
    print(f"phase {'SAB'[phase]}: {len(r)} waves, span {span:.1f} us, wave duration "
          f"p50 {np.median(d):.2f} p90 {np.percentile(d, 90):.2f} p99 {np.percentile(d, 99):.2f} max {d.max():.2f} us; "
          f"sum of wave time {d.sum():.0f} us")
    print(f"  pairs walked per wave: mean {walked.mean():.1f} p99 {np.percentile(walked, 99):.0f} max {walked.max()}; "
          f"list length mean {n.mean():.1f} max {n.max()}; us per walked pair (waves with >= 32): "
          f"{np.median(d[walked >= 32] / walked[walked >= 32]) if (walked >= 32).any() else 0:.3f}")
    # waves in flight over time (20 buckets)
    edges = np.linspace(0, span, 21)
    live = [int(((s <= t) & (e > t)).sum()) for t in edges[:-1] + (edges[1] - edges[0]) / 2]
    print("  waves running at 5%..95% of the span: " + " ".join(str(x) for x in live))
    last = np.argsort(-e)[:8]
    print("  last to finish: " + "; ".join(
        f"tile {r[i, 4]} start {s[i]:.1f} dur {d[i]:.1f} walked {walked[i]}/{n[i]}" for i in last))
    # list scheduling of the measured wave durations on the observed concurrency: XCD order (as
    # launched) vs longest-first by the list length n (known before the launch) vs by the true
    # duration (oracle) — how much of the drain a tile order could recover
    slots = max(live)
    import heapq

    def sched(order):
        h = [0.0] * slots
        for i in order:
            t = heapq.heappop(h)
            heapq.heappush(h, t + d[i])
        return max(h)

    tile = r[:, 4].astype(np.int64)
    print(f"  simulated span on {slots} slots: launch order {sched(np.argsort(s, kind='stable')):.1f} us, "
          f"longest list first {sched(np.argsort(-n, kind='stable')):.1f} us, longest wave first (oracle) "
          f"{sched(np.argsort(-d, kind='stable')):.1f} us; corr(duration, list length) {np.corrcoef(d, n)[0, 1]:.2f}, "
          f"corr(duration, walked) {np.corrcoef(d, walked)[0, 1]:.2f}")
    started_late = s.max()
    print(f"  last wave started at {started_late:.1f} us ({100 * started_late / span:.0f}% of the span)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=1, help="traced frames (gpurun_out/fwd_trace[_k].npy)")
    a = ap.parse_args()
    import torch

    from rain_amd import _native, synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.renderer import PipelineParams, render
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    cams = [c.to(dev) for c in fibonacci_cameras(200, a.width, a.height)][:8]
    extent = 4.4
    pipe = PipelineParams()
    bg = torch.zeros(3, device=dev)
    gt_model = GaussianModel(3, device=dev)
    gt_model.set_params(synthetic.random_gaussians(a.points, sh_degree=3, seed=1, bench=True, device=dev))
    gt_model.active_sh_degree = 3
    with torch.no_grad():
        gts = [render(c, gt_model, pipe, bg)["render"].clamp(0.0, 1.0).contiguous() for c in cams]
    del gt_model
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(a.points, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    g.spatial_lr_scale = extent
    opt = OptimizationParams()
    opt.densify_until_iter = 0
    g.training_setup(opt)
    tr = Trainer(g, cams, gts, opt, pipe, TrainConfig(seed=0), scene_extent=extent)
    T = ((a.width + 15) // 16) * ((a.height + 15) // 16)
    buf = torch.zeros(8 * 8 * T, dtype=torch.int32, device=dev)
    lib = _native.raster()
    for it in range(901, 901 + a.steps):
        tr.step(it)
    torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for k in range(a.frames):
        buf.zero_()
        lib.rr_debug_set_fwd_trace(ctypes.c_void_p(buf.data_ptr()))
        tr.step(901 + a.steps + k)
        torch.cuda.synchronize()
        lib.rr_debug_set_fwd_trace(ctypes.c_void_p(0))
        rec = buf.view(-1, 8).cpu().numpy().view(np.uint32)
        np.save(os.path.join(ROOT, "gpurun_out", "fwd_trace.npy" if k == 0 else f"fwd_trace_{k}.npy"), rec)
        print(f"frame {k}:")
        for phase in (0, 1, 2):  # single-phase, early-stop phase A, phase B
            analyse(rec, phase)


if __name__ == "__main__":
    main()
