#!/usr/bin/env python3
"""A/B timing of rasterizer kernel variants in ONE process (interleaved rounds), on the bench
workload (1M random Gaussians, 1920x1080, SH 3).  Reports per-stage median ms per config and checks
that every config produces the same image / gradients.

    python tools/raster_ab.py --configs 4:1,1:1,2:2,4:4 --rounds 5
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="4:1:1,4:1:0", help="fwd_waves:bwd_waves[:tile_culling]")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--views", type=int, default=4)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--low-pass", type=float, default=0.3)
    ap.add_argument("--knob", default=None, help="compare values of a native tuning key (rr_set_tuning) instead")
    ap.add_argument("--values", default="0,1", help="with --knob: comma-separated values")
    args = ap.parse_args()

    import torch

    from rain_amd import _native, synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.diff_gaussian_rasterization import GaussianRasterizer

    dev = torch.device("cuda:0")
    params = synthetic.random_gaussians(args.points, sh_degree=3, seed=0, bench=True, device=dev)
    act = synthetic.activated(params)
    cams = [c.to(dev) for c in fibonacci_cameras(200, args.width, args.height)][:args.views]
    L = _native.raster()
    from rain_amd.diff_gaussian_rasterization import _C

    if args.knob:
        cfgs = [(0, 0, 1, int(v)) for v in args.values.split(",")]
    else:
        cfgs = [tuple(int(x) for x in (c.split(":") + ["1"])[:3]) for c in args.configs.split(",")]
    times = {c: {} for c in cfgs}
    outs = {}
    for r in range(args.rounds):
        for c in cfgs:
            L.rr_set_blend_config(c[0], c[1])
            _C.TILE_CULLING = bool(c[2])
            if args.knob:
                _native.check(L.rr_set_tuning(args.knob.encode(), c[3]), "tuning")
            L.rr_profile_enable(1)
            _native.Profiler.collect()
            for vi, cam in enumerate(cams):
                st = synthetic.settings_for(cam, 3, low_pass=args.low_pass)
                leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
                m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
                img, radii, depth = GaussianRasterizer(st)(means3D=leaves["means3D"], means2D=m2,
                                                           opacities=leaves["opacities"], shs=leaves["shs"],
                                                           scales=leaves["scales"], rotations=leaves["rotations"])
                g = torch.Generator(device=dev).manual_seed(vi)
                dpix = torch.randn(img.shape, device=dev, generator=g)
                (img * dpix).sum().backward()
                if r == 0 and vi == 0:
                    outs[c] = (img.detach().clone(), leaves["means3D"].grad.clone(), leaves["shs"].grad.clone())
            torch.cuda.synchronize()
            L.rr_profile_enable(0)
            for k, (ms, n) in _native.Profiler.collect().items():
                if n:
                    times[c].setdefault(k, []).append(ms / n)
    L.rr_set_blend_config(0, 0)
    base = outs[cfgs[0]]
    res = {}
    for c in cfgs:
        o = outs[c]
        same_img = bool(torch.equal(o[0], base[0]))
        rel = lambda a, b: float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))  # noqa: E731
        res[f"{args.knob}={c[3]}" if args.knob else f"{c[0]}:{c[1]}:{c[2]}"] = {"stages_ms": {k: round(statistics.median(v), 4) for k, v in times[c].items()},
                                 "image_bitwise_equal": same_img, "dmeans3D_relL1": rel(o[1], base[1]),
                                 "dsh_relL1": rel(o[2], base[2])}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
