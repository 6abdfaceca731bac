#!/usr/bin/env python3
"""Per-stage forward times (HIP events, rr_profile_*) of the bench model with exact tile culling
on and off, to see what the culling's per-row work costs the preprocess and the duplicate.

    python tools/cull_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from rain_amd import _native, fused, synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.diff_gaussian_rasterization import _C
    from rain_amd.gaussian_model import GaussianModel

    dev = torch.device("cuda:0")
    cams = [c.to(dev) for c in fibonacci_cameras(200, 1920, 1080)][:20]
    g = GaussianModel(3, device=dev)
    g.set_params(synthetic.random_gaussians(1_000_000, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    bg = torch.zeros(3, device=dev)
    cache = fused.BinningCache()
    for cull in (True, False, True, False):
        _C.TILE_CULLING = cull
        with torch.no_grad():
            for c in cams[:3]:
                fused.forward(g, c, bg, 0.3, cache=cache)
            torch.cuda.synchronize()
            _native.Profiler.collect()
            with _native.Profiler():
                for c in cams:
                    fused.forward(g, c, bg, 0.3, cache=cache)
            res = _native.Profiler.collect()
        print("cull" if cull else "no-cull", {k: round(v[0] / len(cams), 4) for k, v in res.items()})


if __name__ == "__main__":
    main()
