#!/usr/bin/env python3
"""Per-tile work distribution of the bench frame (1M Gaussians, 1920x1080, SH 3): pairs per tile
(ranges) and blended pairs per tile (tile_max, what the backward walks).  Used to reason about
load balance of the blend kernels."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from rain_amd import synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.diff_gaussian_rasterization import _C

    dev = torch.device("cuda:0")
    params = synthetic.random_gaussians(1_000_000, sh_degree=3, seed=0, bench=True, device=dev)
    act = synthetic.activated(params)
    cams = [c.to(dev) for c in fibonacci_cameras(200, 1920, 1080)]
    out, arrays = {}, {}
    for v in (0, 17, 101):
        s = synthetic.settings_for(cams[v], 3, torch.zeros(3, device=dev))
        e = torch.Tensor([])
        r = _C.rasterize_gaussians(s.bg, act["means3D"], e, act["opacities"], act["scales"], act["rotations"], 1.0,
                                   e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, 1080, 1920, act["shs"], 3,
                                   s.campos, False, False, 0.3)
        dv = _C.debug_views(r[4], r[5], r[6], r[0], 1_000_000, 1920, 1080)
        rng = dv["ranges"].cpu().numpy().astype(np.int64)
        n = rng[:, 1] - rng[:, 0]
        tm = dv["tile_max"].cpu().numpy().astype(np.int64)
        q = lambda a: {p: int(np.percentile(a, p)) for p in (50, 90, 99, 100)}  # noqa: E731
        out[v] = dict(pairs=dict(sum=int(n.sum()), mean=float(n.mean()), pct=q(n)),
                      tile_max=dict(sum=int(tm.sum()), mean=float(tm.mean()), pct=q(tm),
                                    top16=sorted(tm.tolist())[-16:]))
        arrays[f"tile_max_{v}"] = tm
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 1:  # per-tile arrays for offline schedule models
        np.savez_compressed(sys.argv[1], **arrays)


if __name__ == "__main__":
    main()
