#!/usr/bin/env python3
"""Per-bin run lengths of the bench frame's binning (1M Gaussians, 1920x1080, SH 3): the bounds
k_bin_bounds leaves in the image buffer's cleared block (rr_api.hip carve_img), for phase A and
phase B.  What k_sortexpand's per-bin depth sort sees: its LDS path takes runs up to kSxCap
pairs, longer runs go through global scratch in chunks."""
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

    W, H = 1920, 1080
    al = lambda x: (x + 255) & ~255  # noqa: E731  (rr_api.hip align_up)
    N = W * H
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    nbits = (T + 31) // 32
    NB = ((gx + 1) // 2) * ((gy + 1) // 2)
    ranges_off = al(al(N * 4) + N * 4)
    bounds_a = ranges_off + (2 * T + 2 + (nbits + 1) // 2) * 8
    dev = torch.device("cuda:0")
    params = synthetic.random_gaussians(1_000_000, sh_degree=3, seed=0, bench=True, device=dev)
    act = synthetic.activated(params)
    cams = [c.to(dev) for c in fibonacci_cameras(200, W, H)]
    out = {}
    for v in (0, 17, 101):
        s = synthetic.settings_for(cams[v], 3, torch.zeros(3, device=dev))
        e = torch.Tensor([])
        r = _C.rasterize_gaussians(s.bg, act["means3D"], e, act["opacities"], act["scales"], act["rotations"], 1.0,
                                   e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, act["shs"], 3,
                                   s.campos, False, False, 0.3)
        img = r[6]
        torch.cuda.synchronize()
        raw = img[bounds_a:bounds_a + 2 * NB * 8].cpu().numpy().view(np.uint32).reshape(2, NB, 2).astype(np.int64)
        res = {}
        for ph, b in zip("AB", raw):
            lo = np.where(b[:, 1] > 0, 0xFFFFFFFF - b[:, 0], 0)  # {~start, end} (rr_kernels.hpp)
            n = b[:, 1] - lo
            q = {p: int(np.percentile(n, p)) for p in (50, 90, 99, 100)}
            # where the long runs are: each bin's distance from the image centre (in bins,
            # normalised by the half-diagonal), for the longest 2 % against all bins
            bx, by = (gx + 1) // 2, (gy + 1) // 2
            X, Y = np.meshgrid(np.arange(bx), np.arange(by))
            dist = (np.hypot(X + 0.5 - bx / 2, Y + 0.5 - by / 2) / np.hypot(bx / 2, by / 2)).ravel()
            top = np.argsort(n)[-max(1, len(n) // 50):]
            res[ph] = dict(sum=int(n.sum()), nonempty=int((n > 0).sum()), pct=q,
                           over_2048=int((n > 2048).sum()), over_4096=int((n > 4096).sum()),
                           pairs_over_4096=int(n[n > 4096].sum()), top8=sorted(n.tolist())[-8:],
                           dist_all=round(float(dist.mean()), 3), dist_top2pct=round(float(dist[top].mean()), 3),
                           corr_len_dist=round(float(np.corrcoef(n, dist)[0, 1]), 3))
        out[v] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
