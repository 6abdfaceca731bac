#!/usr/bin/env python3
"""How much of the tile binning does blending actually use?  For bench frames (1M Gaussians,
1920x1080, SH 3) this replays every tile's front-to-back blend (torch, vectorised over tiles and
pixels) to find the list position at which the tile's last pixel saturates, maps it to the global
depth rank of that Gaussian, and reports, for depth-prefix cut points R, how many pairs a binning
restricted to ranks < R (all tiles) plus ranks >= R (only tiles still open at R) would emit.
Diagnostic for saturation-aware binning."""
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
    P, W, H = 1_000_000, 1920, 1080
    params = synthetic.random_gaussians(P, sh_degree=3, seed=0, bench=True, device=dev)
    act = synthetic.activated(params)
    cams = [c.to(dev) for c in fibonacci_cameras(200, W, H)]
    out = {}
    gx, gy = (W + 15) // 16, (H + 15) // 16
    for v in (0, 17, 101):
        s = synthetic.settings_for(cams[v], 3, torch.zeros(3, device=dev))
        e = torch.Tensor([])
        r = _C.rasterize_gaussians(s.bg, act["means3D"], e, act["opacities"], act["scales"], act["rotations"], 1.0,
                                   e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, act["shs"], 3,
                                   s.campos, False, False, 0.3)
        dv = _C.debug_views(r[4], r[5], r[6], r[0], P, W, H)
        pl = dv["point_list"].long()
        rg = dv["ranges"].long()
        sp = dv["splats"]
        T = rg.shape[0]
        n = rg[:, 1] - rg[:, 0]
        # depth rank of every Gaussian: stable order of (view depth, index) as the binning sorts
        depth = sp[:, 6]
        order = torch.argsort(depth, stable=True)
        rank = torch.empty_like(order)
        rank[order] = torch.arange(P, device=dev)
        # pixel coordinates per tile
        ty, tx = torch.div(torch.arange(T, device=dev), gx, rounding_mode="floor"), torch.arange(T, device=dev) % gx
        lp = torch.arange(256, device=dev)
        px = (tx[:, None] * 16 + lp[None] % 16).float()
        py = (ty[:, None] * 16 + lp[None] // 16).float()
        valid = (px < W) & (py < H)
        Tr = torch.ones((T, 256), device=dev)
        done = ~valid
        close = torch.full((T,), -1, dtype=torch.long, device=dev)
        j = 0
        maxn = int(n.max())
        while j < maxn:
            act_t = (n > j) & (close < 0)
            if not bool(act_t.any()):
                break
            g = pl[(rg[:, 0] + j).clamp(max=pl.numel() - 1)]
            rec = sp[g]
            dx = rec[:, 0, None] - px
            dy = rec[:, 1, None] - py
            power = -0.5 * (rec[:, 2, None] * dx * dx + rec[:, 4, None] * dy * dy) - rec[:, 3, None] * dx * dy
            alpha = torch.clamp(rec[:, 5, None] * torch.exp(power), max=0.99)
            ok = act_t[:, None] & ~done & (power <= 0) & (alpha >= 1.0 / 255.0)
            testT = Tr * (1 - alpha)
            sat = ok & (testT < 1e-4)
            done = done | sat
            Tr = torch.where(ok & ~sat, testT, Tr)
            newly = act_t & done.all(dim=1) & (close < 0)
            close[newly] = j
            j += 1
        closed = close >= 0
        crank = torch.full((T,), P, dtype=torch.long, device=dev)
        crank[closed] = rank[pl[rg[closed, 0] + close[closed]]]
        pr = rank[pl]  # rank of every pair
        tile_of = torch.repeat_interleave(torch.arange(T, device=dev), n)
        L = int(pl.numel())
        cuts = {}
        R0 = int(pr.min())  # culled Gaussians (no pairs) sort first
        # cut points in pair space: phase A bins the first f*L pairs (depth order) for every tile,
        # phase B the rest only for tiles still open after A
        cum = torch.cumsum(torch.bincount(pr, minlength=P), 0)
        for frac in (1 / 64, 1 / 32, 1 / 16, 1 / 8, 1 / 4):
            R = int(torch.searchsorted(cum, int(frac * L)))
            a_pairs = int((pr < R).sum())
            open_t = crank >= R
            b_pairs = int(((pr >= R) & open_t[tile_of]).sum())
            cuts[f"{frac:.4f}"] = dict(R=R, pairs_prefix=a_pairs, pairs_suffix_open=b_pairs,
                                       open_tiles=int(open_t.sum()), frac_of_L=round((a_pairs + b_pairs) / L, 4))
        used = int(torch.where(closed, close + 1, n).sum())
        out[v] = dict(L=L, tiles=T, tiles_never_closed=int((~closed).sum()), pairs_up_to_close=used,
                      close_rank_pct={p: round(float(np.percentile(crank[closed].cpu().numpy() - R0, p)) / (P - R0), 4)
                                      for p in (50, 90, 99, 100)}
                      if bool(closed.any()) else None, cuts=cuts)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
