#!/usr/bin/env python3
"""How much per-pixel blend work row-band masks could skip on the bench frame (CPU, oracle).

For one 1920x1080 view of the 1M-Gaussian bench model: per tile, the pairs a blend kernel walks
(up to the last contributor of the region's pixels) and, for each pair, which 4-row bands of the
tile contain a pixel centre with alpha >= 1/255 (forward.cu:329-336).  Prints the pixel-pair
evaluations of (a) today's layout (a wave walks its region's pairs for all its pixels) and (b) one
that skips, per pair, the bands the Gaussian does not reach.

    python tools/band_stats.py [--points 1000000] [--view 0]
"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--view", type=int, default=0)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    import torch

    from oracle import oracle as O
    from rain_amd import cameras, synthetic
    from tests.common import oracle_settings

    O.build()
    raw = synthetic.random_gaussians(a.points, sh_degree=3, seed=0, bench=True)
    act = {k: v.float().contiguous().numpy() for k, v in synthetic.activated(raw).items()}
    W, H = a.width, a.height
    cam = cameras.fibonacci_cameras(200, W, H)[a.view]
    st = synthetic.settings_for(cam, 3)._asdict()
    s = oracle_settings(O, {k: (v.float().contiguous() if isinstance(v, torch.Tensor) else v) for k, v in st.items()})
    nr, color, radii, depth, state = O.forward(s, act["means3D"], act["opacities"], shs=act["shs"],
                                               scales=act["scales"], rotations=act["rotations"])
    it = state.internals()
    pl, rg, nc = it["point_list"], it["ranges"], it["n_contrib"]
    xy, co = it["xy"], it["conic_opacity"]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    base_half = base_tile = masked = masked_half = pairs_walk = live_only = band_only = 0
    touched_hist = np.zeros(5, np.int64)
    ys = np.arange(16, dtype=np.float32)
    xs = np.arange(16, dtype=np.float32)
    for t in range(gx * gy):
        tx, ty = t % gx, t // gx
        r0, r1 = int(rg[t, 0]), int(rg[t, 1])
        px = xs + 16 * tx
        py = ys + 16 * ty
        ncp = np.zeros((16, 16), np.int64)
        hh, ww = min(16, H - 16 * ty), min(16, W - 16 * tx)
        ncp[:hh, :ww] = nc[16 * ty:16 * ty + hh, 16 * tx:16 * tx + ww]
        tmax = int(ncp.max())
        if tmax == 0:
            continue
        base_tile += tmax * 256
        base_half += int(ncp[:8].max()) * 128 + int(ncp[8:].max()) * 128
        ids = pl[r0:r0 + tmax]
        pairs_walk += tmax
        g = xy[ids]
        c = co[ids]
        dx = g[:, 0:1, None] - px[None, None, :]          # [n,1,16]
        dy = g[:, 1:2, None] - py[None, :, None]          # [n,16,1]
        power = -0.5 * (c[:, 0, None, None] * dx * dx + c[:, 2, None, None] * dy * dy) - c[:, 1, None, None] * dx * dy
        alpha = np.minimum(0.99, c[:, 3, None, None] * np.exp(power))
        ok = (power <= 0) & (alpha >= 1.0 / 255.0)        # [n,16,16]
        band = ok.reshape(len(ids), 4, 4, 16).any(axis=(2, 3))  # [n,4]
        # a band is walked up to the last contributor of its own pixels
        bmax = ncp.reshape(4, 4, 16).max(axis=(1, 2))
        j = np.arange(len(ids))[:, None]
        live = j < bmax[None, :]
        masked += int((band & live).sum()) * 64
        live_only += int(live.sum()) * 64
        band_only += int(band.sum()) * 64
        touched_hist += np.bincount(band.sum(axis=1), minlength=5)
        hmax = np.array([ncp[:8].max(), ncp[8:].max()])
        hl = j < hmax[None, :]
        hband = np.stack([band[:, :2].any(1), band[:, 2:].any(1)], 1)
        masked_half += int((hband & hl).sum()) * 128
    print(f"view {a.view}: num_rendered {nr}, pairs walked (sum tile_max) {pairs_walk}")
    print(f"pixel-pair evaluations: whole-tile walk {base_tile/1e6:.1f}M, half-tile waves {base_half/1e6:.1f}M, "
          f"half-tile waves + half masks {masked_half/1e6:.1f}M, 4-row band masks {masked/1e6:.1f}M "
          f"(band max n_contrib alone {live_only/1e6:.1f}M, band reach alone {band_only/1e6:.1f}M)")
    print("bands touched per walked pair (0..4):", (touched_hist / touched_hist.sum()).round(3).tolist())


if __name__ == "__main__":
    main()
