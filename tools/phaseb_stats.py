#!/usr/bin/env python3
"""Early-stop binning, phase B at the bench workload (1M Gaussians, 1920x1080, SH 3): per view, the
tiles phase A left open, their phase-B list lengths and their final contributor counts (what the
phase-B blend walks sequentially per tile: the kernel's tail).

    python tools/phaseb_stats.py [--views 0,17,101]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", default="0,17,101,150")
    a = ap.parse_args()
    import numpy as np
    import torch

    from rain_amd import _native, synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.diff_gaussian_rasterization import _C

    dev = torch.device("cuda:0")
    W, H, P = 1920, 1080, 1_000_000
    params = synthetic.random_gaussians(P, sh_degree=3, seed=0, bench=True, device=dev)
    act = synthetic.activated(params)
    cams = [c.to(dev) for c in fibonacci_cameras(200, W, H)]
    L = _native.raster()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    T = gx * gy
    out = {}
    for v in [int(x) for x in a.views.split(",")]:
        s = synthetic.settings_for(cams[v], 3, torch.zeros(3, device=dev))
        e = torch.Tensor([])
        r = _C.rasterize_gaussians(s.bg, act["means3D"], e, act["opacities"], act["scales"], act["rotations"], 1.0,
                                   e, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, act["shs"], 3,
                                   s.campos, False, False, 0.3)
        torch.cuda.synchronize()
        f = _native.RRFrame(P=P, D=3, M=16, width=W, height=H, tan_fovx=s.tanfovx, tan_fovy=s.tanfovy,
                            scale_modifier=1.0, low_pass=0.3, prefiltered=0, debug=0, flags=0)
        dv = _native.RRDebugViews()
        _native.check(L.rr_debug_get_views(ctypes.byref(f), r[4].data_ptr(), r[6].data_ptr(), r[5].data_ptr(), r[0],
                                           ctypes.byref(dv)), "views")
        rg = np.zeros(4 * T, np.uint32)
        tm = np.zeros(T, np.uint32)
        hip.hipMemcpy(rg.ctypes.data, dv.ranges, 16 * T, 2)
        hip.hipMemcpy(tm.ctypes.data, dv.tile_max, 4 * T, 2)
        ra = rg[:2 * T].reshape(T, 2)
        rb = rg[2 * T:].reshape(T, 2)
        la = (ra[:, 1] - ra[:, 0]).astype(np.int64)
        lb = (rb[:, 1] - rb[:, 0]).astype(np.int64)
        opn = lb > 0
        walk_b = np.clip(tm.astype(np.int64) - la, 0, None)[opn]  # phase-B pairs actually blended
        pct = lambda x: {p: int(np.percentile(x, p)) for p in (50, 90, 99, 100)} if len(x) else {}  # noqa: E731
        out[v] = {"open_tiles": int(opn.sum()), "phase_b_pairs": int(lb.sum()), "listB": pct(lb[opn]),
                  "walkedB": pct(walk_b), "tile_max_open": pct(tm[opn].astype(np.int64)),
                  "listA_open": pct(la[opn]), "open_tiles_yx": [(int(t // gx), int(t % gx)) for t in
                                                                  np.nonzero(opn)[0][:12]]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
