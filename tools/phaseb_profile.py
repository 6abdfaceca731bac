#!/usr/bin/env python3
"""Phase-B kernel time against each frame's open-tile region, at the bench workload (1M Gaussians,
1920x1080, SH 3, the bench's camera ring).  Two steps:

    rocprofv3 --kernel-trace -d gpurun_out/pbp -o run --output-format csv \\
        -- python3 tools/phaseb_profile.py run --views 64 > gpurun_out/pbp_views.jsonl
    python tools/phaseb_profile.py join gpurun_out/pbp gpurun_out/pbp_views.jsonl

`run` renders every view once (forward only) and prints, per view, the tiles phase A left open and
their bounding box; `join` pairs the views with the phase-B dispatches of the trace, in launch
order (one forward per view), and prints the per-view kernel durations.
"""
import argparse
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASE_B = {"dup_B": r"k_dup_gather<", "count": r"k_bin_count", "scatter": r"k_bin_scatter",
           "sort_B": r"k_sortexpand<.*1024>", "blend_B": r"k_blend_fwd_s<4"}


def run(a):
    import ctypes

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
    for v in range(a.views):
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
        hip.hipMemcpy(rg.ctypes.data, dv.ranges, 16 * T, 2)
        rb = rg[2 * T:].reshape(T, 2)
        opn = np.nonzero(rb[:, 1] > rb[:, 0])[0]
        rec = {"view": v, "open_tiles": int(len(opn)), "phase_b_pairs": int((rb[:, 1] - rb[:, 0]).astype(np.int64).sum())}
        if len(opn):
            ty, tx = opn // gx, opn % gx
            rec["box"] = [int(tx.min()), int(ty.min()), int(tx.max()) + 1, int(ty.max()) + 1]
        print(json.dumps(rec), flush=True)


def join(a):
    views = [json.loads(x) for x in open(a.views_jsonl) if x.startswith("{")]
    rows = []
    for fn in glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            rows += list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = {k: [] for k in PHASE_B}
    for r in rows:
        for k, pat in PHASE_B.items():
            if re.search(pat, r["Kernel_Name"]):
                per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for i, v in enumerate(views):
        v.update({k: round(per[k][i], 2) for k in PHASE_B if i < len(per[k])})
        print(json.dumps(v))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--views", type=int, default=64)
    j = sub.add_parser("join")
    j.add_argument("trace")
    j.add_argument("views_jsonl")
    a = ap.parse_args()
    run(a) if a.cmd == "run" else join(a)


if __name__ == "__main__":
    main()
