#!/usr/bin/env python3
"""Compare forward-blend implementations (rr_set_tuning "fwd_impl") bitwise on one scene: image,
depth, final_T, n_contrib, tile_max; prints where they first differ.

    python tools/fwd_check.py --impls 0,2 [--points 3000 --width 128 --height 96]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", default="0,2")
    ap.add_argument("--points", type=int, default=3000)
    ap.add_argument("--width", type=int, default=128)
    ap.add_argument("--height", type=int, default=96)
    ap.add_argument("--knob", default="fwd_impl")
    a = ap.parse_args()
    import numpy as np
    import torch

    from rain_amd import _native
    from tests.common import gpu_run, make_scene

    dev = torch.device("cuda:0")
    L = _native.raster()
    inp, st = make_scene(P=a.points, W=a.width, H=a.height, sh_degree=3)

    outs = {}
    for v in [int(x) for x in a.impls.split(",")]:
        _native.check(L.rr_set_tuning(a.knob.encode(), v), "tuning")
        got = gpu_run(inp, st, dev)
        geom, binning, img = got["buffers"]
        H, W = a.height, a.width
        f = _native.RRFrame(P=a.points, D=3, M=16, width=W, height=H, tan_fovx=st["tanfovx"], tan_fovy=st["tanfovy"],
                            scale_modifier=1.0, low_pass=0.3, prefiltered=0, debug=0, flags=0)
        dv = _native.RRDebugViews()
        _native.check(L.rr_debug_get_views(ctypes.byref(f), geom.data_ptr(), img.data_ptr(), binning.data_ptr(),
                                           got["num_rendered"], ctypes.byref(dv)), "views")
        T = ((W + 15) // 16) * ((H + 15) // 16)
        torch.cuda.synchronize()

        final_T = torch.as_tensor(np.zeros(H * W, np.float32))
        n_contrib = torch.as_tensor(np.zeros(H * W, np.int32))
        tile_max = torch.as_tensor(np.zeros(T, np.int32))
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        for dst, src, nb in ((final_T, dv.final_T, H * W * 4), (n_contrib, dv.n_contrib, H * W * 4),
                             (tile_max, dv.tile_max, T * 4)):
            hip.hipMemcpy(dst.data_ptr(), src, nb, 2)
        outs[v] = dict(color=got["color"], depth=got["depth"], final_T=final_T.numpy().reshape(H, W),
                       n_contrib=n_contrib.numpy().reshape(H, W), tile_max=tile_max.numpy())
    _native.check(L.rr_set_tuning(a.knob.encode(), 2 if a.knob == "fwd_impl" else 0), "tuning")
    keys = list(outs)
    base = outs[keys[0]]
    for v in keys[1:]:
        o = outs[v]
        for k in base:
            x, y = base[k], o[k]
            eq = np.array_equal(x, y)
            msg = f"{a.knob}={v} vs {keys[0]}: {k:9s} bitwise_equal={eq}"
            if not eq:
                d = np.argwhere(x != y)
                msg += f" ndiff={len(d)} first={d[:3].tolist()} base={x[tuple(d[0])]} got={y[tuple(d[0])]}"
            print(msg)


if __name__ == "__main__":
    main()
