#!/usr/bin/env python3
"""How much of an HBM-bound in-place stream (the size of the f_rest Adam update: p, m, v of 45
floats per Gaussian) hides under the next frame's forward when the two run on separate streams.
Prints ms for: forward alone, stream alone, both concurrently (forward on the current stream,
the stream on a side stream started just before), and the same with the side stream at high
priority."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from rain_amd import fused, synthetic
    from rain_amd.cameras import fibonacci_cameras
    from rain_amd.gaussian_model import GaussianModel

    dev = torch.device("cuda:0")
    cams = [c.to(dev) for c in fibonacci_cameras(200, 1920, 1080)]
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(1_000_000, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    bg = torch.zeros(3, device=dev)
    cache = fused.BinningCache()
    big = torch.ones(3 * 45 * 1_000_000, device=dev)

    def fwd(i):
        fused.forward(g, cams[i % 200], bg, 0.3, cache=cache)

    def timed(fn, n=30):
        for i in range(5):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t0) / n

    out = {}
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "gpurun_variants", "libgridrmw.so"))
    lib.gridrmw.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p]
    grid = [0]

    def stream_op():
        if grid[0] == 0:
            big.mul_(1.0000001)
        else:
            s = torch.cuda.current_stream()
            lib.gridrmw(big.data_ptr(), big.numel(), grid[0], ctypes.c_void_p(s.cuda_stream))

    out["forward"] = timed(fwd)
    for gsz in (0, 64, 128, 256, 512):
      grid[0] = gsz
      out[f"g{gsz}_stream"] = timed(lambda i: stream_op())
      if gsz == 0:
        out["serial"] = timed(lambda i: (stream_op(), fwd(i)))
      for name, prio in ((f"g{gsz}_overlap", 0),):
        side = torch.cuda.Stream(priority=0)  # noqa
        main = torch.cuda.Stream(priority=prio)

        def both(i):
            with torch.cuda.stream(main):
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    stream_op()
                fwd(i)
                ev2 = torch.cuda.Event()
                ev2.record(side)
                main.wait_event(ev2)

        out[name] = timed(both)
    print({k: round(v, 4) for k, v in out.items()}, flush=True)


if __name__ == "__main__":
    main()
