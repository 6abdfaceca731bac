#!/usr/bin/env python3
"""Owner-kernel time of the Gaussian-sharded step (rr_gauss_backward_views: every view's
per-Gaussian backward of a row block, summed, + Adam) at the bench model size for N = 1, 2, 4, 8,
on one GPU: rank 0's row block (Q = P/N rows) with N views of synthetic records, the exchange
replaced by a local echo (tests/test_sharded_gpu.py).  What an N-GPU step spends in it per rank.

    [RAIN_RASTER_LIB=variant.so] python tools/owner_bench.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Echo:
    def __init__(self, world):
        self.world = world

    def all_to_all(self, recv, send, async_op=False):
        n = send.numel() // self.world
        recv.view(self.world, n).copy_(send.view(self.world, n)[0].expand(self.world, n))
        return None


def main():
    import torch

    from rain_amd import _native, cameras, synthetic
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams
    from rain_amd.sharded import ShardedStep

    dev = torch.device("cuda:0")
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    g.set_params(synthetic.random_gaussians(1_000_000, sh_degree=3, seed=0, bench=True, device=dev))
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    g.training_setup(OptimizationParams())
    cams = [c.to(dev) for c in cameras.fibonacci_cameras(8, 1920, 1080)]
    bg = torch.zeros(3, device=dev)
    keep = [(bg, c.world_view_transform.contiguous(), c.full_proj_transform.contiguous(),
             c.camera_center.contiguous()) for c in cams]
    stats = (g.xyz_gradient_accum, g.denom, g.max_radii2D)
    out = {"lib": os.environ.get("RAIN_RASTER_LIB", "default")}
    for world in (1, 2, 4, 8):
        sh = ShardedStep(Echo(world), 0, world)
        Q, P_pad, lo, nv = sh.layout(g._xyz.shape[0])
        gen = torch.Generator(device=dev).manual_seed(world)
        R = torch.randn(P_pad, 10, generator=gen, device=dev) * 1e-3
        R[:, 9] = (torch.rand(P_pad, generator=gen, device=dev) < 0.68).float() * 3.0  # ~68 % visible
        sh.rec_chunk_rows = Q  # one owner launch (the plain record layout)
        recs = R.reshape(-1)
        for _ in range(3):
            sh.exchange_and_own(g, cams[:world], keep[:world], recs, 0.3, g.optimizer.fused_step(g), stats)
        torch.cuda.synchronize()
        _native.Profiler.collect()
        with _native.Profiler(["gauss_bwd"]):
            for _ in range(10):
                sh.exchange_and_own(g, cams[:world], keep[:world], recs, 0.3, g.optimizer.fused_step(g), stats)
        br = _native.Profiler.collect()
        ms, cnt = br["gauss_bwd"]
        # step 1 of the sharded step: the owner's rows preprocessed for each of the N views
        from rain_amd.diff_gaussian_rasterization import _C
        for _ in range(3):
            sh.preprocess_views(g, cams[:world], bg, 0.3, _C.frame_flags())
        torch.cuda.synchronize()
        _native.Profiler.collect()
        with _native.Profiler(["preprocess"]):
            for _ in range(10):
                sh.preprocess_views(g, cams[:world], bg, 0.3, _C.frame_flags())
        pms, pcnt = _native.Profiler.collect()["preprocess"]
        out[f"N{world}"] = {"Q": Q, "owner_ms": round(ms / cnt, 4), "preprocess_views_ms": round(pms / 10, 4),
                            "preprocess_launches": int(pcnt // 10)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
