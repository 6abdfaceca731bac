#!/usr/bin/env python3
"""Diagnostics of the Gaussian-sharded step (rain_amd/sharded.py) on one GPU: N gloo ranks, one
ordinary iteration at a small scene; each rank prints what crossed the all-to-alls and what its
owner kernel changed, next to one process rendering the same views."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _scene(dev):
    from rain_amd import cameras, synthetic
    from rain_amd.gaussian_model import GaussianModel, OptimizationParams

    cams = [c.to(dev) for c in cameras.fibonacci_cameras(6, 160, 120)]
    gts = [torch.rand(3, 120, 160, generator=torch.Generator().manual_seed(20 + i)).to(dev) for i in range(6)]
    g = GaussianModel(3, divide_ratio=0.8, device=dev)
    p = synthetic.random_gaussians(20000, sh_degree=3, seed=6, bench=True)
    g.set_params(p)
    g.active_sh_degree = 3
    g.spatial_lr_scale = 4.4
    opt = OptimizationParams()
    g.training_setup(opt)
    return g, opt, cams, gts


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from rain_amd.train import TrainConfig, Trainer

    dev = torch.device("cuda:0")
    g, opt, cams, gts = _scene(dev)
    x0 = g._xyz.detach().clone()
    tr = Trainer(g, cams, gts, opt, cfg=TrainConfig(c2f=False, seed=5), scene_extent=4.4)
    tr.step(1001)
    torch.cuda.synchronize()
    o = tr._owner
    Q, P_pad, lo, nv = o.layout(g._xyz.shape[0])
    recs = o._bufs["recs"].view(P_pad, 10)
    recv = o._bufs["recv"].view(world, Q, 10)
    radii = o._bufs["radii"]
    print(rank, o.last, flush=True)
    from rain_amd import fused
    with torch.no_grad():
        c0, r0, d0, st0 = fused.forward(g, cams[tr._views[rank]], torch.zeros(3, device=dev), 0.3)
    print(rank, "fused fwd pairs", st0.num_rendered, "radii>0", (r0 > 0).sum().item(), flush=True)
    print(f"rank {rank}: Q {Q} lo {lo} nv {nv} radii>0 {(radii > 0).sum().item()} recs|.| {recs.abs().sum().item():.4e} "
          f"recs vis {(recs[:, 9] > 0).sum().item()} recs9 {recs[:, :9].abs().sum().item():.4e} recv9 {recv[..., :9].abs().sum().item():.4e} ws {o._bufs['ws'].view(torch.float32).abs().sum().item():.4e} recv vis {(recv[:, :, 9] > 0).sum().item()} "
          f"recv|.| {recv.abs().sum().item():.4e} accum rows {g.xyz_gradient_accum[lo:lo + nv].sum().item():.4e} "
          f"denom rows {g.denom[lo:lo + nv].sum().item()} dxyz rows {(g._xyz[lo:lo + nv] - x0[lo:lo + nv]).abs().sum().item():.4e}",
          flush=True)
    torch.distributed.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(worker, args=(world, port), nprocs=world, join=True, start_method="spawn")


if __name__ == "__main__":
    main()
