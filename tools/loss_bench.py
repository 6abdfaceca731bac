#!/usr/bin/env python3
"""Times the fused L1+SSIM loss kernels (include/rain_loss.h) on a 3x1080x1920 image pair and
saves the loss value and dL/dimg, so builds of rain_amd/csrc/loss.hip can be compared for speed
and for bitwise-equal results.

    python tools/loss_bench.py --tag old --out gpurun_out
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="cur")
    ap.add_argument("--out", default="/tmp/loss_bench", help="where dL/dimg is saved (large: keep out of gpurun_out)")
    ap.add_argument("--ref", default=None, help="tag of an earlier run to compare against bitwise")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    import torch

    from rain_amd.loss import l1_ssim_backward, l1_ssim_forward

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    img = torch.rand(3, 1080, 1920, device=dev, generator=g)
    gt = (img + 0.1 * torch.randn(3, 1080, 1920, device=dev, generator=g)).clamp(0, 1)
    for _ in range(5):
        loss, _p, ws = l1_ssim_forward(img, gt, 0.2)
        dimg = l1_ssim_backward(img, gt, 0.2, ws)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(a.iters):
        e[0].record()
        loss, _p, ws = l1_ssim_forward(img, gt, 0.2)
        e[1].record()
        dimg = l1_ssim_backward(img, gt, 0.2, ws)
        e[2].record()
        e[2].synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    os.makedirs(a.out, exist_ok=True)
    torch.save({"loss": loss.cpu(), "dimg": dimg.cpu()}, os.path.join(a.out, f"loss_{a.tag}.pt"))
    res = {"tag": a.tag, "fwd_ms": tf / a.iters, "bwd_ms": tb / a.iters, "loss": float(loss)}
    if a.ref:
        ref = torch.load(os.path.join(a.out, f"loss_{a.ref}.pt"), weights_only=True)
        d = dimg.cpu()
        res.update(ref=a.ref, loss_diff=float(loss.cpu() - ref["loss"]), dimg_max_abs_diff=float((d - ref["dimg"]).abs().max()),
                   dimg_equal=bool(torch.equal(d, ref["dimg"])))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
