#!/usr/bin/env python3
"""Kernel time of the fused L1+SSIM loss at the bench image size (3 x 1080 x 1920), HIP events."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse

    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None, help="alternative librain_loss.so build (A/B of tile parameters)")
    args = ap.parse_args()
    if args.lib:
        from rain_amd import _native

        _native.LOSS_LIB = os.path.abspath(args.lib)

    from rain_amd.loss import l1_ssim_backward, l1_ssim_forward

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    img = torch.rand((3, 1080, 1920), device=dev, generator=g)
    gt = torch.rand((3, 1080, 1920), device=dev, generator=g)
    for _ in range(5):
        _, _, ws = l1_ssim_forward(img, gt, 0.2)
        l1_ssim_backward(img, gt, 0.2, ws)
    torch.cuda.synchronize()
    n = 50
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    for _ in range(n):
        _, _, ws = l1_ssim_forward(img, gt, 0.2)
    ev[1].record()
    for _ in range(n):
        l1_ssim_backward(img, gt, 0.2, ws)
    ev[2].record()
    torch.cuda.synchronize()
    print(json.dumps({"lib": args.lib, "forward_us": 1e3 * ev[0].elapsed_time(ev[1]) / n,
                      "backward_us": 1e3 * ev[1].elapsed_time(ev[2]) / n}))


if __name__ == "__main__":
    main()
