"""Check the semantics of the DPP / permlane primitives the blend backward relies on."""
import ctypes, os, subprocess, sys
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "lane_probe.so")
if not os.path.exists(so):
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-I", os.path.join(HERE, "..", "rain_amd", "csrc"),
                           os.path.join(HERE, "lane_probe.hip"), "-o", so])
L = ctypes.CDLL(so)
x = torch.arange(64, dtype=torch.float32)
y = 100 + torch.arange(64, dtype=torch.float32)
v = torch.randn(9, 64)
inp = torch.cat([x, y, v.reshape(-1)]).cuda()
out = torch.zeros(400, device="cuda")
assert L.probe(ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr())) == 0
o = out.cpu()
print("swap32 r0:", o[0:64].tolist())
print("swap32 r1:", o[64:128].tolist())
print("swap16 r0:", o[128:192].tolist())
print("swap16 r1:", o[192:256].tolist())
print("row16 lanes 15,31,47,63:", o[256 + 15].item(), o[256 + 31].item(), o[256 + 47].item(), o[256 + 63].item(), "expect", [x[i*16:(i+1)*16].sum().item() for i in range(4)])
print("wave sum lane63:", o[320 + 63].item(), "expect", x.sum().item())
print("sum9:", o[384:393].tolist())
print("expect:", v.sum(1).tolist())
