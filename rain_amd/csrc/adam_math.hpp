// adam_math.hpp — one Adam element update, shared by the standalone optimizer kernel (train.hip)
// and the backward kernel's fused step (rr_backward.hip).
//
// The reference's optimizer is `torch.optim.Adam(l, lr=0.0, eps=1e-15)` (gaussian_model.py:153)
// with torch's defaults, i.e. the multi-tensor (foreach) implementation on GPU tensors
// (torch/optim/adam.py _multi_tensor_adam), which computes in fp32 for fp32 tensors:
//   exp_avg.lerp_(grad, 1 - beta1)                         m += (1 - b1) (g - m)
//   exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)  v = b2 v + (1 - b2) g g
//   denom = exp_avg_sq.sqrt() / bias_correction2_sqrt + eps
//   param.addcdiv_(exp_avg, denom, value=-lr / bias_correction1)
// Restated here in that order in fp32.  The two divisions use the hardware reciprocal (<= 1 ulp
// from torch's IEEE division; the per-element update stays within 1e-6 of torch's, tests/
// test_fused_gpu.py) — about 13 VALU slots per element instead of the ~40 of a double-precision
// moment update with two IEEE divisions.
#pragma once
#include <hip/hip_runtime.h>

// a * b rounded to fp32 (no fma contraction with what consumes it): the sharded step's in-kernel
// gradient scaling must equal torch's separate grad.mul_(scale) bitwise
__device__ __forceinline__ float mul_rounded(float a, float b) {
#pragma clang fp contract(off)
    return a * b;
}

// Per-group constants, formed once per group (not per element).
struct AdamC {
    float w1;        // 1 - beta1 (lerp weight)
    float b2, w2;    // beta2, 1 - beta2
    float inv_bc2s;  // 1 / sqrt(1 - beta2^t)
    float eps;
    float nstep;     // -lr / (1 - beta1^t)
};

__device__ __forceinline__ AdamC adam_consts(double lr, float bc1, float bc2s, double b1, double b2, double eps) {
    AdamC c;
    c.w1 = (float)(1.0 - b1);
    c.b2 = (float)b2;
    c.w2 = (float)(1.0 - b2);
    c.inv_bc2s = 1.0f / bc2s;
    c.eps = (float)eps;
    c.nstep = (float)(-lr / (double)bc1);
    return c;
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamC& c) {
    m = __builtin_fmaf(c.w1, g - m, m);                                        // lerp (weight < 0.5 branch)
    // mul_ then addcmul_: torch's foreach addcmul computes a + value * (b * c), so g * g is
    // rounded on its own before the (contracted) multiply-add
    v = __builtin_fmaf(c.w2, mul_rounded(g, g), v * c.b2);
    const float denom = __builtin_amdgcn_sqrtf(v) * c.inv_bc2s + c.eps;        // sqrt / bc2s + eps
    p = __builtin_fmaf(c.nstep, m * __builtin_amdgcn_rcpf(denom), p);          // addcdiv_
}
