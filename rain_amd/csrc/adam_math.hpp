// adam_math.hpp — one Adam element update, shared by the standalone optimizer kernel (train.hip)
// and the backward kernel's fused step (rr_backward.hip).  Exactly torch's fused Adam
// (ATen/native/cuda/fused_adam_utils.cuh adam_math<float, float, 4, ORIGINAL, false>): the moment
// updates run in double (the betas are doubles there), the step in fp32.
#pragma once
#include <hip/hip_runtime.h>

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, double lr, float bc1, float bc2s,
                                          double b1, double b2, double eps) {
    m = (float)(b1 * (double)m + (1.0 - b1) * (double)g);
    v = (float)(b2 * (double)v + (1.0 - b2) * (double)g * (double)g);
    const float step_size = (float)(lr / (double)bc1);
    const float denom = (float)((double)(sqrtf(v) / bc2s) + eps);
    p -= step_size * m / denom;
}
