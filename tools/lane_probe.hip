// Probe of cross-lane primitives used by rr_blend.hip (run by tools/lane_probe.py on a GPU).
#include <hip/hip_runtime.h>
#include "rr_common.hpp"
using namespace rr;
__global__ void k_probe(const float* in, float* out) {
    const int l = threadIdx.x;
    const float x = in[l], y = in[64 + l];
    unsigned ux = __builtin_bit_cast(unsigned, x), uy = __builtin_bit_cast(unsigned, y);
    auto r = __builtin_amdgcn_permlane32_swap(ux, uy, false, false);
    unsigned r0 = r[0], r1 = r[1];
    out[l] = __builtin_bit_cast(float, r0);
    out[64 + l] = __builtin_bit_cast(float, r1);
    auto s = __builtin_amdgcn_permlane16_swap(ux, uy, false, false);
    unsigned s0 = s[0], s1 = s[1];
    out[128 + l] = __builtin_bit_cast(float, s0);
    out[192 + l] = __builtin_bit_cast(float, s1);
    out[256 + l] = row16_sum(x);
    out[320 + l] = wave_sum_lane63(x);
    float v[9];
    for (int i = 0; i < 9; i++) v[i] = in[128 + i * 64 + l];
    float t0, t1, t2;
    wave_sum9(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], t0, t1, t2);
    __shared__ float sg[9];
    if (l < 9) sg[l] = -1.f;
    __syncthreads();
    red9_store(sg, l, t0, t1, t2);
    __syncthreads();
    if (l < 9) out[384 + l] = sg[l];
}
extern "C" int probe(const float* in, float* out) {
    k_probe<<<1, 64>>>(in, out);
    return hipDeviceSynchronize();
}
