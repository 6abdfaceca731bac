// valu_probe.hip — VALU throughput per instruction kind on gfx950 (cycles per wave-instruction per
// SIMD at full occupancy), to price the blend kernels' op mix.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x + i;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = __builtin_fmaf(x[i], a, b);
    float s = 0;
    for (int i = 0; i < 8; i++) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pkfma(float* out, float a, float b) {
    f2 x[8];
    for (int i = 0; i < 8; i++) x[i] = f2{(float)threadIdx.x + i, (float)i};
    const f2 A{a, a}, Bv{b, b};
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = __builtin_elementwise_fma(x[i], A, Bv);
    float s = 0;
    for (int i = 0; i < 8; i++) s += x[i].x + x[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_exp(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; i++) x[i] = (threadIdx.x + i) * 1e-3f;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = __builtin_amdgcn_exp2f(x[i]) * -1e-3f;  // exp + mul
    float s = 0;
    for (int i = 0; i < 8; i++) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mul(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; i++) x[i] = (threadIdx.x + i) * 1e-3f;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = x[i] * -1.0001f;  // mul only (the exp kernel's partner)
    float s = 0;
    for (int i = 0; i < 8; i++) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_sel(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; i++) x[i] = (threadIdx.x + i) * 1e-3f;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = x[i] < a ? x[i] + b : x[i] - b;  // cmp + add + sub + cndmask
    float s = 0;
    for (int i = 0; i < 8; i++) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    float* out;
    hipMalloc(&out, 1 << 26);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8;  // 8 waves/SIMD worth of 4-wave blocks
    auto run = [&](const char* name, void (*k)(float*, float, float), double ops_per_iter) {
        k<<<blocks, 256>>>(out, 1.0001f, 1e-7f);
        hipEventRecord(e0);
        k<<<blocks, 256>>>(out, 1.0001f, 1e-7f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double winst_per_simd = (double)blocks * 4 * ITERS * ops_per_iter / 1024.0;
        printf("%-8s %7.3f ms  %6.2f ns per 64-lane op per SIMD  (%5.2f cyc @2.4GHz)\n", name, ms,
               ms * 1e6 / winst_per_simd, ms * 1e6 / winst_per_simd * 2.4);
    };
    run("fma", k_fma, 8);
    run("pk_fma", k_pkfma, 8);
    run("mul", k_mul, 8);
    run("exp+mul", k_exp, 16);
    run("sel4", k_sel, 32);
    return 0;
}
