// copy_probe.hip — device-to-device copy variants, 1 GiB, HIP events; picks the yardstick that
// rt_stream_copy (train.hip) implements.  hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o /tmp/copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_one(v4f* __restrict__ d, const v4f* __restrict__ s, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) d[i] = s[i];
}
__global__ __launch_bounds__(256) void k_one_nt(v4f* __restrict__ d, const v4f* __restrict__ s, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}
template <int U>
__global__ __launch_bounds__(256) void k_unroll(v4f* __restrict__ d, const v4f* __restrict__ s, long n) {
    // each block copies U*256 consecutive float4s, lane-strided (coalesced per instruction)
    const long b = (long)blockIdx.x * U * 256 + threadIdx.x;
    v4f r[U];
#pragma unroll
    for (int u = 0; u < U; u++) r[u] = (b + u * 256 < n) ? s[b + u * 256] : v4f{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; u++) if (b + u * 256 < n) d[b + u * 256] = r[u];
}
__global__ __launch_bounds__(256) void k_gs(v4f* __restrict__ d, const v4f* __restrict__ s, long n) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) d[i] = s[i];
}

int main() {
    const long bytes = 1l << 30, n = bytes / 16;
    v4f *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; i++) launch();
        hipEventRecord(e0);
        for (int i = 0; i < 20; i++) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-22s %8.1f GB/s\n", name, 2.0 * bytes / (ms / 20 * 1e-3) / 1e9);
    };
    run("one/thread", [&] { k_one<<<(n + 255) / 256, 256>>>(b, a, n); });
    run("one/thread nt", [&] { k_one_nt<<<(n + 255) / 256, 256>>>(b, a, n); });
    run("unroll4", [&] { k_unroll<4><<<(n + 1023) / 1024, 256>>>(b, a, n); });
    run("unroll8", [&] { k_unroll<8><<<(n + 2047) / 2048, 256>>>(b, a, n); });
    for (int g : {1024, 2048, 4096, 8192, 16384})
        run((std::string("gridstride ") + std::to_string(g)).c_str(), [&] { k_gs<<<g, 256>>>(b, a, n); });
    run("hipMemcpyDtoD", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice); });
    return 0;
}
