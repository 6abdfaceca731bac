// launch_probe.hip — what a dependent kernel launch costs on MI355X, to settle whether the
// binning chain's ~5 us small kernels (k_rs_scan_rows, k_pair_scan_totals, k_window_starts) are
// launch-bound or bound by their own work.  Each probe launches the same kernel N times back to
// back on one stream and reports the wall time per launch (HIP events around the chain); run it
// under `rocprofv3 --kernel-trace --stats` to get the per-kernel durations the trace reports for
// the same kernels.
//
//   hipcc -O3 --offload-arch=gfx950 tools/launch_probe.hip -o tools/launch_probe && tools/launch_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__global__ void k_empty() {}

// one workgroup: one load, one store per thread (the shape of a row-scan block, minus the scan)
__global__ __launch_bounds__(256) void k_load_store(const unsigned* __restrict__ in, unsigned* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    out[i] = in[i] + 1u;
}

// k_rs_scan_rows' shape: one workgroup per digit row of `units` counts, block exclusive scan
__global__ __launch_bounds__(256) void k_row_scan(const unsigned* __restrict__ counts, unsigned* __restrict__ offs,
                                                  int units) {
    __shared__ unsigned wsum[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const unsigned* row = counts + (size_t)blockIdx.x * units;
    const unsigned v = t < units ? row[t] : 0u;
    unsigned incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = (unsigned)__shfl_up((int)incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned pre = 0;
    for (int i = 0; i < w; i++) pre += wsum[i];
    if (t < units) offs[(size_t)blockIdx.x * units + t] = pre + incl - v;
}

int main() {
    const int N = 2000;
    unsigned *a, *b;
    CK(hipMalloc(&a, 1 << 24));
    CK(hipMalloc(&b, 1 << 24));
    CK(hipMemset(a, 0, 1 << 24));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Probe {
        const char* name;
        int kind, blocks, units;
    };
    const std::vector<Probe> probes = {
        {"empty 1x64", 0, 1, 0},          {"empty 256x256", 0, 256, 0},  {"empty 2048x256", 0, 2048, 0},
        {"load+store 1x256", 1, 1, 0},    {"load+store 512x256", 1, 512, 0},
        {"row scan 512 rows x 245", 2, 512, 245}, {"row scan 256 rows x 1024", 2, 256, 256},
    };
    for (const Probe& p : probes) {
        auto launch = [&]() {
            if (p.kind == 0) k_empty<<<p.blocks, p.blocks == 1 ? 64 : 256, 0, st>>>();
            else if (p.kind == 1) k_load_store<<<p.blocks, 256, 0, st>>>(a, b);
            else k_row_scan<<<p.blocks, 256, 0, st>>>(a, b, p.units);
        };
        for (int i = 0; i < 50; i++) launch();
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < N; i++) launch();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"probe\": \"%s\", \"launches\": %d, \"us_per_launch\": %.3f}\n", p.name, N, 1000.0 * ms / N);
    }
    CK(hipFree(a));
    CK(hipFree(b));
    return 0;
}
