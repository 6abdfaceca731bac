// Probe: the SH groups' Adam stream of k_gauss_bwd (48 floats per Gaussian, param / exp_avg /
// exp_avg_sq read and written once) in the kernel's flat, coalesced element order against a
// row-per-thread order (each lane streams its own Gaussian's 192-B rows with float4 accesses:
// 64 rows per wave instruction), which would free the kernel of its LDS row staging.
//
//   hipcc --offload-arch=gfx950 -O3 -o gpurun_variants/probe_rowwise_adam tools/probe_rowwise_adam.hip
//   gpurun_variants/probe_rowwise_adam [rows=1000000]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld(const float* p, bool nt) {
    return nt ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(p)) : *reinterpret_cast<const f4*>(p);
}
__device__ __forceinline__ void st(float* p, f4 v, bool nt) {
    if (nt)
        __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p));
    else
        *reinterpret_cast<f4*>(p) = v;
}
__device__ __forceinline__ void adam4(f4& p, f4 g, f4& m, f4& v) {
    const float w1 = 0.1f, w2 = 0.001f, b2 = 0.999f, ibc = 1.3f, eps = 1e-15f, ns = -1e-3f;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        m[i] = __builtin_fmaf(w1, g[i] - m[i], m[i]);
        v[i] = __builtin_fmaf(w2, g[i] * g[i], v[i] * b2);
        const float d = __builtin_amdgcn_sqrtf(v[i]) * ibc + eps;
        p[i] = __builtin_fmaf(ns, m[i] * __builtin_amdgcn_rcpf(d), p[i]);
    }
}

constexpr int W = 48;  // floats per row

// flat: a 256-row workgroup streams its 256 * 48 floats as float4s, lane-consecutive
template <bool NT>
__global__ __launch_bounds__(256) void k_flat(float* P, float* M, float* V, int rows) {
    const int i0 = blockIdx.x * 256;
    const int nvalid = min(256, rows - i0);
    const int nv = nvalid * W / 4;
    float* p0 = P + (size_t)i0 * W;
    float* m0 = M + (size_t)i0 * W;
    float* v0 = V + (size_t)i0 * W;
    for (int i = threadIdx.x; i < nv; i += 256) {
        f4 p = ld(p0 + 4 * i, NT), m = ld(m0 + 4 * i, NT), v = ld(v0 + 4 * i, NT);
        const f4 g = p * 1e-3f;
        adam4(p, g, m, v);
        st(p0 + 4 * i, p, NT);
        st(m0 + 4 * i, m, NT);
        st(v0 + 4 * i, v, NT);
    }
}

// rowwise: lane t streams row i0 + t, B float4s per array in flight per batch
template <bool NT, int B>
__global__ __launch_bounds__(256) void k_row(float* P, float* M, float* V, int rows) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    float* p0 = P + (size_t)r * W;
    float* m0 = M + (size_t)r * W;
    float* v0 = V + (size_t)r * W;
#pragma unroll
    for (int k0 = 0; k0 < W / 4; k0 += B) {
        f4 p[B], m[B], v[B];
#pragma unroll
        for (int b = 0; b < B; b++) {
            p[b] = ld(p0 + 4 * (k0 + b), NT);
            m[b] = ld(m0 + 4 * (k0 + b), NT);
            v[b] = ld(v0 + 4 * (k0 + b), NT);
        }
#pragma unroll
        for (int b = 0; b < B; b++) {
            const f4 g = p[b] * 1e-3f;
            adam4(p[b], g, m[b], v[b]);
            st(p0 + 4 * (k0 + b), p[b], NT);
            st(m0 + 4 * (k0 + b), m[b], NT);
            st(v0 + 4 * (k0 + b), v[b], NT);
        }
    }
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 1000000;
    const size_t n = (size_t)rows * W;
    float *P, *M, *V;
    CK(hipMalloc(&P, n * 4));
    CK(hipMalloc(&M, n * 4));
    CK(hipMalloc(&V, n * 4));
    std::vector<float> h(n);
    for (size_t i = 0; i < n; i++) h[i] = 0.001f * (float)(i % 977);
    CK(hipMemcpy(P, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(M, 0, n * 4));
    CK(hipMemset(V, 0, n * 4));
    // a 512-MB buffer swept between launches so that no launch starts from warm caches
    float* flush;
    const size_t fl = (size_t)128 << 20;
    CK(hipMalloc(&flush, fl * 4));
    const int nb = (rows + 255) / 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double bytes = 6.0 * 4.0 * (double)n;
    struct K {
        const char* name;
        void (*f)(float*, float*, float*, int);
    } ks[] = {
        {"flat_nt", k_flat<true>},      {"flat", k_flat<false>},         {"row_nt_b1", k_row<true, 1>},
        {"row_nt_b2", k_row<true, 2>},  {"row_nt_b4", k_row<true, 4>},   {"row_nt_b12", k_row<true, 12>},
        {"row_b2", k_row<false, 2>},    {"row_b4", k_row<false, 4>},
    };
    for (int rep = 0; rep < 2; rep++) {
        for (auto& k : ks) {
            float tot = 0.f;
            const int iters = 20;
            for (int it = 0; it < iters; it++) {
                CK(hipMemsetAsync(flush, it & 0xff, fl * 4, 0));
                CK(hipEventRecord(a, 0));
                k.f<<<nb, 256, 0, 0>>>(P, M, V, rows);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0.f;
                CK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
            }
            const float ms = tot / iters;
            printf("{\"kernel\": \"%s\", \"rows\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", k.name, rows, 1000.f * ms,
                   bytes / (ms * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    CK(hipGetLastError());
    return 0;
}
