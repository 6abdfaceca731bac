// rmw_probe.hip — the access pattern of the fused Adam in k_gauss_bwd with no compute in the way:
// three fp32 arrays (param, exp_avg, exp_avg_sq) of the bench's 59M parameters, each read and
// written back in place, float4 per lane.  Prints GB/s of (read + write) bytes: the achievable
// rate for an in-place read-modify-write stream, next to a plain copy of the same byte count.
//   hipcc --offload-arch=gfx950 -O3 tools/rmw_probe.hip -o gpurun_variants/rmw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
typedef float v4f __attribute__((ext_vector_type(4)));

// one float4 of each array per lane
__global__ __launch_bounds__(256) void k_rmw1(v4f* __restrict__ p, v4f* __restrict__ m, v4f* __restrict__ v, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    v4f a = p[i], b = m[i], c = v[i];
    b = b * 0.9f + a * 0.1f;
    c = c * 0.999f + a * a * 0.001f;
    p[i] = a - b * 1e-3f;
    m[i] = b;
    v[i] = c;
}
// U float4s of each array per lane, all loads in flight before the first store
template <int U>
__global__ __launch_bounds__(256) void k_rmwU(v4f* __restrict__ p, v4f* __restrict__ m, v4f* __restrict__ v, long n) {
    const long b0 = (long)blockIdx.x * U * 256 + threadIdx.x;
    v4f a[U], b[U], c[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const long i = b0 + u * 256;
        if (i < n) {
            a[u] = p[i];
            b[u] = m[i];
            c[u] = v[i];
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const long i = b0 + u * 256;
        if (i < n) {
            b[u] = b[u] * 0.9f + a[u] * 0.1f;
            c[u] = c[u] * 0.999f + a[u] * a[u] * 0.001f;
            p[i] = a[u] - b[u] * 1e-3f;
            m[i] = b[u];
            v[i] = c[u];
        }
    }
}
// the same, p / m / v from three distinct 128-Gaussian regions per workgroup like gauss_bwd's
// f_rest stage-out (5760 floats per block, 1440 float4s, 2 float4s per lane per batch)
__global__ __launch_bounds__(128) void k_rmw_blocks(v4f* __restrict__ p, v4f* __restrict__ m, v4f* __restrict__ v,
                                                    long n) {
    const long base = (long)blockIdx.x * 1440;
    const int nv = (int)((n - base) < 1440 ? (n - base) : 1440);
    for (int v0 = threadIdx.x; v0 < nv; v0 += 256) {
        v4f a[2], b[2], c[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int i = min(v0 + q * 128, nv - 1);
            a[q] = p[base + i];
            b[q] = m[base + i];
            c[q] = v[base + i];
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int i = v0 + q * 128;
            if (i >= nv) break;
            b[q] = b[q] * 0.9f + a[q] * 0.1f;
            c[q] = c[q] * 0.999f + a[q] * a[q] * 0.001f;
            p[base + i] = a[q] - b[q] * 1e-3f;
            m[base + i] = b[q];
            v[base + i] = c[q];
        }
    }
}
// out of place: read (p, m, v), write (p2, m2, v2) — ping-pong Adam state
template <bool NT>
__global__ __launch_bounds__(256) void k_pingpong(const v4f* __restrict__ p, const v4f* __restrict__ m,
                                                  const v4f* __restrict__ v, v4f* __restrict__ p2,
                                                  v4f* __restrict__ m2, v4f* __restrict__ v2, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    v4f a = p[i], b = m[i], c = v[i];
    b = b * 0.9f + a * 0.1f;
    c = c * 0.999f + a * a * 0.001f;
    a = a - b * 1e-3f;
    if (NT) {
        __builtin_nontemporal_store(a, p2 + i);
        __builtin_nontemporal_store(b, m2 + i);
        __builtin_nontemporal_store(c, v2 + i);
    } else {
        p2[i] = a;
        m2[i] = b;
        v2[i] = c;
    }
}
// in place with non-temporal stores
__global__ __launch_bounds__(256) void k_rmw_nt(v4f* __restrict__ p, v4f* __restrict__ m, v4f* __restrict__ v, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    v4f a = p[i], b = m[i], c = v[i];
    b = b * 0.9f + a * 0.1f;
    c = c * 0.999f + a * a * 0.001f;
    __builtin_nontemporal_store(a - b * 1e-3f, p + i);
    __builtin_nontemporal_store(b, m + i);
    __builtin_nontemporal_store(c, v + i);
}
// in place, the three arrays interleaved per 64-float4 chunk (one wave's 1 KiB of p, then m, then v):
// one address front instead of three
__global__ __launch_bounds__(256) void k_rmw_inter(v4f* __restrict__ s, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long c = i >> 6, l = i & 63;
    v4f* q = s + c * 192 + l;
    v4f a = q[0], b = q[64], d = q[128];
    b = b * 0.9f + a * 0.1f;
    d = d * 0.999f + a * a * 0.001f;
    q[0] = a - b * 1e-3f;
    q[64] = b;
    q[128] = d;
}
// in place, p separate, (m, v) interleaved per 64-float4 chunk: two fronts
__global__ __launch_bounds__(256) void k_rmw_mv(v4f* __restrict__ p, v4f* __restrict__ s, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long c = i >> 6, l = i & 63;
    v4f* q = s + c * 128 + l;
    v4f a = p[i], b = q[0], d = q[64];
    b = b * 0.9f + a * 0.1f;
    d = d * 0.999f + a * a * 0.001f;
    p[i] = a - b * 1e-3f;
    q[0] = b;
    q[64] = d;
}
// ping-pong with p|m|v interleaved per 64-float4 chunk in both buffers: one read front, one write
// front (the copy's pattern) instead of six
__global__ __launch_bounds__(256) void k_pingpong_inter(const v4f* __restrict__ s, v4f* __restrict__ d, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long c = i >> 6, l = i & 63;
    const v4f* q = s + c * 192 + l;
    v4f* o = d + c * 192 + l;
    v4f a = q[0], b = q[64], e = q[128];
    b = b * 0.9f + a * 0.1f;
    e = e * 0.999f + a * a * 0.001f;
    o[0] = a - b * 1e-3f;
    o[64] = b;
    o[128] = e;
}
__global__ __launch_bounds__(256) void k_copy3(v4f* __restrict__ d, const v4f* __restrict__ s, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

int main() {
    const long floats = 59l * 1000000, n = floats / 4, bytes = floats * 4;
    v4f *p, *d;  // p: the three arrays back to back (the copy reads all of it)
    hipMalloc(&p, 3 * bytes);
    hipMalloc(&d, 3 * bytes);
    hipMemset(p, 0, 3 * bytes);
    hipMemset(d, 0, 3 * bytes);
    v4f *m = p + n, *v = p + 2 * n;
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
        printf("%-26s %7.3f ms %8.1f GB/s\n", name, ms / 20, 6.0 * bytes / (ms / 20 * 1e-3) / 1e9);
    };
    run("rmw 1 float4/lane", [&] { k_rmw1<<<(n + 255) / 256, 256>>>(p, m, v, n); });
    run("rmw 2 float4/lane", [&] { k_rmwU<2><<<(n + 511) / 512, 256>>>(p, m, v, n); });
    run("rmw 4 float4/lane", [&] { k_rmwU<4><<<(n + 1023) / 1024, 256>>>(p, m, v, n); });
    run("rmw 128-Gaussian blocks", [&] { k_rmw_blocks<<<(n + 1439) / 1440, 128>>>(p, m, v, n); });
    run("rmw in place, nt stores", [&] { k_rmw_nt<<<(n + 255) / 256, 256>>>(p, m, v, n); });
    run("ping-pong", [&] { k_pingpong<false><<<(n + 255) / 256, 256>>>(p, m, v, d, d + n, d + 2 * n, n); });
    run("ping-pong nt stores", [&] { k_pingpong<true><<<(n + 255) / 256, 256>>>(p, m, v, d, d + n, d + 2 * n, n); });
    run("ping-pong alternating", [&] {
        static int k = 0;
        v4f* a = (k & 1) ? d : p;
        v4f* b = (k & 1) ? p : d;
        k++;
        k_pingpong<false><<<(n + 255) / 256, 256>>>(a, a + n, a + 2 * n, b, b + n, b + 2 * n, n);
    });
    run("rmw interleaved p|m|v", [&] { k_rmw_inter<<<(n + 255) / 256, 256>>>(p, n); });
    run("rmw p + interleaved m|v", [&] { k_rmw_mv<<<(n + 255) / 256, 256>>>(p, p + n, n); });
    run("ping-pong interleaved", [&] { k_pingpong_inter<<<(n + 255) / 256, 256>>>(p, d, n); });
    run("ping-pong interleaved alt", [&] {
        static int k = 0;
        v4f* a = (k & 1) ? d : p;
        v4f* b = (k & 1) ? p : d;
        k++;
        k_pingpong_inter<<<(n + 255) / 256, 256>>>(a, b, n);
    });
    run("copy nt (same bytes)", [&] { k_copy3<<<(3 * n + 255) / 256, 256>>>(d, p, 3 * n); });
    return 0;
}
