// knn.hip — exact 3-nearest-neighbour mean squared distance (include/rain_knn.h), the MI355X
// replacement of simple-knn's distCUDA2 (submodules/simple-knn/simple_knn.cu:164-207).
//
// Same decomposition as the reference — bbox (origin included), 30-bit Morton codes, stable
// radix sort, boxes of 1024 consecutive sorted points with their AABBs, box-pruned exhaustive
// scan — laid out for CDNA4:
//   * the bbox stays on the device (the reference copies min/max to the host twice);
//   * points are gathered once into Morton order as float4 (16-B coalesced loads afterwards);
//   * k_knn runs one workgroup (4 wave64s) per 256 consecutive sorted points, which are spatially
//     coherent: the workgroup walks the box list in lock-step, a box is staged into LDS only if
//     some lane still needs it (__syncthreads_or), and every lane then reads the staged points
//     as LDS broadcasts — instead of every thread gathering points[indices[i]] from HBM.
// Distances use the reference's expression with FMA contraction off (bitwise equal to the oracle).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <string>

#include "../../include/rain_knn.h"

namespace {

// Onesweep radix sort at every size (rocPRIM's default merge-sorts below 2^20 items)
using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                rocprim::default_config, 0>;

thread_local std::string g_err;
int fail(const std::string& m) {
    g_err = m;
    return 1;
}

constexpr int kBox = 1024;       // BOX_SIZE (simple_knn.cu:1)
constexpr int kThreads = 256;
constexpr int kBBoxBlocks = 256;

struct Box {
    float4 mn, mx;
};

__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

// float -> u32 with CUDA cvt.rzi.u32.f32 semantics (truncate; NaN / negative -> 0; saturate)
__device__ __forceinline__ uint32_t f2u(float v) {
    if (!(v > 0.0f)) return 0u;
    if (v >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)v;
}

__device__ __forceinline__ float sqdist(float4 a, float4 b) {
#pragma clang fp contract(off)
    const float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
    return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ void update3(float4 ref, float4 pt, float& b0, float& b1, float& b2) {
    float d = sqdist(ref, pt);
    if (b0 > d) { const float t = b0; b0 = d; d = t; }
    if (b1 > d) { const float t = b1; b1 = d; d = t; }
    if (b2 > d) { b2 = d; }
}

__device__ __forceinline__ float box_dist(const Box& B, float4 p) {
#pragma clang fp contract(off)
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (p.x < B.mn.x || p.x > B.mx.x) dx = fminf(fabsf(p.x - B.mn.x), fabsf(p.x - B.mx.x));
    if (p.y < B.mn.y || p.y > B.mx.y) dy = fminf(fabsf(p.y - B.mn.y), fabsf(p.y - B.mx.y));
    if (p.z < B.mn.z || p.z > B.mx.z) dz = fminf(fabsf(p.z - B.mn.z), fabsf(p.z - B.mx.z));
    return dx * dx + dy * dy + dz * dz;
}

// block min/max over float3 values (256 threads)
__device__ __forceinline__ void block_minmax(float3& mn, float3& mx) {
    __shared__ float s[6][kThreads];
    const int t = threadIdx.x;
    s[0][t] = mn.x; s[1][t] = mn.y; s[2][t] = mn.z;
    s[3][t] = mx.x; s[4][t] = mx.y; s[5][t] = mx.z;
    __syncthreads();
    for (int off = kThreads / 2; off > 0; off >>= 1) {
        if (t < off) {
            for (int a = 0; a < 3; a++) s[a][t] = fminf(s[a][t], s[a][t + off]);
            for (int a = 3; a < 6; a++) s[a][t] = fmaxf(s[a][t], s[a][t + off]);
        }
        __syncthreads();
    }
    mn = make_float3(s[0][0], s[1][0], s[2][0]);
    mx = make_float3(s[3][0], s[4][0], s[5][0]);
    __syncthreads();
}

__global__ __launch_bounds__(kThreads) void k_bbox_partial(int P, const float* __restrict__ pts, Box* __restrict__ part) {
    float3 mn = make_float3(FLT_MAX, FLT_MAX, FLT_MAX), mx = make_float3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = blockIdx.x * kThreads + threadIdx.x; i < P; i += gridDim.x * kThreads) {
        const float x = pts[3 * (size_t)i], y = pts[3 * (size_t)i + 1], z = pts[3 * (size_t)i + 2];
        mn = make_float3(fminf(mn.x, x), fminf(mn.y, y), fminf(mn.z, z));
        mx = make_float3(fmaxf(mx.x, x), fmaxf(mx.y, y), fmaxf(mx.z, z));
    }
    block_minmax(mn, mx);
    if (threadIdx.x == 0) part[blockIdx.x] = Box{make_float4(mn.x, mn.y, mn.z, 0.f), make_float4(mx.x, mx.y, mx.z, 0.f)};
}

// final reduce, with the reference's init value {0,0,0} folded in (simple_knn.cu:172)
__global__ __launch_bounds__(kThreads) void k_bbox_final(int n, const Box* __restrict__ part, Box* __restrict__ out) {
    float3 mn = make_float3(0.f, 0.f, 0.f), mx = make_float3(0.f, 0.f, 0.f);
    for (int i = threadIdx.x; i < n; i += kThreads) {
        const Box b = part[i];
        mn = make_float3(fminf(mn.x, b.mn.x), fminf(mn.y, b.mn.y), fminf(mn.z, b.mn.z));
        mx = make_float3(fmaxf(mx.x, b.mx.x), fmaxf(mx.y, b.mx.y), fmaxf(mx.z, b.mx.z));
    }
    block_minmax(mn, mx);
    if (threadIdx.x == 0) *out = Box{make_float4(mn.x, mn.y, mn.z, 0.f), make_float4(mx.x, mx.y, mx.z, 0.f)};
}

// coord2Morton (simple_knn.cu:44-62); the bbox is read from device memory
__global__ __launch_bounds__(kThreads) void k_morton(int P, const float* __restrict__ pts, const Box* __restrict__ bb,
                                                     uint32_t* __restrict__ codes) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= P) return;
    const Box b = *bb;
    const float c[3] = {pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2]};
    const float mn[3] = {b.mn.x, b.mn.y, b.mn.z}, mx[3] = {b.mx.x, b.mx.y, b.mx.z};
    uint32_t m[3];
#pragma unroll
    for (int a = 0; a < 3; a++) m[a] = prep_morton(f2u(((c[a] - mn[a]) / (mx[a] - mn[a])) * (float)((1 << 10) - 1)));
    codes[i] = m[0] | (m[1] << 1) | (m[2] << 2);
}

__global__ __launch_bounds__(kThreads) void k_gather(int P, const float* __restrict__ pts,
                                                     const uint32_t* __restrict__ idx, float4* __restrict__ sorted) {
    const int s = blockIdx.x * kThreads + threadIdx.x;
    if (s >= P) return;
    const size_t i = idx[s];
    sorted[s] = make_float4(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], 0.f);
}

// boxMinMax (simple_knn.cu:64-100): one workgroup per box of 1024 sorted points
__global__ __launch_bounds__(kThreads) void k_boxes(int P, const float4* __restrict__ sorted, Box* __restrict__ boxes) {
    float3 mn = make_float3(FLT_MAX, FLT_MAX, FLT_MAX), mx = make_float3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    const int base = blockIdx.x * kBox;
    for (int k = threadIdx.x; k < kBox; k += kThreads) {
        const int s = base + k;
        if (s < P) {
            const float4 p = sorted[s];
            mn = make_float3(fminf(mn.x, p.x), fminf(mn.y, p.y), fminf(mn.z, p.z));
            mx = make_float3(fmaxf(mx.x, p.x), fmaxf(mx.y, p.y), fmaxf(mx.z, p.z));
        }
    }
    block_minmax(mn, mx);
    if (threadIdx.x == 0) boxes[blockIdx.x] = Box{make_float4(mn.x, mn.y, mn.z, 0.f), make_float4(mx.x, mx.y, mx.z, 0.f)};
}

// boxMeanDist (simple_knn.cu:125-157), workgroup-cooperative
__global__ __launch_bounds__(kThreads) void k_knn(int P, int nb, const float4* __restrict__ sorted,
                                                  const uint32_t* __restrict__ idx, const Box* __restrict__ boxes,
                                                  float* __restrict__ out) {
    __shared__ float4 tile[kBox];
    const int s = blockIdx.x * kThreads + threadIdx.x;
    const bool valid = s < P;
    const float4 pt = valid ? sorted[s] : make_float4(0.f, 0.f, 0.f, 0.f);
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    if (valid) {
        const int lo = max(0, s - 3), hi = min(P - 1, s + 3);
        for (int i = lo; i <= hi; i++)
            if (i != s) update3(pt, sorted[i], b0, b1, b2);
    }
    const float reject = b2;
    b0 = b1 = b2 = FLT_MAX;
    for (int b = 0; b < nb; b++) {
        const Box B = boxes[b];
        bool need = false;
        if (valid) {
            const float d = box_dist(B, pt);
            need = !(d > reject || d > b2);
        }
        if (!__syncthreads_or(need)) continue;
        const int base = b * kBox;
        const int n = min(kBox, P - base);
        for (int k = threadIdx.x; k < n; k += kThreads) tile[k] = sorted[base + k];
        __syncthreads();
        if (need) {
            const int self = s - base;
            for (int k = 0; k < n; k++)
                if (k != self) update3(pt, tile[k], b0, b1, b2);
        }
        __syncthreads();
    }
    if (valid) out[idx[s]] = (b0 + b1 + b2) / 3.0f;
}

struct Carve {
    char* p;
    size_t off = 0;
    explicit Carve(void* b) : p(static_cast<char*>(b)) {}
    template <typename T>
    T* take(size_t n) {
        off = (off + 255) & ~size_t(255);
        T* r = p ? reinterpret_cast<T*>(p + off) : nullptr;
        off += n * sizeof(T);
        return r;
    }
};

struct Ws {
    Box* part;
    Box* bbox;
    uint32_t* codes;
    uint32_t* codes_sorted;
    uint32_t* idx;
    float4* sorted;
    Box* boxes;
    void* temp;
    size_t temp_bytes;
    size_t total;
};

Ws carve(void* buf, int P) {
    Carve c(buf);
    Ws w;
    const size_t n = (size_t)(P > 0 ? P : 1);
    const int nb = (P + kBox - 1) / kBox;
    w.part = c.take<Box>(kBBoxBlocks);
    w.bbox = c.take<Box>(1);
    w.codes = c.take<uint32_t>(n);
    w.codes_sorted = c.take<uint32_t>(n);
    w.idx = c.take<uint32_t>(n);
    w.sorted = c.take<float4>(n);
    w.boxes = c.take<Box>((size_t)(nb > 0 ? nb : 1));
    w.temp_bytes = 0;
    if (P > 0)
        (void)rocprim::radix_sort_pairs<OnesweepSort>(nullptr, w.temp_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                        rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr, (size_t)P, 0, 30,
                                        (hipStream_t)0);
    w.temp = c.take<char>(w.temp_bytes > 0 ? w.temp_bytes : 1);
    w.total = (c.off + 255) & ~size_t(255);
    return w;
}

}  // namespace

extern "C" {

const char* sk_last_error(void) { return g_err.c_str(); }

size_t sk_workspace_bytes(int P) { return carve(nullptr, P < 0 ? 0 : P).total; }

int sk_dist_cuda2(int P, const float* points, float* mean_dists, void* workspace, size_t workspace_bytes,
                  void* stream) {
    if (P < 0) return fail("P must be >= 0");
    if (P == 0) return 0;
    if (!points || !mean_dists || !workspace) return fail("null pointer");
    Ws w = carve(workspace, P);
    if (workspace_bytes < w.total) return fail("workspace smaller than sk_workspace_bytes(P)");
    hipStream_t st = (hipStream_t)stream;
    const int nblk = (P + kThreads - 1) / kThreads;
    const int nb = (P + kBox - 1) / kBox;
    const int npart = std::min(kBBoxBlocks, nblk);
    k_bbox_partial<<<npart, kThreads, 0, st>>>(P, points, w.part);
    k_bbox_final<<<1, kThreads, 0, st>>>(npart, w.part, w.bbox);
    k_morton<<<nblk, kThreads, 0, st>>>(P, points, w.bbox, w.codes);
    size_t tb = w.temp_bytes;
    if (rocprim::radix_sort_pairs<OnesweepSort>(w.temp, tb, w.codes, w.codes_sorted, rocprim::counting_iterator<uint32_t>(0), w.idx,
                                  (size_t)P, 0, 30, st) != hipSuccess)
        return fail("morton sort failed");
    k_gather<<<nblk, kThreads, 0, st>>>(P, points, w.idx, w.sorted);
    k_boxes<<<nb, kThreads, 0, st>>>(P, w.sorted, w.boxes);
    k_knn<<<nblk, kThreads, 0, st>>>(P, nb, w.sorted, w.idx, w.boxes, mean_dists);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(std::string("knn launch: ") + hipGetErrorString(e));
    return 0;
}

}  // extern "C"
