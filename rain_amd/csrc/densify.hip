// densify.hip — densify / clone / split / prune as stream compaction (include/rain_train.h
// rt_densify_*; gaussian_model.py:339-415, train.py:136-140).
//
// The reference densifies with a chain of boolean-mask gathers and torch.cat over 6 parameters and
// their 12 Adam moment tensors (clone: cat; split: gather, bmm, cat, then a prune; final prune:
// gather), i.e. several full passes over ~0.7 KB per Gaussian plus a host sync per masked index.
// Here:
//   k_densify_classify  one thread per Gaussian: clone / split / abe / prune decisions -> 5 flag bits
//   rocPRIM scan        exclusive scan of the 5 flags -> every survivor's output row
//   k_densify_apply     one pass over every group's (param, exp_avg, exp_avg_sq) elements, each
//                       element written straight to its rows in the new set (original / clone /
//                       abe copies / n_split children); coalesced reads, contiguous runs of writes.
// One host sync (the counts, to size the outputs and draw the split samples).
//
// Arithmetic is written as torch evaluates the reference's expressions (one rounding per op: fp
// contraction off) — division by a Python scalar as a multiplication by its float reciprocal (as
// ATen does; checked on the device), build_rotation (general_utils.py:52-73) op by op — so
// survivors, clones and the children's other parameters are bitwise those of the torch path; the
// children's xyz differ by the rounding of the reference's 3x3 bmm (a BLAS batched GEMM there, a
// fixed fma order here) and their log-scales by up to an ulp of expf/logf (the device library here,
// ATen's kernels there).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/rain_train.h"

namespace rt_internal {
void set_error(const std::string& m);  // train.hip: the message rt_last_error() returns
}

namespace {

int fail(const std::string& m) {
    rt_internal::set_error(m);
    return 1;
}

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// flag bits per Gaussian
constexpr unsigned kKeepOrig = 1u, kKeepClone = 2u, kKeepChildren = 4u, kSplit = 8u, kKeepAbe = 16u;

// the five ranks of a Gaussian: {orig, clone, children, split, abe copies}
struct Rank5 {
    uint32_t o, c, ch, s, ab;
};
struct Flags5 {
    __host__ __device__ Rank5 operator()(uint8_t f) const {
        return Rank5{f & 1u, (f >> 1) & 1u, (f >> 2) & 1u, (f >> 3) & 1u, (f >> 4) & 1u};
    }
};
struct Add5 {
    __host__ __device__ Rank5 operator()(const Rank5& a, const Rank5& b) const {
        return Rank5{a.o + b.o, a.c + b.c, a.ch + b.ch, a.s + b.s, a.ab + b.ab};
    }
};
using FlagIt = rocprim::transform_iterator<const uint8_t*, Flags5, Rank5>;

struct Workspace {
    uint8_t* flags;
    Rank5* offsets;  // exclusive scan of the flag bits
    Rank5* totals;   // [1]
    void* temp;
    size_t temp_bytes;
    size_t total;
};
size_t scan_temp_bytes(int P) {
    size_t b = 0;
    if (P > 0)
        (void)rocprim::exclusive_scan(nullptr, b, FlagIt((const uint8_t*)nullptr, Flags5()), (Rank5*)nullptr,
                                      Rank5{0u, 0u, 0u, 0u, 0u}, (size_t)P, Add5(), (hipStream_t)0);
    return b;
}
Workspace carve(void* base, int P) {
    char* b = static_cast<char*>(base);
    Workspace w;
    size_t off = 0;
    const size_t n = (size_t)(P > 0 ? P : 1);
    auto take = [&](size_t bytes) {
        off = align_up(off);
        char* p = b ? b + off : nullptr;
        off += bytes;
        return p;
    };
    w.flags = reinterpret_cast<uint8_t*>(take(n));
    w.offsets = reinterpret_cast<Rank5*>(take(n * sizeof(Rank5)));
    w.totals = reinterpret_cast<Rank5*>(take(sizeof(Rank5)));
    w.temp_bytes = scan_temp_bytes(P);
    w.temp = take(w.temp_bytes > 0 ? w.temp_bytes : 1);
    w.total = align_up(off);
    return w;
}

// torch.max(get_scaling, dim=1).values: exp per element, then the max
__device__ __forceinline__ float max_exp3(float a, float b, float c) {
    return fmaxf(fmaxf(expf(a), expf(b)), expf(c));
}

__global__ __launch_bounds__(256) void k_densify_classify(rt_densify_params p, float inv_div,
                                                          const float* __restrict__ accum,
                                                          const float* __restrict__ denom,
                                                          const float* __restrict__ scaling,
                                                          const float* __restrict__ opacity,
                                                          uint8_t* __restrict__ flags) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.P) return;
    float g = accum[i] / denom[i];  // grads = accum / denom; grads[grads.isnan()] = 0
    if (g != g) g = 0.f;
    const float s0 = scaling[3 * i], s1 = scaling[3 * i + 1], s2 = scaling[3 * i + 2];
    const float smax = max_exp3(s0, s1, s2);
    const bool clone = sqrtf(g * g) >= p.grad_threshold && smax <= p.clone_split_scale;  // torch.norm(dim=-1)
    const bool split = g >= p.grad_threshold && smax > p.clone_split_scale;
    const float op = 1.0f / (1.0f + expf(-opacity[i]));  // sigmoid
    const bool low = op < p.min_opacity;
    const bool prune = low || (p.prune_big_world && smax > p.big_world_scale);
    // children: scaling = log(exp(s) / (divide_ratio * N)), pruned on the exp of that
    const float c0 = logf(expf(s0) * inv_div), c1 = logf(expf(s1) * inv_div), c2 = logf(expf(s2) * inv_div);
    const bool prune_child = low || (p.prune_big_world && max_exp3(c0, c1, c2) > p.big_world_scale);
    unsigned f = 0;
    if (!split && !prune) f |= kKeepOrig;
    if (clone && !prune) f |= kKeepClone;
    if (split && !prune_child) f |= kKeepChildren;
    if (split) f |= kSplit;
    if (split && p.abe_split && p.n_split > 1) {  // abe copies: scaling log(exp(s)), pruned on its exp
        const float a0 = logf(expf(s0)), a1 = logf(expf(s1)), a2 = logf(expf(s2));
        if (!(low || (p.prune_big_world && max_exp3(a0, a1, a2) > p.big_world_scale))) f |= kKeepAbe;
    }
    flags[i] = (uint8_t)f;
}

__global__ void k_totals(int P, const uint8_t* __restrict__ flags, const Rank5* __restrict__ offsets,
                         Rank5* __restrict__ totals) {
    *totals = Add5()(offsets[P - 1], Flags5()(flags[P - 1]));
}

constexpr int kMaxGroups = 8;
struct ApplyGroup {
    const float* p;
    const float* m;
    const float* v;
    float* op;
    float* om;
    float* ov;
    int width;
    int kind;
    int64_t n;       // P * width
    int64_t block0;  // first block of this group
};
struct ApplyArgs {
    ApplyGroup grp[kMaxGroups];
    int n_groups;
    int n_split;
    uint32_t A, B, C, S, E;  // counts
    float inv_div;           // 1 / (divide_ratio * N) in fp32
    float abe0, abe1;        // an abe copy's xyz = (xyz * abe0) * abe1
    const uint8_t* flags;
    const Rank5* offsets;
    const float* scaling;
    const float* rotation;
    const float* normals;  // [n_split * S, 3]
};

constexpr int kApplyThreads = 256;

// build_rotation (general_utils.py:52-73): row r of R(q / |q|), op by op as torch evaluates it
__device__ __forceinline__ void rot_row(const float* q4, int r, float& a, float& b, float& c) {
#pragma clang fp contract(off)
    const float w0 = q4[0], x0 = q4[1], y0 = q4[2], z0 = q4[3];
    const float nrm = sqrtf(w0 * w0 + x0 * x0 + y0 * y0 + z0 * z0);
    const float w = w0 / nrm, x = x0 / nrm, y = y0 / nrm, z = z0 / nrm;
    if (r == 0) {
        a = 1.f - 2.f * (y * y + z * z);
        b = 2.f * (x * y - w * z);
        c = 2.f * (x * z + w * y);
    } else if (r == 1) {
        a = 2.f * (x * y + w * z);
        b = 1.f - 2.f * (x * x + z * z);
        c = 2.f * (y * z - w * x);
    } else {
        a = 2.f * (x * z - w * y);
        b = 2.f * (y * z + w * x);
        c = 1.f - 2.f * (x * x + y * y);
    }
}

__global__ __launch_bounds__(kApplyThreads) void k_densify_apply(ApplyArgs a) {
#pragma clang fp contract(off)
    const int64_t blk = blockIdx.x;
    int gi = 0;
#pragma unroll
    for (int k = 1; k < kMaxGroups; k++)
        if (k < a.n_groups && blk >= a.grp[k].block0) gi = k;
    const ApplyGroup& G = a.grp[gi];
    const int64_t e = (blk - G.block0) * kApplyThreads + threadIdx.x;
    if (e >= G.n) return;
    const int w = G.width;
    const int64_t i = e / w;
    const int col = (int)(e - i * w);
    const unsigned f = a.flags[i];
    if (!(f & (kKeepOrig | kKeepClone | kKeepChildren | kKeepAbe))) return;
    const Rank5 off = a.offsets[i];
    const float pv = G.p[e];
    if (f & kKeepOrig) {
        const int64_t d = (int64_t)off.o * w + col;
        G.op[d] = pv;
        if (G.om) {
            G.om[d] = G.m[e];
            G.ov[d] = G.v[e];
        }
    }
    if (f & kKeepClone) {  // densify_and_clone: same values, zero moments
        const int64_t d = ((int64_t)a.A + off.c) * w + col;
        G.op[d] = pv;
        if (G.om) {
            G.om[d] = 0.f;
            G.ov[d] = 0.f;
        }
    }
    if (f & kKeepAbe) {  // the abe copies (copy-major after the clones), zero moments
        float val = pv;
        if (G.kind == RT_GROUP_SCALING) val = logf(expf(pv));  // scaling_inverse_activation(get_scaling)
        if (G.kind == RT_GROUP_XYZ) val = (pv * a.abe0) * a.abe1;
        for (int n = 0; n + 1 < a.n_split; n++) {
            const int64_t d = ((int64_t)a.A + a.B + (int64_t)n * a.E + off.ab) * w + col;
            G.op[d] = val;
            if (G.om) {
                G.om[d] = 0.f;
                G.ov[d] = 0.f;
            }
        }
    }
    if (f & kKeepChildren) {  // densify_and_split children
        float val = pv;
        if (G.kind == RT_GROUP_SCALING) val = logf(expf(pv) * a.inv_div);
        float r0 = 0.f, r1 = 0.f, r2 = 0.f, sd0 = 0.f, sd1 = 0.f, sd2 = 0.f;
        if (G.kind == RT_GROUP_XYZ) {
            rot_row(a.rotation + 4 * i, col, r0, r1, r2);
            sd0 = expf(a.scaling[3 * i]);
            sd1 = expf(a.scaling[3 * i + 1]);
            sd2 = expf(a.scaling[3 * i + 2]);
        }
        for (int n = 0; n < a.n_split; n++) {
            if (G.kind == RT_GROUP_XYZ) {
                // samples = normal(0, 1) * std + 0 (torch.normal); new_xyz = bmm(R, samples) + xyz
                const float* z = a.normals + 3 * ((int64_t)n * a.S + off.s);
                const float q0 = z[0] * sd0 + 0.f, q1 = z[1] * sd1 + 0.f, q2 = z[2] * sd2 + 0.f;
                val = fmaf(r2, q2, fmaf(r1, q1, r0 * q0)) + pv;
            }
            const int64_t d = ((int64_t)a.A + a.B + (int64_t)(a.n_split - 1) * a.E + (int64_t)n * a.C + off.ch) * w +
                              col;
            G.op[d] = val;
            if (G.om) {
                G.om[d] = 0.f;
                G.ov[d] = 0.f;
            }
        }
    }
}

}  // namespace

extern "C" {

size_t rt_densify_workspace_bytes(int P) { return carve(nullptr, P).total; }

int rt_densify_plan(const rt_densify_params* p, const float* xyz_gradient_accum, const float* denom,
                    const float* scaling, const float* opacity, void* workspace, size_t workspace_bytes,
                    int64_t counts[5], void* stream) {
    if (!p || !counts) return fail("rt_densify_plan: null params / counts");
    for (int k = 0; k < 5; k++) counts[k] = 0;
    if (p->P < 0 || p->n_split < 1) return fail("rt_densify_plan: bad P / n_split");
    if (p->P == 0) return 0;
    if (!xyz_gradient_accum || !denom || !scaling || !opacity || !workspace)
        return fail("rt_densify_plan: null array");
    Workspace w = carve(workspace, p->P);
    if (workspace_bytes < w.total) return fail("rt_densify_plan: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const float inv_div = 1.0f / p->split_scale_div;
    k_densify_classify<<<(p->P + 255) / 256, 256, 0, st>>>(*p, inv_div, xyz_gradient_accum, denom, scaling, opacity,
                                                            w.flags);
    size_t tb = w.temp_bytes;
    hipError_t e = rocprim::exclusive_scan(w.temp, tb, FlagIt(w.flags, Flags5()), w.offsets,
                                           Rank5{0u, 0u, 0u, 0u, 0u}, (size_t)p->P, Add5(), st);
    if (e != hipSuccess) return fail(std::string("densify scan: ") + hipGetErrorString(e));
    k_totals<<<1, 1, 0, st>>>(p->P, w.flags, w.offsets, w.totals);
    Rank5 t;
    e = hipMemcpyAsync(&t, w.totals, sizeof(Rank5), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(std::string("densify plan: ") + hipGetErrorString(e));
    counts[0] = t.o;
    counts[1] = t.c;
    counts[2] = t.ch;
    counts[3] = t.s;
    counts[4] = t.ab;
    return 0;
}

int rt_densify_apply(const rt_densify_params* p, const float* scaling, const float* rotation, const float* normals,
                     const void* workspace, const rt_densify_group* groups, int n_groups, const int64_t counts[5],
                     void* stream) {
    if (!p || !counts || (n_groups > 0 && !groups)) return fail("rt_densify_apply: null argument");
    if (n_groups < 0 || n_groups > kMaxGroups) return fail("rt_densify_apply: n_groups must be 0..8");
    if (p->P == 0) return 0;
    if (!workspace || !scaling || !rotation) return fail("rt_densify_apply: null array");
    if (counts[3] > 0 && !normals) return fail("rt_densify_apply: split samples missing");
    for (int k = 0; k < 5; k++)
        if (counts[k] < 0 || counts[k] > p->P) return fail("rt_densify_apply: counts out of range");
    if (counts[4] > 0 && !p->abe_split) return fail("rt_densify_apply: abe copies without abe_split");
    Workspace w = carve(const_cast<void*>(workspace), p->P);
    ApplyArgs a{};
    a.n_groups = n_groups;
    a.n_split = p->n_split;
    a.A = (uint32_t)counts[0];
    a.B = (uint32_t)counts[1];
    a.C = (uint32_t)counts[2];
    a.S = (uint32_t)counts[3];
    a.E = (uint32_t)counts[4];
    a.inv_div = 1.0f / p->split_scale_div;
    a.abe0 = p->abe_xyz_scale0;
    a.abe1 = p->abe_xyz_scale1;
    a.flags = w.flags;
    a.offsets = w.offsets;
    a.scaling = scaling;
    a.rotation = rotation;
    a.normals = normals;
    int64_t blocks = 0;
    for (int k = 0; k < n_groups; k++) {
        const rt_densify_group& g = groups[k];
        if (g.width < 1 || !g.param || !g.out_param) return fail("rt_densify_apply: bad group");
        const bool mom = g.exp_avg != nullptr;
        if ((g.exp_avg_sq != nullptr) != mom || (g.out_exp_avg != nullptr) != mom ||
            (g.out_exp_avg_sq != nullptr) != mom)
            return fail("rt_densify_apply: moments must be given (with outputs) or absent together");
        if (g.kind == RT_GROUP_XYZ && g.width != 3) return fail("rt_densify_apply: the xyz group must have width 3");
        ApplyGroup& d = a.grp[k];
        d.p = g.param;
        d.m = g.exp_avg;
        d.v = g.exp_avg_sq;
        d.op = g.out_param;
        d.om = g.out_exp_avg;
        d.ov = g.out_exp_avg_sq;
        d.width = g.width;
        d.kind = g.kind;
        d.n = (int64_t)p->P * g.width;
        d.block0 = blocks;
        blocks += (d.n + kApplyThreads - 1) / kApplyThreads;
    }
    for (int k = n_groups; k < kMaxGroups; k++) a.grp[k].block0 = INT64_MAX;
    if (blocks == 0) return 0;
    if (blocks > 0x7fffffffLL) return fail("rt_densify_apply: too many elements");
    hipStream_t st = (hipStream_t)stream;
    k_densify_apply<<<(unsigned)blocks, kApplyThreads, 0, st>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(std::string("densify apply: ") + hipGetErrorString(e));
    return 0;
}

}  // extern "C"
