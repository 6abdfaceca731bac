// rr_forward.hip — forward kernels of the MI355X rasterizer.
//
//   k_preprocess<DEG>  one thread per Gaussian (forward.cu:144-246 semantics)
//   k_gather_tiles     tile counts in depth order (input of the prefix sum)
//   k_duplicate<K>     (tile, Gaussian) pairs in depth order, key = tile id only (LDS windows)
//   k_ranges<K>        per-tile [start, end) in the tile-sorted list (rasterizer_impl.cu:105-127)
//   k_blend_fwd        per-tile front-to-back alpha blend (forward.cu:251-369)
//   k_mark_visible     frustum test (rasterizer_impl.cu:43-55)
//
// Binning order: the reference sorts 64-bit (tile << 32 | depth_bits) keys emitted in Gaussian
// index order with a stable radix sort.  Here visible Gaussians are first stable-sorted by
// depth bits (P keys, 32 bits), their pairs are emitted in that order, and the pairs are then
// stable-sorted by tile id only (msb(T) <= 15 bits, 16-bit keys).  Within a tile this yields the
// same (depth, index) order as the reference, at a fraction of the sort traffic.
#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

// No global atomics here: per-Gaussian counts go to tiles[idx] = {pairs, rect area} and are
// prefix-summed in depth order (the rect-area sum is the reference's num_rendered).
template <int DEG>
__device__ __forceinline__ void preprocess_one(const PreArgs& a, int idx) {
    a.radii[idx] = 0;
    a.tiles[idx] = make_uint2(0u, 0u);
    a.depth_keys[idx] = 0xffffffffu;  // culled Gaussians sort behind every visible one

    const v3 p = load3(a.means3D + 3 * (size_t)idx);
    // in_frustum (auxiliary.h:128-153)
    const v3 p_view = xform_point_4x3(p, a.view);
    if (p_view.z <= 0.2f) {
        if (a.prefiltered) __builtin_trap();
        return;
    }
    const float4 p_hom = xform_point_4x4(p, a.proj);
    const float p_w = 1.0f / (p_hom.w + 0.0000001f);
    const float ppx = p_hom.x * p_w, ppy = p_hom.y * p_w;

    float cov[6];
    if (a.cov3D_precomp) {
        const float* c = a.cov3D_precomp + 6 * (size_t)idx;
#pragma unroll
        for (int i = 0; i < 6; i++) cov[i] = c[i];
    } else {
        float4 q = *reinterpret_cast<const float4*>(a.rotations + 4 * (size_t)idx);
        v3 sc = load3(a.scales + 3 * (size_t)idx);
        if (a.raw) {
            q = act_rot(q);
            sc = act_scale(sc);
        }
        cov3d_from_scale_rot(sc, a.scale_modifier, q, cov);
    }
    const Proj2D pr = ewa_setup(p, a.focal_x, a.focal_y, a.tanfovx, a.tanfovy, a.view);
    float ca, cb, cc;
    ewa_cov2d(pr, cov, ca, cb, cc);
    ca += a.low_pass;
    cc += a.low_pass;

    const float det = ca * cc - cb * cb;
    if (det == 0.0f) return;
    const float det_inv = 1.f / det;
    const float cx = cc * det_inv, cy = -cb * det_inv, cz = ca * det_inv;
    const float mid = 0.5f * (ca + cc);
    const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
    const int radius = (int)my_radius;
    const float px = ndc2pix(ppx, a.W), py = ndc2pix(ppy, a.H);
    int x0, y0, x1, y1;
    tile_rect(px, py, radius, a.gx, a.gy, x0, y0, x1, y1);
    const int area = (x1 - x0) * (y1 - y0);
    if (area == 0) return;

    float4 rgb;
    if (a.colors_precomp) {
        const v3 c = load3(a.colors_precomp + 3 * (size_t)idx);
        rgb = make_float4(c.x, c.y, c.z, 0.f);
    } else {
        const v3 cp = load3(a.campos);
        v3 dir = p - cp;
        const float len = sqrtf(dot(dir, dir));
        dir = mk(dir.x / len, dir.y / len, dir.z / len);
        const float* dc = a.raw ? a.shs + 3 * (size_t)idx : a.shs + (size_t)idx * a.M * 3;
        const float* rest = a.raw ? a.shs_rest + (size_t)idx * (a.M - 1) * 3 : dc + 3;
        const v3 c = sh_eval<DEG>(dir, dc, rest);
        rgb = make_float4(fmaxf(c.x, 0.f), fmaxf(c.y, 0.f), fmaxf(c.z, 0.f), 0.f);
    }
    const float opacity = a.raw ? act_opacity(a.opacities[idx]) : a.opacities[idx];
    Splat s;
    s.a = make_float4(px, py, cx, cy);
    s.b = make_float4(cz, opacity, p_view.z, 0.f);
    s.c = rgb;
    a.splats[idx] = s;
    a.radii[idx] = radius;
    uint32_t n = (uint32_t)area;
    if (a.cull) {
        const float qmax = cull_qmax(opacity);
        n = 0;
        for (int y = y0; y < y1; y++) {
            int lo, hi;
            cull_row_span(px, py, cx, cy, cz, qmax, y, x0, x1, &lo, &hi);
            n += hi > lo ? (uint32_t)(hi - lo) : 0u;
        }
    }
    a.tiles[idx] = make_uint2(n, (uint32_t)area);
    a.depth_keys[idx] = __float_as_uint(p_view.z);  // > 0.2, so the bit pattern orders like the value
}

template <int DEG>
__global__ __launch_bounds__(256) void k_preprocess(PreArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < a.P) preprocess_one<DEG>(a, idx);
}

__global__ __launch_bounds__(256) void k_gather_tiles(int P, const uint32_t* __restrict__ idx_sorted,
                                                      const uint2* __restrict__ tiles,
                                                      uint2* __restrict__ tiles_sorted) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P) return;
    tiles_sorted[s] = tiles[idx_sorted[s]];
}

// First Gaussian (depth rank) of every window of `win` consecutive pairs: window k starts inside
// the pair range [a, b) of exactly one Gaussian.
__global__ __launch_bounds__(256) void k_window_starts(int P, const uint2* __restrict__ offsets, uint32_t win,
                                                       int nwin, uint32_t* __restrict__ first) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P) return;
    const uint32_t a = s == 0 ? 0u : offsets[s - 1].x, b = offsets[s].x;
    if (a == b) return;
    for (uint32_t k = (a + win - 1) / win; k <= (b - 1) / win && k < (uint32_t)nwin; k++) first[k] = (uint32_t)s;
}

// duplicateWithKeys (rasterizer_impl.cu:59-100), output-driven: workgroup k produces exactly the
// pairs [k*win, (k+1)*win) of the depth-ordered pair list.  Its Gaussians (from first[k] on) emit
// into an LDS window, which then leaves with coalesced stores — the per-Gaussian form scatters
// every pair to its own cache line — and the window's histogram of the lowest `dbits` key bits is
// written as the tile sort's first-pass digit counts (rr_sort.hip units == windows).
template <typename K>
__global__ __launch_bounds__(256) void k_duplicate(int P, const uint32_t* __restrict__ idx_sorted,
                                                   const uint2* __restrict__ offsets,
                                                   const Splat* __restrict__ splats, const int* __restrict__ radii,
                                                   int gx, int gy, int cull, const uint32_t* __restrict__ first,
                                                   uint32_t win, uint32_t L, K* __restrict__ keys,
                                                   uint32_t* __restrict__ vals, int dbits,
                                                   uint32_t* __restrict__ counts, int units) {
    __shared__ K s_key[kSortMaxUnit];
    __shared__ uint32_t s_val[kSortMaxUnit];
    __shared__ uint32_t hist[256];
    const int t = threadIdx.x;
    const int ndig = 1 << dbits;
    for (int d = t; d < ndig; d += 256) hist[d] = 0;
    const uint32_t w0 = blockIdx.x * win, w1 = min(w0 + win, L);
    const int s0 = (int)first[blockIdx.x];
    for (int base = s0;; base += 256) {
        const int s = base + t;
        if (s < P) {
            const uint32_t a = s == 0 ? 0u : offsets[s - 1].x, b = offsets[s].x;
            const uint32_t lo = max(a, w0), hi = min(b, w1);
            if (lo < hi) {
                const uint32_t g = idx_sorted[s];
                const int r = radii[g];
                const float4 A = splats[g].a;
                int x0, y0, x1, y1;
                tile_rect(A.x, A.y, r, gx, gy, x0, y0, x1, y1);
                const float qmax = cull ? cull_qmax(splats[g].b.y) : 0.f;
                const float cz = cull ? splats[g].b.x : 0.f;
                uint32_t pos = a;
                for (int y = y0; y < y1 && pos < hi; y++) {
                    int l = x0, h = x1;
                    if (cull) cull_row_span(A.x, A.y, A.z, A.w, cz, qmax, y, x0, x1, &l, &h);
                    const uint32_t c = h > l ? (uint32_t)(h - l) : 0u;
                    if (pos + c <= lo) {  // row entirely before the window
                        pos += c;
                        continue;
                    }
                    for (int x = l; x < h && pos < hi; x++, pos++)
                        if (pos >= lo) {
                            s_key[pos - w0] = (K)(y * gx + x);
                            s_val[pos - w0] = g;
                        }
                }
            }
        }
        // another round only if this round's last Gaussian ends before the window does
        const int last = min(base + 255, P - 1);
        if (last >= P - 1 || offsets[last].x >= w1) break;
    }
    __syncthreads();
    const uint32_t mask = (uint32_t)ndig - 1u;
    for (uint32_t j = t; j < w1 - w0; j += 256) {
        const K k = s_key[j];
        keys[w0 + j] = k;
        vals[w0 + j] = s_val[j];
        atomicAdd(&hist[(uint32_t)k & mask], 1u);
    }
    __syncthreads();
    for (int d = t; d < ndig; d += 256) counts[(size_t)d * units + blockIdx.x] = hist[d];
}

template <typename K>
__global__ __launch_bounds__(256) void k_ranges(int L, const K* __restrict__ keys, uint2* __restrict__ ranges) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L) return;
    const uint32_t cur = keys[i];
    if (i == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = keys[i - 1];
        if (cur != prev) {
            ranges[prev].y = i;
            ranges[cur].x = i;
        }
    }
    if (i == L - 1) ranges[cur].y = L;
}

__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means3D,
                                                      const float* __restrict__ view, uint8_t* __restrict__ present) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const v3 pv = xform_point_4x3(load3(means3D + 3 * (size_t)i), view);
    present[i] = pv.z <= 0.2f ? 0 : 1;
}

// ---------------------------------------------------------------------------------------
// host launchers
static inline int blocks_for(long n, int b = 256) { return (int)((n + b - 1) / b); }

void launch_preprocess(const PreArgs& a, hipStream_t st) {
    if (a.P == 0) return;
    const int nb = blocks_for(a.P);
    switch (a.colors_precomp ? 0 : a.D) {
        case 0: k_preprocess<0><<<nb, 256, 0, st>>>(a); break;
        case 1: k_preprocess<1><<<nb, 256, 0, st>>>(a); break;
        case 2: k_preprocess<2><<<nb, 256, 0, st>>>(a); break;
        default: k_preprocess<3><<<nb, 256, 0, st>>>(a); break;
    }
}

void launch_gather_tiles(int P, const uint32_t* idx_sorted, const uint2* tiles, uint2* out, hipStream_t st) {
    if (P == 0) return;
    k_gather_tiles<<<blocks_for(P), 256, 0, st>>>(P, idx_sorted, tiles, out);
}

template <typename K>
void launch_duplicate(int P, const uint32_t* idx_sorted, const uint2* offsets, const Splat* splats, const int* radii,
                      int gx, int gy, int cull, uint32_t* first, uint32_t win, int nwin, uint32_t L, K* keys,
                      uint32_t* vals, int dbits, uint32_t* counts, hipStream_t st) {
    if (P == 0 || L == 0 || win > (uint32_t)kSortMaxUnit) return;  // win comes from radix_sort_plan
    k_window_starts<<<blocks_for(P), 256, 0, st>>>(P, offsets, win, nwin, first);
    k_duplicate<K><<<nwin, 256, 0, st>>>(P, idx_sorted, offsets, splats, radii, gx, gy, cull, first, win, L, keys,
                                          vals, dbits, counts, nwin);
}
template void launch_duplicate<uint16_t>(int, const uint32_t*, const uint2*, const Splat*, const int*, int, int, int,
                                         uint32_t*, uint32_t, int, uint32_t, uint16_t*, uint32_t*, int, uint32_t*,
                                         hipStream_t);
template void launch_duplicate<uint32_t>(int, const uint32_t*, const uint2*, const Splat*, const int*, int, int, int,
                                         uint32_t*, uint32_t, int, uint32_t, uint32_t*, uint32_t*, int, uint32_t*,
                                         hipStream_t);

template <typename K>
void launch_ranges(int L, const K* keys, uint2* ranges, hipStream_t st) {
    if (L == 0) return;
    k_ranges<K><<<blocks_for(L), 256, 0, st>>>(L, keys, ranges);
}
template void launch_ranges<uint16_t>(int, const uint16_t*, uint2*, hipStream_t);
template void launch_ranges<uint32_t>(int, const uint32_t*, uint2*, hipStream_t);

void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st) {
    if (P == 0) return;
    k_mark_visible<<<blocks_for(P), 256, 0, st>>>(P, means3D, view, present);
}

}  // namespace rr
