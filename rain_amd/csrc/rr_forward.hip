// rr_forward.hip — forward kernels of the MI355X rasterizer.
//
//   k_preprocess<DEG>  one thread per Gaussian (forward.cu:144-246 semantics)
//   k_duplicate<K>     (bin, Gaussian) pairs in depth order, key = bin id only, value = Gaussian |
//                      tile mask << BIN_SHIFT (LDS windows; bins: rr_common.hpp)
//   k_expand<K>        per bin of the bin-sorted list: its four per-tile lists (stable) and their
//                      [start, end) (rasterizer_impl.cu:105-127's ranges)
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
__device__ __forceinline__ uint2 preprocess_one(const PreArgs& a, int idx, bool& wide) {
    a.radii[idx] = 0;
    a.tiles[idx] = make_uint2(0u, 0u);
    if (a.depth_keys) a.depth_keys[idx] = 0xffffffffu;  // culled Gaussians sort behind every visible one

    const v3 p = load3(a.means3D + 3 * (size_t)idx);
    // in_frustum (auxiliary.h:128-153)
    const v3 p_view = xform_point_4x3(p, a.view);
    if (p_view.z <= 0.2f) {
        if (a.prefiltered) __builtin_trap();
        return make_uint2(0u, 0u);
    }
    // The row's remaining inputs (but the SH coefficients) in one batch right after the depth
    // test: a wave then waits for one memory round trip where it waited for three (rotation and
    // scale, colour, opacity): preprocess 0.080 -> 0.077 ms/step in an interleaved A/B (the SH rows
    // too: 158 VGPRs, 3 waves/SIMD, 0.086; profiles/r03_preprocess_early_ab.jsonl)
    float4 q = make_float4(1.f, 0.f, 0.f, 0.f);
    v3 sc = mk(0.f, 0.f, 0.f);
    if (!a.cov3D_precomp) {
        q = *reinterpret_cast<const float4*>(a.rotations + 4 * (size_t)idx);
        sc = load3(a.scales + 3 * (size_t)idx);
    }
    const float o_in = a.opacities[idx];
    const float* dc = a.raw ? a.shs + 3 * (size_t)idx : a.shs + (size_t)idx * a.M * 3;
    const v3 c0 = load3(a.colors_precomp ? a.colors_precomp + 3 * (size_t)idx : dc);

    const float4 p_hom = xform_point_4x4(p, a.proj);
    const float p_w = 1.0f / (p_hom.w + 0.0000001f);
    const float ppx = p_hom.x * p_w, ppy = p_hom.y * p_w;

    float cov[6];
    if (a.cov3D_precomp) {
        const float* c = a.cov3D_precomp + 6 * (size_t)idx;
#pragma unroll
        for (int i = 0; i < 6; i++) cov[i] = c[i];
    } else {
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
    if (det == 0.0f) return make_uint2(0u, 0u);
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
    if (area == 0) return make_uint2(0u, 0u);

    float4 rgb;
    if (a.colors_precomp) {
        rgb = make_float4(c0.x, c0.y, c0.z, 0.f);
    } else {
        const v3 cp = load3(a.campos);
        v3 dir = p - cp;
        const float len = sqrtf(dot(dir, dir));
        dir = mk(dir.x / len, dir.y / len, dir.z / len);
        const float* rest = a.raw ? a.shs_rest + (size_t)idx * (a.M - 1) * 3 : dc + 3;
        // the coefficients this degree uses, in 16-B loads (dword-aligned: a record is 180 or 192 B,
        // one lane's loads touch ~4x fewer cache lines per instruction than 45 dword loads)
        constexpr int NR = ((DEG + 1) * (DEG + 1) - 1) * 3;
        float rr[NR > 0 ? NR : 1];
        load_floats_u<NR>(rest, rr);
        const v3 c = sh_eval<DEG>(dir, c0, rr);
        rgb = make_float4(fmaxf(c.x, 0.f), fmaxf(c.y, 0.f), fmaxf(c.z, 0.f), 0.f);
    }
    const float opacity = a.raw ? act_opacity(o_in) : o_in;
    float log2o, inv_o;
    splat_derived(opacity, log2o, inv_o);
    Splat s;
    s.a = make_float4(px, py, kQHalf * cx, kQFull * cy);
    s.b = make_float4(kQHalf * cz, log2o, p_view.z, opacity);
    s.c = make_float4(rgb.x, rgb.y, rgb.z, inv_o);
    if (a.wire) {
        float2* w = reinterpret_cast<float2*>(a.wire + (size_t)kWireFloats * idx);
        w[0] = make_float2(s.a.x, s.a.y);
        w[1] = make_float2(s.a.z, s.a.w);
        w[2] = make_float2(s.b.x, s.b.z);
        w[3] = make_float2(s.b.w, s.c.x);
        w[4] = make_float2(s.c.y, s.c.z);
    } else {
        a.splats[idx] = s;
    }
    if (a.normals) a.normals[idx] = gaussian_normal(sc, q, a.view, p_view);
    a.radii[idx] = radius;
    // (bin, Gaussian) pairs: bins (2 x 2 tiles, rr_common.hpp) holding a tile the Gaussian reaches
    // (exact culling) or a tile of its bounding rect
    // culling on the conic as the duplicate reads it back from the record (splat_conic), so both
    // kernels count the same pairs
    float ccx, ccy, ccz;
    splat_conic(s.a, s.b, ccx, ccy, ccz);
    const CullEll ell = cull_setup(px, py, ccx, ccy, ccz, a.cull ? cull_qmax(opacity) : 0.f);
    uint32_t n = 0;
    for (int Y = y0 >> 1; Y < (y1 + 1) >> 1; Y++) {
        int l0, h0, l1, h1;
        bin_row_spans(ell, a.cull, Y, x0, x1, y0, y1, l0, h0, l1, h1);
        n += bin_count(l0, h0, l1, h1);
    }
    a.tiles[idx] = make_uint2(n, (uint32_t)area);
    // > 0.2, so the bit pattern orders like the value, and so does its offset from kDepthKeyBase
    const uint32_t key = __float_as_uint(p_view.z) - kDepthKeyBase;
    if (a.depth_keys) a.depth_keys[idx] = key;
    wide = key >= (1u << kDepthKeyBits);
    return make_uint2(n, (uint32_t)area);
}

// The block's sums of {pairs, rect tiles} go to a.block_sums[blockIdx.x] (plain stores; a single
// contended 64-bit atomic per block measured +37 us on 1M Gaussians): the frame's pair count is
// then known right after this kernel (rr_api.hip pair_counts_publish reduces them).
template <int DEG>
__device__ __forceinline__ void preprocess_block(const PreArgs& a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    bool wide = false;
    uint2 c = make_uint2(0u, 0u);
    if (idx < a.P) {
        c = preprocess_one<DEG>(a, idx, wide);
    } else if (idx < a.n_out) {  // padding row of a row block: culled
        a.radii[idx] = 0;
        a.tiles[idx] = make_uint2(0u, 0u);
        if (a.depth_keys) a.depth_keys[idx] = 0xffffffffu;
    }
    if (!a.block_sums) return;
    __shared__ uint2 s_sum[4];
    __shared__ uint32_t s_wide[4];
    uint32_t n = c.x, r = c.y;  // per block <= 256 * T, below 2^32 for T < 2^24
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        n += (uint32_t)__shfl_xor((int)n, o);
        r += (uint32_t)__shfl_xor((int)r, o);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool wave_wide = __any(wide);
    if (lane == 0) {
        s_sum[w] = make_uint2(n, r);
        s_wide[w] = wave_wide ? 1u : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a.block_sums[blockIdx.x] = make_uint2(s_sum[0].x + s_sum[1].x + s_sum[2].x + s_sum[3].x,
                                              s_sum[0].y + s_sum[1].y + s_sum[2].y + s_sum[3].y);
        a.block_wide[blockIdx.x] = s_wide[0] | s_wide[1] | s_wide[2] | s_wide[3];
    }
}

// 5 waves per SIMD: the SH-3 instance fits 88 VGPRs without spills (the compiler's own choice,
// 98, gives 4; 6 waves spill 52 B/lane): preprocess 0.094 -> 0.090 ms/step in an interleaved A/B
// (profiles/r03_preprocess_occupancy_ab.txt; 8 waves measured 0.129 vs 0.091 in round 2)
#ifndef RR_PRE_OCC
#define RR_PRE_OCC 5
#endif
template <int DEG>
__global__ __launch_bounds__(256, RR_PRE_OCC) void k_preprocess(PreArgs a) {
    preprocess_block<DEG>(a);
}

template <int DEG>
__global__ __launch_bounds__(256, RR_PRE_OCC) void k_preprocess_views(PreArgs a, PreViews vs) {
    const PreView& c = vs.v[blockIdx.y];
    PreArgs b = a;
    b.view = c.view;
    b.proj = c.proj;
    b.campos = c.campos;
    b.tanfovx = c.tanfovx;
    b.tanfovy = c.tanfovy;
    b.focal_x = c.focal_x;
    b.focal_y = c.focal_y;
    b.low_pass = c.low_pass;
    b.W = c.W;
    b.H = c.H;
    b.gx = c.gx;
    b.gy = c.gy;
    const size_t off = (size_t)blockIdx.y * vs.stride;
    auto at = [&](auto* p) { return reinterpret_cast<decltype(p)>(reinterpret_cast<char*>(p) + off); };
    b.radii = at(a.radii);
    b.splats = at(a.splats);
    b.tiles = at(a.tiles);
    b.depth_keys = a.depth_keys ? at(a.depth_keys) : nullptr;
    b.block_sums = at(a.block_sums);
    b.block_wide = at(a.block_wide);
    b.wire = a.wire ? at(a.wire) : nullptr;
    preprocess_block<DEG>(b);
}

// The receiving side of the sharded step's geometry exchange: rows of `world` chunks (chunk j =
// rank j's rows, wire format) into the geometry arrays in global row order, splats rebuilt with
// splat_derived, depth keys from the depth (0xffffffff for a culled row, radius 0).
__global__ __launch_bounds__(256) void k_unpack_rows(int world, int Q, const char* __restrict__ recv, size_t chunk,
                                                     size_t o_wire, size_t o_tiles, size_t o_radii, size_t o_bsum,
                                                     size_t o_bwide, Splat* __restrict__ splats,
                                                     uint2* __restrict__ tiles, uint32_t* __restrict__ keys,
                                                     int* __restrict__ radii, uint2* __restrict__ bsum,
                                                     uint32_t* __restrict__ bwide) {
    const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= (size_t)world * Q) return;
    const int j = (int)(g / (size_t)Q), r = (int)(g - (size_t)j * Q);
    const char* c = recv + (size_t)j * chunk;
    const float2* w = reinterpret_cast<const float2*>(c + o_wire) + (size_t)(kWireFloats / 2) * r;
    const int radius = reinterpret_cast<const int*>(c + o_radii)[r];
    tiles[g] = reinterpret_cast<const uint2*>(c + o_tiles)[r];
    radii[g] = radius;
    Splat s;
    if (radius > 0) {
        const float2 w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
        float log2o, inv_o;
        splat_derived(w3.x, log2o, inv_o);
        s.a = make_float4(w0.x, w0.y, w1.x, w1.y);
        s.b = make_float4(w2.x, log2o, w2.y, w3.x);
        s.c = make_float4(w3.y, w4.x, w4.y, inv_o);
    } else {
        // a culled row's wire record was never written by its owner (the preprocess returns before
        // the record): a zero record keeps the geometry buffer deterministic
        s.a = s.b = s.c = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    splats[g] = s;
    keys[g] = radius > 0 ? __float_as_uint(s.b.z) - kDepthKeyBase : 0xffffffffu;
    if ((r & 255) == 0) {  // Q is a multiple of 256: rank j's block b is global block g / 256
        bsum[g / 256] = reinterpret_cast<const uint2*>(c + o_bsum)[r / 256];
        bwide[g / 256] = reinterpret_cast<const uint32_t*>(c + o_bwide)[r / 256];
    }
}

void launch_unpack_rows(int world, int rows_per_rank, const char* recv, size_t chunk_bytes,
                        const size_t field_offsets[5], Splat* splats, uint2* tiles, uint32_t* depth_keys, int* radii,
                        uint2* block_sums, uint32_t* block_wide, hipStream_t st) {
    const size_t n = (size_t)world * rows_per_rank;
    if (n == 0) return;
    k_unpack_rows<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
        world, rows_per_rank, recv, chunk_bytes, field_offsets[0], field_offsets[1], field_offsets[2],
        field_offsets[3], field_offsets[4], splats, tiles, depth_keys, radii, block_sums, block_wide);
}

// ---- scan of the pair counts in depth order (replaces a device-wide decoupled-look-back scan:
// its state-init launch plus a look-back chain over ~500 blocks measured 18.5 us per frame) ----
// SatAdd2 (min(a + b, 2^32 - 1) per component) is associative, so the scan equals the exact 64-bit
// prefix sums clamped to 32 bits: both kernels sum in 64 bits and clamp only on output.
__device__ __forceinline__ void block_sum2_u64(unsigned long long& x, unsigned long long& y,
                                               unsigned long long* s) {  // s: [8], 256 threads
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o);
        y += __shfl_xor(y, o);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        s[w] = x;
        s[4 + w] = y;
    }
    __syncthreads();
    x = s[0] + s[1] + s[2] + s[3];
    y = s[4] + s[5] + s[6] + s[7];
}

// n_dev (may be null): only the first min(P, *n_dev) items are read, the rest count as {0, 0}
// (the depth sort that dropped the culled Gaussians leaves its output past its count unwritten)
__device__ __forceinline__ int scan_len(int P, const uint32_t* n_dev) {
    return n_dev ? (int)min((uint32_t)P, *n_dev) : P;
}

__global__ __launch_bounds__(256) void k_pair_scan_totals(const uint2* __restrict__ in, int P,
                                                          ulonglong2* __restrict__ tot, const uint32_t* n_dev) {
    P = scan_len(P, n_dev);
    __shared__ unsigned long long s[8];
    const size_t b0 = (size_t)blockIdx.x * kPairScanItems;
    unsigned long long x = 0, y = 0;
#pragma unroll
    for (int r = 0; r < kPairScanItems / 256; r++) {
        const size_t i = b0 + (size_t)r * 256 + threadIdx.x;
        if (i < (size_t)P) {
            const uint2 v = in[i];
            x += v.x;
            y += v.y;
        }
    }
    block_sum2_u64(x, y, s);
    if (threadIdx.x == 0) tot[blockIdx.x] = make_ulonglong2(x, y);
}

// Exclusive scan, in place, of the nb block totals (one workgroup, 2048 per round, carried in
// 64 bits): the large-P path, where re-summing every earlier total in each block would grow with
// nb^2 (at P = 16.7M that is ~0.5 GB of L2 reads per frame).
__global__ __launch_bounds__(256) void k_pair_scan_prefix(ulonglong2* __restrict__ tot, int nb) {
    constexpr int IPT = kPairScanItems / 256;
    __shared__ unsigned long long s_wx[4], s_wy[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    unsigned long long cx = 0, cy = 0;  // sum of all earlier rounds
    for (int base = 0; base < nb; base += kPairScanItems) {
        ulonglong2 v[IPT];
        unsigned long long tx = 0, ty = 0;
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const int i = base + t * IPT + k;
            v[k] = i < nb ? tot[i] : make_ulonglong2(0ull, 0ull);
            tx += v[k].x;
            ty += v[k].y;
        }
        unsigned long long ix = tx, iy = ty;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long ux = __shfl_up(ix, o), uy = __shfl_up(iy, o);
            if (lane >= o) {
                ix += ux;
                iy += uy;
            }
        }
        __syncthreads();  // the previous round's reads of s_wx / s_wy are done
        if (lane == 63) {
            s_wx[w] = ix;
            s_wy[w] = iy;
        }
        __syncthreads();
        unsigned long long ex = cx + ix - tx, ey = cy + iy - ty;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < w) {
                ex += s_wx[k];
                ey += s_wy[k];
            }
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            const int i = base + t * IPT + k;
            if (i < nb) tot[i] = make_ulonglong2(ex, ey);
            ex += v[k].x;
            ey += v[k].y;
        }
        cx += s_wx[0] + s_wx[1] + s_wx[2] + s_wx[3];
        cy += s_wy[0] + s_wy[1] + s_wy[2] + s_wy[3];
    }
}

// PREFIX: tot[b] already holds the exclusive prefix of the block totals (k_pair_scan_prefix);
// otherwise it holds block b's own total and every block sums those of the blocks before it.
template <bool PREFIX>
__global__ __launch_bounds__(256) void k_pair_scan(const uint2* __restrict__ in, uint2* __restrict__ out, int P,
                                                   const ulonglong2* __restrict__ tot, const uint32_t* n_dev) {
    constexpr int IPT = kPairScanItems / 256;  // 8 consecutive items per thread
    const int n = scan_len(P, n_dev);  // items read; all P are written
    __shared__ unsigned long long s[8];
    __shared__ unsigned long long s_wx[4], s_wy[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const size_t i0 = (size_t)blockIdx.x * kPairScanItems + (size_t)t * IPT;
    // this thread's items: four 16-B loads (two items each) when the run is in range
    uint2 v[IPT];
    if (i0 + IPT <= (size_t)n) {
        const uint4* p = reinterpret_cast<const uint4*>(in + i0);
#pragma unroll
        for (int k = 0; k < IPT / 2; k++) {
            const uint4 q = p[k];
            v[2 * k] = make_uint2(q.x, q.y);
            v[2 * k + 1] = make_uint2(q.z, q.w);
        }
    } else {
#pragma unroll
        for (int k = 0; k < IPT; k++) v[k] = i0 + k < (size_t)n ? in[i0 + k] : make_uint2(0u, 0u);
    }
    // sum of the totals of all earlier blocks
    unsigned long long bx = 0, by = 0;
    if (PREFIX) {
        const ulonglong2 q = tot[blockIdx.x];
        bx = q.x;
        by = q.y;
    } else {
        for (int j = t; j < (int)blockIdx.x; j += 256) {
            const ulonglong2 q = tot[j];
            bx += q.x;
            by += q.y;
        }
        block_sum2_u64(bx, by, s);
    }
    // exclusive scan of the thread sums (wave shuffles, then the 4 wave totals)
    unsigned long long tx = 0, ty = 0;
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        tx += v[k].x;
        ty += v[k].y;
    }
    unsigned long long ix = tx, iy = ty;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long ux = __shfl_up(ix, o), uy = __shfl_up(iy, o);
        if (lane >= o) {
            ix += ux;
            iy += uy;
        }
    }
    if (lane == 63) {
        s_wx[w] = ix;
        s_wy[w] = iy;
    }
    __syncthreads();
    unsigned long long ex = bx + ix - tx, ey = by + iy - ty;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < w) {
            ex += s_wx[k];
            ey += s_wy[k];
        }
    uint2 o[IPT];
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        ex += v[k].x;
        ey += v[k].y;
        o[k] = make_uint2(ex > 0xffffffffull ? 0xffffffffu : (uint32_t)ex, ey > 0xffffffffull ? 0xffffffffu : (uint32_t)ey);
    }
    if (i0 + IPT <= (size_t)P) {
        uint4* p = reinterpret_cast<uint4*>(out + i0);
#pragma unroll
        for (int k = 0; k < IPT / 2; k++) p[k] = make_uint4(o[2 * k].x, o[2 * k].y, o[2 * k + 1].x, o[2 * k + 1].y);
    } else {
#pragma unroll
        for (int k = 0; k < IPT; k++)
            if (i0 + k < (size_t)P) out[i0 + k] = o[k];
    }
}

size_t pair_scan_temp_bytes(int P) {
    return (size_t)std::max((P + kPairScanItems - 1) / kPairScanItems, 1) * sizeof(ulonglong2);
}

namespace {
int g_pair_scan_direct = kPairScanDirectBlocks;
}
void set_pair_scan_direct_blocks(int nb) { g_pair_scan_direct = nb >= 0 ? nb : kPairScanDirectBlocks; }

void launch_pair_scan(const uint2* in, uint2* out, int P, const uint32_t* n_dev, void* temp, hipStream_t st) {
    if (P <= 0) return;
    const int nb = (P + kPairScanItems - 1) / kPairScanItems;
    ulonglong2* tot = static_cast<ulonglong2*>(temp);
    k_pair_scan_totals<<<nb, 256, 0, st>>>(in, P, tot, n_dev);
    if (nb <= g_pair_scan_direct) {
        k_pair_scan<false><<<nb, 256, 0, st>>>(in, out, P, tot, n_dev);
    } else {
        k_pair_scan_prefix<<<1, 256, 0, st>>>(tot, nb);
        k_pair_scan<true><<<nb, 256, 0, st>>>(in, out, P, tot, n_dev);
    }
}

// First Gaussian (depth rank) of every window of `win` consecutive pairs starting at pair0:
// window k = [pair0 + k*win, pair0 + (k+1)*win) starts inside the pair range [a, b) of exactly
// one Gaussian.
// A second window set (pair0_b, win_b, nwin_b, first_b; nwin_b = 0: none) is marked in the same pass.
__global__ __launch_bounds__(256) void k_window_starts(int P, const uint2* __restrict__ offsets, uint32_t pair0,
                                                       uint32_t win, int nwin, uint32_t* __restrict__ first,
                                                       uint32_t pair0_b, uint32_t win_b, int nwin_b,
                                                       uint32_t* __restrict__ first_b, uint32_t* __restrict__ zero,
                                                       int nzero) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = s; i < nzero; i += gridDim.x * blockDim.x) zero[i] = 0u;
    if (s >= P) return;
    const uint32_t a = s == 0 ? 0u : offsets[s - 1].x, b = offsets[s].x;
    if (a == b) return;
    auto mark = [&](uint32_t p0, uint32_t w, int nw, uint32_t* f) {
        if (nw <= 0 || b <= p0) return;
        const uint32_t k0 = a <= p0 ? 0u : (a - p0 + w - 1) / w;
        for (uint32_t k = k0; k <= (b - 1 - p0) / w && k < (uint32_t)nw; k++) f[k] = (uint32_t)s;
    };
    mark(pair0, win, nwin, first);
    mark(pair0_b, win_b, nwin_b, first_b);
}

// duplicateWithKeys (rasterizer_impl.cu:59-100), output-driven: workgroup k produces exactly the
// pairs [pair0 + k*win, pair0 + (k+1)*win) of the depth-ordered pair list.  Its Gaussians (from
// first[k] on) emit into an LDS window, which then leaves with coalesced stores — the
// per-Gaussian form scatters every pair to its own cache line — and the window's histogram of
// the lowest `dbits` key bits is written as the tile sort's first-pass digit counts (rr_sort.hip
// units == windows).  Output of window k goes to [k*win, ...) of keys / vals.
//
// Phase B of early-stop binning (open_bits != nullptr): only pairs whose tile is still open are
// kept.  A Gaussian whose tile rectangle holds no open tile (its rows' words of the open-tile
// bitmask, from LDS) is skipped without enumerating its bins; the kept pairs of the window are
// compacted (order preserved) and the window's length goes to unit_len[k] (a sparse sort unit) and
// into *n_total.  (A two-pass variant — count the kept pairs, one block scan per round, then write
// them compacted — measured slower: 0.104 vs 0.083 ms/step for both duplicate launches.)
template <typename K, bool FILTER>
__global__ __launch_bounds__(256) void k_duplicate(int P, const uint32_t* __restrict__ idx_sorted,
                                                   const uint2* __restrict__ offsets,
                                                   const Splat* __restrict__ splats, const int* __restrict__ radii,
                                                   int gx, int gy, int cull, const uint32_t* __restrict__ first,
                                                   uint32_t pair0, uint32_t win, uint32_t L, K* __restrict__ keys,
                                                   uint32_t* __restrict__ vals, int dbits,
                                                   uint32_t* __restrict__ counts, int units,
                                                   const uint32_t* __restrict__ open_bits,
                                                   uint32_t* __restrict__ unit_len, uint32_t* __restrict__ n_total,
                                                   const uint32_t* __restrict__ order_cost, uint32_t* __restrict__ order_out,
                                                   uint32_t* __restrict__ order_flag, int order_T) {
    // the extra workgroup (block-uniform) is block 0, so that it is dispatched first and runs
    // under the duplicate instead of after it; the windows are blocks 1..units
    if (FILTER && order_out && blockIdx.x == 0) {
        tile_order_body256(order_T, order_cost, open_bits, order_out);
        if (threadIdx.x == 0) *order_flag = (uint32_t)order_T;
        return;
    }
    const int wb = (FILTER && order_out) ? (int)blockIdx.x - 1 : (int)blockIdx.x;  // window
    // open-tile bitmask in LDS for grids of <= 65536 tiles; larger grids read open_bits directly
    // (FILTER: phase B; the unfiltered kernel does without the mask's 8 KiB of LDS)
    const bool kMaskLds = FILTER && gx * gy <= 65536;
    __shared__ K s_key[kSortMaxUnit];
    __shared__ uint32_t s_val[kSortMaxUnit];
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_open[FILTER ? 2048 : 1];
    __shared__ uint32_t wsum[4];
    const int t = threadIdx.x;
    const int ndig = 1 << dbits;
    constexpr bool filter = FILTER;
    for (int d = t; d < ndig; d += 256) hist[d] = 0;
    const uint32_t w0 = pair0 + wb * win, w1 = min(w0 + win, L);
    const uint32_t wn = w1 - w0;
    if (filter) {
        for (uint32_t j = t; j < wn; j += 256) s_val[j] = 0xffffffffu;  // not emitted
        if (kMaskLds)
            for (int i = t; i < (gx * gy + 31) / 32; i += 256) s_open[i] = open_bits[i];
        __syncthreads();
    }
    auto is_open = [&](uint32_t tile) -> bool {
        const uint32_t word = kMaskLds ? s_open[tile >> 5] : open_bits[tile >> 5];
        return ((word >> (tile & 31)) & 1u) != 0;
    };
    // the bin's tiles still open (phase B), as a bin mask
    auto open4 = [&](int X, int Y) -> uint32_t {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int tx = 2 * X + (b & 1), ty = 2 * Y + (b >> 1);
            if (tx < gx && ty < gy && is_open((uint32_t)(ty * gx + tx))) m |= 1u << b;
        }
        return m;
    };
    // any open tile in the rectangle [x0, x1) x [y0, y1): the bitmask words of each row, first hit
    // ends the walk (rows are contiguous bit runs: usually one or two words per row)
    auto rect_open = [&](int x0, int y0, int x1, int y1) -> bool {
        for (int y = y0; y < y1; y++) {
            const uint32_t lo = (uint32_t)(y * gx + x0), hi = (uint32_t)(y * gx + x1);  // bits [lo, hi)
            for (uint32_t wd = lo >> 5; wd <= (hi - 1) >> 5; wd++) {
                uint32_t m = kMaskLds ? s_open[wd] : open_bits[wd];
                if (wd == lo >> 5) m &= ~0u << (lo & 31);
                if (wd == (hi - 1) >> 5) m &= ~0u >> (31 - ((hi - 1) & 31));
                if (m) return true;
            }
        }
        return false;
    };
    const int bgx = bins_x(gx);
    const int s0 = (int)first[wb];
    for (int base = s0;; base += 256) {
        const int s = base + t;
        if (s < P) {
            // two dependent load steps per Gaussian: {offsets, id} then {radius, record} (the id is
            // part of the branch condition and the culling setup precedes the open-tile test, so
            // the compiler cannot sink these loads behind a wait into the branches that use them)
            const uint32_t a = s == 0 ? 0u : offsets[s - 1].x, b = offsets[s].x;
            const uint32_t g = idx_sorted[s];
            const uint32_t lo = max(a, w0), hi = min(b, w1);
            if (lo < hi && g != 0xffffffffu) {
                const int r = radii[g];
                const float4 A = splats[g].a;
                const float4 Bv = splats[g].b;
                // all of the record in one round trip (the compiler otherwise fetches part of it
                // only after waiting for the rest)
                asm volatile("" ::"v"(r), "v"(A.x), "v"(A.y), "v"(A.z), "v"(A.w), "v"(Bv.x), "v"(Bv.w));
                float ccx, ccy, ccz;
                splat_conic(A, Bv, ccx, ccy, ccz);
                const CullEll ell = cull_setup(A.x, A.y, ccx, ccy, ccz, cull ? cull_qmax(Bv.w) : 0.f);
                int x0, y0, x1, y1;
                tile_rect(A.x, A.y, r, gx, gy, x0, y0, x1, y1);
                const bool any_open = !filter || (x0 < x1 && y0 < y1 && rect_open(x0, y0, x1, y1));
                if (any_open) {
                    uint32_t pos = a;
                    for (int Y = y0 >> 1; Y < (y1 + 1) >> 1 && pos < hi; Y++) {
                        int l0, h0, l1, h1, Xa, Xb;
                        bin_row_spans(ell, cull, Y, x0, x1, y0, y1, l0, h0, l1, h1);
                        bin_cols(l0, h0, l1, h1, Xa, Xb);
                        const uint32_t c = bin_count(l0, h0, l1, h1);
                        if (pos + c <= lo) {  // bin row entirely before the window
                            pos += c;
                            continue;
                        }
                        for (int X = Xa; X < Xb && pos < hi; X++) {
                            uint32_t m = bin_mask(X, l0, h0, l1, h1);
                            if (!m) continue;
                            if (pos >= lo) {
                                if (filter) m &= open4(X, Y);
                                if (m) {
                                    s_key[pos - w0] = (K)(Y * bgx + X);
                                    s_val[pos - w0] = g | (m << BIN_SHIFT);
                                }
                            }
                            pos++;
                        }
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
    K* const kout = keys + (size_t)wb * win;
    uint32_t* const vout = vals + (size_t)wb * win;
    if (!filter) {
        for (uint32_t j = t; j < wn; j += 256) {
            const K k = s_key[j];
            kout[j] = k;
            vout[j] = s_val[j];
            atomicAdd(&hist[(uint32_t)k & mask], 1u);
        }
    } else {
        // order-preserving compaction in rounds of 256 slots: wave ballots give each kept pair its
        // rank inside the round, the four wave totals the round's block offsets
        const int lane = t & 63, wv = t >> 6;
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t carry = 0;
        for (uint32_t r0 = 0; r0 < wn; r0 += 256) {
            const uint32_t j = r0 + t;
            const uint32_t v = j < wn ? s_val[j] : 0xffffffffu;
            const bool kept = v != 0xffffffffu;
            const uint64_t m = __ballot(kept);
            if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t pre = carry, tot = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                pre += i < wv ? wsum[i] : 0u;
                tot += wsum[i];
            }
            if (kept) {
                const K k = s_key[j];
                const uint32_t pos = pre + (uint32_t)__popcll(m & lt);
                kout[pos] = k;
                vout[pos] = v;
                atomicAdd(&hist[(uint32_t)k & mask], 1u);
            }
            carry += tot;
            __syncthreads();
        }
        if (t == 0) {
            unit_len[wb] = carry;
            if (carry) atomicAdd(n_total, carry);
        }
    }
    __syncthreads();
    for (int d = t; d < ndig; d += 256) counts[(size_t)d * units + wb] = hist[d];
}

// One workgroup per bin.  The bin's run [lo, hi) of the bin-sorted list (two binary searches over
// the sorted keys) holds its pairs in (depth, index) order with their tile masks; each of the bin's
// (up to) four tiles gets the stable sub-list of the pairs whose mask has its bit, written at
// out_base + 4 lo + b (hi - lo) (capacity 4x the bin pairs, so no global scan), and its range
// (rasterizer_impl.cu:105-127 identifyTileRanges).  Every tile of the grid gets a range, so the
// ranges need no clearing.  n_dev: device-side count of a filtered (phase B) list.
template <typename K>
__global__ __launch_bounds__(256) void k_expand(uint32_t n_host, const uint32_t* __restrict__ n_dev,
                                                const K* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                int gx, int gy, uint32_t out_base, uint32_t* __restrict__ point_list,
                                                uint2* __restrict__ ranges, const uint32_t* __restrict__ open_bits) {
    __shared__ uint32_t wsum[4][4];
    const int bgx = bins_x(gx);
    const int bin = blockIdx.x;
    const int X = bin % bgx, Y = bin / bgx;
    if (open_bits) {  // phase B: a bin whose tiles all closed in phase A holds no pair, and its
                      // tiles' ranges were cleared with the frame's: nothing to search or write
        bool any = false;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int tx = 2 * X + (b & 1), ty = 2 * Y + (b >> 1);
            if (tx < gx && ty < gy) {
                const uint32_t tile = (uint32_t)(ty * gx + tx);
                any = any || ((open_bits[tile >> 5] >> (tile & 31)) & 1u);
            }
        }
        if (!any) return;  // block-uniform
    }
    const uint32_t n = n_dev ? *n_dev : n_host;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // 256-ary searches for the bin's first pair and the next bin's: each round probes 256 evenly
    // spaced keys at once (one load latency per round, 3 rounds for 16M pairs, instead of a 24-deep
    // chain of dependent loads), and the two searches share their rounds (their loads in flight
    // together)
    const uint32_t v0 = (uint32_t)bin, v1 = (uint32_t)bin + 1u;
    uint32_t l0 = 0, h0 = n, l1 = 0, h1 = n;  // answers in [l, h]
    while (h0 - l0 > 1 || h1 - l1 > 1) {
        const bool a0 = h0 - l0 > 1, a1 = h1 - l1 > 1;
        const uint32_t s0 = (h0 - l0 + 255) / 256, s1 = (h1 - l1 + 255) / 256;
        const uint32_t i0 = l0 + (uint32_t)t * s0, i1 = l1 + (uint32_t)t * s1;
        const bool q0 = a0 && i0 < h0, q1 = a1 && i1 < h1;
        const uint32_t k0 = q0 ? (uint32_t)keys[i0] : 0u, k1 = q1 ? (uint32_t)keys[i1] : 0u;
        const int c0 = __syncthreads_count(q0 && k0 < v0);  // probes below v
        const int c1 = __syncthreads_count(q1 && k1 < v1);
        // probes 0..c-1 are below v: the answer lies in (l + (c-1) step, l + c step]
        if (a0) {
            const uint32_t nl = c0 == 0 ? l0 : l0 + (uint32_t)(c0 - 1) * s0 + 1u;
            h0 = min(h0, l0 + (uint32_t)c0 * s0);
            l0 = nl;
        }
        if (a1) {
            const uint32_t nl = c1 == 0 ? l1 : l1 + (uint32_t)(c1 - 1) * s1 + 1u;
            h1 = min(h1, l1 + (uint32_t)c1 * s1);
            l1 = nl;
        }
    }
    {
        const uint32_t k0 = l0 < h0 ? (uint32_t)keys[l0] : 0u, k1 = l1 < h1 ? (uint32_t)keys[l1] : 0u;
        if (l0 < h0) l0 += k0 < v0 ? 1u : 0u;  // block-uniform: every thread read the same key
        if (l1 < h1) l1 += k1 < v1 ? 1u : 0u;
    }
    const uint32_t lo = l0, hi = l1;
    const uint32_t len = hi - lo;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t dst0 = out_base + 4u * lo;
    uint32_t carry[4] = {0u, 0u, 0u, 0u};
    for (uint32_t r0 = 0; r0 < len; r0 += 256) {
        const uint32_t j = r0 + (uint32_t)t;
        const uint32_t v = j < len ? vals[lo + j] : 0u;
        const uint32_t m = j < len ? v >> BIN_SHIFT : 0u;
        uint32_t rank[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint64_t bal = __ballot((m >> b) & 1u);
            rank[b] = (uint32_t)__popcll(bal & lt);
            if (lane == 0) wsum[w][b] = (uint32_t)__popcll(bal);
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 4; b++) {
            uint32_t pre = carry[b], tot = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                pre += i < w ? wsum[i][b] : 0u;
                tot += wsum[i][b];
            }
            if ((m >> b) & 1u) point_list[dst0 + (uint32_t)b * len + pre + rank[b]] = v & BIN_ID_MASK;
            carry[b] += tot;
        }
        __syncthreads();
    }
    if (t < 4) {
        const int tx = 2 * X + (t & 1), ty = 2 * Y + (t >> 1);
        const uint32_t s = dst0 + (uint32_t)t * len;
        if (tx < gx && ty < gy) ranges[ty * gx + tx] = make_uint2(s, s + carry[t]);
    }
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

void launch_preprocess_views(const PreArgs& a, const PreViews& vs, hipStream_t st) {
    const int rows = a.n_out > a.P ? a.n_out : a.P;
    if (rows == 0 || vs.V <= 0) return;
    const dim3 grid(blocks_for(rows), vs.V);
    switch (a.colors_precomp ? 0 : a.D) {
        case 0: k_preprocess_views<0><<<grid, 256, 0, st>>>(a, vs); break;
        case 1: k_preprocess_views<1><<<grid, 256, 0, st>>>(a, vs); break;
        case 2: k_preprocess_views<2><<<grid, 256, 0, st>>>(a, vs); break;
        default: k_preprocess_views<3><<<grid, 256, 0, st>>>(a, vs); break;
    }
}

void launch_preprocess(const PreArgs& a, hipStream_t st) {
    const int rows = a.n_out > a.P ? a.n_out : a.P;
    if (rows == 0) return;
    const int nb = blocks_for(rows);
    // (staging the SH coefficients through LDS was measured slower: 1.68 vs 1.66 ms per step)
    switch (a.colors_precomp ? 0 : a.D) {
        case 0: k_preprocess<0><<<nb, 256, 0, st>>>(a); break;
        case 1: k_preprocess<1><<<nb, 256, 0, st>>>(a); break;
        case 2: k_preprocess<2><<<nb, 256, 0, st>>>(a); break;
        default: k_preprocess<3><<<nb, 256, 0, st>>>(a); break;
    }
}

template <typename K>
bool launch_duplicate(const DupArgs<K>& d, hipStream_t st) {
    if (d.P == 0 || d.nwin == 0 || d.win > (uint32_t)kSortMaxUnit) {  // win comes from radix_sort_plan
        if (d.zero && d.nzero > 0) (void)hipMemsetAsync(d.zero, 0, (size_t)d.nzero * sizeof(uint32_t), st);
        return false;
    }
    const bool second = d.first_b && d.nwin_b > 0 && d.win_b > 0 && d.win_b <= (uint32_t)kSortMaxUnit;
    if (!d.starts_done)
        k_window_starts<<<blocks_for(d.P), 256, 0, st>>>(d.P, d.offsets, d.pair0, d.win, d.nwin, d.first, d.pair0_b,
                                                         second ? d.win_b : 1u, second ? d.nwin_b : 0,
                                                         d.first_b, d.zero, d.zero ? d.nzero : 0);
    auto kern = d.open_bits ? k_duplicate<K, true> : k_duplicate<K, false>;
    const bool ord = d.open_bits && d.order_out && d.order_cost && d.order_flag && d.order_T > 0;
    kern<<<d.nwin + (ord ? 1 : 0), 256, 0, st>>>(d.P, d.idx_sorted, d.offsets, d.splats, d.radii, d.gx, d.gy, d.cull,
                                                  d.first, d.pair0, d.win, d.L, d.keys, d.vals, d.dbits, d.counts,
                                                  d.nwin, d.open_bits, d.unit_len, d.n_total, ord ? d.order_cost : nullptr,
                                                  ord ? d.order_out : nullptr, d.order_flag, d.order_T);
    return !d.starts_done && second;
}
template bool launch_duplicate<uint16_t>(const DupArgs<uint16_t>&, hipStream_t);
template bool launch_duplicate<uint32_t>(const DupArgs<uint32_t>&, hipStream_t);

template <typename K>
void launch_expand(uint32_t L, const uint32_t* n_dev, const K* keys, const uint32_t* vals, int gx, int gy,
                   uint32_t out_base, uint32_t* point_list, uint2* ranges, const uint32_t* open_bits, hipStream_t st) {
    const int nb = bins_x(gx) * bins_y(gy);
    if (nb > 0) k_expand<K><<<nb, 256, 0, st>>>(L, n_dev, keys, vals, gx, gy, out_base, point_list, ranges, open_bits);
}
template void launch_expand<uint16_t>(uint32_t, const uint32_t*, const uint16_t*, const uint32_t*, int, int, uint32_t,
                                      uint32_t*, uint2*, const uint32_t*, hipStream_t);
template void launch_expand<uint32_t>(uint32_t, const uint32_t*, const uint32_t*, const uint32_t*, int, int, uint32_t,
                                      uint32_t*, uint2*, const uint32_t*, hipStream_t);

void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st) {
    if (P == 0) return;
    k_mark_visible<<<blocks_for(P), 256, 0, st>>>(P, means3D, view, present);
}

}  // namespace rr
