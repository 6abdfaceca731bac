// rr_preprocess.hpp — one Gaussian's preprocess (forward.cu:144-246 preprocessCUDA semantics), shared
// by the forward preprocess kernels (rr_forward.hip) and by the per-Gaussian backward when it runs
// the next frame's preprocess on the parameters it has just updated (rr_backward.hip, rr_next_frame).
#pragma once
#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

// The culled outputs of row idx (radius 0, no pairs, the largest depth key).
__device__ __forceinline__ void preprocess_clear(const PreArgs& a, int idx) {
    a.radii[idx] = 0;
    a.tiles[idx] = make_uint2(0u, 0u);
    if (a.depth_keys) a.depth_keys[idx] = 0xffffffffu;  // culled Gaussians sort behind every visible one
}

// Everything after the frustum test, on inputs already in registers: p (mean), p_view, q / sc
// (raw in raw mode), o_in (opacity or its logit), c0 (SH DC or precomputed colour) and `rest`
// (SH coefficients 1.., read as VEC_REST ? 16-B loads of global memory : scalars, e.g. an LDS row).
template <int DEG, bool VEC_REST>
__device__ __forceinline__ uint2 preprocess_finish(const PreArgs& a, int idx, v3 p, v3 p_view, float4 q, v3 sc,
                                                   float o_in, v3 c0, const float* rest, bool& wide) {
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
        // the coefficients this degree uses, in 16-B loads (dword-aligned: a record is 180 or 192 B,
        // one lane's loads touch ~4x fewer cache lines per instruction than 45 dword loads)
        constexpr int NR = ((DEG + 1) * (DEG + 1) - 1) * 3;
        float rr[NR > 0 ? NR : 1];
        if (VEC_REST) {
            load_floats_u<NR>(rest, rr);
        } else {
#pragma unroll
            for (int i = 0; i < NR; i++) rr[i] = rest[i];
        }
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

// The sums of {pairs, rect tiles} of a block of 256 Gaussians go to a.block_sums[blk] and its
// wide-key flag to a.block_wide[blk] (plain stores; a single contended 64-bit atomic per block
// measured +37 us on 1M Gaussians).  256 threads; c / wide: this thread's Gaussian's values.
__device__ __forceinline__ void preprocess_block_sums(const PreArgs& a, int blk, uint2 c, bool wide) {
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
        a.block_sums[blk] = make_uint2(s_sum[0].x + s_sum[1].x + s_sum[2].x + s_sum[3].x,
                                       s_sum[0].y + s_sum[1].y + s_sum[2].y + s_sum[3].y);
        a.block_wide[blk] = s_wide[0] | s_wide[1] | s_wide[2] | s_wide[3];
    }
}

}  // namespace rr
