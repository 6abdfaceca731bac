// rr_blend_fwd_s.hip — per-tile front-to-back alpha blend, forward (forward.cu:251-369), scalar-
// record / scalar-arithmetic variant.
//
// Written for the scalar VALU with as few vector instructions per (pixel, pair) as possible (a
// packed v_pk_fma_f32 costs ~2x a plain v_fma_f32 on gfx950 and needs operand shuffles, so packing
// buys nothing here):
//   * every lane of a wave blends the same pair at the same time, so the pair's 48-B Splat is
//     wave-uniform.  The workgroup stages a round of 64 NW records in LDS (one per thread,
//     gathered by id) while the previous round blends, and the waves read them as LDS
//     broadcasts — one exposed gather latency per tile: the records come from a 48 B x P array
//     that no L2 holds, ~1-2 us away (round 2 measured scalar loads per group of pairs, batched
//     or software-pipelined, at 0.203-0.229 vs 0.176 ms/step for this staging);
//   * alpha in log2 units from the pre-scaled conic (rr_common.hpp blend_e2): per pixel 3 fma-class
//     ops and one exp2;
//   * a lane owns PIX pixels of one column (rows l/16 + 4k): the x-terms of the falloff are
//     computed once per lane and pair;
//   * no per-pixel "open" flag: a saturated pixel keeps -T (T >= 1e-4 > 0 while open), so every
//     later pair finds T*(1 - alpha) < 1e-4, re-saturates and changes nothing (wgt = 0, T kept by
//     one select with a -|x| source modifier); the masks of the compares combine on the scalar unit;
//   * a pixel row k whose 16 x 4 pixels are all closed (or that no lane reaches with alpha >=
//     1/255) skips the pair's blend with a uniform branch; a wave leaves when all its pixels closed.
// Measured (tools/fwd_trace.py, per-wave s_memrealtime records): phase A runs ~6 waves per SIMD
// for ~2/3 of its span, then drains; a wave walks ~100 pairs (its 8 rows saturate) in ~40 us.
#include <algorithm>

#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

typedef float v4f __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const u2v cu2v_s;

// NW waves per 16x16 tile, PIX = 4/NW pixels per lane: lane l of wave w owns column l%16 and rows
// l/16 + 4*(w*PIX + k), k < PIX.  G pairs per group (their alphas formed before the blend).
template <int NW, bool AUX>
#ifndef RR_FWD_S_OCC
#define RR_FWD_S_OCC 1
#endif
__global__ __launch_bounds__(64 * NW, RR_FWD_S_OCC) void k_blend_fwd_s(BlendFwdArgs a) {
#pragma clang fp contract(off)  // blend_e2's rounding: every fma below is explicit
    constexpr int PIX = 4 / NW;
#ifndef RR_FWD_S_GROUP
#define RR_FWD_S_GROUP 3
#endif
#ifndef RR_FWD_TRACE
#define RR_FWD_TRACE 0
#endif
    constexpr int G = RR_FWD_S_GROUP;
    const int ntiles = a.gx * a.gy;
    if ((int)blockIdx.x >= ntiles) {  // the workspace clear (block-uniform, after every tile's block)
        const size_t nb = gridDim.x - (unsigned)ntiles, i0 = (blockIdx.x - (unsigned)ntiles) * (size_t)blockDim.x;
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        for (size_t i = i0 + threadIdx.x; i < a.clear_n4; i += nb * blockDim.x) a.clear[i] = z;
        return;
    }
    const int tile = xcd_tile(blockIdx.x, ntiles);
    if (a.phase == kBlendPhaseB && !a.open[tile]) return;  // finished in phase A
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int px = tx * TILE_X + (lane & 15);
    const float pfx = (float)px;
    const size_t HW = (size_t)a.H * a.W;

    int py[PIX];
    float pfy[PIX], T[PIX], C0[PIX], C1[PIX], C2[PIX], Dp[PIX], N0[PIX], N1[PIX], N2[PIX];
    uint32_t last[PIX];
    bool inside[PIX];
#pragma unroll
    for (int k = 0; k < PIX; k++) {
        py[k] = ty * TILE_Y + (lane >> 4) + 4 * (w * PIX + k);
        pfy[k] = (float)py[k];
        inside[k] = px < a.W && py[k] < a.H;
        T[k] = inside[k] ? 1.f : -1.f;  // T < 0: closed (pixels outside the image start closed)
        C0[k] = C1[k] = C2[k] = Dp[k] = N0[k] = N1[k] = N2[k] = 0.f;
        last[k] = 0;
    }
    const u2v r0 = ((cu2v_s*)a.ranges)[tile];
    uint32_t lo = r0.x, hi = r0.y;
    uint32_t koff = 0;  // contributor index of the list's first pair
    if (a.phase == kBlendPhaseB) {
        // resume from the state phase A left for this open tile, then walk the phase-B list
        koff = hi - lo;
        const u2v rb = ((cu2v_s*)a.ranges_b)[tile];
        lo = rb.x;
        hi = rb.y;
#pragma unroll
        for (int k = 0; k < PIX; k++) {
            if (inside[k]) {
                const int pix = a.W * py[k] + px;
                const uint32_t nc = a.n_contrib[pix];
                T[k] = (nc & kDoneBit) ? -a.final_T[pix] : a.final_T[pix];
                C0[k] = a.out_color[pix];
                C1[k] = a.out_color[HW + pix];
                C2[k] = a.out_color[2 * HW + pix];
                Dp[k] = a.out_depth[pix];
                if (AUX) {
                    N0[k] = a.out_normal[pix];
                    N1[k] = a.out_normal[HW + pix];
                    N2[k] = a.out_normal[2 * HW + pix];
                }
                last[k] = nc & ~kDoneBit;
            }
        }
        // retire the resume loads here: left pending, the compiler's wait analysis carries them
        // into the pair loop and waits for the next round's record prefetch at every group
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    const int n = (int)(hi - lo);
#if RR_FWD_TRACE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    int walked = 0;
#endif

    // One group of G pairs: their alphas first (independent of T), then the sequential blend.
    // ra/rb/rc/rn: the pairs' records as wave-uniform values (SGPR operands).
    auto blend_group = [&](int j0, int jlim, const v4f (&ra)[G], const v4f (&rb)[G], const v4f (&rc)[G],
                           const v4f (&rn)[G]) {
        bool open[PIX];  // as of the group's start (only used to skip work)
#pragma unroll
        for (int k = 0; k < PIX; k++) open[k] = T[k] > 0.f;
        // alphas of the group (independent of T): forward.cu:329-336 as blend_e2 (rr_common.hpp)
        float al[G][PIX];
        bool ok[G][PIX];
        uint64_t okm[G][PIX];  // ok as a wave mask (ballots of the compares themselves: v_cmp into SGPRs)
        P2X px2[G];
#pragma unroll
        for (int u = 0; u < G; u++) px2[u] = blend_p2_x(ra[u].z, ra[u].w, rb[u].y, ra[u].x - pfx);
#pragma unroll
        for (int k = 0; k < PIX; k++) {
#pragma unroll
            for (int u = 0; u < G; u++) {
                const float e2 = blend_e2(px2[u], rb[u].x, ra[u].y - pfy[k]);
                const float a99 = fminf(0.99f, __builtin_amdgcn_exp2f(e2));
                // non-short-circuit: both compares become lane masks combined on the scalar unit
                ok[u][k] = (e2 <= rb[u].y) & (a99 >= 1.0f / 255.0f) & open[k];
                okm[u][k] = __builtin_amdgcn_ballot_w64(e2 <= rb[u].y) &
                            __builtin_amdgcn_ballot_w64(a99 >= 1.0f / 255.0f) & __builtin_amdgcn_ballot_w64(open[k]);
                al[u][k] = a99;
            }
        }
#pragma unroll
        for (int u = 0; u < G; u++) {
            if (j0 + u >= jlim) break;
            const uint32_t k1 = koff + (uint32_t)(j0 + u + 1);
#pragma unroll
            for (int k = 0; k < PIX; k++) {
                if (!okm[u][k]) continue;  // this pixel row: nothing to blend
                const float alpha = ok[u][k] ? al[u][k] : 0.f;
                const float testT = T[k] * (1.f - alpha);
                // forward.cu:337-341: saturation closes the pixel without blending this Gaussian
                // (a closed pixel, T < 0, always lands here)
                const bool sat = testT < 0.0001f;
                const bool blend = ok[u][k] & !sat;
                const float wgt = sat ? 0.f : alpha * T[k];
                C0[k] = __builtin_fmaf(rc[u].x, wgt, C0[k]);
                C1[k] = __builtin_fmaf(rc[u].y, wgt, C1[k]);
                C2[k] = __builtin_fmaf(rc[u].z, wgt, C2[k]);
                Dp[k] = __builtin_fmaf(rb[u].z, wgt, Dp[k]);
                if (AUX) {
                    N0[k] = __builtin_fmaf(rn[u].x, wgt, N0[k]);
                    N1[k] = __builtin_fmaf(rn[u].y, wgt, N1[k]);
                    N2[k] = __builtin_fmaf(rn[u].z, wgt, N2[k]);
                }
                T[k] = sat ? -fabsf(T[k]) : testT;
                last[k] = blend ? k1 : last[k];
            }
        }
    };
    auto wave_open = [&]() {
        uint64_t any_open = 0;
#pragma unroll
        for (int k = 0; k < PIX; k++) any_open |= __builtin_amdgcn_ballot_w64(T[k] > 0.f);
        return any_open != 0;
    };
    // Records staged through LDS a round of 64 NW pairs at a time, the next round's gathered into
    // registers while this one blends (one exposed load latency per tile instead of one per group:
    // the records are gathered from a 48-B x P array no L2 holds).  Reads are wave-uniform LDS
    // broadcasts; the arithmetic is the scalar path's (blend_group) on VGPR operands.
    {
        constexpr int RND = 64 * NW;
        __shared__ v4f s_ra[RND], s_rb[RND], s_rc[RND], s_rn[AUX ? RND : 1];
        v4f pa = {}, pb = {}, pc = {}, pn = {};
        auto fetch = [&](int j) {
            if (j < n) {
                const uint32_t id = ((const uint32_t*)a.point_list)[lo + j];
                const v4f* r = (const v4f*)a.splats + 3 * (size_t)id;
                pa = r[0];
                pb = r[1];
                pc = r[2];
                if (AUX) pn = ((const v4f*)a.normals)[id];
            }
        };
        fetch(t);
        for (int r0 = 0; r0 < n; r0 += RND) {
            bool mine = false;
#pragma unroll
            for (int k = 0; k < PIX; k++) mine |= T[k] > 0.f;
            // every wave reaches this barrier each round (it also guards the LDS reuse)
            if (!__syncthreads_or(mine)) break;
            if (r0 + t < n) {
                s_ra[t] = pa;
                s_rb[t] = pb;
                s_rc[t] = pc;
                if (AUX) s_rn[t] = pn;
            }
            __syncthreads();
            fetch(r0 + RND + t);  // next round in flight while this one blends
            const int cnt = min(RND, n - r0);
            for (int j = 0; j < cnt; j += G) {
                if (!wave_open()) break;  // this wave's pixels all saturated
#if RR_FWD_TRACE
                walked = r0 + j + G;
#endif
                v4f ra[G], rb[G], rc[G], rn[G];
#pragma unroll
                for (int u = 0; u < G; u++) {
                    const int q = min(j + u, cnt - 1);
                    ra[u] = s_ra[q];
                    rb[u] = s_rb[q];
                    rc[u] = s_rc[q];
                    if (AUX) rn[u] = s_rn[q];
                }
                blend_group(r0 + j, r0 + cnt, ra, rb, rc, rn);
            }
        }
    }
#if RR_FWD_TRACE
    if (a.trace && lane == 0) {  // timing record of this wave (tools/fwd_trace.py)
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const int ntl = a.gx * a.gy;
        uint32_t* r = a.trace + 8 * ((size_t)(a.phase == kBlendPhaseB ? 4 * ntl : 0) + (size_t)blockIdx.x * NW + w);
        r[0] = (uint32_t)t_start;
        r[1] = (uint32_t)(t_start >> 32);
        r[2] = (uint32_t)t_end;
        r[3] = (uint32_t)(t_end >> 32);
        r[4] = (uint32_t)tile;
        r[5] = (uint32_t)min(walked, n);
        r[6] = (uint32_t)n;
        r[7] = (uint32_t)a.phase | ((uint32_t)w << 8) | ((uint32_t)NW << 16);
    }
#endif

    if (a.phase == kBlendPhaseA) {
        // still open somewhere in the tile: leave the raw state (no background) for phase B
        bool any_open = false;
#pragma unroll
        for (int k = 0; k < PIX; k++) any_open |= T[k] > 0.f;
        const bool tile_open = NW == 1 ? __builtin_amdgcn_ballot_w64(any_open) != 0
                                       : __syncthreads_or(any_open) != 0;
        if (threadIdx.x == 0) {
            a.open[tile] = tile_open ? 1 : 0;
            // phase B's open-tile bitmask (zeroed with the frame's ranges): replaces a one-workgroup
            // pass over the flags between the two phases
            if (tile_open) atomicOr(&a.open_bits[tile >> 5], 1u << (tile & 31));
        }
        if (tile_open) {
#pragma unroll
            for (int k = 0; k < PIX; k++) {
                if (px < a.W && py[k] < a.H) {
                    const int pix = a.W * py[k] + px;
                    a.final_T[pix] = fabsf(T[k]);
                    a.n_contrib[pix] = last[k] | (T[k] > 0.f ? 0u : kDoneBit);
                    a.out_color[pix] = C0[k];
                    a.out_color[HW + pix] = C1[k];
                    a.out_color[2 * HW + pix] = C2[k];
                    a.out_depth[pix] = Dp[k];
                    if (AUX) {
                        a.out_normal[pix] = N0[k];
                        a.out_normal[HW + pix] = N1[k];
                        a.out_normal[2 * HW + pix] = N2[k];
                    }
                }
            }
            return;
        }
    }
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < PIX; k++) {
        if (px < a.W && py[k] < a.H) {
            m = max(m, last[k]);
            const int pix = a.W * py[k] + px;
            const float Tk = fabsf(T[k]);
            a.final_T[pix] = Tk;
            a.n_contrib[pix] = last[k];
            a.out_color[pix] = C0[k] + Tk * bg0;
            a.out_color[HW + pix] = C1[k] + Tk * bg1;
            a.out_color[2 * HW + pix] = C2[k] + Tk * bg2;
            a.out_depth[pix] = Dp[k];
            if (AUX) {
                a.out_normal[pix] = N0[k];
                a.out_normal[HW + pix] = N1[k];
                a.out_normal[2 * HW + pix] = N2[k];
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if (NW == 1) {
        if (lane == 0) a.tile_max[tile] = m;
    } else {
        __shared__ uint32_t s_m[NW];
        if (lane == 0) s_m[w] = m;
        __syncthreads();
        if (t == 0) {
            uint32_t mm = s_m[0];
#pragma unroll
            for (int i = 1; i < NW; i++) mm = max(mm, s_m[i]);
            a.tile_max[tile] = mm;
        }
    }
}

namespace {
uint32_t* g_fwd_trace = nullptr;
}
void set_fwd_trace(void* dev_buf) { g_fwd_trace = static_cast<uint32_t*>(dev_buf); }

// Phase A (or a single-phase frame): 2 waves per tile (2 pixels per lane); phase B, whose few open
// tiles each set the launch's length: 4 (1 pixel per lane).
void launch_blend_fwd(const BlendFwdArgs& a_in, hipStream_t st) {
    BlendFwdArgs a = a_in;
    a.trace = g_fwd_trace;
    const int T = a.gx * a.gy;
    if (T == 0) return;
    const bool aux = a.out_normal != nullptr;
    const int waves = a.phase == kBlendPhaseB ? 4 : 2;
    // workspace clear: ~16 float4 stores per thread, at most 4096 extra workgroups
    const size_t per_block = (size_t)64 * waves * 16;
    const int nc = (a.clear && a.clear_n4) ? (int)std::min<size_t>((a.clear_n4 + per_block - 1) / per_block, 4096) : 0;
    const int nb = T + nc;
    if (waves == 4) {
        if (aux) k_blend_fwd_s<4, true><<<nb, 256, 0, st>>>(a);
        else k_blend_fwd_s<4, false><<<nb, 256, 0, st>>>(a);
    } else {
        if (aux) k_blend_fwd_s<2, true><<<nb, 128, 0, st>>>(a);
        else k_blend_fwd_s<2, false><<<nb, 128, 0, st>>>(a);
    }
}

}  // namespace rr
