// rr_blend_fwd.hip — per-tile front-to-back alpha blend, forward (forward.cu:251-369).
//
// The kernel is VALU-issue bound (SQ counters: the SIMDs issue a VALU op nearly every cycle), so
// it is written for CDNA4's packed fp32 pipe: every lane owns PAIRS x 2 pixels of one column and
// evaluates each pair of pixels with v_pk_{fma,mul,add}_f32 (one instruction, two pixels).  The
// two pixels of a pair share dx (same column), so the x-terms of the falloff are scalar.
//
// Layout: NW wave64s per 16x16 tile (NW = 2: one pixel pair per lane; NW = 1: two pairs), lane l
// of wave w owns column l%16 and rows l/16 + 4k, k in the wave's share of {0,1,2,3}; pair p holds
// rows (l/16 + 8p' + {0, 4}) with p' = w * PAIRS + p.
//   * Each round stages 64*NW records (48 B, rr_common.hpp Splat) in LDS; the next round's
//     records are prefetched into registers while the current one is blended.
//   * A round starts only if some pixel of the tile is still open (__syncthreads_count,
//     forward.cu:302-304); inside a round a wave leaves as soon as all its pixels are saturated.
//   * The falloff uses blend_power/blend_G (rr_common.hpp), the same op sequence as the backward.
//   * n_contrib: a pixel that is still open has processed every pair before the current one, so its
//     contributor count is just (pair index + 1) — no per-pixel counter.
#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Scalar-record stream (SC): every lane of a wave blends the same pair at the same time, so the
// pair's id and its 48-B Splat are wave-uniform.  They are read through the constant address space
// (s_load into SGPRs, straight into the VALU ops as scalar operands): no LDS staging, no
// workgroup barrier per round, no VGPRs for the record, and each wave walks its tile's list on its
// own (a wave whose pixels have all saturated stops without waiting for the others).
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const v4f cv4f;
typedef __attribute__((address_space(4))) const uint32_t cu32;
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const u2v cu2v;

__device__ __forceinline__ uint2 load_range(const uint2* p, int i, bool scalar) {
    if (scalar) {
        const u2v v = ((cu2v*)p)[i];
        return make_uint2(v.x, v.y);
    }
    return p[i];
}

// AUX: also blend the per-Gaussian view-space normals into out_normal (RR_FLAG_AUX_NORMAL).
template <int NW, bool AUX, bool SC>
__global__ __launch_bounds__(64 * NW) void k_blend_fwd(BlendFwdArgs a) {
#pragma clang fp contract(off)  // exactly blend_power's rounding: every fma below is explicit
    // NW = 4 (phase B of early-stop binning: few open tiles with long lists, so per-tile latency
    // rules): each lane owns ONE pixel, the packed pair's second half is a masked dummy
    constexpr bool HALF = NW == 4;
    constexpr int PAIRS = HALF ? 1 : 2 / NW;  // pixel pairs per lane
    constexpr int B = 64 * NW;                // records per round
#ifndef RR_FWD_GROUP
#define RR_FWD_GROUP 4
#endif
    constexpr int kGroup = RR_FWD_GROUP;      // pairs whose alphas are formed together (8: neutral)
    static_assert(B % kGroup == 0, "group size");
    const int ntiles = a.gx * a.gy;
    const int tile = a.order ? (int)a.order[blockIdx.x] : xcd_tile(blockIdx.x, ntiles);
    if (a.phase == kBlendPhaseB && !a.open[tile]) return;  // finished in phase A
    (void)ntiles;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int px = tx * TILE_X + (lane & 15);
    const float pfx = (float)px;

    __shared__ float4 s_a[SC ? 1 : B];
    __shared__ float4 s_b[SC ? 1 : B];
    __shared__ float4 s_c[SC ? 1 : B];
    __shared__ float4 s_n[(AUX && !SC) ? B : 1];

    // per pixel pair: T (transmittance), om (1 while the pixel is open, 0 once saturated: it zeroes
    // alpha, so a closed pixel neither blends nor changes T), colour / depth accumulators
    int py[PAIRS][2];
    f2 pfy[PAIRS], T[PAIRS], om[PAIRS], C0[PAIRS], C1[PAIRS], C2[PAIRS], Dp[PAIRS];
    f2 N0[PAIRS], N1[PAIRS], N2[PAIRS];  // AUX only
    uint32_t last[PAIRS][2];
#pragma unroll
    for (int p = 0; p < PAIRS; p++) {
        const int row0 = ty * TILE_Y + (lane >> 4) + (HALF ? 4 * w : 8 * (w * PAIRS + p));
        py[p][0] = row0;
        py[p][1] = HALF ? 0x3fffffff : row0 + 4;  // HALF: never inside the image
        pfy[p] = f2{(float)row0, (float)(HALF ? row0 : row0 + 4)};
        T[p] = f2{1.f, 1.f};
        om[p] = f2{(px < a.W && row0 < a.H) ? 1.f : 0.f, (px < a.W && py[p][1] < a.H) ? 1.f : 0.f};
        C0[p] = C1[p] = C2[p] = Dp[p] = f2{0.f, 0.f};
        N0[p] = N1[p] = N2[p] = f2{0.f, 0.f};
        last[p][0] = last[p][1] = 0;
    }
    const size_t HW = (size_t)a.H * a.W;
    uint2 range = load_range(a.ranges, tile, SC);
    uint32_t koff = 0;  // contributor index of the list's first pair
    if (a.phase == kBlendPhaseB) {
        // resume: the state phase A left for this open tile (raw colour / depth sums, T, last
        // contributor, saturated flag), then continue over the phase-B list
        koff = range.y - range.x;
        range = load_range(a.ranges_b, tile, SC);
#pragma unroll
        for (int p = 0; p < PAIRS; p++)
#pragma unroll
            for (int k = 0; k < 2; k++) {
                if (px < a.W && py[p][k] < a.H) {
                    const int pix = a.W * py[p][k] + px;
                    const uint32_t nc = a.n_contrib[pix];
                    const float tv = a.final_T[pix], c0 = a.out_color[pix], c1 = a.out_color[HW + pix],
                                c2 = a.out_color[2 * HW + pix], dv = a.out_depth[pix];
                    if (k) {
                        T[p].y = tv; C0[p].y = c0; C1[p].y = c1; C2[p].y = c2; Dp[p].y = dv;
                        om[p].y = (nc & kDoneBit) ? 0.f : 1.f;
                    } else {
                        T[p].x = tv; C0[p].x = c0; C1[p].x = c1; C2[p].x = c2; Dp[p].x = dv;
                        om[p].x = (nc & kDoneBit) ? 0.f : 1.f;
                    }
                    if (AUX) {
                        const float n0 = a.out_normal[pix], n1 = a.out_normal[HW + pix], n2 = a.out_normal[2 * HW + pix];
                        if (k) { N0[p].y = n0; N1[p].y = n1; N2[p].y = n2; }
                        else { N0[p].x = n0; N1[p].x = n1; N2[p].x = n2; }
                    }
                    last[p][k] = nc & ~kDoneBit;
                }
            }
    }
    const int n = (int)(range.y - range.x);
    auto all_closed = [&]() {
        bool c = true;
#pragma unroll
        for (int p = 0; p < PAIRS; p++) c = c && om[p].x == 0.f && om[p].y == 0.f;
        return c;
    };

    // one pair of the group: falloff + alpha of both pixels of every pixel pair (blend_power's op
    // sequence; the x-terms are shared by the two pixels of a pair)
    auto alpha_of = [&](const float ax, const float ay, const float acx, const float acy, const float bcz,
                        const float bop, f2 (&al_out)[PAIRS]) {
        const float dx = ax - pfx;
        const float cxdx2 = (acx * dx) * dx;
        const float wdx = acy * dx;
#pragma unroll
        for (int p = 0; p < PAIRS; p++) {
            const f2 dy = f2{ay, ay} - pfy[p];
            const f2 tq = fma2(f2{bcz, bcz} * dy, dy, f2{cxdx2, cxdx2});
            const f2 u = f2{wdx, wdx} * dy;
            const f2 power = fma2(f2{-0.5f, -0.5f}, tq, -u);
            const f2 pl = power * f2{kLog2e, kLog2e};
            f2 al = f2{bop, bop} * f2{__builtin_amdgcn_exp2f(pl.x), __builtin_amdgcn_exp2f(pl.y)};
            // forward.cu:333-336: skip power > 0 and alpha < 1/255 (alpha := 0)
            al.x = (power.x <= 0.0f && fminf(0.99f, al.x) >= 1.0f / 255.0f) ? fminf(0.99f, al.x) : 0.f;
            al.y = (power.y <= 0.0f && fminf(0.99f, al.y) >= 1.0f / 255.0f) ? fminf(0.99f, al.y) : 0.f;
            al_out[p] = al;
        }
    };
    // the sequential blend of one pair into every pixel pair (forward.cu:337-349)
    auto blend_one = [&](const f2 (&alg)[PAIRS], const float bdepth, const float cr, const float cg, const float cb,
                         const float4 nv, const uint32_t k1) {
#pragma unroll
        for (int p = 0; p < PAIRS; p++) {
            const f2 al = alg[p] * om[p];
            const f2 testT = T[p] * (f2{1.f, 1.f} - al);
            // forward.cu:337-341: saturation closes the pixel without blending this Gaussian
            const bool sat0 = testT.x < 0.0001f, sat1 = testT.y < 0.0001f;
            f2 wgt = al * T[p];
            wgt.x = sat0 ? 0.f : wgt.x;
            wgt.y = sat1 ? 0.f : wgt.y;
            C0[p] = fma2(f2{cr, cr}, wgt, C0[p]);
            C1[p] = fma2(f2{cg, cg}, wgt, C1[p]);
            C2[p] = fma2(f2{cb, cb}, wgt, C2[p]);
            Dp[p] = fma2(f2{bdepth, bdepth}, wgt, Dp[p]);
            if (AUX) {
                N0[p] = fma2(f2{nv.x, nv.x}, wgt, N0[p]);
                N1[p] = fma2(f2{nv.y, nv.y}, wgt, N1[p]);
                N2[p] = fma2(f2{nv.z, nv.z}, wgt, N2[p]);
            }
            T[p].x = sat0 ? T[p].x : testT.x;
            T[p].y = sat1 ? T[p].y : testT.y;
            om[p].x = sat0 ? 0.f : om[p].x;
            om[p].y = sat1 ? 0.f : om[p].y;
            last[p][0] = wgt.x > 0.f ? k1 : last[p][0];
            last[p][1] = wgt.y > 0.f ? k1 : last[p][1];
        }
    };

    if constexpr (SC) {
        cu32* plist = (cu32*)a.point_list + range.x;  // padded by kPointListPad entries
        cv4f* recs = (cv4f*)a.splats;
        cv4f* nrm = (cv4f*)a.normals;
        for (int j0 = 0; j0 < n; j0 += kGroup) {
            if (__all(all_closed())) break;
            uint32_t id[kGroup];
#pragma unroll
            for (int uu = 0; uu < kGroup; uu++) id[uu] = plist[j0 + uu];
#pragma unroll
            for (int uu = 1; uu < kGroup; uu++) id[uu] = (j0 + uu < n) ? id[uu] : id[0];  // past the list end
            v4f ra[kGroup], rb[kGroup], rc[kGroup], rn[kGroup];
#pragma unroll
            for (int uu = 0; uu < kGroup; uu++) {
                ra[uu] = recs[3 * id[uu]];
                rb[uu] = recs[3 * id[uu] + 1];
                rc[uu] = recs[3 * id[uu] + 2];
                if (AUX) rn[uu] = nrm[id[uu]];
            }
            f2 alq[kGroup][PAIRS];
#pragma unroll
            for (int uu = 0; uu < kGroup; uu++)
                alpha_of(ra[uu].x, ra[uu].y, ra[uu].z, ra[uu].w, rb[uu].x, rb[uu].y, alq[uu]);
#pragma unroll
            for (int uu = 0; uu < kGroup; uu++) {
                if (j0 + uu >= n) break;
                const float4 nv = AUX ? make_float4(rn[uu].x, rn[uu].y, rn[uu].z, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
                blend_one(alq[uu], rb[uu].z, rc[uu].x, rc[uu].y, rc[uu].z, nv, koff + (uint32_t)(j0 + uu + 1));
            }
        }
    } else {
    float4 na = make_float4(0.f, 0.f, 0.f, 0.f), nb = na, nc = na, nn = na;
    if (t < n) {
        const uint32_t id = a.point_list[range.x + t];
        load_splat(a.splats, id, na, nb, nc);
        if (AUX) nn = a.normals[id];
    }
    for (int base = 0; base < n; base += B) {
        if (__syncthreads_count(all_closed()) == B) break;
        if (base + t < n) {
            s_a[t] = na;
            s_b[t] = nb;
            s_c[t] = nc;
            if (AUX) s_n[t] = nn;
        }
        __syncthreads();
        if (base + B + t < n) {
            const uint32_t id = a.point_list[range.x + base + B + t];
            load_splat(a.splats, id, na, nb, nc);
            if (AUX) nn = a.normals[id];
        }
        const int cnt = min(B, n - base);
        for (int j0 = 0; j0 < cnt; j0 += kGroup) {
            if (__all(all_closed())) break;
            // groups of kGroup pairs: the falloff / alpha of the group (independent of T) are formed
            // first, so their exp / compare chains overlap; only the blend below is sequential.
            // A slot past cnt (stale / uninitialised LDS, j < B still) is computed but never blended.
            f2 alq[kGroup][PAIRS];
#pragma unroll
            for (int uu = 0; uu < kGroup; uu++) {
                const float4 A = s_a[j0 + uu];
                const float4 Bv = s_b[j0 + uu];
                alpha_of(A.x, A.y, A.z, A.w, Bv.x, Bv.y, alq[uu]);
            }
#pragma unroll
            for (int uu = 0; uu < kGroup; uu++) {
                const int j = j0 + uu;
                if (j >= cnt) break;
                const float4 Bv = s_b[j];
                const float4 Cc = s_c[j];
                blend_one(alq[uu], Bv.z, Cc.x, Cc.y, Cc.z, AUX ? s_n[j] : make_float4(0.f, 0.f, 0.f, 0.f),
                          koff + (uint32_t)(base + j + 1));
            }
        }
        __syncthreads();
    }
    }  // LDS-staged rounds

    if (a.phase == kBlendPhaseA) {
        // still open: leave the raw state for phase B (no background yet)
        const bool closed = __syncthreads_count(all_closed()) == B;
        if (threadIdx.x == 0) a.open[tile] = closed ? 0 : 1;
        if (!closed) {
#pragma unroll
            for (int p = 0; p < PAIRS; p++)
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    if (px < a.W && py[p][k] < a.H) {
                        const int pix = a.W * py[p][k] + px;
                        const bool done = (k ? om[p].y : om[p].x) == 0.f;
                        a.final_T[pix] = k ? T[p].y : T[p].x;
                        a.n_contrib[pix] = last[p][k] | (done ? kDoneBit : 0u);
                        a.out_color[pix] = k ? C0[p].y : C0[p].x;
                        a.out_color[HW + pix] = k ? C1[p].y : C1[p].x;
                        a.out_color[2 * HW + pix] = k ? C2[p].y : C2[p].x;
                        a.out_depth[pix] = k ? Dp[p].y : Dp[p].x;
                        if (AUX) {
                            a.out_normal[pix] = k ? N0[p].y : N0[p].x;
                            a.out_normal[HW + pix] = k ? N1[p].y : N1[p].x;
                            a.out_normal[2 * HW + pix] = k ? N2[p].y : N2[p].x;
                        }
                    }
                }
            return;
        }
    }
    uint32_t m = 0;
#pragma unroll
    for (int p = 0; p < PAIRS; p++)
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (px < a.W && py[p][k] < a.H) {
                const float Tk = k ? T[p].y : T[p].x;
                m = max(m, last[p][k]);
                const int pix = a.W * py[p][k] + px;
                a.final_T[pix] = Tk;
                a.n_contrib[pix] = last[p][k];
                a.out_color[pix] = (k ? C0[p].y : C0[p].x) + Tk * a.bg[0];
                a.out_color[HW + pix] = (k ? C1[p].y : C1[p].x) + Tk * a.bg[1];
                a.out_color[2 * HW + pix] = (k ? C2[p].y : C2[p].x) + Tk * a.bg[2];
                a.out_depth[pix] = k ? Dp[p].y : Dp[p].x;
                if (AUX) {
                    a.out_normal[pix] = k ? N0[p].y : N0[p].x;
                    a.out_normal[HW + pix] = k ? N1[p].y : N1[p].x;
                    a.out_normal[2 * HW + pix] = k ? N2[p].y : N2[p].x;
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

template <bool SC>
void launch_blend_fwd_t(const BlendFwdArgs& a, hipStream_t st) {
    const int T = a.gx * a.gy;
    const bool aux = a.out_normal != nullptr;
    if (a.phase == kBlendPhaseB && blend_fwd_b_waves() == 4) {
        if (aux) k_blend_fwd<4, true, SC><<<T, 256, 0, st>>>(a);
        else k_blend_fwd<4, false, SC><<<T, 256, 0, st>>>(a);
    } else if (blend_fwd_waves() == 1) {
        if (aux) k_blend_fwd<1, true, SC><<<T, 64, 0, st>>>(a);
        else k_blend_fwd<1, false, SC><<<T, 64, 0, st>>>(a);
    } else {
        if (aux) k_blend_fwd<2, true, SC><<<T, 128, 0, st>>>(a);
        else k_blend_fwd<2, false, SC><<<T, 128, 0, st>>>(a);
    }
}

void launch_blend_fwd(const BlendFwdArgs& a, hipStream_t st) {
    if (a.gx * a.gy == 0) return;
    const int impl = blend_fwd_impl(a.phase == kBlendPhaseB);
    if (impl == 2) launch_blend_fwd_s(a, blend_fwd_s_waves(a.phase == kBlendPhaseB), st);
    else if (impl == 1) launch_blend_fwd_t<true>(a, st);
    else launch_blend_fwd_t<false>(a, st);
}

}  // namespace rr
