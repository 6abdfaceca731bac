// rr_blend.hip — per-tile alpha blending backward (backward.cu:389-547); the forward blend lives in
// rr_blend_fwd_s.hip.
//
// CDNA4 mapping.  A 16x16 tile is processed by one wave64, each lane owning PPL = 4 pixels of one
// column: lane l owns column l%16 of rows l/16 + 4q, q < 4.
//   * Each round stages 64 (tile, Gaussian) records (48 B each, rr_common.hpp Splat) in LDS; the
//     NEXT round's records go global -> LDS directly (global_load_lds_dwordx4 into the other half of
//     a double-buffered stage) while the current round is blended, so the dependent id -> record
//     gather latency is hidden behind compute and costs no prefetch VGPRs.
//   * All lanes read a staged record as an LDS broadcast and apply it to their PPL pixels.
//   * Each lane sums its PPL pixels' contributions in registers, the wave reduces the 9 gradient
//     components of two pairs together across its 64 lanes with DPP / permlane (no LDS), lane 63
//     parks the sums in LDS, and after each round ONE global float atomic per (tile, Gaussian,
//     component) is issued, consecutive lanes on consecutive components of a Gaussian's 64-B
//     accumulator line (the reference issues 9 atomics per contributing PIXEL).  Only the first
//     max(n_contrib) pairs of a tile are walked (recorded by the forward).
//   * Tiles are dispatched heaviest first (the order the phase-B duplicate or the prologue wrote),
//     else XCD-contiguously (the dispatcher sends block b to XCD b % 8), so tiles sharing Gaussians
//     share an L2.
#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

// Measured choices (interleaved A/B on the bench step, profiles/):
//   * records staged global -> LDS directly (global_load_lds_dwordx4, double-buffered) instead of
//     through 12 prefetch VGPRs and a ds_write: 159 -> 121 VGPRs, 3 -> 4 waves per SIMD; blend
//     backward 0.2427 / 0.2449 -> 0.2384 / 0.2401 ms (r05_bwd_glds_ab.jsonl; the same staging in the
//     forward blend measured slower, r05_fwd_glds_ab.jsonl);
//   * two pairs' gradient components reduced across the wave together (wave_sum18, 48 instead of
//     56 VALU per two pairs, bitwise the same sums) at 4 waves per SIMD (128 VGPRs): 0.2383 / 0.2361
//     -> 0.2260 / 0.2276 ms (r05_bwd_pair2_ab.jsonl);
//   * one wave per tile: 2 or 4 waves per tile, a software-pipelined pair loop and branch-free pixel
//     bodies all measured slower (r03_blend_bwd_waves_ab.jsonl, r03_blend_bwd_branchless_ab.jsonl).
__global__ __launch_bounds__(64, 4) void k_blend_bwd(BlendBwdArgs a) {
    constexpr int PPL = 4;
    constexpr int B = 64;
    const int ntiles = a.gx * a.gy;
    const int tile = a.order ? (int)a.order[blockIdx.x] : xcd_tile(blockIdx.x, ntiles);
    const int nmax = (int)a.tile_max[tile];  // pairs past this index were blended by no pixel
    if (nmax == 0) return;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int t = threadIdx.x;
    const int lane = t;
    const int px = tx * TILE_X + (lane & 15);
    const int py0 = ty * TILE_Y + (lane >> 4);
    const float pfx = (float)px;

    __shared__ float4 s_a2[2][B];
    __shared__ float4 s_b2[2][B];
    __shared__ float4 s_c2[2][B];
    __shared__ uint32_t s_id2[2][B];
    __shared__ float s_g[B * NGRAD];

    const size_t HW = (size_t)a.H * a.W;
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
    // The reference keeps accum_rec per channel (backward.cu:497-507) and only ever uses its dot
    // product with dL/dpix; by linearity the same convex-combination recurrence runs on the scalar
    // R = accum_rec . dL/dpix (8 fewer VALU ops and 4 fewer VGPRs per pixel and pair, and as well
    // conditioned as the per-channel form), advanced at each contributing pair right after its use.
    float T[PPL], tfbg[PPL], dp0[PPL], dp1[PPL], dp2[PPL], R[PPL];
    int last[PPL];
#pragma unroll
    for (int q = 0; q < PPL; q++) {
        const int py = py0 + 4 * q;
        const bool inside = px < a.W && py < a.H;
        const int pix = a.W * py + px;
        const float Tf = inside ? a.final_T[pix] : 0.f;
        T[q] = Tf;
        last[q] = inside ? (int)a.n_contrib[pix] : 0;
        dp0[q] = inside ? a.dL_dpix[pix] : 0.f;
        dp1[q] = inside ? a.dL_dpix[HW + pix] : 0.f;
        dp2[q] = inside ? a.dL_dpix[2 * HW + pix] : 0.f;
        // -T_final * (bg . dL/dpixel): numerator of the background term (backward.cu:521-524)
        tfbg[q] = -Tf * (bg0 * dp0[q] + bg1 * dp1[q] + bg2 * dp2[q]);
        R[q] = 0.f;
    }
    const uint2 range = a.ranges[tile];
    const uint2 range_b = a.ranges_b[tile];
    const uint32_t na_len = range.y - range.x;  // list = A-list ++ B-list (early-stop binning)
    auto pair_at = [&](int idx) -> uint32_t {
        return (uint32_t)idx < na_len ? range.x + idx : range_b.x + ((uint32_t)idx - na_len);
    };
    const float ddelx_dx = 0.5f * a.W;
    const float ddely_dy = 0.5f * a.H;

    // round r's records land in stage r & 1: issued (global -> LDS) one round ahead; the wave writes
    // its 64 lanes' records contiguously, which is the stage's layout (record t at [t])
    auto glds_round = [&](int buf, uint32_t id) {
        typedef __attribute__((address_space(1))) const void* gp;
        typedef __attribute__((address_space(3))) void* lp;
        const float4* src = reinterpret_cast<const float4*>(a.splats) + 3 * (size_t)id;
        __builtin_amdgcn_global_load_lds((gp)(src + 0), (lp)&s_a2[buf][0], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gp)(src + 1), (lp)&s_b2[buf][0], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gp)(src + 2), (lp)&s_c2[buf][0], 16, 0, 0);
    };
    // ids: lanes past the list load record 0 (staged, never read); the next round's id is loaded
    // a round ahead of its records
    uint32_t cid = t < nmax ? a.point_list[pair_at(nmax - 1 - t)] : 0u;
    glds_round(0, cid);
    uint32_t nid = B + t < nmax ? a.point_list[pair_at(nmax - 1 - (B + t))] : 0u;
    for (int base = 0, cur = 0; base < nmax; base += B, cur ^= 1) {
        float4* const s_a = s_a2[cur];
        float4* const s_b = s_b2[cur];
        float4* const s_c = s_c2[cur];
        uint32_t* const s_id = s_id2[cur];
        s_id[t] = cid;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this round's records are in LDS
        __syncthreads();
        if (base + B < nmax) {  // block-uniform: the next round's records and the one after's ids
            glds_round(cur ^ 1, nid);
            cid = nid;
            const int k3 = base + 2 * B + t;
            nid = k3 < nmax ? a.point_list[pair_at(nmax - 1 - k3)] : 0u;
        }
        const int cnt = min(B, nmax - base);
        // two pairs per reduction (wave_sum18): each pair's pixel work in order (T and R advance
        // pair by pair), then one interleaved reduction of their 18 sums
        auto pair_grads = [&](int j, float (&g)[NGRAD]) -> bool {
            const int contributor = nmax - 1 - (base + j);
            const float4 A = s_a[j];
            const float4 Bv = s_b[j];
            float g0, g1, g2, g3, g4, g5, g6 = 0.f, g7 = 0.f, g8 = 0.f;
            bool any = false;
            // The conic-side terms are linear in v = e * dL/dalpha with e = opacity G (the unclamped
            // alpha), and a lane's PPL pixels share its column (dx): per pixel only S_v, S_v.dy,
            // S_v.dy^2 are accumulated, and the six components follow once per lane and pair
            // (g0 = S_v dx, g1 = S_vdy, g2 = dx g0, g3 = dx g1, g4 = S_vdy2, g5 = S_v / opacity):
            // 5 VALU per pixel instead of 11.
            const float dx = A.x - pfx;
            const P2X px2 = blend_p2_x(A.z, A.w, Bv.y, dx);  // identical to the forward's values
            float sv = 0.f, svdy = 0.f, svdy2 = 0.f;
            const float4 Cc = s_c[j];  // once per pair (not per active row)
            // every pixel's alpha first, in one basic block, so that the PPL exp chains interleave
            // instead of each waiting behind the previous pixel's branched body (LLVM sinks each
            // back into its pixel's block without the opaque uses): blend bwd 0.2453 -> 0.2435 ms
            // per step in an interleaved A/B; the reciprocals hoisted too (paid for inactive pixels
            // as well) measured 0.2491 (profiles/r03_blend_bwd_hoist_ab.jsonl)
            float ev[PPL], av[PPL];
            bool acv[PPL];
#pragma unroll
            for (int q = 0; q < PPL; q++) {
                const float dy = A.y - (float)(py0 + 4 * q);
                const float e2 = blend_e2(px2, Bv.x, dy);
                ev[q] = __builtin_amdgcn_exp2f(e2);  // o G
                av[q] = fminf(0.99f, ev[q]);
                acv[q] = contributor < last[q] && e2 <= Bv.y && av[q] >= 1.0f / 255.0f;
            }
#pragma unroll
            for (int q = 0; q < PPL; q++) asm volatile("" : "+v"(ev[q]), "+v"(av[q]));
#pragma unroll
            for (int q = 0; q < PPL; q++) {
                const float dy = A.y - (float)(py0 + 4 * q);
                const float e = ev[q], alpha = av[q];
                const bool act = acv[q];
                if (act) {
                    any = true;
                    // both divisions by (1 - alpha) share one reciprocal; the Newton step keeps T's
                    // recovery within an ulp per pair over lists of thousands of pairs (the bare
                    // v_rcp_f32 measured 2 % faster on this kernel, 0.238 vs 0.243 ms)
                    const float inv = rcp_nr(1.f - alpha);
                    T[q] = T[q] * inv;                // T_i, the transmittance in front of this Gaussian
                    const float dchannel_dcolor = alpha * T[q];
                    const float cdp = Cc.x * dp0[q] + Cc.y * dp1[q] + Cc.z * dp2[q];
                    g6 += dchannel_dcolor * dp0[q];
                    g7 += dchannel_dcolor * dp1[q];
                    g8 += dchannel_dcolor * dp2[q];
                    const float d = cdp - R[q];  // R: accum_rec . dL/dpix in front of this Gaussian
                    // dL/dalpha = T_i (c - accum_rec) . dL/dpix - T_final (bg . dL/dpix) / (1 - alpha)
                    const float dL_dalpha = d * T[q] + tfbg[q] * inv;
                    // the reference's next accum_rec update (last_alpha = alpha, last_color = c),
                    // applied now instead of at the next contributing pair: the same fma on the
                    // same values, without carrying last_alpha / last_color
                    R[q] = __builtin_fmaf(alpha, d, R[q]);
                    const float v = e * dL_dalpha;
                    const float vdy = v * dy;
                    sv += v;
                    svdy += vdy;
                    svdy2 = __builtin_fmaf(vdy, dy, svdy2);
                }
            }
            // unconditionally: with no active pixel the sums are 0 and so are these (a branch here
            // costs a zero-initialising move per component and pair)
            g0 = sv * dx;
            g1 = svdy;
            g2 = g0 * dx;
            g3 = g1 * dx;
            g4 = svdy2;
            g5 = sv * s_c[j].w;  // 1 / opacity
            g[0] = g0;
            g[1] = g1;
            g[2] = g2;
            g[3] = g3;
            g[4] = g4;
            g[5] = g5;
            g[6] = g6;
            g[7] = g7;
            g[8] = g8;
            return any;
        };
        for (int j = 0; j < cnt; j += 2) {
            float ga[NGRAD], gb[NGRAD];
            const bool anya = pair_grads(j, ga);
            const bool has_b = j + 1 < cnt;  // block-uniform
            bool anyb = false;
            if (has_b) {
                anyb = pair_grads(j + 1, gb);
            } else {
#pragma unroll
                for (int k = 0; k < NGRAD; k++) gb[k] = 0.f;
            }
            float t[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
            if (__ballot(anya || anyb) != 0ull) wave_sum18(ga, gb, t);
            red18_store(&s_g[j * NGRAD], lane, t, has_b);
        }
        __syncthreads();
        // one atomic per (pair, component); consecutive lanes hit consecutive components of a pair
#pragma unroll
        for (int c = 0; c < NGRAD; c++) {
            const int e = c * B + t;
            const int pair = e / NGRAD;
            if (pair < cnt) {
                float v = s_g[e];
                const int comp = e - pair * NGRAD;
                if (comp <= 1) {  // dL/dmean2D from (Sx, Sy): -(conic . S), then the NDC factor
                    const float sx = s_g[pair * NGRAD], sy = s_g[pair * NGRAD + 1];
                    float ccx, ccy, ccz;
                    splat_conic(s_a[pair], s_b[pair], ccx, ccy, ccz);
                    v = comp == 0 ? -(ccx * sx + ccy * sy) * ddelx_dx : -(ccz * sy + ccy * sx) * ddely_dy;
                } else {
                    v *= comp <= 4 ? -0.5f : 1.f;
                }
                if (v != 0.f) atomicAdd(a.gacc + (size_t)s_id[pair] * GACC_STRIDE + comp, v);
            }
        }
        __syncthreads();
    }
}

// Heaviest tiles first ("longest processing time" order) for the backward blend: a tile costs
// tile_max pairs, which varies by more than 10x across a frame, and in XCD order a dense tile
// dispatched late runs alone on its SIMD after the rest of the grid has drained.  One workgroup:
// counting sort of the tiles by descending min(tile_max / 4, 1023) (order inside a bucket free).
__device__ __forceinline__ void tile_order_body(int T, const uint32_t* __restrict__ cost, uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[1024];
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    auto bucket = [&](int i) {
        const uint32_t c = cost[i];
        return 1023u - min(c >> 2, 1023u);
    };
    // up to kReg tiles per thread stay in registers between the two passes (one read of the costs,
    // all loads in flight together); larger grids fall back to re-reading
    constexpr int kReg = 16;
    uint32_t bk[kReg];
#pragma unroll
    for (int r = 0; r < kReg; r++) bk[r] = (t + r * 1024 < T) ? bucket(t + r * 1024) : 0u;
    hist[t] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kReg; r++)
        if (t + r * 1024 < T) atomicAdd(&hist[bk[r]], 1u);
    for (int i = t + kReg * 1024; i < T; i += 1024) atomicAdd(&hist[bucket(i)], 1u);
    __syncthreads();
    const uint32_t v = hist[t];
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t pre = 0;
    for (int i = 0; i < w; i++) pre += wsum[i];
    hist[t] = pre + incl - v;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kReg; r++)
        if (t + r * 1024 < T) order[atomicAdd(&hist[bk[r]], 1u)] = (uint32_t)(t + r * 1024);
    for (int i = t + kReg * 1024; i < T; i += 1024) order[atomicAdd(&hist[bucket(i)], 1u)] = (uint32_t)i;
}

// Backward prologue: the gradient accumulators are cleared by every workgroup but the first,
// which computes the backward's tile order meanwhile (a one-workgroup job that otherwise ran
// alone on the GPU for ~11 us between the clear and the blend).
__global__ __launch_bounds__(1024) void k_bwd_prologue(float4* __restrict__ gacc, size_t n4, int T,
                                                       const uint32_t* __restrict__ tile_max,
                                                       uint32_t* __restrict__ order,
                                                       const uint32_t* __restrict__ order_flag) {
    if (order) {
        if (blockIdx.x == 0) {
            // the phase-B duplicate launch already sorted this frame's tiles (DupArgs::order_out)
            if (order_flag && *order_flag == (uint32_t)T) return;
            tile_order_body(T, tile_max, order);
            return;
        }
    }
    const size_t zb = order ? blockIdx.x - 1 : blockIdx.x, nzb = order ? gridDim.x - 1 : gridDim.x;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (size_t i = zb * 1024 + threadIdx.x; i < n4; i += nzb * 1024) gacc[i] = z;
}

void launch_bwd_prologue(float* gacc, size_t nfloats, int T, const uint32_t* tile_max, uint32_t* order,
                         const uint32_t* order_flag, hipStream_t st) {
    const size_t n4 = nfloats / 4;  // P * GACC_STRIDE, a multiple of 4 (0: already clear)
    const size_t zb = n4 ? std::max<size_t>(1, std::min<size_t>((n4 + 1023) / 1024, 2048)) : 0;
    const bool ord = order && T > 0;
    if (zb + (ord ? 1 : 0) == 0) return;
    k_bwd_prologue<<<(unsigned)(zb + (ord ? 1 : 0)), 1024, 0, st>>>(reinterpret_cast<float4*>(gacc), n4, T, tile_max,
                                                                    ord ? order : nullptr, order_flag);
}

void launch_blend_bwd(const BlendBwdArgs& a, hipStream_t st) {
    const int T = a.gx * a.gy;
    if (T > 0) k_blend_bwd<<<T, 64, 0, st>>>(a);  // a.order: from the prologue or the phase-B duplicate
}

}  // namespace rr
