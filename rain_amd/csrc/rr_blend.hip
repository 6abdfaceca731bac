// rr_blend.hip — per-tile alpha blending backward (backward.cu:389-547); the forward blend lives in
// rr_blend_fwd_s.hip.
//
// CDNA4 mapping.  A 16x16 tile is processed by NW wave64s (NW = 1, 2 or 4, chosen per kernel at
// run time, see rr_set_blend_config), each lane owning PPL = 4/NW pixels of one column: thread t
// (lane l = t%64, wave w = t/64) owns column l%16 of rows l/16 + 4*(w*PPL + q), q < PPL.
//   * Each round stages 64*NW (tile, Gaussian) records (48 B each, rr_common.hpp Splat) in LDS; the
//     NEXT round's records are fetched into registers while the current round is blended, so the
//     dependent id -> record gather latency is hidden behind compute.
//   * All lanes read a staged record as an LDS broadcast and apply it to their PPL pixels.
//   * Forward early termination: a round starts only if some pixel of the tile is open
//     (__syncthreads_count, forward.cu:302-304); inside a round each wave leaves as soon as all its
//     pixels are saturated (wave vote), pixel groups that are done are skipped by exec mask.
//   * Backward: each lane sums its PPL pixels' contributions in registers, each wave reduces the 9
//     gradient components across its 64 lanes with DPP (no LDS), lane 63 parks the wave sums in
//     LDS, and after each round ONE global float atomic per (tile, Gaussian, component) is issued,
//     consecutive lanes on consecutive components of a Gaussian's 64-B accumulator line (the
//     reference issues 9 atomics per contributing PIXEL).  The backward only walks the first
//     max(n_contrib) pairs of a tile (recorded by the forward).
//   * Tiles are assigned XCD-contiguously (the dispatcher sends block b to XCD b % 8), so tiles
//     sharing Gaussians share an L2.
#include <cstdlib>
#include <string>

#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

#ifndef RR_BWD_DEFER
#define RR_BWD_DEFER 0
#endif
#ifndef RR_BWD_BF
#define RR_BWD_BF 0
#endif
// RR_BWD_GLDS: the next round's records go global -> LDS directly (global_load_lds_dwordx4 into the
// other half of a double-buffered stage) instead of through 12 prefetch VGPRs and a ds_write:
// 159 -> 121 VGPRs, 3 -> 4 waves per SIMD; blend backward 0.2427 / 0.2449 -> 0.2384 / 0.2401 ms,
// step 1.0600 / 1.0597 -> 1.0523 / 1.0527 ms (profiles/r05_bwd_glds_ab.jsonl).  (The same staging
// in the forward blend measured slower, 0.188 vs 0.170 ms: profiles/r05_fwd_glds_ab.jsonl.)
#ifndef RR_BWD_GLDS
#define RR_BWD_GLDS 1
#endif
// RR_BWD_PAIR2: two pairs' gradient components reduced across the wave together (wave_sum18, 48
// instead of 56 VALU per two pairs, bitwise the same sums), with the default kernel held at 4 waves
// per SIMD (RR_BWD_OCC: 128 VGPRs, 20 B/lane of scratch): blend backward 0.2383 / 0.2361 ->
// 0.2260 / 0.2276 ms, step 1.0514 / 1.0499 -> 1.0406 / 1.0415 ms; at 3 waves (134 VGPRs) 0.2333 /
// 0.2339 (profiles/r05_bwd_pair2_ab.jsonl)
#ifndef RR_BWD_OCC
#define RR_BWD_OCC 4  // the default kernel's minimum waves per SIMD (launch bounds)
#endif
#ifndef RR_BWD_PAIR2
#define RR_BWD_PAIR2 1
#endif

// OCC: minimum waves per SIMD requested from the register allocator.  The default 3 leaves the
// compiler its 132 VGPRs without spills; 4 caps it at 128 with 96 B/lane of scratch in the
// per-round flush (0.2446 / 0.2424 vs 0.2411 / 0.2413 ms/step in an interleaved A/B; a variant
// that also read the next pair's record from LDS one pair ahead was neutral at 3 waves and slower
// at 4: profiles/r03_blend_bwd_occupancy_ab.txt).
template <int NW, int OCC>
__global__ __launch_bounds__(64 * NW, OCC) void k_blend_bwd(BlendBwdArgs a) {
    constexpr int PPL = 4 / NW;
    constexpr int B = 64 * NW;
    const int ntiles = a.gx * a.gy;
    const int tile = a.order ? (int)a.order[blockIdx.x] : xcd_tile(blockIdx.x, ntiles);
    const int nmax = (int)a.tile_max[tile];  // pairs past this index were blended by no pixel
    if (nmax == 0) return;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int px = tx * TILE_X + (lane & 15);
    const int py0 = ty * TILE_Y + (lane >> 4) + 4 * w * PPL;
    const float pfx = (float)px;

#if RR_BWD_GLDS
    __shared__ float4 s_a2[2][B];
    __shared__ float4 s_b2[2][B];
    __shared__ float4 s_c2[2][B];
    __shared__ uint32_t s_id2[2][B];
#else
    __shared__ float4 s_a[B];
    __shared__ float4 s_b[B];
    __shared__ float4 s_c[B];
    __shared__ uint32_t s_id[B];
#endif
    __shared__ float s_g[NW][B * NGRAD];

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

#if RR_BWD_GLDS
    // round r's records land in stage r & 1: issued (global -> LDS) one round ahead; each wave
    // writes its 64 lanes' records contiguously, which is the stage's layout (record t at [t])
    auto glds_round = [&](int buf, uint32_t id) {
        typedef __attribute__((address_space(1))) const void* gp;
        typedef __attribute__((address_space(3))) void* lp;
        const float4* src = reinterpret_cast<const float4*>(a.splats) + 3 * (size_t)id;
        __builtin_amdgcn_global_load_lds((gp)(src + 0), (lp)&s_a2[buf][64 * w], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gp)(src + 1), (lp)&s_b2[buf][64 * w], 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gp)(src + 2), (lp)&s_c2[buf][64 * w], 16, 0, 0);
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
#else
    uint32_t nid = 0;
    float4 na = make_float4(0.f, 0.f, 0.f, 0.f), nb = na, nc = na;
    if (t < nmax) {
        nid = a.point_list[pair_at(nmax - 1 - t)];
        load_splat(a.splats, nid, na, nb, nc);
    }
    for (int base = 0; base < nmax; base += B) {
        if (base + t < nmax) {
            s_id[t] = nid;
            s_a[t] = na;
            s_b[t] = nb;
            s_c[t] = nc;
        }
        __syncthreads();
        const int k2 = base + B + t;  // prefetch the next round while this one is blended
        if (k2 < nmax) {
            nid = a.point_list[pair_at(nmax - 1 - k2)];
            load_splat(a.splats, nid, na, nb, nc);
        }
        const int cnt = min(B, nmax - base);
#endif
#if RR_BWD_DEFER
        // Software-pipelined by hand: the block after pair j's branched pixel bodies holds pair
        // j's nine per-lane sums, the LDS record reads and the four exp2 chains of pair j + 1, and
        // the wave reduction of pair j — independent dependency chains for the scheduler to
        // interleave, where the reduction's permlane / DPP chain and the next record's LDS latency
        // otherwise each ran alone.  The reduction is unconditional (skipping an empty pair measured
        // neutral, and its branch would split the block); the last pair reads its own record again.
        float4 A = s_a[0], Bv = s_b[0], Cc = s_c[0];
        float ev[PPL], av[PPL];
        bool ok[PPL];
        auto alphas = [&](int jp) {
            const int contrib_next = nmax - 1 - (base + jp);
            (void)contrib_next;
            const float dx = A.x - pfx;
            const P2X px2 = blend_p2_x(A.z, A.w, Bv.y, dx);
#pragma unroll
            for (int q = 0; q < PPL; q++) {
                const float dy = A.y - (float)(py0 + 4 * q);
                const float e2 = blend_e2(px2, Bv.x, dy);
                ev[q] = __builtin_amdgcn_exp2f(e2);  // o G
                av[q] = fminf(0.99f, ev[q]);
                // keep every exp chain in this block (LLVM would sink each into its pixel's branch)
                asm volatile("" : "+v"(ev[q]), "+v"(av[q]));
                ok[q] = (e2 <= Bv.y) & (av[q] >= 1.0f / 255.0f);
#if RR_BWD_BF
                // branch-free bodies: an inactive pixel runs the body with alpha = e = 0, which
                // leaves T (1 / (1 - 0) = 1 exactly), R and every sum bit for bit unchanged
                ok[q] = ok[q] & (contrib_next < last[q]);
                av[q] = ok[q] ? av[q] : 0.f;
                ev[q] = ok[q] ? ev[q] : 0.f;
#endif
            }
        };
        alphas(0);
        for (int j = 0; j < cnt; j++) {
            const int contributor = nmax - 1 - (base + j);
            (void)contributor;
            const float dx = A.x - pfx;
            float sv = 0.f, svdy = 0.f, svdy2 = 0.f, g6 = 0.f, g7 = 0.f, g8 = 0.f;
            auto body = [&](int q) {
                const float dy = A.y - (float)(py0 + 4 * q);
                const float e = ev[q], alpha = av[q];
                const float inv = rcp_nr(1.f - alpha);
                T[q] = T[q] * inv;
                const float dchannel_dcolor = alpha * T[q];
                const float cdp = Cc.x * dp0[q] + Cc.y * dp1[q] + Cc.z * dp2[q];
                g6 += dchannel_dcolor * dp0[q];
                g7 += dchannel_dcolor * dp1[q];
                g8 += dchannel_dcolor * dp2[q];
                const float d = cdp - R[q];
                const float dL_dalpha = d * T[q] + tfbg[q] * inv;
                R[q] = __builtin_fmaf(alpha, d, R[q]);
                const float v = e * dL_dalpha;
                const float vdy = v * dy;
                sv += v;
                svdy += vdy;
                svdy2 = __builtin_fmaf(vdy, dy, svdy2);
            };
#if RR_BWD_BF == 1
#pragma unroll
            for (int q = 0; q < PPL; q++) body(q);
#elif RR_BWD_BF == 2
            // one branch per two pixels of the lane (tile rows 0-7 / 8-15)
#pragma unroll
            for (int q = 0; q < PPL; q += 2) {
                if (q + 1 >= PPL) {
                    if (ok[q]) body(q);
                } else if (ok[q] | ok[q + 1]) {
                    body(q);
                    body(q + 1);
                }
            }
#else
#pragma unroll
            for (int q = 0; q < PPL; q++)
                if ((contributor < last[q]) & ok[q]) body(q);
#endif
            const float p0 = sv * dx, p1 = svdy, p2 = p0 * dx, p3 = p1 * dx, p4 = svdy2;
            const float p5 = sv * Cc.w;  // 1 / opacity
            const int jn = min(j + 1, cnt - 1);
            A = s_a[jn];
            Bv = s_b[jn];
            Cc = s_c[jn];
            alphas(jn);
            float t0, t1, t2;
            wave_sum9(p0, p1, p2, p3, p4, p5, g6, g7, g8, t0, t1, t2);
            red9_store(&s_g[w][j * NGRAD], lane, t0, t1, t2);
        }
#elif RR_BWD_PAIR2
        // two pairs per reduction (wave_sum18): each pair's pixel work as in the loop below, in
        // order (T and R advance pair by pair), then one interleaved reduction of their 18 sums
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
            red18_store(&s_g[w][j * NGRAD], lane, t, has_b);
        }
#else
        for (int j = 0; j < cnt; j++) {
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
            float* sg = &s_g[w][j * NGRAD];
            float t0 = 0.f, t1 = 0.f, t2 = 0.f;
            if (__ballot(any) != 0ull) wave_sum9(g0, g1, g2, g3, g4, g5, g6, g7, g8, t0, t1, t2);
            red9_store(sg, lane, t0, t1, t2);
        }
#endif
        __syncthreads();
        // one atomic per (pair, component); consecutive lanes hit consecutive components of a pair
#pragma unroll
        for (int c = 0; c < NGRAD; c++) {
            const int e = c * B + t;
            const int pair = e / NGRAD;
            if (pair < cnt) {
                float v = s_g[0][e];
#pragma unroll
                for (int i = 1; i < NW; i++) v += s_g[i][e];
                const int comp = e - pair * NGRAD;
                if (comp <= 1) {  // dL/dmean2D from (Sx, Sy): -(conic . S), then the NDC factor
                    float sx = s_g[0][pair * NGRAD], sy = s_g[0][pair * NGRAD + 1];
#pragma unroll
                    for (int i = 1; i < NW; i++) {
                        sx += s_g[i][pair * NGRAD];
                        sy += s_g[i][pair * NGRAD + 1];
                    }
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
// The forward blends use the same order with the tile's list length as its cost (ranges != null).
__device__ __forceinline__ void tile_order_body(int T, const uint32_t* __restrict__ cost,
                                                const uint2* __restrict__ ranges, uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[1024];
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    auto bucket = [&](int i) {
        const uint32_t c = ranges ? ranges[i].y - ranges[i].x : cost[i];
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

__global__ __launch_bounds__(1024) void k_tile_order(int T, const uint32_t* __restrict__ cost,
                                                     const uint2* __restrict__ ranges,
                                                     uint32_t* __restrict__ order) {
    tile_order_body(T, cost, ranges, order);
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
            tile_order_body(T, tile_max, nullptr, order);
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

namespace {
int g_bwd_waves = 0;
int g_dup_order = 1;
int g_bwd_order = -1;  // -1: RAIN_BWD_TILE_ORDER or the default (on)
int g_fwd_order = -1;  // -1: RAIN_FWD_TILE_ORDER or the default (off)
int g_fwd_s_waves = 2, g_fwd_s_b_waves = 4;
int env_waves(const char* name, int dflt) {
    const char* s = std::getenv(name);
    if (!s) return dflt;
    const int v = std::atoi(s);
    return (v >= 1 && v <= 4) ? v : dflt;
}
}  // namespace

// Defaults: measured on MI355X (profiles/).  The forward blend (rr_blend_fwd_s.hip)
// runs 2 waves per tile in phase A (2 pixels per lane), 4 in phase B (1 pixel per lane).
constexpr int kBwdWavesDefault = 1;

void set_blend_config(int fwd_waves, int bwd_waves) {
    g_fwd_s_waves = (fwd_waves == 1 || fwd_waves == 4) ? fwd_waves : 2;
    g_bwd_waves = bwd_waves;
}

bool bwd_tile_order() {
    if (g_bwd_order < 0) {
        const char* s = std::getenv("RAIN_BWD_TILE_ORDER");
        g_bwd_order = s ? (std::atoi(s) != 0) : 1;
    }
    return g_bwd_order != 0;
}

// the backward's tile order computed by an extra workgroup of the phase-B duplicate (default) or
// by the backward prologue (rr_set_tuning "dup_tile_order" 0)
bool dup_tile_order() { return g_dup_order != 0; }

bool fwd_tile_order() {
    if (g_fwd_order < 0) {
        // default off: list length is not what a forward tile costs (saturation is); measured
        // 1.585 vs 1.581 ms per training step with / without, and in a wave-timing trace of phase A
        // (tools/fwd_trace.py) the duration of a tile is uncorrelated with its list length (-0.07)
        const char* s = std::getenv("RAIN_FWD_TILE_ORDER");
        g_fwd_order = s ? (std::atoi(s) != 0) : 0;
    }
    return g_fwd_order != 0;
}

int blend_fwd_s_waves(bool phase_b) { return phase_b ? g_fwd_s_b_waves : g_fwd_s_waves; }

void launch_tile_order_by_length(int T, const uint2* ranges, uint32_t* order, hipStream_t st) {
    if (T > 0) k_tile_order<<<1, 1024, 0, st>>>(T, nullptr, ranges, order);
}

int set_tuning(const char* key, int value) {
    if (!key) return 1;
    const std::string k(key);
    if (k == "bwd_tile_order") g_bwd_order = value != 0;
    else if (k == "fwd_tile_order") g_fwd_order = value != 0;
    else if (k == "fwd_b_waves") g_fwd_s_b_waves = value ? 4 : g_fwd_s_waves;
    else if (k == "fwd_waves" || k == "fwd_s_waves") g_fwd_s_waves = (value == 1 || value == 4) ? value : 2;
    else if (k == "fwd_s_b_waves") g_fwd_s_b_waves = (value == 1 || value == 2) ? value : 4;
    else if (k == "bwd_waves") g_bwd_waves = value;
    else if (k == "sort_min_units") set_sort_min_units(value);
    else if (k == "sort_min_units_tile") set_sort_min_units_tile(value);
    else if (k == "sort_max_rounds") set_sort_max_rounds(value);
    else if (k == "pair_scan_direct_blocks") set_pair_scan_direct_blocks(value);
    else if (k == "wide_bin_keys") set_wide_bin_keys(value != 0);
    else if (k == "dup_tile_order") g_dup_order = value != 0;
    else if (k == "sx_bucket") set_sx_bucket(value != 0);
    else return 1;
    return 0;
}

void launch_blend_bwd(const BlendBwdArgs& a, hipStream_t st) {
    const int T = a.gx * a.gy;
    if (T == 0) return;
    // a.order was filled by the prologue (launch_bwd_prologue)
    const int nw = g_bwd_waves ? g_bwd_waves : env_waves("RAIN_BLEND_BWD_WAVES", kBwdWavesDefault);
    switch (nw) {
        case 2: k_blend_bwd<2, 1><<<T, 128, 0, st>>>(a); break;
        case 3: k_blend_bwd<1, 3><<<T, 64, 0, st>>>(a); break;  // A/B variant: 1 wave, up to 168 VGPRs
        case 4: k_blend_bwd<4, 1><<<T, 256, 0, st>>>(a); break;
        default: k_blend_bwd<1, RR_BWD_OCC><<<T, 64, 0, st>>>(a); break;
    }
}

}  // namespace rr
