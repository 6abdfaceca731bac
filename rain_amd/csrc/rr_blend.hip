// rr_blend.hip — per-tile alpha blending, forward and backward (forward.cu:251-369, backward.cu:389-547).
//
// CDNA4 mapping: ONE wave64 per 16x16 tile, FOUR pixels per lane (lane l owns column l%16 of rows
// l/16, l/16+4, l/16+8, l/16+12).  Compared with the reference's 256-thread block per tile:
//   * the per-pair record (48 B) is staged once in LDS and read as a broadcast by 64 lanes that
//     each use it for 4 pixels (4x less LDS/VALU overhead per pixel);
//   * a workgroup is a single wave: no cross-wave barrier cost, no __syncthreads_count; early
//     termination is a wave vote (`__all`) checked per pair;
//   * backward: each lane first sums its 4 pixels' contributions in registers, then ONE wave-wide
//     DPP reduction per (tile, Gaussian) pair (the reference issues 9 atomics per pixel), and the
//     pair sums are flushed with one coalesced batch of global float atomics per 64 pairs;
//   * tiles are assigned XCD-contiguously (blockIdx % 8 selects an XCD on MI355X), so tiles that
//     share Gaussians share an L2.
#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

constexpr int WPIX = 4;  // pixels per lane

// Bijective block -> tile remap: the blocks the dispatcher sends to one XCD (b % 8) get one
// contiguous run of tiles (cdna_hip_programming.md §5, "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_tile(int b, int n) {
    const int q = n >> 3, r = n & 7;
    const int x = b & 7, s = b >> 3;
    return x < r ? x * (q + 1) + s : r * (q + 1) + (x - r) * q + s;
}

__global__ __launch_bounds__(64) void k_blend_fwd(BlendFwdArgs a) {
    const int ntiles = a.gx * a.gy;
    const int tile = xcd_tile(blockIdx.x, ntiles);
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x;
    const int px = tx * TILE_X + (lane & 15);
    const int py0 = ty * TILE_Y + (lane >> 4);
    const float pfx = (float)px;

    __shared__ float4 s_a[64];
    __shared__ float4 s_b[64];
    __shared__ float4 s_c[64];

    float T[WPIX], C0[WPIX], C1[WPIX], C2[WPIX], Dp[WPIX];
    uint32_t contrib[WPIX], last[WPIX];
    bool done[WPIX];
#pragma unroll
    for (int q = 0; q < WPIX; q++) {
        T[q] = 1.0f;
        C0[q] = C1[q] = C2[q] = Dp[q] = 0.f;
        contrib[q] = last[q] = 0;
        done[q] = !(px < a.W && py0 + 4 * q < a.H);
    }
    const uint2 range = a.ranges[tile];
    const int n = (int)(range.y - range.x);

    for (int base = 0; base < n; base += 64) {
        bool lane_done = done[0] && done[1] && done[2] && done[3];
        if (__all(lane_done)) break;
        const int k = base + lane;
        if (k < n) {
            const Splat s = a.splats[a.point_list[range.x + k]];
            s_a[lane] = s.a;
            s_b[lane] = s.b;
            s_c[lane] = s.c;
        }
        __syncthreads();
        const int cnt = min(64, n - base);
        for (int j = 0; j < cnt; j++) {
            lane_done = done[0] && done[1] && done[2] && done[3];
            if (__all(lane_done)) break;
            const float4 A = s_a[j];
            const float4 B = s_b[j];
#pragma unroll
            for (int q = 0; q < WPIX; q++) {
                if (!done[q]) {
                    contrib[q]++;
                    const float dx = A.x - pfx, dy = A.y - (float)(py0 + 4 * q);
                    const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
                    if (power <= 0.0f) {
                        const float alpha = fminf(0.99f, B.y * __expf(power));
                        if (alpha >= 1.0f / 255.0f) {
                            const float test_T = T[q] * (1 - alpha);
                            if (test_T < 0.0001f) {
                                done[q] = true;
                            } else {
                                const float4 Cc = s_c[j];
                                C0[q] += Cc.x * alpha * T[q];
                                C1[q] += Cc.y * alpha * T[q];
                                C2[q] += Cc.z * alpha * T[q];
                                Dp[q] += B.z * alpha * T[q];
                                T[q] = test_T;
                                last[q] = contrib[q];
                            }
                        }
                    }
                }
            }
        }
        __syncthreads();
    }

    uint32_t m = 0;
    const size_t HW = (size_t)a.H * a.W;
#pragma unroll
    for (int q = 0; q < WPIX; q++) {
        const int py = py0 + 4 * q;
        if (px < a.W && py < a.H) {
            m = max(m, last[q]);
            const int pix = a.W * py + px;
            a.final_T[pix] = T[q];
            a.n_contrib[pix] = last[q];
            a.out_color[pix] = C0[q] + T[q] * a.bg[0];
            a.out_color[HW + pix] = C1[q] + T[q] * a.bg[1];
            a.out_color[2 * HW + pix] = C2[q] + T[q] * a.bg[2];
            a.out_depth[pix] = Dp[q];
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if (lane == 0) a.tile_max[tile] = m;
}

__global__ __launch_bounds__(64) void k_blend_bwd(BlendBwdArgs a) {
    const int ntiles = a.gx * a.gy;
    const int tile = xcd_tile(blockIdx.x, ntiles);
    const int nmax = (int)a.tile_max[tile];  // pairs past this index were blended by no pixel
    if (nmax == 0) return;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x;
    const int px = tx * TILE_X + (lane & 15);
    const int py0 = ty * TILE_Y + (lane >> 4);
    const float pfx = (float)px;

    __shared__ float4 s_a[64];
    __shared__ float4 s_b[64];
    __shared__ float4 s_c[64];
    __shared__ uint32_t s_id[64];
    __shared__ float s_g[64 * NGRAD];

    const size_t HW = (size_t)a.H * a.W;
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
    float T[WPIX], Tf[WPIX], dp0[WPIX], dp1[WPIX], dp2[WPIX], bgd[WPIX];
    float ar0[WPIX], ar1[WPIX], ar2[WPIX], lc0[WPIX], lc1[WPIX], lc2[WPIX], la[WPIX];
    int last[WPIX];
#pragma unroll
    for (int q = 0; q < WPIX; q++) {
        const int py = py0 + 4 * q;
        const bool inside = px < a.W && py < a.H;
        const int pix = a.W * py + px;
        Tf[q] = inside ? a.final_T[pix] : 0.f;
        T[q] = Tf[q];
        last[q] = inside ? (int)a.n_contrib[pix] : 0;
        dp0[q] = inside ? a.dL_dpix[pix] : 0.f;
        dp1[q] = inside ? a.dL_dpix[HW + pix] : 0.f;
        dp2[q] = inside ? a.dL_dpix[2 * HW + pix] : 0.f;
        bgd[q] = bg0 * dp0[q] + bg1 * dp1[q] + bg2 * dp2[q];
        ar0[q] = ar1[q] = ar2[q] = lc0[q] = lc1[q] = lc2[q] = la[q] = 0.f;
    }
    const uint2 range = a.ranges[tile];
    const float ddelx_dx = 0.5f * a.W;
    const float ddely_dy = 0.5f * a.H;

    for (int base = 0; base < nmax; base += 64) {
        const int k = base + lane;
        if (k < nmax) {
            const uint32_t g = a.point_list[range.x + nmax - 1 - k];
            const Splat s = a.splats[g];
            s_id[lane] = g;
            s_a[lane] = s.a;
            s_b[lane] = s.b;
            s_c[lane] = s.c;
        }
        __syncthreads();
        const int cnt = min(64, nmax - base);
        for (int j = 0; j < cnt; j++) {
            const int contributor = nmax - 1 - (base + j);
            const float4 A = s_a[j];
            const float4 B = s_b[j];
            float g0 = 0.f, g1 = 0.f, g2 = 0.f, g3 = 0.f, g4 = 0.f, g5 = 0.f, g6 = 0.f, g7 = 0.f, g8 = 0.f;
            bool any = false;
#pragma unroll
            for (int q = 0; q < WPIX; q++) {
                const float dx = A.x - pfx, dy = A.y - (float)(py0 + 4 * q);
                const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
                const float G = __expf(power);
                const float alpha = fminf(0.99f, B.y * G);
                const bool act = contributor < last[q] && power <= 0.0f && alpha >= 1.0f / 255.0f;
                if (act) {
                    any = true;
                    const float one_m = 1.f - alpha;
                    T[q] = __fdividef(T[q], one_m);
                    const float dchannel_dcolor = alpha * T[q];
                    const float4 Cc = s_c[j];
                    ar0[q] = la[q] * lc0[q] + (1.f - la[q]) * ar0[q];
                    ar1[q] = la[q] * lc1[q] + (1.f - la[q]) * ar1[q];
                    ar2[q] = la[q] * lc2[q] + (1.f - la[q]) * ar2[q];
                    lc0[q] = Cc.x;
                    lc1[q] = Cc.y;
                    lc2[q] = Cc.z;
                    float dL_dalpha = (Cc.x - ar0[q]) * dp0[q] + (Cc.y - ar1[q]) * dp1[q] + (Cc.z - ar2[q]) * dp2[q];
                    g6 += dchannel_dcolor * dp0[q];
                    g7 += dchannel_dcolor * dp1[q];
                    g8 += dchannel_dcolor * dp2[q];
                    dL_dalpha *= T[q];
                    la[q] = alpha;
                    dL_dalpha += __fdividef(-Tf[q], one_m) * bgd[q];
                    const float dL_dG = B.y * dL_dalpha;
                    const float gdx = G * dx, gdy = G * dy;
                    const float dG_ddelx = -gdx * A.z - gdy * A.w;
                    const float dG_ddely = -gdy * B.x - gdx * A.w;
                    g0 += dL_dG * dG_ddelx * ddelx_dx;
                    g1 += dL_dG * dG_ddely * ddely_dy;
                    g2 += -0.5f * gdx * dx * dL_dG;
                    g3 += -0.5f * gdx * dy * dL_dG;
                    g4 += -0.5f * gdy * dy * dL_dG;
                    g5 += G * dL_dalpha;
                }
            }
            float* sg = &s_g[j * NGRAD];
            if (__ballot(any) != 0ull) {
                g0 = wave_sum_lane63(g0);
                g1 = wave_sum_lane63(g1);
                g2 = wave_sum_lane63(g2);
                g3 = wave_sum_lane63(g3);
                g4 = wave_sum_lane63(g4);
                g5 = wave_sum_lane63(g5);
                g6 = wave_sum_lane63(g6);
                g7 = wave_sum_lane63(g7);
                g8 = wave_sum_lane63(g8);
                if (lane == 63) {
                    sg[0] = g0; sg[1] = g1; sg[2] = g2; sg[3] = g3; sg[4] = g4;
                    sg[5] = g5; sg[6] = g6; sg[7] = g7; sg[8] = g8;
                }
            } else if (lane == 63) {
#pragma unroll
                for (int c = 0; c < NGRAD; c++) sg[c] = 0.f;
            }
        }
        __syncthreads();
        // one atomic per (pair, component); consecutive lanes hit consecutive components of a pair
#pragma unroll
        for (int c = 0; c < NGRAD; c++) {
            const int e = c * 64 + lane;
            const int pair = e / NGRAD;
            if (pair < cnt) {
                const float v = s_g[e];
                if (v != 0.f) atomicAdd(a.gacc + (size_t)s_id[pair] * GACC_STRIDE + (e - pair * NGRAD), v);
            }
        }
        __syncthreads();
    }
}

void launch_blend_fwd(const BlendFwdArgs& a, hipStream_t st) {
    const int T = a.gx * a.gy;
    if (T == 0) return;
    k_blend_fwd<<<T, 64, 0, st>>>(a);
}

void launch_blend_bwd(const BlendBwdArgs& a, hipStream_t st) {
    const int T = a.gx * a.gy;
    if (T == 0) return;
    k_blend_bwd<<<T, 64, 0, st>>>(a);
}

}  // namespace rr
