// loss.hip — fused L1 + SSIM training loss, forward and backward (include/rain_loss.h).
//
// Replaces the reference's five depthwise 11x11 conv2d calls per SSIM evaluation plus their
// autograd (utils/loss_utils.py:22-53, train.py:113-115), which on ROCm go through MIOpen's
// generic convolution paths.  One wave64 per 64x32 output tile and channel: the band's 42 input
// rows (5-pixel halo, zero padded like conv2d padding=5) stream through a two-row LDS ring; each
// lane applies the separable Gaussian as an 11-tap horizontal pass (LDS) and an 11-tap vertical
// pass (an 11-row register ring), and all five moment maps (E[x], E[y], E[x^2], E[y^2], E[xy])
// come out of the same pass.  3x1080x1920 on MI355X: forward 51 us, backward 46 us (the
// 16x16-tile / 26x26-patch version: 92 / 64 us).
//
//   S = (2 m1 m2 + C1)(2 s12 + C2) / ((m1^2 + m2^2 + C1)(s11 + s22 + C2)),  s.. = E[..] - m.m.
//   dS/dm1 = 2 m2 (B - A) / (Cd Dd) - 2 m1 S (1/Cd - 1/Dd),  dS/dE[x^2] = -S / Dd,
//   dS/dE[xy] = 2 A / (Cd Dd)
// dL/dx = blur(G1) + 2 x blur(G11) + y blur(G12) + (1-lambda) sign(x-y)/(CHW)   (blur is self-adjoint:
// symmetric window, zero padding), with G.. = -lambda/(CHW) dS/d.. stored by the forward.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/rain_loss.h"

namespace {

// Tiling: one wave64 per block; lane l owns output column l of a 64-wide tile and TH consecutive
// output rows.  The block streams the TH + 10 input rows of its band through an NR-row LDS ring,
// and global loads run LA rows ahead of the ring in a small register queue, so memory latency
// hides behind LA rows of arithmetic while a wave needs only NR x 74 floats of LDS per plane
// (LA 2..6 and TH 16..64 measured: TH 32 best, LA within 5%; per kernel in round 3, standalone
// 3x1080x1920: backward TH 8/16/32/48/64 = 62/54/45/51/57 us, forward TH 16/32/48 = 55/52/65 us,
// profiles/r03_ssim_band_ab.jsonl).
// The row loop is fully unrolled (build flag -pragma-unroll-threshold, rain_amd/_build.py): every
// ring / queue slot is a compile-time register.
constexpr int R = 5;             // window radius (11 taps)
constexpr int TW = 64;           // output columns per block
#ifndef RL_TH
#define RL_TH 32
#endif
#ifndef RL_TH_BWD
#define RL_TH_BWD RL_TH
#endif
#ifndef RL_LA_FWD
#define RL_LA_FWD 2
#endif
#ifndef RL_LA_BWD
#define RL_LA_BWD 4
#endif
constexpr int TH_FWD = RL_TH;     // output rows per block, forward
constexpr int TH_BWD = RL_TH_BWD; // and backward
constexpr int PW = TW + 2 * R;   // 74: patch row width (halo of 5 each side, zero padded)
constexpr int NR = 2;            // LDS row ring (double buffer)
constexpr int LA_FWD = RL_LA_FWD; // rows of global-load lookahead (register queue), forward
constexpr int LA_BWD = RL_LA_BWD; // and backward (fewer live values: deeper queue fits)
constexpr int NQ = 2;            // 64-column chunks per patch row
constexpr int NB_MAX = 1 << 20;  // partial-sum slots

thread_local std::string g_err;

struct Win {
    float w[11];
};

// 1/x: v_rcp_f32 (1 ulp) plus one Newton step
__device__ __forceinline__ float rcp_nr(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(r, __builtin_fmaf(-x, r, 1.0f), r);
}

// Loads go through buffer descriptors (one per plane, built from wave-uniform values): the
// per-lane column offset is fixed for the whole band and the row offset is a scalar, so a row
// costs no address VGPRs, and out-of-image rows / columns read 0 through the range check
// (conv2d's zero padding).
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr int kOOB = 0x3FFFFFF0;  // offset that fails the range check (plane bytes < 2^30)

__device__ __forceinline__ Rsrc plane_rsrc(const float* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float load_f32(Rsrc r, int voff, int soff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void store_f32(float v, Rsrc r, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, 0);
}
// Opaque use: the row's horizontal sums are computed here, not sunk to their first (later) use,
// which would keep the row's LDS reads live across rows.
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }

// Per-row LDS base, laundered so that the compiler cannot keep every row's tap addresses alive
// across the unrolled band (it CSEs them otherwise: ~60 extra VGPRs).  Taps then fold into the
// ds_read immediate offsets.
typedef __attribute__((address_space(3))) const float* lds_ptr;
__device__ __forceinline__ lds_ptr row_base(const float* p) {
    lds_ptr q = (lds_ptr)p;
    asm volatile("" : "+v"(q));
    return q;
}

// One patch row of NP planes in registers.
template <int NP>
struct PatchRow {
    float v[NP][NQ];
    __device__ __forceinline__ void load(const Rsrc (&rs)[NP], const int (&voff)[NQ], int soff) {
#pragma unroll
        for (int h = 0; h < NQ; h++)
#pragma unroll
            for (int k = 0; k < NP; k++)
                v[k][h] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs[k], voff[h], soff, 0));
    }
    __device__ __forceinline__ void store(float (*dst)[NR][PW], int slot, int lane) const {
#pragma unroll
        for (int h = 0; h < NQ; h++) {
            const int q = lane + 64 * h;
            if (q < PW)
#pragma unroll
                for (int k = 0; k < NP; k++) dst[k][slot][q] = v[k][h];
        }
    }
};

// Per-band addressing: lane column offsets (bytes) and the scalar row offset of band row r.
struct Band {
    int voff[NQ];
    int y0, H, rowbytes;
    __device__ __forceinline__ Band(int x0, int y0_, int H_, int W, int lane) : y0(y0_), H(H_), rowbytes(4 * W) {
#pragma unroll
        for (int h = 0; h < NQ; h++) {
            const int gx = x0 + lane + 64 * h;
            voff[h] = (gx >= 0 && gx < W && lane + 64 * h < PW) ? 4 * gx : kOOB;
        }
    }
    __device__ __forceinline__ int soff(int r) const {
        const int gy = y0 + r;
        return (gy >= 0 && gy < H) ? gy * rowbytes : kOOB;
    }
};

// Rows 0..NR-1 into the LDS ring, rows NR..NR+LA-1 into the register queue.
template <int NP, int LA, int PH>
__device__ __forceinline__ void prime(const Rsrc (&rs)[NP], const Band& bd, float (*dst)[NR][PW],
                                      PatchRow<NP> (&q)[LA + 1], int lane) {
    PatchRow<NP> rows[NR];
#pragma unroll
    for (int i = 0; i < NR; i++) rows[i].load(rs, bd.voff, bd.soff(i));
#pragma unroll
    for (int i = 0; i < LA; i++)
        if (NR + i < PH) q[(NR + i) % (LA + 1)].load(rs, bd.voff, bd.soff(NR + i));
#pragma unroll
    for (int i = 0; i < NR; i++) rows[i].store(dst, i, lane);
    __syncthreads();
}

// Per band row r (compile time): issue the load of row r + NR + LA, and after the row has been
// read from the ring move row r + NR from the queue into its slot.
template <int NP, int LA, int PH>
__device__ __forceinline__ void queue_issue(const Rsrc (&rs)[NP], const Band& bd, PatchRow<NP> (&q)[LA + 1], int r) {
    __builtin_amdgcn_sched_barrier(0);  // rows stay in program order (bounded register lifetimes)
    if (r + NR + LA < PH) q[(r + NR + LA) % (LA + 1)].load(rs, bd.voff, bd.soff(r + NR + LA));
}
template <int NP, int LA, int PH>
__device__ __forceinline__ void queue_retire(float (*dst)[NR][PW], const PatchRow<NP> (&q)[LA + 1], int r, int lane) {
    __syncthreads();  // every lane's reads of slot r % NR are done before it is refilled
    if (r + NR < PH) q[(r + NR) % (LA + 1)].store(dst, r % NR, lane);
}

// Forward: the lane walks the PH band rows of its column top to bottom.  An 11-tap horizontal
// pass over the LDS ring gives the five row moments (x, y, x^2, y^2, xy), kept in an 11-row
// register ring; once it is full each new row completes one output row through the 11-tap
// vertical pass, followed by the SSIM term and the three gradient maps.
template <int TH>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k_ssim_fwd(const float* __restrict__ img, const float* __restrict__ gt, int H,
                                                 int W, float lambda, float inv_n, Win win, float* __restrict__ g1,
                                                 float* __restrict__ g11, float* __restrict__ g12,
                                                 float2* __restrict__ partial) {
    __shared__ float sp[2][NR][PW];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * TW - R, y0 = blockIdx.y * TH - R;
    const size_t plane = (size_t)H * W;
    const int lane = threadIdx.x;
    constexpr int PH = TH + 2 * R;  // input rows per band
    const Rsrc rs[2] = {plane_rsrc(img + c * plane, 4 * (int)plane), plane_rsrc(gt + c * plane, 4 * (int)plane)};
    const Rsrc ws[3] = {plane_rsrc(g1 + c * plane, 4 * (int)plane), plane_rsrc(g11 + c * plane, 4 * (int)plane),
                        plane_rsrc(g12 + c * plane, 4 * (int)plane)};
    const Band bd(x0, y0, H, W, lane);
    constexpr int LA = LA_FWD;
    PatchRow<2> q[LA + 1];
    prime<2, LA, PH>(rs, bd, sp, q, lane);
    const int gx = blockIdx.x * TW + lane;
    const bool col_in = gx < W;
    const int vo = col_in ? 4 * gx : kOOB;
    const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
    const float k = -lambda * inv_n;
    float r0[11], r1[11], r2[11], r3[11], r4[11];  // register ring, one array per moment
    float s_val = 0.f, l1 = 0.f;
#pragma unroll
    for (int r = 0; r < PH; r++) {
        queue_issue<2, LA, PH>(rs, bd, q, r);
        const int slot = r % NR;
        const lds_ptr px = row_base(&sp[0][slot][lane]);
        const lds_ptr py = px + NR * PW;  // plane 1, same slot
        float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
        for (int j = 0; j < 11; j++) {
            const float xv = px[j], yv = py[j], wj = win.w[j];
            a += wj * xv;
            b += wj * yv;
            aa += wj * (xv * xv);
            bb += wj * (yv * yv);
            ab += wj * (xv * yv);
        }
        pin(a);
        pin(b);
        pin(aa);
        pin(bb);
        pin(ab);
        // L1 at this row's centre pixel (output row r - R); selects, not branches, so that the
        // compiler cannot sink the row's arithmetic into conditional blocks (the LDS reads would
        // then stay live across rows and spill)
        if (r >= R && r < TH + R) l1 += (col_in && y0 + r < H) ? fabsf(px[R] - py[R]) : 0.f;
        queue_retire<2, LA, PH>(sp, q, r, lane);
        r0[r % 11] = a;
        r1[r % 11] = b;
        r2[r % 11] = aa;
        r3[r % 11] = bb;
        r4[r % 11] = ab;
        if (r >= 2 * R) {
            const int o = r - 2 * R;  // output row within the tile
            float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
            for (int i = 0; i < 11; i++) {
                const int qs = (o + i) % 11;
                const float wi = win.w[i];
                m1 += wi * r0[qs];
                m2 += wi * r1[qs];
                e11 += wi * r2[qs];
                e22 += wi * r3[qs];
                e12 += wi * r4[qs];
            }
            const int gy = blockIdx.y * TH + o;
            {
                const float m1s = m1 * m1, m2s = m2 * m2, m12 = m1 * m2;
                const float s11 = e11 - m1s, s22 = e22 - m2s, s12 = e12 - m12;
                const float A = 2.f * m12 + C1, B = 2.f * s12 + C2;
                const float Cd = m1s + m2s + C1, Dd = s11 + s22 + C2;
                const float inv_cd = rcp_nr(Cd), inv_dd = rcp_nr(Dd);
                const float cdd = inv_cd * inv_dd;
                const float S = (A * B) * cdd;
                s_val += (col_in && gy < H) ? S : 0.f;
                // buffer stores: lane offset fixed, row offset scalar; outside the image the
                // offsets fail the range check and the stores are dropped
                const int so = gy < H ? gy * 4 * W : kOOB;
                store_f32(k * (2.f * m2 * (B - A) * cdd - 2.f * m1 * S * (inv_cd - inv_dd)), ws[0], vo, so);
                store_f32(k * (-S * inv_dd), ws[1], vo, so);
                store_f32(k * (2.f * A * cdd), ws[2], vo, so);
            }
        }
    }
    // block partial sums (fixed order -> deterministic)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s_val += __shfl_xor(s_val, o);
        l1 += __shfl_xor(l1, o);
    }
    if (lane == 0) {
        const int bid = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partial[bid] = make_float2(s_val, l1);
    }
}

// One block of 1024 threads; every thread keeps four independent double accumulators per sum so
// its loads are all in flight (a single chain of dependent adds made this a 25 us latency-bound
// kernel).  Fixed summation order: the result is deterministic.
constexpr int kFinT = 1024;
// Thread i's two sums of the fixed-order reduction, then its wave's butterfly (shared by the
// 1024-thread kernel and the one-wave form that rides on the backward launch: same order, same bits).
__device__ __forceinline__ void finalize_wave_sums(const float2* __restrict__ partial, int nb, int i, double& ss,
                                                   double& ll) {
    double s[4] = {0.0, 0.0, 0.0, 0.0}, l[4] = {0.0, 0.0, 0.0, 0.0};
    for (; i + 3 * kFinT < nb; i += 4 * kFinT) {
        float2 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = partial[i + k * kFinT];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            s[k] += v[k].x;
            l[k] += v[k].y;
        }
    }
    for (int k = 0; i < nb; i += kFinT, k++) {
        s[k] += partial[i].x;
        l[k] += partial[i].y;
    }
    ss = (s[0] + s[1]) + (s[2] + s[3]);
    ll = (l[0] + l[1]) + (l[2] + l[3]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ss += __shfl_xor(ss, o);
        ll += __shfl_xor(ll, o);
    }
}
// S, Lv: the 16 wave totals added in wave order
__device__ __forceinline__ void finalize_store(double S, double Lv, float lambda, float inv_n, float* __restrict__ loss,
                                               float* __restrict__ parts) {
    const float ssim = (float)(S * inv_n);
    const float l1 = (float)(Lv * inv_n);
    const float total = (1.0f - lambda) * l1 + lambda * (1.0f - ssim);
    loss[0] = total;
    if (parts) {
        parts[0] = total;
        parts[1] = l1;
        parts[2] = ssim;
    }
}
__global__ __launch_bounds__(kFinT) void k_loss_finalize(const float2* __restrict__ partial, int nb, float lambda,
                                                         float inv_n, float* __restrict__ loss,
                                                         float* __restrict__ parts) {
    __shared__ double rs[kFinT / 64], rl[kFinT / 64];
    double ss, ll;
    finalize_wave_sums(partial, nb, threadIdx.x, ss, ll);
    if ((threadIdx.x & 63) == 0) {
        rs[threadIdx.x >> 6] = ss;
        rl[threadIdx.x >> 6] = ll;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double S = 0.0, Lv = 0.0;
        for (int w = 0; w < kFinT / 64; w++) {
            S += rs[w];
            Lv += rl[w];
        }
        finalize_store(S, Lv, lambda, inv_n, loss, parts);
    }
}
// The same reduction by ONE wave standing in for the 16 waves in turn (an extra workgroup of the
// backward launch in rl_l1_ssim_forward_backward: one launch less per training step).
__device__ void loss_finalize_one_wave(const float2* __restrict__ partial, int nb, float lambda, float inv_n,
                                       float* __restrict__ loss, float* __restrict__ parts) {
    double S = 0.0, Lv = 0.0;
    for (int w = 0; w < kFinT / 64; w++) {
        double ss, ll;
        finalize_wave_sums(partial, nb, w * 64 + (int)threadIdx.x, ss, ll);
        S += ss;  // the butterfly left every lane with the wave total: the same additions in order
        Lv += ll;
    }
    if (threadIdx.x == 0) finalize_store(S, Lv, lambda, inv_n, loss, parts);
}

// Backward: the same streamed walk over the three forward maps (G1, G11, G12): horizontal pass
// from the LDS ring into an 11-row register ring, vertical pass from registers, then the
// pointwise chain rule.
template <int TH>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_ssim_bwd(const float* __restrict__ img, const float* __restrict__ gt, int H,
                                                 int W, float lambda, float inv_n, Win win,
                                                 const float* __restrict__ g1, const float* __restrict__ g11,
                                                 const float* __restrict__ g12, const float* __restrict__ grad_loss,
                                                 float* __restrict__ dimg, const float2* __restrict__ partial,
                                                 int nb, float* __restrict__ loss, float* __restrict__ parts) {
    if (loss && blockIdx.x == gridDim.x - 1) {  // the extra column (block-uniform): the forward's finalize
        if (blockIdx.y == 0 && blockIdx.z == 0) loss_finalize_one_wave(partial, nb, lambda, inv_n, loss, parts);
        return;
    }
    __shared__ float sg[3][NR][PW];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * TW - R, y0 = blockIdx.y * TH - R;
    const size_t plane = (size_t)H * W;
    const int lane = threadIdx.x;
    constexpr int PH = TH + 2 * R;  // input rows per band
    const Rsrc rs[3] = {plane_rsrc(g1 + c * plane, 4 * (int)plane), plane_rsrc(g11 + c * plane, 4 * (int)plane),
                        plane_rsrc(g12 + c * plane, 4 * (int)plane)};
    const Rsrc ps[3] = {plane_rsrc(img + c * plane, 4 * (int)plane), plane_rsrc(gt + c * plane, 4 * (int)plane),
                        plane_rsrc(dimg + c * plane, 4 * (int)plane)};
    const Band bd(x0, y0, H, W, lane);
    constexpr int LA = LA_BWD;
    PatchRow<3> q[LA + 1];
    prime<3, LA, PH>(rs, bd, sg, q, lane);
    const int gx = blockIdx.x * TW + lane;
    const int vo = gx < W ? 4 * gx : kOOB;
    const float gl = grad_loss[0];
    const float l1k = (1.f - lambda) * inv_n;
    float r0[11], r1[11], r2[11];
#pragma unroll
    for (int r = 0; r < PH; r++) {
        queue_issue<3, LA, PH>(rs, bd, q, r);
        const int slot = r % NR;
        const lds_ptr pa = row_base(&sg[0][slot][lane]);
        float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
        for (int j = 0; j < 11; j++) {
            const float wj = win.w[j];
            a += wj * pa[j];
            b += wj * pa[NR * PW + j];
            d += wj * pa[2 * NR * PW + j];
        }
        pin(a);
        pin(b);
        pin(d);
        queue_retire<3, LA, PH>(sg, q, r, lane);
        r0[r % 11] = a;
        r1[r % 11] = b;
        r2[r % 11] = d;
        if (r >= 2 * R) {
            const int o = r - 2 * R;
            const int gy = blockIdx.y * TH + o;
            float b1 = 0.f, b11 = 0.f, b12 = 0.f;
#pragma unroll
            for (int i = 0; i < 11; i++) {
                const int qs = (o + i) % 11;
                const float wi = win.w[i];
                b1 += wi * r0[qs];
                b11 += wi * r1[qs];
                b12 += wi * r2[qs];
            }
            {  // branch-free (see the forward): out-of-image offsets fail the range check
                const int so = gy < H ? gy * 4 * W : kOOB;
                const float xv = load_f32(ps[0], vo, so);
                const float yv = load_f32(ps[1], vo, so);
                const float dd = xv - yv;
                const float sgn = dd > 0.f ? 1.f : (dd < 0.f ? -1.f : 0.f);
                store_f32(gl * (b1 + 2.f * xv * b11 + yv * b12 + l1k * sgn), ps[2], vo, so);
            }
        }
    }
}

int nblocks(int C, int H, int W) { return ((W + TW - 1) / TW) * ((H + TH_FWD - 1) / TH_FWD) * C; }

// The two-pass forward + backward (the backward grid's extra column finalizes the loss, bitwise
// rl_l1_ssim_forward's, when `loss` is given).
void launch_fwd_bwd(const float* img, const float* gt, int C, int H, int W, float lambda, const Win& win, float* g1,
                    float2* partial, float* loss, float* parts, const float* grad_loss, float* dimg, hipStream_t st) {
    const size_t n = (size_t)C * H * W;
    const float inv_n = (float)(1.0 / (double)n);
    const dim3 gf((W + TW - 1) / TW, (H + TH_FWD - 1) / TH_FWD, C);
    k_ssim_fwd<TH_FWD><<<gf, 64, 0, st>>>(img, gt, H, W, lambda, inv_n, win, g1, g1 + n, g1 + 2 * n, partial);
    const dim3 gb((W + TW - 1) / TW + (loss ? 1 : 0), (H + TH_BWD - 1) / TH_BWD, C);
    k_ssim_bwd<TH_BWD><<<gb, 64, 0, st>>>(img, gt, H, W, lambda, inv_n, win, g1, g1 + n, g1 + 2 * n, grad_loss, dimg,
                                          partial, nblocks(C, H, W), loss, parts);
}

}  // namespace

extern "C" {

const char* rl_last_error(void) { return g_err.c_str(); }

size_t rl_workspace_bytes(int C, int H, int W) {
    return (size_t)3 * C * H * W * sizeof(float) + (size_t)nblocks(C, H, W) * sizeof(float2) + 256;
}

int rl_l1_ssim_forward(const float* img, const float* gt, int C, int H, int W, float lambda, const float* window,
                       void* workspace, size_t workspace_bytes, float* loss, float* parts, void* stream) {
    if (!img || !gt || !window || !workspace || !loss || C <= 0 || H <= 0 || W <= 0) {
        g_err = "rl_l1_ssim_forward: bad argument";
        return 1;
    }
    if ((size_t)H * W * 4 >= (size_t)kOOB) {  // buffer-descriptor range (one channel plane)
        g_err = "rl_l1_ssim_forward: image plane larger than 2^30 bytes";
        return 1;
    }
    if (workspace_bytes < rl_workspace_bytes(C, H, W) || nblocks(C, H, W) > NB_MAX) {
        g_err = "rl_l1_ssim_forward: workspace too small";
        return 3;
    }
    Win win;
    for (int i = 0; i < 11; i++) win.w[i] = window[i];
    const size_t n = (size_t)C * H * W;
    float* g1 = static_cast<float*>(workspace);
    float* g11 = g1 + n;
    float* g12 = g11 + n;
    float2* partial = reinterpret_cast<float2*>(g12 + n);
    const float inv_n = (float)(1.0 / (double)n);
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((W + TW - 1) / TW, (H + TH_FWD - 1) / TH_FWD, C);
    k_ssim_fwd<TH_FWD><<<grid, 64, 0, st>>>(img, gt, H, W, lambda, inv_n, win, g1, g11, g12, partial);
    k_loss_finalize<<<1, kFinT, 0, st>>>(partial, nblocks(C, H, W), lambda, inv_n, loss, parts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("rl_l1_ssim_forward: ") + hipGetErrorString(e);
        return 2;
    }
    return 0;
}

int rl_l1_ssim_backward(const float* img, const float* gt, int C, int H, int W, float lambda, const float* window,
                        const void* workspace, const float* grad_loss, float* dimg, void* stream) {
    if (!img || !gt || !window || !workspace || !grad_loss || !dimg || C <= 0 || H <= 0 || W <= 0) {
        g_err = "rl_l1_ssim_backward: bad argument";
        return 1;
    }
    if ((size_t)H * W * 4 >= (size_t)kOOB) {
        g_err = "rl_l1_ssim_backward: image plane larger than 2^30 bytes";
        return 1;
    }
    Win win;
    for (int i = 0; i < 11; i++) win.w[i] = window[i];
    const size_t n = (size_t)C * H * W;
    const float* g1 = static_cast<const float*>(workspace);
    const float inv_n = (float)(1.0 / (double)n);
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((W + TW - 1) / TW, (H + TH_BWD - 1) / TH_BWD, C);
    k_ssim_bwd<TH_BWD><<<grid, 64, 0, st>>>(img, gt, H, W, lambda, inv_n, win, g1, g1 + n, g1 + 2 * n, grad_loss, dimg,
                                            nullptr, 0, nullptr, nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("rl_l1_ssim_backward: ") + hipGetErrorString(e);
        return 2;
    }
    return 0;
}

int rl_l1_ssim_forward_backward(const float* img, const float* gt, int C, int H, int W, float lambda,
                                const float* window, void* workspace, size_t workspace_bytes, float* loss,
                                float* parts, const float* grad_loss, float* dimg, void* stream) {
    if (!img || !gt || !window || !workspace || !loss || !grad_loss || !dimg || C <= 0 || H <= 0 || W <= 0) {
        g_err = "rl_l1_ssim_forward_backward: bad argument";
        return 1;
    }
    if ((size_t)H * W * 4 >= (size_t)kOOB) {
        g_err = "rl_l1_ssim_forward_backward: image plane larger than 2^30 bytes";
        return 1;
    }
    if (workspace_bytes < rl_workspace_bytes(C, H, W) || nblocks(C, H, W) > NB_MAX) {
        g_err = "rl_l1_ssim_forward_backward: workspace too small";
        return 3;
    }
    Win win;
    for (int i = 0; i < 11; i++) win.w[i] = window[i];
    const size_t n = (size_t)C * H * W;
    float* g1 = static_cast<float*>(workspace);
    float2* partial = reinterpret_cast<float2*>(g1 + 3 * n);
    const float inv_n = (float)(1.0 / (double)n);
    hipStream_t st = (hipStream_t)stream;
    launch_fwd_bwd(img, gt, C, H, W, lambda, win, g1, partial, loss, parts, grad_loss, dimg, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("rl_l1_ssim_forward_backward: ") + hipGetErrorString(e);
        return 2;
    }
    return 0;
}

}  // extern "C"
