// loss.hip — fused L1 + SSIM training loss, forward and backward (include/rain_loss.h).
//
// Replaces the reference's five depthwise 11x11 conv2d calls per SSIM evaluation plus their
// autograd (utils/loss_utils.py:22-53, train.py:113-115), which on ROCm go through MIOpen's
// generic convolution paths.  One workgroup per 16x16 output tile and channel: the 26x26 input
// patch (5-pixel halo, zero padded like conv2d padding=5) is staged in LDS, the separable Gaussian
// is applied as an 11-tap horizontal pass over 26 rows and an 11-tap vertical pass, and all five
// moment maps (E[x], E[y], E[x^2], E[y^2], E[xy]) come out of the same pass.
//
//   S = (2 m1 m2 + C1)(2 s12 + C2) / ((m1^2 + m2^2 + C1)(s11 + s22 + C2)),  s.. = E[..] - m.m.
//   dS/dm1 = 2 m2 (B - A) / (Cd Dd) - 2 m1 S (1/Cd - 1/Dd),  dS/dE[x^2] = -S / Dd,
//   dS/dE[xy] = 2 A / (Cd Dd)
// dL/dx = blur(G1) + 2 x blur(G11) + y blur(G12) + (1-lambda) sign(x-y)/(CHW)   (blur is self-adjoint:
// symmetric window, zero padding), with G.. = -lambda/(CHW) dS/d.. stored by the forward.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/rain_loss.h"

namespace {

constexpr int TS = 16;           // output tile
constexpr int R = 5;             // window radius (11 taps)
constexpr int PT = TS + 2 * R;   // 26: patch with halo
constexpr int NB_MAX = 1 << 20;  // partial-sum slots

thread_local std::string g_err;

struct Win {
    float w[11];
};

__device__ __forceinline__ int tile_blocks(int W) { return (W + TS - 1) / TS; }

__global__ __launch_bounds__(256) void k_ssim_fwd(const float* __restrict__ img, const float* __restrict__ gt, int H,
                                                  int W, float lambda, float inv_n, Win win, float* __restrict__ g1,
                                                  float* __restrict__ g11, float* __restrict__ g12,
                                                  float2* __restrict__ partial) {
    __shared__ float sx[PT][PT + 1];
    __shared__ float sy[PT][PT + 1];
    __shared__ float hs[5][PT][TS];
    __shared__ float red[2][4];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * TS - R, y0 = blockIdx.y * TS - R;
    const size_t plane = (size_t)H * W;
    const float* X = img + c * plane;
    const float* Y = gt + c * plane;
    const int t = threadIdx.x;
    for (int i = t; i < PT * PT; i += 256) {
        const int r = i / PT, q = i % PT;
        const int gy = y0 + r, gx = x0 + q;
        const bool in = gx >= 0 && gx < W && gy >= 0 && gy < H;
        sx[r][q] = in ? X[(size_t)gy * W + gx] : 0.f;
        sy[r][q] = in ? Y[(size_t)gy * W + gx] : 0.f;
    }
    __syncthreads();
    for (int i = t; i < PT * TS; i += 256) {
        const int r = i / TS, q = i % TS;
        float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
        for (int j = 0; j < 11; j++) {
            const float xv = sx[r][q + j], yv = sy[r][q + j], w = win.w[j];
            a += w * xv;
            b += w * yv;
            aa += w * (xv * xv);
            bb += w * (yv * yv);
            ab += w * (xv * yv);
        }
        hs[0][r][q] = a;
        hs[1][r][q] = b;
        hs[2][r][q] = aa;
        hs[3][r][q] = bb;
        hs[4][r][q] = ab;
    }
    __syncthreads();
    const int tx = t % TS, ty = t / TS;
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const float w = win.w[i];
        m1 += w * hs[0][ty + i][tx];
        m2 += w * hs[1][ty + i][tx];
        e11 += w * hs[2][ty + i][tx];
        e22 += w * hs[3][ty + i][tx];
        e12 += w * hs[4][ty + i][tx];
    }
    const int gx = blockIdx.x * TS + tx, gy = blockIdx.y * TS + ty;
    const bool inside = gx < W && gy < H;
    float s_val = 0.f, l1 = 0.f;
    if (inside) {
        const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
        const float m1s = m1 * m1, m2s = m2 * m2, m12 = m1 * m2;
        const float s11 = e11 - m1s, s22 = e22 - m2s, s12 = e12 - m12;
        const float A = 2.f * m12 + C1, B = 2.f * s12 + C2;
        const float Cd = m1s + m2s + C1, Dd = s11 + s22 + C2;
        const float inv_cd = 1.f / Cd, inv_dd = 1.f / Dd;
        const float S = (A * B) * (inv_cd * inv_dd);
        s_val = S;
        const float xv = sx[ty + R][tx + R], yv = sy[ty + R][tx + R];
        l1 = fabsf(xv - yv);
        const float k = -lambda * inv_n;
        const size_t o = c * plane + (size_t)gy * W + gx;
        g1[o] = k * (2.f * m2 * (B - A) * inv_cd * inv_dd - 2.f * m1 * S * (inv_cd - inv_dd));
        g11[o] = k * (-S * inv_dd);
        g12[o] = k * (2.f * A * inv_cd * inv_dd);
    }
    // block partial sums (fixed order -> deterministic)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s_val += __shfl_xor(s_val, o);
        l1 += __shfl_xor(l1, o);
    }
    if ((t & 63) == 0) {
        red[0][t >> 6] = s_val;
        red[1][t >> 6] = l1;
    }
    __syncthreads();
    if (t == 0) {
        const int bid = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partial[bid] = make_float2(red[0][0] + red[0][1] + red[0][2] + red[0][3],
                                   red[1][0] + red[1][1] + red[1][2] + red[1][3]);
    }
}

// One block of 1024 threads; every thread keeps four independent double accumulators per sum so
// its loads are all in flight (a single chain of dependent adds made this a 25 us latency-bound
// kernel).  Fixed summation order: the result is deterministic.
constexpr int kFinT = 1024;
__global__ __launch_bounds__(kFinT) void k_loss_finalize(const float2* __restrict__ partial, int nb, float lambda,
                                                         float inv_n, float* __restrict__ loss,
                                                         float* __restrict__ parts) {
    __shared__ double rs[kFinT / 64], rl[kFinT / 64];
    double s[4] = {0.0, 0.0, 0.0, 0.0}, l[4] = {0.0, 0.0, 0.0, 0.0};
    int i = threadIdx.x;
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
    double ss = (s[0] + s[1]) + (s[2] + s[3]), ll = (l[0] + l[1]) + (l[2] + l[3]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ss += __shfl_xor(ss, o);
        ll += __shfl_xor(ll, o);
    }
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
}

__global__ __launch_bounds__(256) void k_ssim_bwd(const float* __restrict__ img, const float* __restrict__ gt, int H,
                                                  int W, float lambda, float inv_n, Win win,
                                                  const float* __restrict__ g1, const float* __restrict__ g11,
                                                  const float* __restrict__ g12, const float* __restrict__ grad_loss,
                                                  float* __restrict__ dimg) {
    __shared__ float sg[3][PT][PT + 1];
    __shared__ float hs[3][PT][TS];
    const int c = blockIdx.z;
    const int x0 = blockIdx.x * TS - R, y0 = blockIdx.y * TS - R;
    const size_t plane = (size_t)H * W;
    const int t = threadIdx.x;
    for (int i = t; i < PT * PT; i += 256) {
        const int r = i / PT, q = i % PT;
        const int gy = y0 + r, gx = x0 + q;
        const bool in = gx >= 0 && gx < W && gy >= 0 && gy < H;
        const size_t o = c * plane + (size_t)gy * W + gx;
        sg[0][r][q] = in ? g1[o] : 0.f;
        sg[1][r][q] = in ? g11[o] : 0.f;
        sg[2][r][q] = in ? g12[o] : 0.f;
    }
    __syncthreads();
    for (int i = t; i < PT * TS; i += 256) {
        const int r = i / TS, q = i % TS;
        float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
        for (int j = 0; j < 11; j++) {
            const float w = win.w[j];
            a += w * sg[0][r][q + j];
            b += w * sg[1][r][q + j];
            d += w * sg[2][r][q + j];
        }
        hs[0][r][q] = a;
        hs[1][r][q] = b;
        hs[2][r][q] = d;
    }
    __syncthreads();
    const int tx = t % TS, ty = t / TS;
    const int gx = blockIdx.x * TS + tx, gy = blockIdx.y * TS + ty;
    if (gx >= W || gy >= H) return;
    float b1 = 0.f, b11 = 0.f, b12 = 0.f;
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const float w = win.w[i];
        b1 += w * hs[0][ty + i][tx];
        b11 += w * hs[1][ty + i][tx];
        b12 += w * hs[2][ty + i][tx];
    }
    const size_t o = c * plane + (size_t)gy * W + gx;
    const float xv = img[o], yv = gt[o];
    const float d = xv - yv;
    const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    const float g = b1 + 2.f * xv * b11 + yv * b12 + (1.f - lambda) * inv_n * sgn;
    dimg[o] = grad_loss[0] * g;
}

int nblocks(int C, int H, int W) { return ((W + TS - 1) / TS) * ((H + TS - 1) / TS) * C; }

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
    dim3 grid((W + TS - 1) / TS, (H + TS - 1) / TS, C);
    k_ssim_fwd<<<grid, 256, 0, st>>>(img, gt, H, W, lambda, inv_n, win, g1, g11, g12, partial);
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
    Win win;
    for (int i = 0; i < 11; i++) win.w[i] = window[i];
    const size_t n = (size_t)C * H * W;
    const float* g1 = static_cast<const float*>(workspace);
    const float inv_n = (float)(1.0 / (double)n);
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((W + TS - 1) / TS, (H + TS - 1) / TS, C);
    k_ssim_bwd<<<grid, 256, 0, st>>>(img, gt, H, W, lambda, inv_n, win, g1, g1 + n, g1 + 2 * n, grad_loss, dimg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("rl_l1_ssim_backward: ") + hipGetErrorString(e);
        return 2;
    }
    return 0;
}

}  // extern "C"
