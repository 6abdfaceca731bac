// rr_common.hpp — shared device helpers and data layout of the MI355X rasterizer.
//
// Layout decisions (see DESIGN.md §Data layout in HBM):
//   * Splat (48 B, AoS, 16-B aligned): everything the per-tile blend kernels need for one
//     Gaussian, so a (tile, Gaussian) pair costs one 4-B id load plus three 16-B loads of one
//     record, instead of the reference's id + xy + conic_opacity + per-use rgb/depth gathers
//     (forward.cu:310-349).
//       a = {x_pix, y_pix, qa, qb}
//       b = {qc, log2(opacity), depth(view z), opacity}
//       c = {r, g, b, 1/opacity}   (SH colour, or colors_precomp copied in)
//     with the conic pre-scaled into the exponent's log2 units (blend_p2): qa = -log2(e)/2 conic.x,
//     qb = -log2(e) conic.y, qc = -log2(e)/2 conic.z, so a pixel's alpha costs 3 fma-class ops and
//     one exp2 of (p2 + log2 opacity) instead of the reference's 6 ops, a scaling and a multiply.
//   * Backward accumulators: 16 floats (one 64-B line) per Gaussian, components
//     0..1 dL/dmean2D(ndc), 2..4 dL/dconic (x,y,w), 5 dL/dopacity, 6..8 dL/dcolor.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rr {

constexpr int TILE_X = 16;
constexpr int TILE_Y = 16;
constexpr int TILE_PIX = TILE_X * TILE_Y;  // 256 threads = 4 wave64 per tile
constexpr int GACC_STRIDE = 16;            // floats per Gaussian in the backward accumulator
constexpr int NGRAD = 9;                   // accumulated components per (tile, Gaussian) pair

struct alignas(16) Splat {
    float4 a;
    float4 b;
    float4 c;
};

// auxiliary.h:11-28
#define RR_SH_C0 0.28209479177387814f
#define RR_SH_C1 0.4886025119029199f
#define RR_SH_C2_0 1.0925484305920792f
#define RR_SH_C2_1 -1.0925484305920792f
#define RR_SH_C2_2 0.31539156525252005f
#define RR_SH_C2_3 -1.0925484305920792f
#define RR_SH_C2_4 0.5462742152960396f
#define RR_SH_C3_0 -0.5900435899266435f
#define RR_SH_C3_1 2.890611442640554f
#define RR_SH_C3_2 -0.4570457994644658f
#define RR_SH_C3_3 0.3731763325901154f
#define RR_SH_C3_4 -0.4570457994644658f
#define RR_SH_C3_5 1.445305721320277f
#define RR_SH_C3_6 -0.5900435899266435f

struct v3 {
    float x, y, z;
};
__device__ __forceinline__ v3 mk(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 operator*(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

__device__ __forceinline__ v3 load3(const float* p) { return mk(p[0], p[1], p[2]); }

// ndc2Pix (auxiliary.h:30-33): evaluated in double like the reference.
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// getRect (auxiliary.h:35-45): C truncation toward zero, clamped to [0, grid].
__device__ __forceinline__ void tile_rect(float px, float py, int r, int gx, int gy, int& x0, int& y0, int& x1,
                                          int& y1) {
    x0 = min(gx, max(0, (int)((px - r) / TILE_X)));
    y0 = min(gy, max(0, (int)((py - r) / TILE_Y)));
    x1 = min(gx, max(0, (int)((px + r + TILE_X - 1) / TILE_X)));
    y1 = min(gy, max(0, (int)((py + r + TILE_Y - 1) / TILE_Y)));
}

// ---- exact tile culling ---------------------------------------------------------------
// The reference emits a (tile, Gaussian) pair for every tile of the 3-sigma bounding square.  A
// pair whose Gaussian reaches no pixel of the tile with alpha >= 1/255 is skipped by every pixel
// in both blend kernels (forward.cu:329-338, backward.cu:485-491) and so changes no output.  Such
// pairs are dropped here with a conservative test: a tile is kept iff the ellipse
// {d : d^T conic d <= 2 ln(255 o) + margin} meets the continuous rectangle spanned by the tile's
// pixel centres (a superset of the discrete pixels); the margin covers fp32 / fast-exp rounding
// in the blend.  Non positive-definite conics are never culled.
__device__ __forceinline__ float cull_qmax(float opacity) {
    // alpha = o*exp(-q/2) >= 1/255  <=>  q <= 2 ln(255 o); +0.02 absolute / +1e-4 relative margin
    const float t = 2.0f * (logf(255.0f * opacity) + 0.01f);
    return t + 1e-4f * fabsf(t);
}
// Evaluated per tile row, O(rows) instead of O(tiles): the set {q <= qmax} is an
// ellipse, its intersection with tile row ty's pixel-centre band [y0, y1] is convex, so its
// x-projection is one interval [xl, xr] and the row's touched tiles are the contiguous columns
// whose pixel-centre span [16 tx, 16 tx + 15] meets it.  xr over the band is the concave
// x_right(y) = (-cb y + sqrt(ca qmax - D y^2)) / ca maximised at y clamped to the ellipse's
// rightmost point y* = -cb xmax / cc (mirror for xl).  Slack of 1e-3 px + 1e-5 relative keeps
// it conservative against rounding — including that of the hardware square root and reciprocal
// (<= 1-2 ulp) used here — and the q margin of cull_qmax covers the blend's.
// The per-Gaussian part (cull_setup) is computed once; cull_row_span is the per-row part.  The
// preprocess (counting) and the duplicate (emitting) evaluate both on the same inputs with the
// same op sequence (no contraction), so they agree on every Gaussian's pair count bit for bit.
struct CullEll {
    float mx, my, ca, cb, qmax, D, yext, xmax, ystar, inv_ca, slack_y, slack_x;
    int mode;  // 0 ellipse, 1 not a proper ellipse (keep the rect row), 2 opacity < 1/255 everywhere (empty)
};
__device__ __forceinline__ CullEll cull_setup(float mx, float my, float ca, float cb, float cc, float qmax) {
#pragma clang fp contract(off)
    CullEll e;
    e.mx = mx;
    e.my = my;
    e.ca = ca;
    e.cb = cb;
    e.qmax = qmax;
    e.D = ca * cc - cb * cb;
    e.mode = !(ca > 0.f && cc > 0.f && e.D > 0.f) ? 1 : !(qmax > 0.f) ? 2 : 0;
    const float qd = qmax * __builtin_amdgcn_rcpf(e.D);
    e.yext = __builtin_amdgcn_sqrtf(ca * qd);
    e.xmax = __builtin_amdgcn_sqrtf(cc * qd);
    e.ystar = -cb * e.xmax * __builtin_amdgcn_rcpf(cc);  // rightmost point; leftmost is at -ystar
    e.inv_ca = __builtin_amdgcn_rcpf(ca);
    e.slack_y = 1e-3f + 1e-5f * e.yext;
    e.slack_x = 1e-3f + 1e-5f * e.xmax;
    return e;
}
// Column range [*lo, *hi) of tile row ty, clipped to the bounding rect [x0, x1); empty rows give
// lo >= hi.
__device__ __forceinline__ void cull_row_span(const CullEll& e, int ty, int x0, int x1, int* lo, int* hi) {
#pragma clang fp contract(off)
    if (e.mode == 1) {
        *lo = x0;
        *hi = x1;
        return;
    }
    const float by0 = (float)(ty * TILE_Y) - e.my, by1 = by0 + (float)(TILE_Y - 1);
    const float ya = fmaxf(by0, -e.yext), yb = fminf(by1, e.yext);
    if (e.mode == 2 || ya > yb + e.slack_y) {
        *lo = x1;
        *hi = x1;
        return;
    }
    const float yr = fminf(fmaxf(e.ystar, ya), yb);
    const float yl = fminf(fmaxf(-e.ystar, ya), yb);
    const float cq = e.ca * e.qmax;
    const float xr = (-e.cb * yr + __builtin_amdgcn_sqrtf(fmaxf(cq - e.D * yr * yr, 0.f))) * e.inv_ca;
    const float xl = (-e.cb * yl - __builtin_amdgcn_sqrtf(fmaxf(cq - e.D * yl * yl, 0.f))) * e.inv_ca;
    if (!(xr >= xl) || !(xr - xl < 3.0e38f)) {  // non-finite arithmetic: stay conservative
        *lo = x0;
        *hi = x1;
        return;
    }
    // tile tx is touched iff 16 tx - mx <= xr and 16 tx + 15 - mx >= xl
    const float vl = (xl - e.slack_x + e.mx - (float)(TILE_X - 1)) * (1.0f / TILE_X);
    const float vh = (xr + e.slack_x + e.mx) * (1.0f / TILE_X);
    *lo = (int)ceilf(fminf(fmaxf(vl, (float)x0), (float)x1));
    *hi = (int)floorf(fminf(fmaxf(vh, (float)x0 - 1.f), (float)x1 - 1.f)) + 1;
}

// ---- bins: 2 x 2 blend tiles (32 x 32 px) ------------------------------------------------------
// The binning sorts (bin, Gaussian) pairs instead of (tile, Gaussian) pairs: a Gaussian that
// covers a 3 x 3 block of tiles covers ~2 x 2 bins, so about half as many pairs are emitted,
// sorted and stored, on fewer key bits.  A pair carries the 4-bit mask of the bin's tiles the
// Gaussian reaches (bit 2 r + c: tile row r, column c of the bin) in the top bits of its value;
// after the sort, k_expand splits every bin's list into its four per-tile lists (stable), so the
// blend kernels still walk exact per-tile lists in (depth, index) order.
constexpr int BIN_SHIFT = 28;                     // value = gaussian | mask << BIN_SHIFT (P < 2^28)
constexpr uint32_t BIN_ID_MASK = (1u << BIN_SHIFT) - 1u;
__host__ __device__ __forceinline__ int bins_x(int gx) { return (gx + 1) >> 1; }
__host__ __device__ __forceinline__ int bins_y(int gy) { return (gy + 1) >> 1; }

// The two tile rows 2Y, 2Y+1 of bin row Y: the tile-column span [l, h) each row's pixels are
// reached in (exact culling, cull_row_span) or the bounding rect's columns; rows outside [y0, y1)
// are empty.
__device__ __forceinline__ void bin_row_spans(const CullEll& e, int cull, int Y, int x0, int x1, int y0, int y1,
                                              int& l0, int& h0, int& l1, int& h1) {
    l0 = h0 = l1 = h1 = x0;
    const int ya = 2 * Y, yb = 2 * Y + 1;
    if (ya >= y0 && ya < y1) {
        l0 = x0;
        h0 = x1;
        if (cull) cull_row_span(e, ya, x0, x1, &l0, &h0);
    }
    if (yb >= y0 && yb < y1) {
        l1 = x0;
        h1 = x1;
        if (cull) cull_row_span(e, yb, x0, x1, &l1, &h1);
    }
}
// Mask of bin column X given its two rows' spans (bit 2 r + c = tile (2Y + r, 2X + c) reached).
__device__ __forceinline__ uint32_t bin_mask(int X, int l0, int h0, int l1, int h1) {
    const int c0 = 2 * X, c1 = 2 * X + 1;
    return (uint32_t)(c0 >= l0 && c0 < h0) | ((uint32_t)(c1 >= l0 && c1 < h0) << 1) |
           ((uint32_t)(c0 >= l1 && c0 < h1) << 2) | ((uint32_t)(c1 >= l1 && c1 < h1) << 3);
}
// Bin columns [Xa, Xb) that can hold a non-zero mask in a bin row.
__device__ __forceinline__ void bin_cols(int l0, int h0, int l1, int h1, int& Xa, int& Xb) {
    const bool e0 = h0 <= l0, e1 = h1 <= l1;
    const int lo = e0 ? l1 : (e1 ? l0 : min(l0, l1));
    const int hi = e0 ? h1 : (e1 ? h0 : max(h0, h1));
    Xa = lo >> 1;
    Xb = (e0 && e1) ? Xa : (hi + 1) >> 1;
}

// Number of bin columns X with bin_mask(X, ...) != 0, in closed form: the bins a non-empty span
// [l, h) touches are [l / 2, (h - 1) / 2], and a bin counts once if both rows touch it.  (A loop
// over the columns makes a wave wait for its widest Gaussian's row length times every row.)
__device__ __forceinline__ uint32_t bin_count(int l0, int h0, int l1, int h1) {
    const bool e0 = h0 <= l0, e1 = h1 <= l1;
    const int a0 = l0 >> 1, b0 = (h0 - 1) >> 1, a1 = l1 >> 1, b1 = (h1 - 1) >> 1;
    const int n0 = e0 ? 0 : b0 - a0 + 1, n1 = e1 ? 0 : b1 - a1 + 1;
    const int ov = (e0 || e1) ? 0 : max(0, min(b0, b1) - max(a0, a1) + 1);
    return (uint32_t)(n0 + n1 - ov);
}

// Column-major 4x4 transforms (auxiliary.h:47-86).  Matrices live in device memory and are
// indexed with wave-uniform offsets, so the compiler keeps them in SGPRs (s_load).
__device__ __forceinline__ v3 xform_point_4x3(v3 p, const float* m) {
    return mk(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
              m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ __forceinline__ float4 xform_point_4x4(v3 p, const float* m) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}
__device__ __forceinline__ v3 xform_vec_4x3_T(v3 p, const float* m) {
    return mk(m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
              m[8] * p.x + m[9] * p.y + m[10] * p.z);
}

// GaussianModel getters (gaussian_model.py:85-105) for raw-parameter mode, written as torch
// evaluates them: exp, x / clamp_min(|x|_2, 1e-12) (F.normalize), 1 / (1 + exp(-x)).
__device__ __forceinline__ v3 act_scale(v3 s) { return mk(expf(s.x), expf(s.y), expf(s.z)); }
__device__ __forceinline__ float4 act_rot(float4 q) {
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
    return make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}
__device__ __forceinline__ float act_opacity(float o) { return 1.0f / (1.0f + expf(-o)); }

// Quaternion (r,x,y,z) -> row-major rotation (forward.cu:116-127 builds its transpose in glm).
__device__ __forceinline__ void quat_rot(float4 q, float R[3][3]) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

// Auxiliary surface normal (BASELINE configs[4] depth + normal outputs; the reference renders no
// normals): the world axis of the Gaussian's smallest scale (a column of R), rotated into view
// space, flipped to face the camera, unit length.  Same op order as gaussian_normal in
// oracle/raster_oracle.c.
__device__ __forceinline__ float4 gaussian_normal(v3 sc, float4 q, const float* view, v3 p_view) {
    float R[3][3];
    quat_rot(q, R);
    int k = 0;
    if (sc.y < (k == 0 ? sc.x : sc.y)) k = 1;
    if (sc.z < (k == 0 ? sc.x : sc.y)) k = 2;
    const v3 n = k == 0 ? mk(R[0][0], R[1][0], R[2][0]) : k == 1 ? mk(R[0][1], R[1][1], R[2][1])
                                                                 : mk(R[0][2], R[1][2], R[2][2]);
    v3 nv = mk(view[0] * n.x + view[4] * n.y + view[8] * n.z, view[1] * n.x + view[5] * n.y + view[9] * n.z,
               view[2] * n.x + view[6] * n.y + view[10] * n.z);
    if (dot(nv, p_view) > 0.f) nv = mk(-nv.x, -nv.y, -nv.z);
    const float len = sqrtf(dot(nv, nv));
    return len > 0.f ? make_float4(nv.x / len, nv.y / len, nv.z / len, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Sigma = M^T M with M[i][j] = s_i R[j][i]  (forward.cu:129-140).  Used by the forward
// preprocess AND recomputed by the backward (no cov3D round trip through HBM).
__device__ __forceinline__ void cov3d_from_scale_rot(v3 scale, float mod, float4 q, float cov[6]) {
    float R[3][3];
    quat_rot(q, R);
    const float s[3] = {mod * scale.x, mod * scale.y, mod * scale.z};
    float M[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) M[i][j] = s[i] * R[j][i];
    cov[0] = M[0][0] * M[0][0] + M[1][0] * M[1][0] + M[2][0] * M[2][0];
    cov[1] = M[0][0] * M[0][1] + M[1][0] * M[1][1] + M[2][0] * M[2][1];
    cov[2] = M[0][0] * M[0][2] + M[1][0] * M[1][2] + M[2][0] * M[2][2];
    cov[3] = M[0][1] * M[0][1] + M[1][1] * M[1][1] + M[2][1] * M[2][1];
    cov[4] = M[0][1] * M[0][2] + M[1][1] * M[1][2] + M[2][1] * M[2][2];
    cov[5] = M[0][2] * M[0][2] + M[1][2] * M[1][2] + M[2][2] * M[2][2];
}

// EWA projection pieces shared by forward preprocess (forward.cu:63-102) and the backward
// (backward.cu:154-189): clamped view-space mean t, A = J·W (glm's T[i][j] == A[i][j]).
struct Proj2D {
    v3 t;
    float txtz, tytz, limx, limy;
    float A[2][3];
};
__device__ __forceinline__ Proj2D ewa_setup(v3 mean, float fx, float fy, float tanfovx, float tanfovy,
                                            const float* view) {
    Proj2D p;
    v3 t = xform_point_4x3(mean, view);
    p.limx = 1.3f * tanfovx;
    p.limy = 1.3f * tanfovy;
    p.txtz = t.x / t.z;
    p.tytz = t.y / t.z;
    t.x = fminf(p.limx, fmaxf(-p.limx, p.txtz)) * t.z;
    t.y = fminf(p.limy, fmaxf(-p.limy, p.tytz)) * t.z;
    p.t = t;
    const float J00 = fx / t.z, J02 = -(fx * t.x) / (t.z * t.z);
    const float J11 = fy / t.z, J12 = -(fy * t.y) / (t.z * t.z);
#pragma unroll
    for (int j = 0; j < 3; j++) {
        p.A[0][j] = J00 * view[4 * j + 0] + J02 * view[4 * j + 2];
        p.A[1][j] = J11 * view[4 * j + 1] + J12 * view[4 * j + 2];
    }
    return p;
}
// (a, b, c) of A V A^T before dilation, associated as glm evaluates transpose(T) * transpose(Vrk) * T
// (forward.cu:95): B = A V is (T^T Vrk^T)[k][r] = B[r][k], and cov[c][r] = sum_k B[r][k] A[c][k], so
// the returned cov[0][1] is B[1] . A[0] (not B[0] . A[1], equal only in exact arithmetic).
__device__ __forceinline__ void ewa_cov2d(const Proj2D& p, const float cov[6], float& a, float& b, float& c) {
    const float V[3][3] = {{cov[0], cov[1], cov[2]}, {cov[1], cov[3], cov[4]}, {cov[2], cov[4], cov[5]}};
    float B[2][3];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) B[i][j] = p.A[i][0] * V[0][j] + p.A[i][1] * V[1][j] + p.A[i][2] * V[2][j];
    a = B[0][0] * p.A[0][0] + B[0][1] * p.A[0][1] + B[0][2] * p.A[0][2];
    b = B[1][0] * p.A[0][0] + B[1][1] * p.A[0][1] + B[1][2] * p.A[0][2];
    c = B[1][0] * p.A[1][0] + B[1][1] * p.A[1][1] + B[1][2] * p.A[1][2];
}

// SH -> RGB (forward.cu:9-60), degree known at compile time.  Returns the pre-clamp value.
// Coefficient 0 is dc[0..3), coefficient k >= 1 is rest[3(k-1)..): one contiguous [M,3] block
// (dc = sh, rest = sh + 3) or the model's separate f_dc / f_rest tensors (raw-parameter mode).
template <int DEG>
__device__ __forceinline__ v3 sh_eval(v3 dir, v3 dc, const float* rest) {
    v3 r = RR_SH_C0 * dc;
    if (DEG > 0) {
        const float x = dir.x, y = dir.y, z = dir.z;
        r = r - (RR_SH_C1 * y) * load3(rest + 0) + (RR_SH_C1 * z) * load3(rest + 3) - (RR_SH_C1 * x) * load3(rest + 6);
        if (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            r = r + (RR_SH_C2_0 * xy) * load3(rest + 9);
            r = r + (RR_SH_C2_1 * yz) * load3(rest + 12);
            r = r + (RR_SH_C2_2 * (2.0f * zz - xx - yy)) * load3(rest + 15);
            r = r + (RR_SH_C2_3 * xz) * load3(rest + 18);
            r = r + (RR_SH_C2_4 * (xx - yy)) * load3(rest + 21);
            if (DEG > 2) {
                r = r + (RR_SH_C3_0 * y * (3.0f * xx - yy)) * load3(rest + 24);
                r = r + (RR_SH_C3_1 * xy * z) * load3(rest + 27);
                r = r + (RR_SH_C3_2 * y * (4.0f * zz - xx - yy)) * load3(rest + 30);
                r = r + (RR_SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy)) * load3(rest + 33);
                r = r + (RR_SH_C3_4 * x * (4.0f * zz - xx - yy)) * load3(rest + 36);
                r = r + (RR_SH_C3_5 * z * (xx - yy)) * load3(rest + 39);
                r = r + (RR_SH_C3_6 * x * (xx - 3.0f * yy)) * load3(rest + 42);
            }
        }
    }
    return mk(r.x + 0.5f, r.y + 0.5f, r.z + 0.5f);
}
template <int DEG>
__device__ __forceinline__ v3 sh_eval(v3 dir, const float* dc, const float* rest) {
    return sh_eval<DEG>(dir, load3(dc), rest);
}

// N consecutive floats at a dword-aligned address, as 16-B loads (the target runs in unaligned
// access mode, so a 16-B global load needs only dword alignment) plus a scalar tail.
template <int N>
__device__ __forceinline__ void load_floats_u(const float* p, float (&out)[N > 0 ? N : 1]) {
    typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
#pragma unroll
    for (int i = 0; i + 4 <= N; i += 4) {
        const f4u v = *reinterpret_cast<const f4u*>(p + i);
        out[i] = v.x;
        out[i + 1] = v.y;
        out[i + 2] = v.z;
        out[i + 3] = v.w;
    }
#pragma unroll
    for (int i = N & ~3; i < N; i++) out[i] = p[i];
}

// Prefetch of one Splat record into three float4 registers.  Plain float4 variables: keeping
// the prefetched record in a struct made hipcc place it in scratch (private memory).
__device__ __forceinline__ void load_splat(const Splat* __restrict__ s, uint32_t i, float4& a, float4& b, float4& c) {
    const float4* p = reinterpret_cast<const float4*>(s + i);
    a = p[0];
    b = p[1];
    c = p[2];
}

// 1/x from v_rcp_f32 (1 ulp) refined by one Newton step (~0.5 ulp): 4 VALU ops instead of the
// ~10-op IEEE division sequence hipcc emits for '/' and __fdividef.  x = 1 - alpha is in [0.01, 1).
__device__ __forceinline__ float rcp_nr(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(r, __builtin_fmaf(-x, r, 1.0f), r);
}

// Bijective block -> tile remap (cdna_hip_programming.md §5, "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_tile(int b, int n) {
    const int q = n >> 3, r = n & 7;
    const int x = b & 7, s = b >> 3;
    return x < r ? x * (q + 1) + s : r * (q + 1) + (x - r) * q + s;
}

// Falloff of a (pair, pixel) (forward.cu:329-336 / backward.cu:481-491) in log2 units:
//   power = -0.5 (cx dx^2 + cz dy^2) - cy dx dy,   p2 = log2(e) power = qa dx^2 + qb dx dy + qc dy^2,
//   alpha = min(0.99, opacity exp(power)) = min(0.99, exp2(p2 + log2 opacity)),
// evaluated with one fixed op sequence (blend_p2_x per pair and lane, then blend_e2 per pixel;
// explicit fmas, no contraction) by both blend kernels, so forward and backward take
// bitwise-identical alpha decisions.  log2 opacity is folded into the per-lane x term, so a pixel
// gets e2 = p2 + log2 o from two fmas; the reference's power <= 0 test is e2 <= log2 o.
// dx, dy = mean - pixel.
constexpr float kLog2e = 1.44269504088896340736f;
constexpr float kQHalf = -0.5f * kLog2e;          // qa = kQHalf cx, qc = kQHalf cz
constexpr float kQFull = -kLog2e;                 // qb = kQFull cy
constexpr float kQHalfInv = -1.38629436111989061883f;  // -2 ln 2: cx = kQHalfInv qa (back-conversion, <= 2 ulp)
constexpr float kQFullInv = -0.69314718055994530942f;  // -ln 2
struct P2X {  // the x terms of e2, once per (pair, lane)
    float ax, bx;
};
__device__ __forceinline__ P2X blend_p2_x(float qa, float qb, float lo, float dx) {
#pragma clang fp contract(off)
    return P2X{(qa * dx) * dx + lo, qb * dx};
}
__device__ __forceinline__ float blend_e2(P2X x, float qc, float dy) {
    return __builtin_fmaf(__builtin_fmaf(qc, dy, x.bx), dy, x.ax);
}
// The raw conic (cx, cy, cz) and opacity of a record, for the tile culling and the backward's
// conic-gradient flush.
__device__ __forceinline__ void splat_conic(float4 a, float4 b, float& cx, float& cy, float& cz) {
    cx = a.z * kQHalfInv;
    cy = a.w * kQFullInv;
    cz = b.x * kQHalfInv;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Wave64 sum with DPP row shifts + row broadcasts; the total lands in lane 63.
// 6 DPP-fused adds (row_shr 1/2/4/8, row_bcast15, row_bcast31) — no LDS traffic.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK,
                                                                     0xf, true));
}
__device__ __forceinline__ float wave_sum_lane63(float v) {
    v = dpp_add<0x111, 0xf>(v);  // row_shr:1
    v = dpp_add<0x112, 0xf>(v);  // row_shr:2
    v = dpp_add<0x114, 0xf>(v);  // row_shr:4
    v = dpp_add<0x118, 0xf>(v);  // row_shr:8
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1,3
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2,3
    return v;
}

// Row-of-16 sum with DPP row shifts: lane 15 of each row ends up with that row's total.
__device__ __forceinline__ float row16_sum(float v) {
    v = dpp_add<0x111, 0xf>(v);  // row_shr:1
    v = dpp_add<0x112, 0xf>(v);  // row_shr:2
    v = dpp_add<0x114, 0xf>(v);  // row_shr:4
    v = dpp_add<0x118, 0xf>(v);  // row_shr:8
    return v;
}

// a + b after v_permlane32_swap(a, b): lanes 0-31 get a_lo + a_hi, lanes 32-63 get b_lo + b_hi.
// NOTE (ROCm 7.2 hipcc): bit-casting the builtin's vector elements directly miscompiles (both
// results alias the vdst register, see tools/lane_probe.py); going through named unsigned
// temporaries, as below, generates the intended `v_permlane*_swap v_a, v_b; v_add v_a, v_a, v_b`.
__device__ __forceinline__ float swap32_add(float a, float b) {
    unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
    const auto r = __builtin_amdgcn_permlane32_swap(ua, ub, false, false);
    ua = r[0];
    ub = r[1];
    return __builtin_bit_cast(float, ua) + __builtin_bit_cast(float, ub);
}
// a + b after v_permlane16_swap(a, b): rows (16 lanes) become [a0+a1, b0+b1, a2+a3, b2+b3].
__device__ __forceinline__ float swap16_add(float a, float b) {
    unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
    const auto r = __builtin_amdgcn_permlane16_swap(ua, ub, false, false);
    ua = r[0];
    ub = r[1];
    return __builtin_bit_cast(float, ua) + __builtin_bit_cast(float, ub);
}

// Wave64 sums of 9 values in 28 VALU ops (vs 54 for nine independent DPP reductions): two
// lane-halving swap stages pack two components per register, then one row reduction per
// register.  Result: lane 16r+15 holds component ((r&1)<<1 | r>>1) in t0, that +4 in t1, and
// lane 15 holds component 8 in t2 (see red9_store).
__device__ __forceinline__ void wave_sum9(float v0, float v1, float v2, float v3, float v4, float v5, float v6,
                                          float v7, float v8, float& t0, float& t1, float& t2) {
    const float r0 = swap32_add(v0, v1), r1 = swap32_add(v2, v3), r2 = swap32_add(v4, v5), r3 = swap32_add(v6, v7),
                r4 = swap32_add(v8, 0.f);
    t0 = row16_sum(swap16_add(r0, r1));
    t1 = row16_sum(swap16_add(r2, r3));
    t2 = row16_sum(swap16_add(r4, 0.f));
}
// Two pairs' nine components (a, b) at once: 48 VALU ops instead of 2 x 28 — the swap stages pair
// a's and b's components instead of two of one pair's, so the row sums run on 5 registers, not 6.
// The same adds on the same values as two wave_sum9 calls (bitwise the same sums).  Result: lane
// 16r+15 holds component 2i + (r & 1) of pair r >> 1 in t[i] (i < 4), and lanes 15 / 47 hold
// component 8 of a / b in t[4] (see red18_store).
__device__ __forceinline__ void wave_sum18(const float (&a)[NGRAD], const float (&b)[NGRAD], float (&t)[5]) {
    float r[NGRAD];
#pragma unroll
    for (int k = 0; k < NGRAD; k++) r[k] = swap32_add(a[k], b[k]);
#pragma unroll
    for (int i = 0; i < 4; i++) t[i] = row16_sum(swap16_add(r[2 * i], r[2 * i + 1]));
    t[4] = row16_sum(swap16_add(r[8], 0.f));
}
__device__ __forceinline__ void red18_store(float* dst, int lane, const float (&t)[5], bool has_b) {
    if ((lane & 15) == 15) {
        const int row = lane >> 4, sel = row >> 1, odd = row & 1;
        if (sel == 0 || has_b) {
            float* d = dst + sel * NGRAD;
#pragma unroll
            for (int i = 0; i < 4; i++) d[2 * i + odd] = t[i];
            if (!odd) d[8] = t[4];
        }
    }
}
__device__ __forceinline__ void red9_store(float* dst, int lane, float t0, float t1, float t2) {
    if ((lane & 15) == 15) {
        const int row = lane >> 4;
        const int c = ((row & 1) << 1) | (row >> 1);
        dst[c] = t0;
        dst[c + 4] = t1;
        if (row == 0) dst[8] = t2;
    }
}

// The backward blend's tile order (heaviest first, rr_blend.hip tile_order_body: counting sort by
// 1023 - min(cost / 4, 1023), order inside a bucket free) by ONE 256-thread workgroup: the extra
// workgroup of the phase-B duplicate launch, where it runs beside the duplicate instead of on the
// backward prologue's critical path.  There the costs are phase A's: a tile phase A left open
// (open_bits) goes on walking in phase B and counts as heaviest (bucket 0).
__device__ __forceinline__ void tile_order_body256(int T, const uint32_t* __restrict__ cost,
                                                   const uint32_t* __restrict__ open_bits,
                                                   uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[1024];
    __shared__ uint32_t wsum[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // the buckets of a batch of kTB tiles per thread, every load in flight at once (clamped
    // indices, no per-tile condition: a load inside the atomic loop made each of the T / 256
    // iterations wait for its own memory round trip, ~50 us at T = 8160)
    constexpr int kTB = 16;
    auto buckets = [&](int base, uint32_t (&bk)[kTB]) {
        uint32_t c[kTB], ob[kTB];
#pragma unroll
        for (int k = 0; k < kTB; k++) {
            const int i = min(base + k * 256 + t, T - 1);
            c[k] = cost[i];
            ob[k] = open_bits ? open_bits[i >> 5] : 0u;
        }
#pragma unroll
        for (int k = 0; k < kTB; k++) {
            const int i = min(base + k * 256 + t, T - 1);
            bk[k] = ((ob[k] >> (i & 31)) & 1u) ? 0u : 1023u - min(c[k] >> 2, 1023u);
        }
    };
#pragma unroll
    for (int k = 0; k < 4; k++) hist[4 * t + k] = 0;
    __syncthreads();
    for (int base = 0; base < T; base += kTB * 256) {
        uint32_t bk[kTB];
        buckets(base, bk);
#pragma unroll
        for (int k = 0; k < kTB; k++)
            if (base + k * 256 + t < T) atomicAdd(&hist[bk[k]], 1u);
    }
    __syncthreads();
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = hist[4 * t + k];
        sum += v[k];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int i = 0; i < w; i++) run += wsum[i];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        hist[4 * t + k] = run;
        run += v[k];
    }
    __syncthreads();
    // order inside a bucket is free (atomic slot claims)
    for (int base = 0; base < T; base += kTB * 256) {
        uint32_t bk[kTB];
        buckets(base, bk);
#pragma unroll
        for (int k = 0; k < kTB; k++) {
            const int i = base + k * 256 + t;
            if (i < T) order[atomicAdd(&hist[bk[k]], 1u)] = (uint32_t)i;
        }
    }
}

}  // namespace rr
