// rr_backward.hip — backward kernels of the MI355X rasterizer.
//
//   k_gauss_bwd<DEG>   one thread per Gaussian: the reference's computeCov2DCUDA
//                      (backward.cu:133-264) + preprocessCUDA (backward.cu:336-386, SH bwd :9-128,
//                      cov3D bwd :268-331) fused, writing every gradient output exactly once
//                      (so the host allocates them uninitialised — no zero-fill pass).  It consumes
//                      the per-Gaussian accumulators the blend backward (rr_blend.hip) filled.
#include "adam_math.hpp"
#include "rr_common.hpp"
#include "rr_kernels.hpp"
#include "rr_preprocess.hpp"

namespace rr {

// ---- per-Gaussian backward -------------------------------------------------------------

// SH backward (backward.cu:9-128), split in two so that the coefficient gradients can overwrite
// the staged coefficients in LDS: sh_dir_grad only reads the coefficients (rest[3(k-1)..] holds
// coefficient k >= 1) and returns dL/d(dir); sh_coeff_grads only writes dL/dsh_k = Y_k(dir) dL/dRGB
// into row[3k..3k+2] for k < K and zeros for K <= k < M.
template <int DEG>
__device__ __forceinline__ v3 sh_dir_grad(v3 dir, const float* rest, v3 dL_dRGB) {
    const float x = dir.x, y = dir.y, z = dir.z;
    v3 dRGBdx = mk(0, 0, 0), dRGBdy = mk(0, 0, 0), dRGBdz = mk(0, 0, 0);
    if (DEG > 0) {
        dRGBdx = -RR_SH_C1 * load3(rest + 6);
        dRGBdy = -RR_SH_C1 * load3(rest + 0);
        dRGBdz = RR_SH_C1 * load3(rest + 3);
        if (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            const v3 s4 = load3(rest + 9), s5 = load3(rest + 12), s6 = load3(rest + 15), s7 = load3(rest + 18),
                     s8 = load3(rest + 21);
            dRGBdx = dRGBdx + ((RR_SH_C2_0 * y) * s4 + (RR_SH_C2_2 * 2.f * -x) * s6 + (RR_SH_C2_3 * z) * s7 +
                               (RR_SH_C2_4 * 2.f * x) * s8);
            dRGBdy = dRGBdy + ((RR_SH_C2_0 * x) * s4 + (RR_SH_C2_1 * z) * s5 + (RR_SH_C2_2 * 2.f * -y) * s6 +
                               (RR_SH_C2_4 * 2.f * -y) * s8);
            dRGBdz = dRGBdz + ((RR_SH_C2_1 * y) * s5 + (RR_SH_C2_2 * 2.f * 2.f * z) * s6 + (RR_SH_C2_3 * x) * s7);
            if (DEG > 2) {
                const v3 s9 = load3(rest + 24), s10 = load3(rest + 27), s11 = load3(rest + 30), s12 = load3(rest + 33),
                         s13 = load3(rest + 36), s14 = load3(rest + 39), s15 = load3(rest + 42);
                dRGBdx = dRGBdx + ((RR_SH_C3_0 * 3.f * 2.f * xy) * s9 + (RR_SH_C3_1 * yz) * s10 +
                                   (RR_SH_C3_2 * -2.f * xy) * s11 + (RR_SH_C3_3 * -3.f * 2.f * xz) * s12 +
                                   (RR_SH_C3_4 * (-3.f * xx + 4.f * zz - yy)) * s13 + (RR_SH_C3_5 * 2.f * xz) * s14 +
                                   (RR_SH_C3_6 * 3.f * (xx - yy)) * s15);
                dRGBdy = dRGBdy + ((RR_SH_C3_0 * 3.f * (xx - yy)) * s9 + (RR_SH_C3_1 * xz) * s10 +
                                   (RR_SH_C3_2 * (-3.f * yy + 4.f * zz - xx)) * s11 +
                                   (RR_SH_C3_3 * -3.f * 2.f * yz) * s12 + (RR_SH_C3_4 * -2.f * xy) * s13 +
                                   (RR_SH_C3_5 * -2.f * yz) * s14 + (RR_SH_C3_6 * -3.f * 2.f * xy) * s15);
                dRGBdz = dRGBdz + ((RR_SH_C3_1 * xy) * s10 + (RR_SH_C3_2 * 4.f * 2.f * yz) * s11 +
                                   (RR_SH_C3_3 * 3.f * (2.f * zz - xx - yy)) * s12 +
                                   (RR_SH_C3_4 * 4.f * 2.f * xz) * s13 + (RR_SH_C3_5 * (xx - yy)) * s14);
            }
        }
    }
    return mk(dot(dRGBdx, dL_dRGB), dot(dRGBdy, dL_dRGB), dot(dRGBdz, dL_dRGB));
}

template <int DEG>
__device__ __forceinline__ void sh_coeff_grads(v3 dir, v3 dL_dRGB, float* row, int M, bool acc) {
    const float x = dir.x, y = dir.y, z = dir.z;
    auto W = [&](int k, float s) {
        const float g0 = s * dL_dRGB.x, g1 = s * dL_dRGB.y, g2 = s * dL_dRGB.z;
        if (acc) {  // the multi-view kernel: add this view's gradient (rounded on its own first)
            row[3 * k + 0] += g0;
            row[3 * k + 1] += g1;
            row[3 * k + 2] += g2;
        } else {
            row[3 * k + 0] = g0;
            row[3 * k + 1] = g1;
            row[3 * k + 2] = g2;
        }
    };
    W(0, RR_SH_C0);
    if (DEG > 0) {
        W(1, -RR_SH_C1 * y);
        W(2, RR_SH_C1 * z);
        W(3, -RR_SH_C1 * x);
        if (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            W(4, RR_SH_C2_0 * xy);
            W(5, RR_SH_C2_1 * yz);
            W(6, RR_SH_C2_2 * (2.f * zz - xx - yy));
            W(7, RR_SH_C2_3 * xz);
            W(8, RR_SH_C2_4 * (xx - yy));
            if (DEG > 2) {
                W(9, RR_SH_C3_0 * y * (3.f * xx - yy));
                W(10, RR_SH_C3_1 * xy * z);
                W(11, RR_SH_C3_2 * y * (4.f * zz - xx - yy));
                W(12, RR_SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy));
                W(13, RR_SH_C3_4 * x * (4.f * zz - xx - yy));
                W(14, RR_SH_C3_5 * z * (xx - yy));
                W(15, RR_SH_C3_6 * x * (xx - 3.f * yy));
            }
        }
    }
    constexpr int K = (DEG + 1) * (DEG + 1);
    if (!acc)
        for (int i = 3 * K; i < 3 * M; i++) row[i] = 0.f;
}

// The 11 per-Gaussian gradients of the small groups (xyz 3, opacity 1, scaling 3, rotation 4),
// kept in registers so that the fused Adam step can batch its loads (rr_grads.adam).
struct SmallGrads {
    float v[11];
};
__device__ __forceinline__ void put(float* grad, size_t e, float g) {
    if (grad) grad[e] = g;
}

// Stores of the optimizer state (parameters and moments).  (Written through with sc1 vector
// stores, so that the lines leave the XCD's L2 instead of staying dirty until the kernel-end
// write-back, the kernel took 0.66 vs 0.37 ms: profiles/r05_gauss_bwd_variants_ab.jsonl.)
__device__ __forceinline__ void st_state(float* p, float v) { *p = v; }
// The SH groups' Adam stream (59 % of the kernel's bytes, each read once and written once) goes
// through non-temporal loads and stores: its lines no longer displace what the caches hold for
// the rest of the step, and the kernel runs 0.369 -> 0.326 ms with batches of one float4 per
// array (0.346 at two), step 1.0406 -> 0.9847 ms; non-temporal loads of the coefficient staging
// or of the small groups' state measured slower (profiles/r06f_gauss_bwd_nt_ab.jsonl).
typedef float nt4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_ld4(const float* p) {
    const nt4f v = __builtin_nontemporal_load(reinterpret_cast<const nt4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_state4(float* p, float4 v) {
    const nt4f w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<nt4f*>(p));
}

// Adam over n elements whose (param, moment) addresses are given: all loads first, then the
// math, then the stores (the compiler cannot batch them itself: the arrays may alias).
template <int N>
__device__ __forceinline__ void adam_batch(float* const (&pp)[N], float* const (&mp)[N], float* const (&vp)[N],
                                           const float (&g)[N], const AdamC (&c)[N], float (&p)[N]) {
    float m[N], v[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
        p[i] = *pp[i];
        m[i] = *mp[i];
        v[i] = *vp[i];
    }
#pragma unroll
    for (int i = 0; i < N; i++) adam_elem(p[i], g[i], m[i], v[i], c[i]);
#pragma unroll
    for (int i = 0; i < N; i++) {
        st_state(pp[i], p[i]);
        st_state(mp[i], m[i]);
        st_state(vp[i], v[i]);
    }
}

// upd: the 11 parameters after the step (xyz 3, opacity 1, scaling 3, rotation 4), for the next
// frame's preprocess (rr_next_frame); a group that is not stepped keeps its value.
__device__ __forceinline__ void adam_small(const GaussBwdArgs& a, int idx, const SmallGrads& sg, SmallGrads& upd) {
    const rr_adam& ad = a.adam;
    auto consts = [&](const rr_adam_group& G) {
        return adam_consts(G.lr, G.bias_correction1, G.bias_correction2_sqrt, ad.beta1, ad.beta2, ad.eps);
    };
    const AdamC c_xyz = consts(ad.xyz), c_sc = consts(ad.scaling), c_op = consts(ad.opacity),
                c_rot = consts(ad.rotation);
    const rr_adam_group* gr[11];
    AdamC cc[11];  // values (indices are compile-time after unrolling: stays in registers)
    size_t e[11];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        gr[i] = &ad.xyz;
        cc[i] = c_xyz;
        e[i] = 3 * (size_t)idx + i;
        gr[4 + i] = &ad.scaling;
        cc[4 + i] = c_sc;
        e[4 + i] = 3 * (size_t)idx + i;
    }
    gr[3] = &ad.opacity;
    cc[3] = c_op;
    e[3] = idx;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        gr[7 + i] = &ad.rotation;
        cc[7 + i] = c_rot;
        e[7 + i] = 4 * (size_t)idx + i;
    }
    if (ad.xyz.param && ad.scaling.param && ad.opacity.param && ad.rotation.param) {  // the usual case
        float* pp[11];
        float* mp[11];
        float* vp[11];
#pragma unroll
        for (int i = 0; i < 11; i++) {
            pp[i] = gr[i]->param + e[i];
            mp[i] = gr[i]->exp_avg + e[i];
            vp[i] = gr[i]->exp_avg_sq + e[i];
        }
        adam_batch<11>(pp, mp, vp, sg.v, cc, upd.v);
        return;
    }
    // a group without param is not stepped (the sharded step of an opacity-reset iteration)
#pragma unroll
    for (int i = 0; i < 11; i++) {
        upd.v[i] = 0.f;
        if (!gr[i]->param) continue;
        float p = gr[i]->param[e[i]], m = gr[i]->exp_avg[e[i]], v = gr[i]->exp_avg_sq[e[i]];
        adam_elem(p, sg.v[i], m, v, cc[i]);
        gr[i]->param[e[i]] = p;
        gr[i]->exp_avg[e[i]] = m;
        gr[i]->exp_avg_sq[e[i]] = v;
        upd.v[i] = p;
    }
}

// What the per-Gaussian backward needs of one view: its camera, and the Gaussian's accumulators
// from that view's blend backward (GACC layout: dmean2D.xy, dconic.xyz, dopacity, dcolor.rgb) with
// its radius.
struct GaccRec {
    const float* gp;  // GACC_STRIDE floats (single view, read when radius > 0)
    int radius;
    const float2* q;  // a packed kRecFloats record already in registers (multi-view kernel)
};
__device__ __forceinline__ ViewCam view_cam(const GaussBwdArgs& a) {
    return ViewCam{a.view, a.proj, a.campos, a.tanfovx, a.tanfovy, a.focal_x, a.focal_y, a.low_pass};
}

// One Gaussian, one view.  `coef` is this thread's LDS row holding its SH coefficients (staged by
// the kernel; coefficient k at coef[3k..3k+2]); the SH gradients go to `gsh` in the same layout,
// stored (acc_sh false) or added (acc_sh true: the multi-view kernel sums the views in order).
// coef == gsh (the single-view kernel) is allowed: every coefficient is read before the first
// gradient is written.  Both are nullptr when there are neither SH inputs nor SH gradients.
template <int DEG, bool PACKED>
__device__ __forceinline__ void gauss_bwd_one(const GaussBwdArgs& a, const ViewCam& c, int idx, const GaccRec& rec,
                                              const float* coef, float* gsh, bool acc_sh, SmallGrads& sg) {
    const int M = a.M;
    float* dmean2 = a.dL_dmeans2D ? a.dL_dmeans2D + 3 * (size_t)idx : nullptr;
    float* dcol = a.dL_dcolors ? a.dL_dcolors + 3 * (size_t)idx : nullptr;
    float* dcov = a.dL_dcov3D ? a.dL_dcov3D + 6 * (size_t)idx : nullptr;
    // small-group gradients: written out if requested, and kept in sg for the fused Adam step
    auto emit3 = [&](float* out, int slot, v3 g) {
        sg.v[slot] = g.x;
        sg.v[slot + 1] = g.y;
        sg.v[slot + 2] = g.z;
        put(out, 3 * (size_t)idx + 0, g.x);
        put(out, 3 * (size_t)idx + 1, g.y);
        put(out, 3 * (size_t)idx + 2, g.z);
    };
    auto emit_rot = [&](float4 g) {
        sg.v[7] = g.x;
        sg.v[8] = g.y;
        sg.v[9] = g.z;
        sg.v[10] = g.w;
        put(a.dL_drot, 4 * (size_t)idx + 0, g.x);
        put(a.dL_drot, 4 * (size_t)idx + 1, g.y);
        put(a.dL_drot, 4 * (size_t)idx + 2, g.z);
        put(a.dL_drot, 4 * (size_t)idx + 3, g.w);
    };
    auto emit_op = [&](float g) {
        sg.v[3] = g;
        put(a.dL_dopacity, idx, g);
    };

    const int radius = rec.radius;
    if (!(radius > 0)) {  // untouched Gaussians: exact zeros (backward.cu:146,357)
        if (dmean2) dmean2[0] = dmean2[1] = dmean2[2] = 0.f;
        if (dcol) dcol[0] = dcol[1] = dcol[2] = 0.f;
        emit_op(0.f);
        emit3(a.dL_dmeans3D, 0, mk(0.f, 0.f, 0.f));
        if (dcov)
#pragma unroll
            for (int i = 0; i < 6; i++) dcov[i] = 0.f;
        if (gsh && !acc_sh)
            for (int i = 0; i < 3 * M; i++) gsh[i] = 0.f;
        emit3(a.dL_dscales, 4, mk(0.f, 0.f, 0.f));
        emit_rot(make_float4(0.f, 0.f, 0.f, 0.f));
        return;
    }

    float4 ga, gb;
    float g8;
    if (PACKED) {  // 40-B record, loaded by the caller
        const float2* q = rec.q;
        const float2 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
        ga = make_float4(q0.x, q0.y, q1.x, q1.y);
        gb = make_float4(q2.x, q2.y, q3.x, q3.y);
        g8 = q4.x;
    } else {
        ga = *reinterpret_cast<const float4*>(rec.gp);
        gb = *reinterpret_cast<const float4*>(rec.gp + 4);
        g8 = rec.gp[8];
    }
    const float dm2x = ga.x, dm2y = ga.y;
    const float dcx = ga.z, dcy = ga.w, dcz = gb.x;
    if (dmean2) {
        dmean2[0] = dm2x;
        dmean2[1] = dm2y;
        dmean2[2] = 0.f;
    }
    if (dcol) {
        dcol[0] = gb.z;
        dcol[1] = gb.w;
        dcol[2] = g8;
    }
    if (a.raw) {  // sigmoid backward (torch: grad * (1 - y) * y)
        const float o = act_opacity(a.opacities[idx]);
        emit_op(gb.y * (1.0f - o) * o);
    } else {
        emit_op(gb.y);
    }
    if (a.grad_accum) {  // densification statistics (gaussian_model.py:419-421, train.py:133)
        a.grad_accum[idx] += sqrtf(dm2x * dm2x + dm2y * dm2y);
        a.denom[idx] += 1.0f;
        a.max_radii2D[idx] = fmaxf(a.max_radii2D[idx], (float)radius);
    }

    const v3 mean = load3(a.means3D + 3 * (size_t)idx);
    float cov[6];
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f), q_raw = q;
    v3 scale = mk(0.f, 0.f, 0.f);
    if (a.cov3D_precomp) {
        const float* c = a.cov3D_precomp + 6 * (size_t)idx;
#pragma unroll
        for (int i = 0; i < 6; i++) cov[i] = c[i];
    } else {
        q = q_raw = *reinterpret_cast<const float4*>(a.rotations + 4 * (size_t)idx);
        scale = load3(a.scales + 3 * (size_t)idx);
        if (a.raw) {
            q = act_rot(q_raw);
            scale = act_scale(scale);
        }
        cov3d_from_scale_rot(scale, a.scale_modifier, q, cov);  // identical to the forward's value
    }

    // ---- computeCov2DCUDA (backward.cu:154-263) ----
    const Proj2D pr = ewa_setup(mean, c.focal_x, c.focal_y, c.tanfovx, c.tanfovy, c.view);
    const float x_grad_mul = pr.txtz < -pr.limx || pr.txtz > pr.limx ? 0.f : 1.f;
    const float y_grad_mul = pr.tytz < -pr.limy || pr.tytz > pr.limy ? 0.f : 1.f;
    float ca, cb, cc;
    ewa_cov2d(pr, cov, ca, cb, cc);
    ca += c.low_pass;
    cc += c.low_pass;
    const float denom = ca * cc - cb * cb;
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float(&T)[2][3] = pr.A;
    float dc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (denom2inv != 0.f) {
        dL_da = denom2inv * (-cc * cc * dcx + 2 * cb * cc * dcy + (denom - ca * cc) * dcz);
        dL_dc = denom2inv * (-ca * ca * dcz + 2 * ca * cb * dcy + (denom - ca * cc) * dcx);
        dL_db = denom2inv * 2 * (cb * cc * dcx - (denom + 2 * cb * cb) * dcy + ca * cb * dcz);
        dc[0] = (T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc);
        dc[3] = (T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc);
        dc[5] = (T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc);
        dc[1] = 2 * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db +
                2 * T[1][0] * T[1][1] * dL_dc;
        dc[2] = 2 * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db +
                2 * T[1][0] * T[1][2] * dL_dc;
        dc[4] = 2 * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db +
                2 * T[1][1] * T[1][2] * dL_dc;
    }
    if (dcov)
#pragma unroll
        for (int i = 0; i < 6; i++) dcov[i] = dc[i];
    const float V[3][3] = {{cov[0], cov[1], cov[2]}, {cov[1], cov[3], cov[4]}, {cov[2], cov[4], cov[5]}};
    const float dL_dT00 = 2 * (T[0][0] * V[0][0] + T[0][1] * V[0][1] + T[0][2] * V[0][2]) * dL_da +
                          (T[1][0] * V[0][0] + T[1][1] * V[0][1] + T[1][2] * V[0][2]) * dL_db;
    const float dL_dT01 = 2 * (T[0][0] * V[1][0] + T[0][1] * V[1][1] + T[0][2] * V[1][2]) * dL_da +
                          (T[1][0] * V[1][0] + T[1][1] * V[1][1] + T[1][2] * V[1][2]) * dL_db;
    const float dL_dT02 = 2 * (T[0][0] * V[2][0] + T[0][1] * V[2][1] + T[0][2] * V[2][2]) * dL_da +
                          (T[1][0] * V[2][0] + T[1][1] * V[2][1] + T[1][2] * V[2][2]) * dL_db;
    const float dL_dT10 = 2 * (T[1][0] * V[0][0] + T[1][1] * V[0][1] + T[1][2] * V[0][2]) * dL_dc +
                          (T[0][0] * V[0][0] + T[0][1] * V[0][1] + T[0][2] * V[0][2]) * dL_db;
    const float dL_dT11 = 2 * (T[1][0] * V[1][0] + T[1][1] * V[1][1] + T[1][2] * V[1][2]) * dL_dc +
                          (T[0][0] * V[1][0] + T[0][1] * V[1][1] + T[0][2] * V[1][2]) * dL_db;
    const float dL_dT12 = 2 * (T[1][0] * V[2][0] + T[1][1] * V[2][1] + T[1][2] * V[2][2]) * dL_dc +
                          (T[0][0] * V[2][0] + T[0][1] * V[2][1] + T[0][2] * V[2][2]) * dL_db;
    const float* vm = c.view;  // glm W[i][j] == vm[4j+i]
    const float dL_dJ00 = vm[0] * dL_dT00 + vm[4] * dL_dT01 + vm[8] * dL_dT02;
    const float dL_dJ02 = vm[2] * dL_dT00 + vm[6] * dL_dT01 + vm[10] * dL_dT02;
    const float dL_dJ11 = vm[1] * dL_dT10 + vm[5] * dL_dT11 + vm[9] * dL_dT12;
    const float dL_dJ12 = vm[2] * dL_dT10 + vm[6] * dL_dT11 + vm[10] * dL_dT12;
    const v3 t = pr.t;
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -c.focal_x * tz2 * dL_dJ02;
    const float dL_dty = y_grad_mul * -c.focal_y * tz2 * dL_dJ12;
    const float dL_dtz = -c.focal_x * tz2 * dL_dJ00 - c.focal_y * tz2 * dL_dJ11 +
                         (2 * c.focal_x * t.x) * tz3 * dL_dJ02 + (2 * c.focal_y * t.y) * tz3 * dL_dJ12;
    v3 dmean = xform_vec_4x3_T(mk(dL_dtx, dL_dty, dL_dtz), c.view);

    // ---- preprocessCUDA bwd: mean2D -> mean3D (backward.cu:360-377) ----
    const float* pj = c.proj;
    const float4 m_hom = xform_point_4x4(mean, pj);
    const float m_w = 1.0f / (m_hom.w + 0.0000001f);
    const float mul1 = (pj[0] * mean.x + pj[4] * mean.y + pj[8] * mean.z + pj[12]) * m_w * m_w;
    const float mul2 = (pj[1] * mean.x + pj[5] * mean.y + pj[9] * mean.z + pj[13]) * m_w * m_w;
    dmean.x += (pj[0] * m_w - pj[3] * mul1) * dm2x + (pj[1] * m_w - pj[3] * mul2) * dm2y;
    dmean.y += (pj[4] * m_w - pj[7] * mul1) * dm2x + (pj[5] * m_w - pj[7] * mul2) * dm2y;
    dmean.z += (pj[8] * m_w - pj[11] * mul1) * dm2x + (pj[9] * m_w - pj[11] * mul2) * dm2y;

    // ---- SH bwd (backward.cu:9-128); the clamp mask is recomputed from the forward SH value ----
    if (a.shs) {
        const float* dc = coef;  // staged coefficients (same values as shs / f_dc + f_rest)
        const float* rest = coef + 3;
        const v3 cp = load3(c.campos);
        const v3 dir_orig = mean - cp;
        const float len = sqrtf(dot(dir_orig, dir_orig));
        const v3 dir = mk(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
        const v3 rgb = sh_eval<DEG>(dir, dc, rest);
        v3 dL_dRGB = mk(gb.z, gb.w, g8);
        dL_dRGB.x *= rgb.x < 0 ? 0.f : 1.f;
        dL_dRGB.y *= rgb.y < 0 ? 0.f : 1.f;
        dL_dRGB.z *= rgb.z < 0 ? 0.f : 1.f;
        const v3 dL_ddir = sh_dir_grad<DEG>(dir, rest, dL_dRGB);  // last read of the staged coefficients
        sh_coeff_grads<DEG>(dir, dL_dRGB, gsh, M, acc_sh);        // (may overwrite them with dL/dsh)
        // dnormvdv (auxiliary.h:96-106)
        const v3 v = dir_orig;
        const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
        const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
        dmean.x += ((+sum2 - v.x * v.x) * dL_ddir.x - v.y * v.x * dL_ddir.y - v.z * v.x * dL_ddir.z) * invsum32;
        dmean.y += (-v.x * v.y * dL_ddir.x + (sum2 - v.y * v.y) * dL_ddir.y - v.z * v.y * dL_ddir.z) * invsum32;
        dmean.z += (-v.x * v.z * dL_ddir.x - v.y * v.z * dL_ddir.y + (sum2 - v.z * v.z) * dL_ddir.z) * invsum32;
    } else if (gsh && !acc_sh) {
        for (int i = 0; i < 3 * M; i++) gsh[i] = 0.f;
    }
    emit3(a.dL_dmeans3D, 0, dmean);

    // ---- cov3D bwd (backward.cu:268-331) ----
    if (a.scales) {
        const float r = q.x, x = q.y, y = q.z, z = q.w;
        float R[3][3];
        quat_rot(q, R);
        const float s[3] = {a.scale_modifier * scale.x, a.scale_modifier * scale.y, a.scale_modifier * scale.z};
        float Mm[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) Mm[i][j] = s[i] * R[j][i];
        const float dS[3][3] = {{dc[0], 0.5f * dc[1], 0.5f * dc[2]},
                                {0.5f * dc[1], dc[3], 0.5f * dc[4]},
                                {0.5f * dc[2], 0.5f * dc[4], dc[5]}};
        float dM[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                dM[i][j] = 2.0f * Mm[i][0] * dS[0][j] + 2.0f * Mm[i][1] * dS[1][j] + 2.0f * Mm[i][2] * dS[2][j];
        float ds[3];
#pragma unroll
        for (int i = 0; i < 3; i++) ds[i] = R[0][i] * dM[i][0] + R[1][i] * dM[i][1] + R[2][i] * dM[i][2];
        // raw mode: exp backward (torch: grad * result)
        emit3(a.dL_dscales, 4,
              a.raw ? mk(ds[0] * scale.x, ds[1] * scale.y, ds[2] * scale.z) : mk(ds[0], ds[1], ds[2]));
        float Gm[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) Gm[i][j] = dM[i][j] * s[i];
        float4 dq;
        dq.x = 2 * z * (Gm[0][1] - Gm[1][0]) + 2 * y * (Gm[2][0] - Gm[0][2]) + 2 * x * (Gm[1][2] - Gm[2][1]);
        dq.y = 2 * y * (Gm[1][0] + Gm[0][1]) + 2 * z * (Gm[2][0] + Gm[0][2]) + 2 * r * (Gm[1][2] - Gm[2][1]) -
               4 * x * (Gm[2][2] + Gm[1][1]);
        dq.z = 2 * x * (Gm[1][0] + Gm[0][1]) + 2 * r * (Gm[2][0] - Gm[0][2]) + 2 * z * (Gm[1][2] + Gm[2][1]) -
               4 * y * (Gm[2][2] + Gm[0][0]);
        dq.w = 2 * r * (Gm[0][1] - Gm[1][0]) + 2 * x * (Gm[2][0] + Gm[0][2]) + 2 * y * (Gm[1][2] + Gm[2][1]) -
               4 * z * (Gm[1][1] + Gm[0][0]);
        if (a.raw) {
            // F.normalize backward: x / clamp_min(n, eps) -> g / n' - x (g.x) / n'^2 / n  (n >= eps)
            const float4 x = q_raw;
            const float n = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
            const float nd = fmaxf(n, 1e-12f);
            const float gx = dq.x * x.x + dq.y * x.y + dq.z * x.z + dq.w * x.w;
            const float c = n >= 1e-12f ? -gx / (nd * nd) / n : 0.f;
            dq = make_float4(dq.x / nd + x.x * c, dq.y / nd + x.y * c, dq.z / nd + x.z * c, dq.w / nd + x.w * c);
        }
        emit_rot(dq);
    } else {
        emit3(a.dL_dscales, 4, mk(0.f, 0.f, 0.f));
        emit_rot(make_float4(0.f, 0.f, 0.f, 0.f));
    }
}

// Workgroup of kGB Gaussians.  The SH coefficients (the bulk of the per-Gaussian bytes: 192 B at
// M = 16) are staged into LDS one Gaussian row per wave instruction (coalesced 192-B reads instead
// of 64 lanes each walking its own 192-B record), and dL/dsh leaves the same way.  Row stride
// kShStride is odd, so the per-thread row accesses are LDS-bank-conflict free.
// Single-view kernel: 256 Gaussians per workgroup (the preprocess's block size, so the next frame's
// per-256-row block sums come out of the same workgroup, rr_next_frame; 128 and 256 measured the
// same, round 3); multi-view kernel: 128 (it holds two LDS row blocks).
#ifndef RR_GB_THREADS
#define RR_GB_THREADS 256
#endif
constexpr int kGB1 = RR_GB_THREADS;
constexpr int kGB = 128;
constexpr int kShStride = 49;

// The per-Gaussian backward of one workgroup of kGB Gaussians.  Single view (MULTI false): the
// gradients of this view, written out and / or stepped by the fused Adam; s_gr == s_sh.
// MULTI (k_gauss_bwd_views, the Gaussian-sharded multi-GPU step): every view of va->cams in
// order, each from its packed accumulator record, summed per element in view order into registers
// (11 small-group values) and into s_gr (the SH gradients; s_sh keeps the coefficients), then
// scaled by va->grad_scale (1/N, rounded like grad.mul_(1/N)) before the Adam step.
struct GaussBwdViewsArgs;
template <int DEG, bool MULTI, int KGB>
__device__ __forceinline__ void gauss_bwd_block(const GaussBwdArgs& a, const GaussBwdViewsArgs* va, float* s_sh,
                                                float* s_gr);

template <int DEG>
// Occupancy: 3 waves per SIMD, set by LDS (a 196-B coefficient row per Gaussian, 12.5 KiB per
// wave at either workgroup size), not by the 144 VGPRs.
__global__ __launch_bounds__(kGB1) void k_gauss_bwd(GaussBwdArgs a) {
    __shared__ float s_sh[kGB1 * kShStride];
    gauss_bwd_block<DEG, false, kGB1>(a, nullptr, s_sh, s_sh);
}

constexpr int kMaxViews = 16;
constexpr int kRecFloats = 10;  // packed accumulator record: GACC slots 0..8, radius (as a float)
struct GaussBwdViewsArgs {
    GaussBwdArgs g;  // the row block: P rows, raw parameters / Adam / statistics offset to it
    ViewCam cams[kMaxViews];
    int V;
    const float* records;  // [V][rec_rows][kRecFloats]
    int rec_rows;
    float grad_scale;
};

template <int DEG>
__global__ __launch_bounds__(kGB) void k_gauss_bwd_views(GaussBwdViewsArgs va) {
    __shared__ float s_sh[kGB * kShStride];
    __shared__ float s_gr[kGB * kShStride];
    gauss_bwd_block<DEG, true, kGB>(va.g, &va, s_sh, s_gr);
}

template <int DEG, bool MULTI, int KGB>
__device__ __forceinline__ void gauss_bwd_block(const GaussBwdArgs& a, const GaussBwdViewsArgs* va, float* s_sh,
                                                float* s_gr) {
    const int t = threadIdx.x, lane = t & 63;
    const int i0 = blockIdx.x * KGB;
    const int nvalid = min(KGB, a.P - i0);
    const int M = a.M, nf = 3 * M;  // floats per Gaussian
    const bool stage = M > 0 && (a.shs != nullptr || a.dL_dsh != nullptr || a.use_adam);
    if (stage && a.shs) {
        // flat, coalesced loads of the block's coefficient region(s), all in flight at once, then
        // scattered into the padded LDS rows; j = e / w via a float reciprocal (exact: e < 2^13)
        // float4 per lane when the region is 16-B aligned (1 KiB per wave instruction instead of 256 B)
        auto stage_in = [&](const float* src, int w, int koff) {
            const int total = nvalid * w;
            const float inv = 1.0f / (float)w;
            const float* base = src + (size_t)i0 * w;
            auto put_lds = [&](int e, float x) {
                const int j = (int)(((float)e + 0.5f) * inv);
                s_sh[j * kShStride + koff + (e - j * w)] = x;
            };
            if (((uintptr_t)base & 15u) == 0) {
                const int nv = total >> 2;
                float4 buf[12];
#pragma unroll
                for (int q = 0; q < 12; q++) {
                    const int i = t + q * KGB;
                    buf[q] = i < nv ? reinterpret_cast<const float4*>(base)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
                }
#pragma unroll
                for (int q = 0; q < 12; q++) {
                    const int i = t + q * KGB;
                    if (i < nv) {
                        put_lds(4 * i, buf[q].x);
                        put_lds(4 * i + 1, buf[q].y);
                        put_lds(4 * i + 2, buf[q].z);
                        put_lds(4 * i + 3, buf[q].w);
                    }
                }
                for (int e = 4 * nv + t; e < total; e += KGB) put_lds(e, base[e]);
                return;
            }
            float buf[48];
#pragma unroll
            for (int q = 0; q < 48; q++) {
                const int e = t + q * KGB;
                buf[q] = e < total ? base[e] : 0.f;
            }
#pragma unroll
            for (int q = 0; q < 48; q++) {
                const int e = t + q * KGB;
                if (e < total) put_lds(e, buf[q]);
            }
        };
        if (!a.raw) {
            stage_in(a.shs, nf, 0);
        } else {
            stage_in(a.shs, 3, 0);
            if (nf > 3) stage_in(a.shs_rest, nf - 3, 3);
        }
    }
    __syncthreads();
    SmallGrads upd;  // the small groups' parameters after the fused Adam step (rr_next_frame)
    if (t < nvalid) {
        SmallGrads sg;
        const int idx = i0 + t;
        float* row = stage ? s_sh + t * kShStride : nullptr;
        if (!MULTI) {
            const GaccRec rec{a.gacc + (size_t)idx * GACC_STRIDE, a.radii[idx], nullptr};
            gauss_bwd_one<DEG, false>(a, view_cam(a), idx, rec, row, row, false, sg);
        } else {
            float* grow = stage ? s_gr + t * kShStride : nullptr;
            // each view's 40-B record is loaded while the previous view is processed (one record
            // in flight ahead instead of a radius load then a dependent record load per view)
            const float2* rp = reinterpret_cast<const float2*>(va->records) + (size_t)idx * (kRecFloats / 2);
            const size_t vstride = (size_t)va->rec_rows * (kRecFloats / 2);
            float2 nq[kRecFloats / 2];
#pragma unroll
            for (int k = 0; k < kRecFloats / 2; k++) nq[k] = rp[k];
            for (int v = 0; v < va->V; v++) {
                float2 cq[kRecFloats / 2];
#pragma unroll
                for (int k = 0; k < kRecFloats / 2; k++) cq[k] = nq[k];
                if (v + 1 < va->V) {
#pragma unroll
                    for (int k = 0; k < kRecFloats / 2; k++) nq[k] = rp[(size_t)(v + 1) * vstride + k];
                }
                const GaccRec rec{nullptr, (int)cq[4].y, cq};
                SmallGrads gv;
                gauss_bwd_one<DEG, true>(a, va->cams[v], idx, rec, row, grow, v > 0, gv);
#pragma unroll
                for (int i = 0; i < 11; i++) sg.v[i] = v > 0 ? sg.v[i] + gv.v[i] : gv.v[i];
            }
#pragma unroll
            for (int i = 0; i < 11; i++) sg.v[i] = mul_rounded(sg.v[i], va->grad_scale);
        }
        if (a.use_adam) adam_small(a, i0 + t, sg, upd);
    }
    __syncthreads();
    // the next frame's preprocess reads the updated SH coefficients back from the LDS rows
    const bool back = !MULTI && a.has_next;
    if (stage && (a.dL_dsh || a.use_adam)) {
        // gradients leave coalesced; with the fused step the SH groups' Adam runs here, on the
        // same flat element order
        auto stage_out = [&](float* dst, const rr_adam_group* grp, int w, int koff) {
            const int total = nvalid * w;
            const float inv = 1.0f / (float)w;
            const AdamC c = grp ? adam_consts(grp->lr, grp->bias_correction1, grp->bias_correction2_sqrt, a.adam.beta1,
                                              a.adam.beta2, a.adam.eps)
                                : AdamC{};
#ifndef RR_GB_ADAM_BATCH
#define RR_GB_ADAM_BATCH 4
#endif
            constexpr int kB = RR_GB_ADAM_BATCH;  // Adam elements per batch of loads
            auto grad_at = [&](int e) {
                const int j = (int)(((float)e + 0.5f) * inv);
                const float g = s_gr[j * kShStride + koff + (e - j * w)];
                return MULTI ? mul_rounded(g, va->grad_scale) : g;
            };
            auto put_back = [&](int e, float x) {  // the updated coefficient into its LDS row slot
                const int j = (int)(((float)e + 0.5f) * inv);
                s_gr[j * kShStride + koff + (e - j * w)] = x;
            };
            const size_t gb = (size_t)i0 * w;
            const uintptr_t al = (grp ? ((uintptr_t)(grp->param + gb) | (uintptr_t)(grp->exp_avg + gb) |
                                         (uintptr_t)(grp->exp_avg_sq + gb))
                                      : 0u) |
                                 (dst ? (uintptr_t)(dst + gb) : 0u);
            if ((al & 15u) == 0) {
                // float4 per lane: kB / 4 vectors per batch, (param, m, v) loads all in flight
#ifndef RR_GB_ADAM_VEC
#define RR_GB_ADAM_VEC (kB / 4 > 0 ? kB / 4 : 1)
#endif
                constexpr int kV = RR_GB_ADAM_VEC;
                const int nv = total >> 2;
                for (int v0 = t; v0 < nv; v0 += kV * KGB) {
                    float4 g4[kV], p4[kV], m4[kV], s4[kV];
#pragma unroll
                    for (int q = 0; q < kV; q++) {
                        const int i = min(v0 + q * KGB, nv - 1);  // clamped duplicates are not stored
                        g4[q] = make_float4(grad_at(4 * i), grad_at(4 * i + 1), grad_at(4 * i + 2), grad_at(4 * i + 3));
                        if (grp) {
                            p4[q] = nt_ld4(grp->param + gb + 4 * (size_t)i);
                            m4[q] = nt_ld4(grp->exp_avg + gb + 4 * (size_t)i);
                            s4[q] = nt_ld4(grp->exp_avg_sq + gb + 4 * (size_t)i);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < kV; q++) {
                        const int i = v0 + q * KGB;
                        if (i >= nv) break;
                        if (dst) reinterpret_cast<float4*>(dst + gb)[i] = g4[q];
                        if (grp) {
                            adam_elem(p4[q].x, g4[q].x, m4[q].x, s4[q].x, c);
                            adam_elem(p4[q].y, g4[q].y, m4[q].y, s4[q].y, c);
                            adam_elem(p4[q].z, g4[q].z, m4[q].z, s4[q].z, c);
                            adam_elem(p4[q].w, g4[q].w, m4[q].w, s4[q].w, c);
                            st_state4(grp->param + gb + 4 * (size_t)i, p4[q]);
                            st_state4(grp->exp_avg + gb + 4 * (size_t)i, m4[q]);
                            st_state4(grp->exp_avg_sq + gb + 4 * (size_t)i, s4[q]);
                            if (back) {
                                put_back(4 * i, p4[q].x);
                                put_back(4 * i + 1, p4[q].y);
                                put_back(4 * i + 2, p4[q].z);
                                put_back(4 * i + 3, p4[q].w);
                            }
                        }
                    }
                }
                for (int e = 4 * nv + t; e < total; e += KGB) {  // tail (< 4 elements)
                    const float g = grad_at(e);
                    put(dst, gb + e, g);
                    if (grp) {
                        float p = grp->param[gb + e], m = grp->exp_avg[gb + e], v = grp->exp_avg_sq[gb + e];
                        adam_elem(p, g, m, v, c);
                        grp->param[gb + e] = p;
                        grp->exp_avg[gb + e] = m;
                        grp->exp_avg_sq[gb + e] = v;
                        if (back) put_back(e, p);
                    }
                }
                return;
            }
            for (int e0 = t; e0 < total; e0 += kB * KGB) {
                float g[kB];
                float* pp[kB];
                float* mp[kB];
                float* vp[kB];
                AdamC cq[kB];
                int n = 0;
#pragma unroll
                for (int q = 0; q < kB; q++) {
                    const int e = e0 + q * KGB;
                    const bool ok = e < total;
                    const int ee = ok ? e : e0;  // e0 < total: a valid dummy for the unused lanes of the batch
                    g[q] = grad_at(ee);
                    const size_t ge = (size_t)i0 * w + ee;
                    if (ok) put(dst, ge, g[q]);
                    n += ok;
                    if (grp) {
                        pp[q] = grp->param + ge;
                        mp[q] = grp->exp_avg + ge;
                        vp[q] = grp->exp_avg_sq + ge;
                        cq[q] = c;
                    }
                }
                float pn[kB];
                if (grp) {
                    if (n == kB) {
                        adam_batch<kB>(pp, mp, vp, g, cq, pn);
                    } else {  // tail: one at a time, never touching an element twice
                        for (int q = 0; q < n; q++) {
                            float p = *pp[q], m = *mp[q], v = *vp[q];
                            adam_elem(p, g[q], m, v, c);
                            *pp[q] = p;
                            *mp[q] = m;
                            *vp[q] = v;
                            pn[q] = p;
                        }
                    }
                    if (back)
                        for (int q = 0; q < n; q++) put_back(e0 + q * KGB, pn[q]);
                }
            }
        };
        const rr_adam* ad = a.use_adam ? &a.adam : nullptr;
        if (!a.raw) {
            stage_out(a.dL_dsh, nullptr, nf, 0);
        } else {
            stage_out(a.dL_dsh, ad ? &ad->f_dc : nullptr, 3, 0);
            if (nf > 3) stage_out(a.dL_dsh_rest, ad ? &ad->f_rest : nullptr, nf - 3, 3);
        }
    }
    if constexpr (!MULTI) {
        if (back) {
            // Cross-step fusion (include/rain_raster.h rr_next_frame): the next frame's preprocess
            // (forward.cu:144-246) of this block's Gaussians on the parameters this pass has just
            // stepped — xyz / opacity / scaling / rotation from registers, the SH coefficients from
            // the LDS rows — with the forward preprocess's own code (rr_preprocess.hpp), so the
            // geometry equals what k_preprocess would compute from the stored parameters.
            __syncthreads();
            const PreArgs& nx = a.next;
            bool wide = false;
            uint2 c = make_uint2(0u, 0u);
            if (t < nvalid) {
                const int idx = i0 + t;
                preprocess_clear(nx, idx);
                const v3 p = mk(upd.v[0], upd.v[1], upd.v[2]);
                const v3 p_view = xform_point_4x3(p, nx.view);  // in_frustum (auxiliary.h:128-153)
                if (p_view.z > 0.2f) {
                    const float* row = s_sh + t * kShStride;
                    c = preprocess_finish<DEG, false>(nx, idx, p, p_view,
                                                      make_float4(upd.v[7], upd.v[8], upd.v[9], upd.v[10]),
                                                      mk(upd.v[4], upd.v[5], upd.v[6]), upd.v[3],
                                                      mk(row[0], row[1], row[2]), row + 3, wide);
                }
            }
            if constexpr (KGB == 256) {
                preprocess_block_sums(nx, blockIdx.x, c, wide);
            } else {
                // a 256-row block sum from 256 / KGB workgroups: atomic adds into the entries the
                // launcher zeroed (launch_gauss_bwd)
                static_assert(256 % KGB == 0, "workgroups must tile the 256-row block sums");
                uint32_t n = c.x, r = c.y;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    n += (uint32_t)__shfl_xor((int)n, o);
                    r += (uint32_t)__shfl_xor((int)r, o);
                }
                const bool wave_wide = __any(wide);
                if (lane == 0) {
                    const int blk = (blockIdx.x * KGB) / 256;
                    if (n) atomicAdd(&nx.block_sums[blk].x, n);
                    if (r) atomicAdd(&nx.block_sums[blk].y, r);
                    if (wave_wide) atomicOr(&nx.block_wide[blk], 1u);
                }
            }
        }
    }
}

int launch_gauss_bwd_views(const GaussBwdArgs& a, const ViewCam* cams, int V, const float* records, int rec_rows,
                           float grad_scale, hipStream_t st) {
    if (V < 1 || V > kMaxViews) return 1;
    if (a.P == 0) return 0;
    GaussBwdViewsArgs va{};
    va.g = a;
    for (int v = 0; v < V; v++) va.cams[v] = cams[v];
    va.V = V;
    va.records = records;
    va.rec_rows = rec_rows;
    va.grad_scale = grad_scale;
    const int nb = (a.P + kGB - 1) / kGB;
    switch (a.shs ? a.D : 0) {
        case 0: k_gauss_bwd_views<0><<<nb, kGB, 0, st>>>(va); break;
        case 1: k_gauss_bwd_views<1><<<nb, kGB, 0, st>>>(va); break;
        case 2: k_gauss_bwd_views<2><<<nb, kGB, 0, st>>>(va); break;
        default: k_gauss_bwd_views<3><<<nb, kGB, 0, st>>>(va); break;
    }
    return 0;
}

// Packed per-(Gaussian, view) record for the sharded step: accumulator slots 0..8 and the radius.
// Q > 0: rows are grouped for a chunked exchange (rr_backward_records) — row i = j*Q + r of owner
// j lands in chunk c = r / CR at N*r0 + j*rows_c + (r - r0) (r0 = c*CR, rows_c = min(CR, Q - r0)).
__global__ __launch_bounds__(256) void k_pack_records(const float* __restrict__ gacc, const int* __restrict__ radii,
                                                      int P, int Q, int CR, float* __restrict__ rec) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    size_t pos = (size_t)i;
    if (Q > 0) {
        const int j = i / Q, r = i - j * Q, r0 = (r / CR) * CR;
        pos = (size_t)(P / Q) * r0 + (size_t)j * min(CR, Q - r0) + (r - r0);
    }
    const int r = radii[i];
    float v[kRecFloats];
    if (r > 0) {
        const float4 a = reinterpret_cast<const float4*>(gacc + (size_t)i * GACC_STRIDE)[0];
        const float4 b = reinterpret_cast<const float4*>(gacc + (size_t)i * GACC_STRIDE)[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        v[8] = gacc[(size_t)i * GACC_STRIDE + 8];
    } else {
#pragma unroll
        for (int k = 0; k < 9; k++) v[k] = 0.f;
    }
    v[9] = (float)r;
    float2* o = reinterpret_cast<float2*>(rec + pos * kRecFloats);
#pragma unroll
    for (int k = 0; k < kRecFloats / 2; k++) o[k] = make_float2(v[2 * k], v[2 * k + 1]);
}

void launch_pack_records(const float* gacc, const int* radii, int P, int Q, int chunk_rows, float* rec,
                         hipStream_t st) {
    if (P > 0) k_pack_records<<<(P + 255) / 256, 256, 0, st>>>(gacc, radii, P, Q, chunk_rows, rec);
}

void launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t st) {
    if (a.P == 0) return;
    if (kGB1 != 256 && a.has_next) {  // the next frame's block sums are accumulated atomically
        const size_t nbs = ((size_t)a.P + 255) / 256;
        (void)hipMemsetAsync(a.next.block_sums, 0, nbs * sizeof(uint2), st);
        (void)hipMemsetAsync(a.next.block_wide, 0, nbs * sizeof(uint32_t), st);
    }
    // a.M <= 16 is validated by the API: the LDS row holds at most 16 coefficients
    const int nb = (a.P + kGB1 - 1) / kGB1;
    switch (a.shs ? a.D : 0) {
        case 0: k_gauss_bwd<0><<<nb, kGB1, 0, st>>>(a); break;
        case 1: k_gauss_bwd<1><<<nb, kGB1, 0, st>>>(a); break;
        case 2: k_gauss_bwd<2><<<nb, kGB1, 0, st>>>(a); break;
        default: k_gauss_bwd<3><<<nb, kGB1, 0, st>>>(a); break;
    }
}

}  // namespace rr
