/*
 * rain_train.h — C ABI of the fused training-step kernels around the rasterizer.
 *
 * rt_adam_step replaces the reference's optimizer.step() (train.py:145-146) on
 * torch.optim.Adam(param_groups, lr=0.0, eps=1e-15) (scene/gaussian_model.py:153-157): one launch
 * updates every parameter group, with the fp32 arithmetic of torch's default (multi-tensor,
 * foreach) Adam that the reference's optimizer runs on GPU tensors (torch/optim/adam.py
 * _multi_tensor_adam; no weight decay, no amsgrad; rain_amd/csrc/adam_math.hpp):
 *   m.lerp_(g, 1 - b1) ;  v = b2*v + (1-b2)*g*g
 *   p += (-lr / bc1) * m / (sqrt(v) / bc2_sqrt + eps)   (hardware sqrt / reciprocal, <= 1 ulp)
 * with bc1 = 1 - b1^step and bc2_sqrt = sqrt(1 - b2^step) computed by the caller per group.
 *
 * Plain device pointers and sizes; the HIP stream is passed as void*.  Returns 0 on success,
 * otherwise non-zero with rt_last_error() describing the problem.
 */
#ifndef RAIN_TRAIN_H
#define RAIN_TRAIN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_MAX_GROUPS 8

typedef struct rt_adam_group {
    float* param;        /* [numel] updated in place */
    const float* grad;   /* [numel] */
    float* exp_avg;      /* [numel] updated in place */
    float* exp_avg_sq;   /* [numel] updated in place */
    int64_t numel;
    double lr;
    float bias_correction1;      /* 1 - beta1^step */
    float bias_correction2_sqrt; /* sqrt(1 - beta2^step) */
} rt_adam_group;

int rt_adam_step(const rt_adam_group* groups, int n_groups, double beta1, double beta2, double eps, void* stream);

/* The same step on gradient SUMS: every gradient element is multiplied by grad_scale (fp32) before
 * the update -- bitwise the reference's grad.mul_(1/N) followed by step().  Used by the view-sharded
 * step, where each rank updates only its 1/N slice of the flat parameter buffer after a
 * reduce-scatter of the gradient sums (rain_amd/train.py ShardedAdam). */
int rt_adam_step_scaled(const rt_adam_group* groups, int n_groups, double beta1, double beta2, double eps,
                        float grad_scale, void* stream);

/*
 * Densification as stream compaction (replaces GaussianModel.densify_and_prune's boolean-mask
 * cat / index chain, gaussian_model.py:339-415 via train.py:136-140).
 *
 * With g = xyz_gradient_accum / denom (NaN -> 0) and s = exp(scaling):
 *   clone  = |g| >= grad_threshold && max(s) <= clone_split_scale          (densify_and_clone)
 *   split  =  g  >= grad_threshold && max(s) >  clone_split_scale          (densify_and_split)
 *   prune(x) = sigmoid(opacity_x) < min_opacity || (prune_big_world && max(s_x) > big_world_scale)
 * (max_radii2D never prunes: densification_postfix has zeroed it before the prune, as in the
 * reference).  The result is, in the reference's order: the originals that are neither split nor
 * pruned, then the clones not pruned, then for n = 0..n_split-1 the n-th child of every split
 * Gaussian not pruned.  A child of Gaussian i has xyz = R(q_i) (z * s_i) + xyz_i, with z the i-th
 * row (in split order) of block n of standard normals drawn by the caller exactly as torch.normal
 * draws them, scaling = log(s_i * (1 / split_scale_div)) (torch divides by a scalar through its
 * reciprocal), and the parameters of i otherwise; clones and children get zero Adam moments.
 *
 * With abe_split (RAIN-GS warm-up, train.py:138-140, gaussian_model.py:342-364) the split
 * Gaussians first get n_split - 1 copies each, appended after the clones (copy-major, like
 * repeat(BACK_N, 1)): xyz = (xyz * abe_xyz_scale0) * abe_xyz_scale1, scaling = log(exp(s)), the
 * other parameters as they are, zero moments, pruned like any row; the caller draws (and drops)
 * the (n_split - 1) * counts[3] rows of normals the reference draws for them before the split's.
 *
 * rt_densify_plan: flags + offsets into the workspace and the five counts (host, after a sync):
 *   counts[0] = originals kept, [1] = clones kept, [2] = split Gaussians whose children are kept,
 *   [3] = split Gaussians (rows of standard normals per child block), [4] = split Gaussians whose
 *   abe copies are kept (0 without abe_split).
 * rt_densify_apply: writes every group's parameter / exp_avg / exp_avg_sq rows for the new set of
 *   counts[0] + counts[1] + (n_split - 1) * counts[4] + n_split * counts[2] Gaussians.
 */
typedef struct rt_densify_params {
    int P;                    /* Gaussians before densification */
    int n_split;              /* children per split Gaussian (N = 2) */
    float grad_threshold;     /* max_grad */
    float clone_split_scale;  /* percent_dense * scene_extent */
    float min_opacity;
    float big_world_scale;    /* 0.1 * extent */
    int prune_big_world;      /* max_screen_size given */
    float split_scale_div;    /* divide_ratio * N */
    int abe_split;            /* RAIN-GS warm-up split (gaussian_model.py:342-364): n_split - 1 extra copies */
    float abe_xyz_scale0;     /* 0.3: an abe copy's xyz = (xyz * abe_xyz_scale0) * abe_xyz_scale1 */
    float abe_xyz_scale1;     /* scene_extent */
} rt_densify_params;

typedef struct rt_densify_group {
    const float* param;       /* [P, width] */
    const float* exp_avg;     /* [P, width] or NULL (no optimizer state yet) */
    const float* exp_avg_sq;
    float* out_param;         /* [P_new, width] */
    float* out_exp_avg;       /* NULL when exp_avg is NULL */
    float* out_exp_avg_sq;
    int width;                /* floats per Gaussian: xyz 3, f_dc 3, f_rest 3(M-1), opacity 1, scaling 3, rotation 4 */
    int kind;                 /* RT_GROUP_* */
} rt_densify_group;

#define RT_GROUP_OTHER 0
#define RT_GROUP_XYZ 1
#define RT_GROUP_SCALING 2

size_t rt_densify_workspace_bytes(int P);
int rt_densify_plan(const rt_densify_params* p, const float* xyz_gradient_accum, const float* denom,
                    const float* scaling, const float* opacity, void* workspace, size_t workspace_bytes,
                    int64_t counts[5], void* stream);
int rt_densify_apply(const rt_densify_params* p, const float* scaling, const float* rotation, const float* normals,
                     const void* workspace, const rt_densify_group* groups, int n_groups, const int64_t counts[5],
                     void* stream);

/* Streaming device-to-device copy of n_bytes (multiple of 16; both pointers 16-B aligned): 16-B
 * loads/stores per lane, grid sized to fill every CU several times.  Not on the training path: it
 * is the achievable-HBM yardstick bench.py prices the HBM-bound kernels against (the guide's
 * float4 copy, ~6.3 TB/s read + write on MI355X). */
int rt_stream_copy(void* dst, const void* src, size_t n_bytes, void* stream);

/* In-place read-modify-write stream over three arrays of n_floats (multiple of 4; 16-B aligned):
 * the access pattern of an Adam step (param, exp_avg, exp_avg_sq read and written back) with a
 * few FMAs for arithmetic.  Not on the training path: the achievable rate for that pattern
 * (~5.3-5.5 TB/s read + write on MI355X, below the copy's ~6.6: tools/rmw_probe.hip), which
 * bench.py prices the fused-Adam backward kernel against. */
int rt_stream_rmw(float* p, float* m, float* v, size_t n_floats, void* stream);

/* Densification statistics of the reference-API step (gaussian_model.py:419-421,
 * add_densification_stats; train.py:133), one launch each, for the rows with vis[i] != 0:
 * xyz_gradient_accum[i] += ||grad2d[i, 0:2]|| (torch.norm's rounding), denom[i] += 1;
 * max_radii2D[i] = max(max_radii2D[i], radii[i]).  grad2d rows are grad_stride floats apart. */
int rt_densify_stats(int P, const float* grad2d, int grad_stride, const uint8_t* vis, float* xyz_gradient_accum,
                     float* denom, void* stream);
int rt_max_radii(int P, const int* radii, const uint8_t* vis, float* max_radii2D, void* stream);

/* Trace markers (not on the training path): launches an empty one-wave kernel named
 * k_trace_mark_begin (which == 0) or k_trace_mark_end (which != 0) on `stream`, so that a
 * rocprofv3 kernel trace can be cut to the launches between them (bench.py's timed loop). */
int rt_trace_marker(int which, int tag, void* stream);

const char* rt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RAIN_TRAIN_H */
