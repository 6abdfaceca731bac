/*
 * rain_train.h — C ABI of the fused training-step kernels around the rasterizer.
 *
 * rt_adam_step replaces the reference's optimizer.step() (train.py:145-146) on
 * torch.optim.Adam(param_groups, lr=0.0, eps=1e-15) (scene/gaussian_model.py:153-157): one launch
 * updates every parameter group, with the arithmetic of torch's fused Adam
 * (ATen/native/cuda/fused_adam_utils.cuh adam_math, ORIGINAL mode, no weight decay, no amsgrad):
 *   m = b1*m + (1-b1)*g ;  v = b2*v + (1-b2)*g*g            (double, stored fp32)
 *   p -= (lr / bc1) * m / (sqrt(v) / bc2_sqrt + eps)        (fp32)
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

const char* rt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RAIN_TRAIN_H */
