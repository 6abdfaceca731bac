/*
 * rain_loss.h — C ABI of the fused training loss:
 *   loss = (1 - lambda) * mean|img - gt| + lambda * (1 - SSIM(img, gt))
 * with the reference's SSIM (utils/loss_utils.py:22-53: 11x11 Gaussian window, sigma 1.5, zero
 * padding, C1 = 0.01^2, C2 = 0.03^2) and L1 (loss_utils.py:6-7), as used by train.py:113-114.
 *
 * Forward writes the scalar loss and three per-pixel maps (dS/dmu1, dS/dE[x^2], dS/dE[xy], already
 * scaled by -lambda/(C*H*W)) that the backward blurs back onto the image.  Deterministic: block
 * partial sums are reduced in a fixed order.
 */
#ifndef RAIN_LOSS_H
#define RAIN_LOSS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* bytes of workspace the forward needs: 3*C*H*W floats of maps + per-block partial sums */
size_t rl_workspace_bytes(int C, int H, int W);

/* img, gt: [C,H,W] fp32 contiguous device arrays; window: 11 HOST floats (the reference's 1-D
 * gaussian(11, 1.5), normalised in fp32); out: loss[0] = total loss (device scalar); parts (device,
 * optional) = {total, L1 term, mean SSIM}. */
int rl_l1_ssim_forward(const float* img, const float* gt, int C, int H, int W, float lambda, const float* window,
                       void* workspace, size_t workspace_bytes, float* loss, float* parts, void* stream);

/* dimg = grad_loss[0] * dLoss/dimg (grad_loss: device scalar). */
int rl_l1_ssim_backward(const float* img, const float* gt, int C, int H, int W, float lambda, const float* window,
                        const void* workspace, const float* grad_loss, float* dimg, void* stream);

/* Forward and backward in one call, for a caller that needs both at once (a training step):
 * loss / parts exactly as rl_l1_ssim_forward, dimg exactly as rl_l1_ssim_backward; the finalize of
 * the loss rides on the backward launch (one launch less).  Not in the reference: its loss is
 * autograd over utils/loss_utils.py:22-53; this entry is the fused step's shortcut. */
int rl_l1_ssim_forward_backward(const float* img, const float* gt, int C, int H, int W, float lambda,
                                const float* window, void* workspace, size_t workspace_bytes, float* loss,
                                float* parts, const float* grad_loss, float* dimg, void* stream);

const char* rl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
