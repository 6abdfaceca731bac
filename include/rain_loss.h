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

/* rl_l1_ssim_forward_backward split in two around the rasterizer's early-stop phase B, so that the
 * loss of the image rows phase A finished overlaps phase B on another stream.  open_bits: the
 * frame's open-tile bitmask (rr_frame_open_tiles: bit ty * tiles_x + tx of the 16 x 16-px tiles
 * phase A left open); part 1 runs the forward and backward bands whose rows (with the 11 x 11
 * window's halo, twice for the backward) hold no open tile, part 2 the others and the loss
 * finalize (loss required) — called after phase B and after part 1 (e.g. the stream of part 2
 * waits for an event recorded after part 1).  wait_event (optional, a hipEvent_t): the stream waits
 * for it first (rr_phase_a_event).  Together the two parts write bitwise rl_l1_ssim_forward_backward's
 * loss, parts and dimg into the same workspace.  The two-pass form only (rl_set_fused_band 0).
 * Not in the reference. */
int rl_l1_ssim_forward_backward_part(const float* img, const float* gt, int C, int H, int W, float lambda,
                                     const float* window, void* workspace, size_t workspace_bytes, float* loss,
                                     float* parts, const float* grad_loss, float* dimg, const void* open_bits,
                                     int tiles_x, int tiles_y, int part, void* wait_event, void* stream);

/* rl_l1_ssim_forward_backward's form: the forward + backward passes over maps in the workspace
 * (rows = 0, default), or one band walk of `rows` output rows per block (16, 24, 32, 48 or 64) that
 * forms the derivative maps on chip and blurs them back in the same pass (measured slower: its
 * per-row dependency chain is twice as long).  dimg agrees between the two to float contraction and
 * the loss to float rounding (the one-walk form sums its partials over another block partition). */
int rl_set_fused_band(int rows);

const char* rl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
