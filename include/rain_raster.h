/*
 * rain_raster.h — C ABI of the MI355X-native differentiable Gaussian-splat rasterizer.
 *
 * This is the drop-in boundary for the reference's `_C` extension
 * (sharonal10/rain submodules/diff_gaussian_rasterization/ext.cpp:4-7, rasterize_points.cu:24-212).
 * Every entry point takes plain device pointers, sizes and a HIP stream handle (as void*);
 * no torch types cross this boundary.  The Python host side (rain_amd/diff_gaussian_rasterization)
 * mirrors the reference's pybind signatures on top of these functions; INTEGRATION.md shows the
 * ctypes binding a maintainer would add to the reference instead of its pybind module.
 *
 * Conventions (identical to the reference kernels):
 *   - all float tensors are fp32, contiguous; means3D/scales [P,3], rotations [P,4] (w,x,y,z),
 *     opacities [P,1], shs [P,M,3], colors_precomp [P,3], cov3D_precomp [P,6];
 *   - viewmatrix/projmatrix are 16 floats, column-major (the transposed torch matrices);
 *   - optional inputs are NULL (the reference passes empty tensors, i.e. nullptr);
 *   - image outputs are planar CHW.
 * Return value: 0 on success, otherwise an rr_status code; rr_last_error() gives the text
 * (the reference raises std::runtime_error / AT_ERROR in the same situations).
 */
#ifndef RAIN_RASTER_H
#define RAIN_RASTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum rr_status {
    RR_OK = 0,
    RR_ERR_ARG = 1,     /* bad sizes / missing required pointer  (reference: AT_ERROR, rasterize_points.cu:47-49) */
    RR_ERR_HIP = 2,     /* HIP runtime / kernel error            (reference: CHECK_CUDA, auxiliary.h:155-162) */
    RR_ERR_CAPACITY = 3 /* workspace smaller than the *_bytes() query */
};

/* Per-frame settings: the scalar fields of GaussianRasterizationSettings
 * (diff_gaussian_rasterization/__init__.py:148-161) plus P, D, M. */
typedef struct rr_frame {
    int P;              /* number of Gaussians (means3D.size(0)) */
    int D;              /* active SH degree (settings.sh_degree) */
    int M;              /* SH coefficient stride, sh.size(1), 0 if no SH */
    int width, height;  /* image_width, image_height */
    float tan_fovx, tan_fovy;
    float scale_modifier;
    float low_pass;     /* RAIN-GS 2D dilation (forward.cu:99-100); 0.3 in vanilla 3DGS */
    int prefiltered;
    int debug;          /* sync + check after every launch (auxiliary.h:155-162) */
    int flags;          /* RR_FLAG_* (0 = defaults) */
} rr_frame;

/* Exact tile culling (default ON): (tile, Gaussian) pairs whose Gaussian provably reaches no
 * pixel of the tile with alpha >= 1/255 are not emitted.  Every pixel of such a tile skips the pair
 * in the reference too (forward.cu:329-338, backward.cu:485-491), so images, depth, radii and
 * gradients are unchanged; only the internal pair list is shorter.  The flag restores the
 * reference's full bounding-square binning (used by the pair-order parity test). */
#define RR_FLAG_NO_TILE_CULLING 1

/* Raw-parameter (training) mode: the Gaussian inputs are GaussianModel's pre-activation
 * parameters (scene/gaussian_model.py:131-136) and the rasterizer applies the getters itself
 * (gaussian_model.py:85-105): scales = exp(scales), rotations = rotations / max(|rotations|, 1e-12),
 * opacities = sigmoid(opacities), SH = cat(shs [P,1,3], shs_rest [P,M-1,3]).  The backward then
 * writes gradients w.r.t. those raw parameters (chain rule through the getters fused into the
 * per-Gaussian kernel), splitting dL/dSH into dL_dsh [P,1,3] and dL_dsh_rest [P,M-1,3], and can
 * fold the densification statistics (train.py:132-134, gaussian_model.py:419-421) into the same
 * pass.  Requires shs and scales/rotations (no precomputed colours or covariances). */
#define RR_FLAG_RAW_PARAMS 2

/* Early-stop binning (default ON for frames of >= 2^16 pairs; rr_set_binning_config): the tile
 * lists are built in two phases.  The pairs of the Gaussians nearer than a per-frame depth cut
 * (~1/3 of the pairs; rr_set_binning_config's denominator) are binned and blended for every tile;
 * the rest are binned only for tiles with a pixel still unsaturated, and their blend resumes
 * where it stopped.  Pairs past a tile's saturation are never blended by any pixel
 * (forward.cu:337-341; the backward walk starts at the last contributor), so images, depth and
 * gradients are those of the full lists; only the internal lists are shorter.  The flag bins
 * every pair in one phase (the pair-order tests compare full lists with the reference's). */
#define RR_FLAG_FULL_BINNING 4

/* Auxiliary normal map (BASELINE configs[4]: depth + normal aux outputs; the reference has no
 * normal output, so this has no reference counterpart -- parity is against oracle/raster_oracle.c).
 * Each visible Gaussian's normal is the world axis of its smallest scale, rotated into view space,
 * flipped to face the camera, unit length; the map is sum_i alpha_i T_i n_i per pixel (like depth:
 * no background term, not normalised by 1 - T).  Forward only (no gradient, like depth).  Needs
 * scales/rotations; set the flag on both forward stages and pass out_normal to
 * rr_forward_render_aux. */
#define RR_FLAG_AUX_NORMAL 8

/* Backward only: the workspace is the one registered with rr_set_forward_workspace before this
 * frame's forward render (already zero-filled there; see rr_set_forward_workspace).  Without it, or
 * when the workspace is not that registered buffer, rr_backward clears the workspace itself. */
#define RR_FLAG_WORKSPACE_REGISTERED 16

/* Camera / per-frame device arrays (reference args of the same names). */
typedef struct rr_camera {
    const float* background; /* [3] */
    const float* viewmatrix; /* [16] */
    const float* projmatrix; /* [16] */
    const float* campos;     /* [3] */
} rr_camera;

/* Gaussian inputs.  Exactly one of shs / colors_precomp, and one of (scales, rotations) /
 * cov3D_precomp must be non-NULL (checked by the Python layer, __init__.py:183-187). */
typedef struct rr_gaussians {
    const float* means3D;
    const float* shs;
    const float* colors_precomp;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const float* shs_rest;  /* RR_FLAG_RAW_PARAMS only: f_rest [P,M-1,3] (shs is then f_dc [P,1,3]) */
} rr_gaussians;

/* ---- scratch sizing (replaces GeometryState/ImageState/BinningState::fromChunk,
 *      rasterizer_impl.cu:144-183, and required<T>() rasterizer_impl.h:56-62) ---- */
size_t rr_geometry_bytes(int P);
size_t rr_image_bytes(int width, int height);
size_t rr_binning_bytes(int num_rendered, int width, int height);
size_t rr_backward_workspace_bytes(int P);

/*
 * Forward, stage 1 (replaces Rasterizer::forward rasterizer_impl.cu:213-277):
 * preprocess every Gaussian, total their (bin, Gaussian) pair counts, choose the early-stop depth
 * cut, and read back the pair counts (the one device->host sync the reference also has,
 * rasterizer_impl.cu:273).  Writes radii[P] (int32), *num_rendered = the reference's value (sum
 * of bounding-square tile counts, returned to Python unchanged) and *num_pairs = the pairs that
 * will actually be binned (after exact tile culling; size the binning buffer with it).  The image
 * buffer's per-frame block (tile ranges, counters) is reset here: render the frame (stage 2) into
 * the same image buffer.
 */
int rr_forward_geometry(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, int* radii,
                        void* geom_buffer, size_t geom_bytes, void* image_buffer, size_t image_bytes,
                        int* num_rendered, int* num_pairs, void* stream);

/*
 * Forward, stage 2 (replaces rasterizer_impl.cu:279-329): emit the (bin, Gaussian) pairs, put
 * each bin's pairs in the reference's (depth, index) order, split them into the bin's tile lists
 * and ranges, and alpha-blend every tile (two early-stop phases on large frames).
 * out_color [3,H,W], out_depth [1,H,W] are fully written.  `f` must carry the same flags as in
 * stage 1.
 */
int rr_forward_render(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, const int* radii,
                      void* geom_buffer, void* image_buffer, void* binning_buffer, size_t binning_bytes,
                      int num_pairs, float* out_color, float* out_depth, void* stream);

/* rr_forward_render plus the aux normal map out_normal [3,H,W] (RR_FLAG_AUX_NORMAL; NULL otherwise). */
int rr_forward_render_aux(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, const int* radii,
                          void* geom_buffer, void* image_buffer, void* binning_buffer, size_t binning_bytes,
                          int num_pairs, float* out_color, float* out_depth, float* out_normal, void* stream);

/*
 * Both forward stages in one call, for callers that keep a reusable binning buffer (the training
 * loop): stage 1, the pair-count read-back, then stage 2 straight away if `binning_bytes` is at
 * least rr_binning_bytes(*num_pairs, W, H) -- no return to the caller between the sync and the
 * binning launches, so the device idles only for the read-back itself.  If the buffer is too
 * small, *binning_needed receives the required size and RR_INCOMPLETE is returned with stage 1
 * done: the caller grows its buffer and finishes with rr_forward_render.
 */
#define RR_INCOMPLETE 4
int rr_forward(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, int* radii, void* geom_buffer,
               size_t geom_bytes, void* image_buffer, size_t image_bytes, void* binning_buffer, size_t binning_bytes,
               int* num_rendered, int* num_pairs, size_t* binning_needed, float* out_color, float* out_depth,
               void* stream);

/* Optional fused optimizer step for RR_FLAG_RAW_PARAMS backwards (rr_grads.adam): Adam over the six
 * GaussianModel parameter groups (gaussian_model.py:144-153), applied in the same pass that forms
 * the gradients, so the gradients never travel through HBM.  Same arithmetic as rain_train.h's
 * rt_adam_step / torch's fused Adam; the caller supplies each group's lr and bias corrections
 * (1 - beta1^step, sqrt(1 - beta2^step)).  param must be the array passed as the matching input
 * (means3D, shs, shs_rest, opacities, scales, rotations); it is updated in place. */
typedef struct rr_adam_group {
    float* param;
    float* exp_avg;
    float* exp_avg_sq;
    double lr;
    float bias_correction1;
    float bias_correction2_sqrt;
} rr_adam_group;
typedef struct rr_adam {
    rr_adam_group xyz, f_dc, f_rest, opacity, scaling, rotation;
    double beta1, beta2, eps;
} rr_adam;

/* Gradient outputs of _C.rasterize_gaussians_backward (rasterize_points.cu:145-153,190).
 * All arrays are fully written (no pre-zeroing needed). */
typedef struct rr_grads {
    float* dL_dmeans2D;   /* [P,3]  (z stays 0) */
    float* dL_dcolors;    /* [P,3] */
    float* dL_dopacity;   /* [P,1] */
    float* dL_dmeans3D;   /* [P,3] */
    float* dL_dcov3D;     /* [P,6] */
    float* dL_dsh;        /* [P,M,3] (may be NULL when M == 0) */
    float* dL_dscales;    /* [P,3] */
    float* dL_drotations; /* [P,4] */
    /* RR_FLAG_RAW_PARAMS only (all optional; dL_dmeans2D / dL_dcolors / dL_dcov3D may then be NULL):
     * dL_dsh -> f_dc grad [P,1,3], dL_dsh_rest -> f_rest grad [P,M-1,3]; dL_dopacity, dL_dscales,
     * dL_drotations are w.r.t. the raw logit / log-scale / unnormalised quaternion.
     * Densification statistics, updated in place for radii > 0 (gaussian_model.py:419-421,
     * train.py:133): grad_accum[i] += |dL/dmean2D[i].xy|, denom[i] += 1,
     * max_radii2D[i] = max(max_radii2D[i], radii[i]). */
    float* dL_dsh_rest;
    float* grad_accum;    /* [P] */
    float* denom;         /* [P] */
    float* max_radii2D;   /* [P] */
    /* RR_FLAG_RAW_PARAMS only, optional: apply Adam in place; the six gradient outputs may then be NULL */
    const rr_adam* adam;
    /* Optional, with adam: the NEXT frame's preprocess, run by the per-Gaussian backward on the
     * parameters it has just updated (struct below) */
    const struct rr_next_frame* next;
} rr_grads;

/* Cross-step fusion of the training loop: the per-Gaussian backward kernel of step s holds every
 * Gaussian's parameters right after its Adam update, which is exactly the input of step s+1's
 * preprocess (forward.cu:144-246: projection, covariance, SH colour, tile counts).  With
 * rr_grads.next it runs that preprocess in the same pass — the parameters are not read again — and
 * fills the next frame's geometry buffer and radii; step s+1 then renders with
 * rr_forward_from_geometry.  Requires rr_grads.adam, RR_FLAG_RAW_PARAMS, and the same P, M and SH
 * degree D in both frames (the caller renders normally when the degree steps up or a densify /
 * opacity reset replaces the parameters). */
typedef struct rr_next_frame {
    const rr_frame* frame;   /* the next frame: width, height, tan_fov, scale_modifier, low_pass, flags */
    const rr_camera* cam;    /* its camera (background unused) */
    int* radii;              /* [P] out */
    void* geom_buffer;       /* rr_geometry_bytes(P), filled as rr_forward_geometry's preprocess does */
    size_t geom_bytes;
} rr_next_frame;

/*
 * Backward (replaces Rasterizer::backward rasterizer_impl.cu:334-430 and the zero-filled
 * allocations of rasterize_points.cu:145-153).  dL_dpix is [3,H,W].
 */
/* Optional: the workspace (rr_backward_workspace_bytes, 16-B aligned) of the backward that will
 * follow the NEXT forward render on this thread.  That render zero-fills it inside its blend launch
 * (workgroups dispatched after the tiles', in the blend's drain), and an rr_backward given the same
 * workspace skips its own clear (one launch's worth of stores less between the loss and the blend
 * backward, with RR_FLAG_WORKSPACE_REGISTERED).  The caller must not write the workspace in
 * between.  NULL: drop a registration. */
int rr_set_forward_workspace(void* workspace, size_t workspace_bytes);

int rr_backward(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, const int* radii,
                const void* geom_buffer, const void* image_buffer, const void* binning_buffer,
                int num_rendered, const float* dL_dpix, void* workspace, size_t workspace_bytes,
                const rr_grads* out, void* stream);

/*
 * ---- Gaussian-sharded view-parallel training step (N ranks; no reference counterpart: the
 * reference is single-GPU).  Rank r owns the Gaussian rows
 * [r*Q, (r+1)*Q) (Q a multiple of 256, N*Q >= P) and renders one view per step; the bytes that
 * cross xGMI per step are per-(Gaussian, view) records, not parameters or gradients:
 *   1. owner:  rr_preprocess_rows for each of the step's N views over its rows -> that view's
 *              splat records, pair counts, depth keys, radii, per-256-row block sums;
 *   2. all-to-all: rank v receives view v's arrays of every row block, assembling them at
 *              rr_geometry_layout's offsets of a P_pad = N*Q geometry buffer (+ radii [P_pad]);
 *   3. rank v: rr_forward_from_geometry (depth sort, binning, blend: rr_forward minus the
 *              preprocess), loss, rr_backward_records -> one 10-float record per Gaussian
 *              (the blend backward's dmean2D.xy, dconic.xyz, dopacity, dcolor.rgb and the radius);
 *   4. all-to-all: the owner receives its rows' records of all N views;
 *   5. owner:  rr_gauss_backward_views: per Gaussian, the reference's per-view gradient
 *              (cov2D / projection / SH / cov3D backward, raw-parameter chain) for each view in
 *              order, summed per element in that order, scaled by grad_scale (1/N, rounded like
 *              grad.mul_(1/N)), then Adam on the owner's rows and the densification statistics.
 * The arithmetic of one step equals one process rendering the N views, summing their raw-parameter
 * gradients in view order, dividing by N and stepping Adam (up to the blend backward's float-atomic
 * order).  Parameters and moments are current only on their owner's rows between steps; callers
 * all-gather them where a full replica is read (densification, checkpoints, evaluation).
 */
#define RR_MAX_VIEWS 16
typedef struct rr_view {
    const float* viewmatrix; /* [16] device, column-major world->view (as rr_camera) */
    const float* projmatrix; /* [16] device, full projection */
    const float* campos;     /* [3] device */
    float tan_fovx, tan_fovy, low_pass;
    int width, height;
} rr_view;
/* Byte offsets, inside a geometry buffer carved for P rows (rr_geometry_bytes(P)), of the arrays
 * the preprocess writes: offsets[0] splat records (48 B each), [1] pair counts (uint2),
 * [2] depth keys (u32), [3] per-256-row block sums (uint2), [4] per-block wide-key flags (u32). */
int rr_geometry_layout(int P, size_t* offsets);
/* Preprocess of one row block for one camera: frame.P valid rows (gaussians pointers offset to the
 * block's first row), n_rows (a multiple of 256, >= P) rows written; rows P..n_rows-1 are culled
 * padding.  Outputs are the caller's arrays of n_rows entries (block sums: n_rows/256). */
int rr_preprocess_rows(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, int n_rows, int* radii,
                       void* splats, void* tiles, void* depth_keys, void* block_sums, void* block_wide, void* stream);
/* rr_preprocess_rows for num_views views of the same rows in one launch: view v's camera from
 * views[v] (the frame's width / height / tan_fov / low_pass are replaced by the view's), its arrays
 * at out + v * view_stride + field_offsets[k] for k = radii, splats, tiles, depth keys, block
 * sums, wide flags (the owner's send chunks of the Gaussian-sharded step).  wire != 0: instead of
 * the 48-B splat records and the depth keys, one 40-B wire record per row at field_offsets[1]
 * (the 10 floats a splat record holds that cannot be recomputed; field_offsets[3] unused), which
 * rr_unpack_rows turns back into the geometry arrays bitwise. */
int rr_preprocess_rows_views(const rr_frame* f, const rr_view* views, int num_views, const rr_gaussians* g,
                             int n_rows, void* out, size_t view_stride, const size_t field_offsets[6], int wire,
                             void* stream);
/* The receiving side of the geometry all-to-all: world chunks of chunk_bytes at recv (chunk j =
 * rank j's rows_per_rank rows in wire form, fields at field_offsets = wire records, tiles, radii,
 * block sums, wide flags) into a geometry buffer of world * rows_per_rank rows (splat records,
 * pair counts, depth keys, block sums at rr_geometry_layout's offsets) and radii[]. */
int rr_unpack_rows(int world, int rows_per_rank, const void* recv, size_t chunk_bytes, const size_t field_offsets[5],
                   void* geom_buffer, size_t geom_bytes, int* radii, void* stream);
/* rr_forward over a geometry buffer whose preprocess arrays are already filled (frame.P rows;
 * radii [P]) — by the sharded step's unpack or by the previous step's backward (rr_next_frame);
 * same outputs, same RR_INCOMPLETE / binning_needed protocol, with rr_forward_render_geometry as the
 * second stage. */
int rr_forward_from_geometry(const rr_frame* f, const rr_camera* cam, const int* radii, void* geom_buffer,
                             size_t geom_bytes, void* image_buffer, size_t image_bytes, void* binning_buffer,
                             size_t binning_bytes, int* num_rendered, int* num_pairs, size_t* binning_needed,
                             float* out_color, float* out_depth, void* stream);
int rr_forward_render_geometry(const rr_frame* f, const rr_camera* cam, const int* radii, void* geom_buffer,
                               void* image_buffer, void* binning_buffer, size_t binning_bytes, int num_pairs,
                               float* out_color, float* out_depth, void* stream);
/* Blend backward of a frame into one record of 10 floats per row (dmean2D.xy, dconic.xyz,
 * dopacity, dcolor.rgb, radius); workspace as rr_backward.  rows_per_rank = 0: records [P][10].
 * rows_per_rank = Q > 0 (dividing P = N*Q): grouped for an exchange in row chunks of chunk_rows —
 * chunk c (owner rows [r0, r0 + n_c), r0 = c*chunk_rows, n_c = min(chunk_rows, Q - r0)) is the
 * contiguous block [N][n_c][10] at row offset N*r0, so that its all-to-all can start while the
 * owners already run the previous chunk (rr_gauss_backward_views on n_c rows, record_rows n_c). */
int rr_backward_records(const rr_frame* f, const rr_camera* cam, const int* radii, const void* geom_buffer,
                        const void* image_buffer, const void* binning_buffer, int num_rendered, const float* dL_dpix,
                        void* workspace, size_t workspace_bytes, int rows_per_rank, int chunk_rows, float* records,
                        void* stream);
/* Per-Gaussian backward of a row block over num_views views (records [num_views][record_rows][10]),
 * RR_FLAG_RAW_PARAMS only: frame.P rows, frame.D / M / scale_modifier; gaussians = raw parameters
 * offset to the block.  out: no gradient arrays; optional densification statistics (offset to the
 * block); optional Adam (param pointers = the matching inputs; a group whose param is NULL is not
 * stepped, e.g. the replaced opacity of an opacity-reset iteration). */
int rr_gauss_backward_views(const rr_frame* f, const rr_view* views, int num_views, const rr_gaussians* g,
                            const float* records, int record_rows, float grad_scale, const rr_grads* out,
                            void* stream);

/* markVisible (rasterize_points.cu:193-212, rasterizer_impl.cu:43-55,130-142): present[P] as 0/1 bytes. */
int rr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                    uint8_t* present, void* stream);

/* ---- diagnostics ---- */
const char* rr_last_error(void);
const char* rr_version(void);

/* Per-stage frame statistics of the last forward on this thread (L, visible count, L_eff...). */
typedef struct rr_frame_stats {
    int64_t num_rendered;  /* L: the reference's pair count (bounding-square tiles) */
    int64_t num_visible;   /* V */
    int64_t l_eff;         /* sum over tiles of max n_contrib (needs rr_read_frame_stats) */
    int64_t tiles;         /* T */
    int64_t num_pairs;     /* pairs emitted by exact tile culling (before early-stop binning) */
    int64_t num_binned;    /* pairs actually sorted into tile lists (phase A + phase B) */
    int64_t phase_b_pairs; /* pairs of the Gaussians behind the early-stop cut (0: one phase) */
    int64_t phase_b_slots; /* phase-B slots the duplicate reserved (<= phase_b_pairs: its region's size) */
} rr_frame_stats;
int rr_read_frame_stats(const rr_frame* f, const void* geom_buffer, const void* image_buffer, rr_frame_stats* out,
                        void* stream);

/* Device pointers into the private scratch layout (tests compare them with the oracle's
 * binning state: per-tile pair order, ranges, n_contrib, final_T). */
typedef struct rr_debug_views {
    const uint32_t* point_list; /* [L] Gaussian ids in per-tile depth order */
    const uint32_t* ranges;     /* [T][2] */
    const uint32_t* tile_max;   /* [T] max n_contrib per tile */
    const float* final_T;       /* [H*W] */
    const uint32_t* n_contrib;  /* [H*W] */
    const float* splats;        /* [P][12] packed per-Gaussian records (see rr_common.hpp) */
} rr_debug_views;
int rr_debug_get_views(const rr_frame* f, const void* geom_buffer, const void* image_buffer,
                       const void* binning_buffer, int num_rendered, rr_debug_views* out);

/* Kernel timing with HIP events on the launch stream (bench.py's live roofline numbers).
 * rr_profile_enable(1) starts recording the selected stages (rr_profile_select: bit s = stage s,
 * default all); rr_profile_collect() synchronizes, adds the elapsed ms per stage into
 * ms[RR_NUM_STAGES] / counts, and clears the record.  Each recorded stage costs two event records
 * on the stream, so a timed loop selects only the kernel it reports. */
enum rr_stage {
    RR_STAGE_PREPROCESS = 0,
    RR_STAGE_DEPTH_SORT,
    RR_STAGE_SCAN,
    RR_STAGE_DUPLICATE,
    RR_STAGE_TILE_SORT,
    RR_STAGE_RANGES,
    RR_STAGE_BLEND_FWD,
    RR_STAGE_BLEND_BWD,
    RR_STAGE_GAUSS_BWD,
    RR_STAGE_MEMSET,
    RR_NUM_STAGES
};
int rr_profile_enable(int enable);
int rr_profile_select(unsigned stage_mask);

/* Runtime tuning knobs: each forces a product path that larger frames or scenes take onto the
 * small frames of the tests (every setting gives the same lists, images and gradients).  Kept per
 * HIP device (the device current at the call); a CPU-only process sets those of device 0.
 *   "pair_scan_direct_blocks" n  pair-count scans of up to n blocks of 2048 Gaussians let every
 *                         block sum the earlier block totals itself (2 launches); larger ones scan
 *                         the totals in one workgroup first (3 launches); default 512, <0 resets,
 *   "wide_bin_keys" 0/1   32-bit bin keys even when the bins fit 16 bits (default 0: only frames
 *                         with more than 65536 bins of 32x32 px use them),
 *   "phase_b_gather" 0/1  phase B by the gather path when the bins fit one workgroup's count
 *                         (default 1) or always by the windowed path (frames of > 16384 bins),
 *   "dup_b_rows" 0/1      phase-B gather on frames up to 128 x 256 tiles: open tiles as per-row bit
 *                         masks (default 1), or the flat mask of wider frames,
 *   "dup_big_bins" n      phase-B gather: Gaussians spanning more than n bins (default 32) emitted
 *                         by their whole workgroup; 0: each by its own thread; <0 resets,
 *   "sx_bucket" 0/1       per-bin order by one bucket pass + per-bucket insertion sort (default 1)
 *                         or by the 9-bit LSD passes of crowded buckets only,
 *   "sx_lds_cap" n        per-bin runs of more than n pairs (default, 0: 2048 in phase A, 4096 in
 *                         phase B's 1024-thread sort-expand) depth-sorted through their own
 *                         point_list region instead of LDS,
 *   "sort_min_units" n / "sort_min_units_tile" n  radix sorts pick the largest unit with >= n units
 *                         (defaults 128 / 1024 for the bin sorts; 0 resets),
 *   "sort_max_rounds" r   cap on 64-item rounds per wave in a sort unit: 1, 2, 4, 8 (16 otherwise),
 *   "early_den" n         early-stop split: phase A holds ~1/n of the pairs (default 3).
 * Unknown keys return RR_ERR_ARG. */
int rr_set_tuning(const char* key, int value);
/* Diagnostics: device buffer of >= 8 * 8 * tiles u32 receiving one timing record per forward-blend
 * wave (start / end s_memrealtime, tile, pairs walked, list length, phase) — only builds compiled
 * with -DRR_FWD_TRACE=1 write it (tools/fwd_trace.py); NULL turns it off. */
int rr_debug_set_fwd_trace(void* dev_buf);

/* Tuning knob (diagnostics / tests): early-stop binning bins L / split_denominator pairs in phase A
 * (1 = one phase) for frames of at least min_pairs pairs; 0 restores a default (3, 2^16).  Results
 * are identical for every choice.  Applies to frames rendered after the call (a backward finds its
 * frame's lists in the image buffer). */
int rr_set_binning_config(int split_denominator, int min_pairs);
int rr_profile_collect(double* ms, int64_t* counts);
const char* rr_stage_name(int stage);
/* Diagnostics: host time this thread spent waiting for forwards' pair counts (the one device->host
 * read per frame) since the last reset, in ns, and the number of waits; reset != 0 clears both
 * after reading.  Near zero per frame means the host, not the device, paces the loop. */
int rr_host_wait_stats(int reset, int64_t* wait_ns, int64_t* waits);

#ifdef __cplusplus
}
#endif
#endif /* RAIN_RASTER_H */
