/*
 * raster_oracle.c — CPU restatement of the reference differentiable Gaussian rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle and the CPU baseline
 * (`cpu_baseline.kind = "port"` in bench.py).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path (rain_amd/) never does.
 *
 * It restates, in plain C (float32, same operation order as the reference source),
 * the algorithm of sharonal10/rain submodules/diff_gaussian_rasterization:
 *   - preprocess            cuda_rasterizer/forward.cu:144-246 (+ computeCov3D :107-141,
 *                           computeCov2D :63-102, computeColorFromSH :9-60,
 *                           in_frustum / getRect / ndc2Pix auxiliary.h:30-45,128-153)
 *   - binning               cuda_rasterizer/rasterizer_impl.cu:59-127,266-310
 *                           (duplicateWithKeys, CUB InclusiveSum + stable radix SortPairs
 *                           on 32+msb(T) key bits, identifyTileRanges)
 *   - forward blend         cuda_rasterizer/forward.cu:251-369
 *   - backward blend        cuda_rasterizer/backward.cu:389-547
 *   - backward cov2D        cuda_rasterizer/backward.cu:133-264
 *   - backward preprocess   cuda_rasterizer/backward.cu:336-386 (+ SH bwd :9-128,
 *                           cov3D bwd :268-331, dnormvdv auxiliary.h:96-106)
 *   - markVisible           cuda_rasterizer/rasterizer_impl.cu:43-55,130-142
 *
 * Binning is done the way the reference does it (64-bit (tile|depth) keys in Gaussian
 * index order, stable LSD radix sort) — deliberately NOT the depth-first scheme the HIP
 * path uses — so the oracle also checks that the two orderings agree.
 *
 * Parity status: the reference CUDA code cannot be built here (needs nvcc, the CUDA
 * runtime, cooperative_groups and CUB), and the reference ships no tests or fixtures for
 * this path.  The SH polynomial and camera matrices are pinned against the reference's
 * importable Python (tests/golden/make_golden.py); the rest is "parity unpinned" against
 * the reference binary and is validated by autograd/finite differences of a differentiable
 * torch restatement (oracle/torch_ref.py).  See DESIGN.md §Oracle.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BLOCK_X 16
#define BLOCK_Y 16
#define BLOCK_SIZE (BLOCK_X * BLOCK_Y)

/* auxiliary.h:11-28 */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

typedef struct { float x, y, z; } f3;

static inline f3 mk3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 add3(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub3(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 scl3(float s, f3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
static inline float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float minf(float a, float b) { return a < b ? a : b; }
static inline float maxf(float a, float b) { return a > b ? a : b; }
static inline int mini(int a, int b) { return a < b ? a : b; }
static inline int maxi(int a, int b) { return a > b ? a : b; }

/* auxiliary.h:30-33 — computed in double, returned as float */
static inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

/* auxiliary.h:35-45 — C truncation, clamped to [0, grid] */
static inline void get_rect(float px, float py, int r, int gx, int gy, int* minx, int* miny, int* maxx,
                            int* maxy) {
    *minx = mini(gx, maxi(0, (int)((px - r) / BLOCK_X)));
    *miny = mini(gy, maxi(0, (int)((py - r) / BLOCK_Y)));
    *maxx = mini(gx, maxi(0, (int)((px + r + BLOCK_X - 1) / BLOCK_X)));
    *maxy = mini(gy, maxi(0, (int)((py + r + BLOCK_Y - 1) / BLOCK_Y)));
}

/* auxiliary.h:47-66 (column-major 4x4) */
static inline f3 xform_point_4x3(f3 p, const float* m) {
    return mk3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
               m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
static inline void xform_point_4x4(f3 p, const float* m, float out[4]) {
    out[0] = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
    out[1] = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
    out[2] = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
    out[3] = m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15];
}
/* auxiliary.h:78-86 */
static inline f3 xform_vec_4x3_T(f3 p, const float* m) {
    return mk3(m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
               m[8] * p.x + m[9] * p.y + m[10] * p.z);
}
/* auxiliary.h:96-106 */
static inline f3 dnormvdv(f3 v, f3 dv) {
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    f3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

/* Rotation matrix from an (r,x,y,z) quaternion, standard row-major math form.
 * forward.cu:116-127 builds glm::mat3 with these entries column-by-column, i.e. the glm
 * matrix is the transpose of Rs below; Sigma = Rs diag(s^2) Rs^T either way. */
static inline void quat_to_rot(const float* q, float Rs[3][3]) {
    float r = q[0], x = q[1], y = q[2], z = q[3];
    Rs[0][0] = 1.f - 2.f * (y * y + z * z); Rs[0][1] = 2.f * (x * y - r * z); Rs[0][2] = 2.f * (x * z + r * y);
    Rs[1][0] = 2.f * (x * y + r * z); Rs[1][1] = 1.f - 2.f * (x * x + z * z); Rs[1][2] = 2.f * (y * z - r * x);
    Rs[2][0] = 2.f * (x * z - r * y); Rs[2][1] = 2.f * (y * z + r * x); Rs[2][2] = 1.f - 2.f * (x * x + y * y);
}

/* forward.cu:107-141.  glm: M = S*R (math S·Rs^T), Sigma = M^T M. */
static void compute_cov3d(const float* scale, float mod, const float* rot, float* cov3D) {
    float Rs[3][3];
    quat_to_rot(rot, Rs);
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    float Mm[3][3]; /* math M[i][j] = s_i * Rs[j][i] */
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Mm[i][j] = s[i] * Rs[j][i];
    float Sg[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Sg[i][j] = Mm[0][i] * Mm[0][j] + Mm[1][i] * Mm[1][j] + Mm[2][i] * Mm[2][j];
    cov3D[0] = Sg[0][0]; cov3D[1] = Sg[0][1]; cov3D[2] = Sg[0][2];
    cov3D[3] = Sg[1][1]; cov3D[4] = Sg[1][2]; cov3D[5] = Sg[2][2];
}

/* Exported for the golden test (tests/test_golden.py): Sigma3D of n Gaussians, 6 floats each. */
void orc_cov3d(int n, const float* scales, float mod, const float* rots, float* out) {
    for (int i = 0; i < n; i++) compute_cov3d(scales + 3 * (size_t)i, mod, rots + 4 * (size_t)i, out + 6 * (size_t)i);
}

/* Auxiliary normal (BASELINE configs[4] "depth+normal aux outputs"; the reference renders no
 * normals, so this follows the build's own definition in include/rain_raster.h RR_FLAG_AUX_NORMAL):
 * the world axis of the smallest scale (column k of Rs), rotated into view space by R_w2c
 * (transformVec4x3, auxiliary.h:68-76), flipped to face the camera, unit length. */
static f3 gaussian_normal(const float* scale, const float* rot, const float* view, f3 p_view) {
    float Rs[3][3];
    quat_to_rot(rot, Rs);
    int k = 0;
    if (scale[1] < scale[k]) k = 1;
    if (scale[2] < scale[k]) k = 2;
    f3 n = mk3(Rs[0][k], Rs[1][k], Rs[2][k]);
    f3 nv = mk3(view[0] * n.x + view[4] * n.y + view[8] * n.z, view[1] * n.x + view[5] * n.y + view[9] * n.z,
                view[2] * n.x + view[6] * n.y + view[10] * n.z);
    if (dot3(nv, p_view) > 0.f) nv = mk3(-nv.x, -nv.y, -nv.z);
    float len = sqrtf(dot3(nv, nv));
    if (!(len > 0.f)) return mk3(0.f, 0.f, 0.f);
    return mk3(nv.x / len, nv.y / len, nv.z / len);
}

/* Shared between forward.cu:63-102 and backward.cu:156-189: the clamped view-space mean,
 * the 2x3 block A = J·W (glm's T is A laid out so that glm T[i][j] == A[i][j]), and the
 * un-dilated 2D covariance A V A^T. */
typedef struct {
    f3 t;            /* clamped view-space mean */
    float txtz, tytz; /* unclamped ratios (for the backward clamp mask) */
    float limx, limy;
    float A[2][3];
    float V[3][3];
} cov2d_ctx;

static void cov2d_setup(f3 mean, float fx, float fy, float tanfovx, float tanfovy, const float* cov3D,
                        const float* view, cov2d_ctx* c) {
    f3 t = xform_point_4x3(mean, view);
    c->limx = 1.3f * tanfovx;
    c->limy = 1.3f * tanfovy;
    c->txtz = t.x / t.z;
    c->tytz = t.y / t.z;
    t.x = minf(c->limx, maxf(-c->limx, c->txtz)) * t.z;
    t.y = minf(c->limy, maxf(-c->limy, c->tytz)) * t.z;
    c->t = t;
    float J00 = fx / t.z, J02 = -(fx * t.x) / (t.z * t.z);
    float J11 = fy / t.z, J12 = -(fy * t.y) / (t.z * t.z);
    /* W[i][j] = R_w2c[i][j] = view[4j+i] */
    float W[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) W[i][j] = view[4 * j + i];
    for (int j = 0; j < 3; j++) {
        c->A[0][j] = J00 * W[0][j] + J02 * W[2][j];
        c->A[1][j] = J11 * W[1][j] + J12 * W[2][j];
    }
    c->V[0][0] = cov3D[0]; c->V[0][1] = cov3D[1]; c->V[0][2] = cov3D[2];
    c->V[1][0] = cov3D[1]; c->V[1][1] = cov3D[3]; c->V[1][2] = cov3D[4];
    c->V[2][0] = cov3D[2]; c->V[2][1] = cov3D[4]; c->V[2][2] = cov3D[5];
}

/* cov = A V A^T (upper 2x2), before the low-pass dilation, in glm's association of
 * transpose(T) * transpose(Vrk) * T (forward.cu:95, backward.cu:184): (T^T Vrk^T)[k][r] = B[r][k] and
 * cov[c][r] = sum_k B[r][k] * A[c][k] (k = 0, 1, 2 left to right), so the off-diagonal the reference
 * returns, cov[0][1], is B[1] . A[0]. */
static void cov2d_eval(const cov2d_ctx* c, float* a, float* b, float* cc) {
    float B[2][3];
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 3; j++) B[i][j] = c->A[i][0] * c->V[0][j] + c->A[i][1] * c->V[1][j] + c->A[i][2] * c->V[2][j];
    *a = B[0][0] * c->A[0][0] + B[0][1] * c->A[0][1] + B[0][2] * c->A[0][2];
    *b = B[1][0] * c->A[0][0] + B[1][1] * c->A[0][1] + B[1][2] * c->A[0][2];
    *cc = B[1][0] * c->A[1][0] + B[1][1] * c->A[1][1] + B[1][2] * c->A[1][2];
}

/* forward.cu:9-60 */
static f3 color_from_sh(int deg, int max_coeffs, f3 pos, f3 campos, const float* shs, unsigned char* clamped3) {
    f3 dir = sub3(pos, campos);
    float len = sqrtf(dot3(dir, dir));
    dir = mk3(dir.x / len, dir.y / len, dir.z / len);
    const float* sh = shs;
#define SH(k) mk3(sh[3 * (k) + 0], sh[3 * (k) + 1], sh[3 * (k) + 2])
    f3 result = scl3(SH_C0, SH(0));
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        result = sub3(add3(sub3(result, scl3(SH_C1 * y, SH(1))), scl3(SH_C1 * z, SH(2))), scl3(SH_C1 * x, SH(3)));
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            result = add3(result, scl3(SH_C2[0] * xy, SH(4)));
            result = add3(result, scl3(SH_C2[1] * yz, SH(5)));
            result = add3(result, scl3(SH_C2[2] * (2.0f * zz - xx - yy), SH(6)));
            result = add3(result, scl3(SH_C2[3] * xz, SH(7)));
            result = add3(result, scl3(SH_C2[4] * (xx - yy), SH(8)));
            if (deg > 2) {
                result = add3(result, scl3(SH_C3[0] * y * (3.0f * xx - yy), SH(9)));
                result = add3(result, scl3(SH_C3[1] * xy * z, SH(10)));
                result = add3(result, scl3(SH_C3[2] * y * (4.0f * zz - xx - yy), SH(11)));
                result = add3(result, scl3(SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), SH(12)));
                result = add3(result, scl3(SH_C3[4] * x * (4.0f * zz - xx - yy), SH(13)));
                result = add3(result, scl3(SH_C3[5] * z * (xx - yy), SH(14)));
                result = add3(result, scl3(SH_C3[6] * x * (xx - 3.0f * yy), SH(15)));
            }
        }
    }
#undef SH
    result = mk3(result.x + 0.5f, result.y + 0.5f, result.z + 0.5f);
    clamped3[0] = result.x < 0; clamped3[1] = result.y < 0; clamped3[2] = result.z < 0;
    return mk3(maxf(result.x, 0.f), maxf(result.y, 0.f), maxf(result.z, 0.f));
}

/* SH colour for a given unit direction (forward.cu:18-59 after the normalisation at :14-16):
 * out = max(SH(dir) + 0.5, 0), clamped = (SH(dir) + 0.5 < 0).  Test entry point. */
void orc_sh_eval(int deg, int max_coeffs, int n, const float* dirs, const float* shs, float* out,
                 unsigned char* clamped) {
    for (int i = 0; i < n; i++) {
        /* campos = 0, pos = dir: color_from_sh re-normalises an (already unit) direction */
        f3 d = mk3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        f3 rgb = color_from_sh(deg, max_coeffs, d, mk3(0.f, 0.f, 0.f), shs + (size_t)i * max_coeffs * 3,
                               clamped + 3 * (size_t)i);
        out[3 * i] = rgb.x; out[3 * i + 1] = rgb.y; out[3 * i + 2] = rgb.z;
    }
}

/* ------------------------------------------------------------------------------------ */

typedef struct orc_state {
    int P, D, M, W, H, gx, gy;
    int num_rendered;
    /* geometry (rasterizer_impl.cu:144-159) */
    float* depths;
    int* radii;
    float* xy;            /* 2P */
    float* cov3D;         /* 6P */
    float* conic_opacity; /* 4P */
    float* rgb;           /* 3P */
    unsigned char* clamped; /* 3P */
    uint32_t* tiles_touched;
    uint32_t* point_offsets;
    /* binning */
    uint32_t* point_list; /* L */
    uint64_t* keys;       /* L (sorted) */
    /* image */
    uint32_t* ranges; /* 2T */
    float* final_T;   /* W*H */
    uint32_t* n_contrib;
} orc_state;

void orc_free(orc_state* s) {
    if (!s) return;
    free(s->depths); free(s->radii); free(s->xy); free(s->cov3D); free(s->conic_opacity); free(s->rgb);
    free(s->clamped); free(s->tiles_touched); free(s->point_offsets); free(s->point_list); free(s->keys);
    free(s->ranges); free(s->final_T); free(s->n_contrib);
    free(s);
}

static int set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
    return omp_get_max_threads();
#else
    (void)nthreads;
    return 1;
#endif
}

/* auxiliary.h:128-153 + rasterizer_impl.cu:43-55 */
void orc_mark_visible(int P, const float* means3D, const float* view, const float* proj, unsigned char* present) {
    for (int i = 0; i < P; i++) {
        f3 p = mk3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
        f3 pv = xform_point_4x3(p, view);
        (void)proj;
        present[i] = !(pv.z <= 0.2f);
    }
}

/* stable LSD radix sort of (key, value) pairs on bits [0, nbits) — CUB SortPairs semantics */
static void radix_sort_pairs_u64(uint64_t* keys, uint32_t* vals, size_t n, int nbits) {
    if (n == 0) return;
    uint64_t* k2 = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint32_t* v2 = (uint32_t*)malloc(n * sizeof(uint32_t));
    uint64_t *ks = keys, *kd = k2;
    uint32_t *vs = vals, *vd = v2;
    for (int shift = 0; shift < nbits; shift += 8) {
        int bits = nbits - shift < 8 ? nbits - shift : 8;
        uint64_t mask = (1ull << bits) - 1;
        size_t count[257];
        memset(count, 0, sizeof(count));
        for (size_t i = 0; i < n; i++) count[((ks[i] >> shift) & mask) + 1]++;
        for (int b = 0; b < 256; b++) count[b + 1] += count[b];
        for (size_t i = 0; i < n; i++) {
            size_t d = count[(ks[i] >> shift) & mask]++;
            kd[d] = ks[i];
            vd[d] = vs[i];
        }
        uint64_t* tk = ks; ks = kd; kd = tk;
        uint32_t* tv = vs; vs = vd; vd = tv;
    }
    if (ks != keys) {
        memcpy(keys, ks, n * sizeof(uint64_t));
        memcpy(vals, vs, n * sizeof(uint32_t));
    }
    free(k2);
    free(v2);
}

/* rasterizer_impl.cu:24-39 */
static uint32_t get_higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

uint32_t orc_get_higher_msb(uint32_t n) { return get_higher_msb(n); }

/*
 * Full forward (rasterizer_impl.cu:187-330).  Returns a state handle for the backward,
 * writes out_color [3,H,W], out_depth [H,W], radii [P]; *num_rendered_out = L.
 * shs / colors_precomp / scales / rotations / cov3D_precomp may be NULL (empty tensor).
 */
orc_state* orc_forward(int P, int D, int M, const float* bg, int W, int H, const float* means3D,
                       const float* shs, const float* colors_precomp, const float* opacities, const float* scales,
                       float scale_modifier, const float* rotations, const float* cov3D_precomp,
                       const float* view, const float* proj, const float* campos, float tanfovx, float tanfovy,
                       int prefiltered, float low_pass, float* out_color, float* out_depth, int* radii_out,
                       int* num_rendered_out, int nthreads, float* out_normal) {
    (void)prefiltered;
    set_threads(nthreads);
    orc_state* s = (orc_state*)calloc(1, sizeof(orc_state));
    s->P = P; s->D = D; s->M = M; s->W = W; s->H = H;
    s->gx = (W + BLOCK_X - 1) / BLOCK_X;
    s->gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    const int gx = s->gx, gy = s->gy, T = gx * gy;
    const float focal_y = H / (2.0f * tanfovy);
    const float focal_x = W / (2.0f * tanfovx);
    size_t Pz = P > 0 ? (size_t)P : 1;
    s->depths = (float*)calloc(Pz, sizeof(float));
    s->radii = (int*)calloc(Pz, sizeof(int));
    s->xy = (float*)calloc(2 * Pz, sizeof(float));
    s->cov3D = (float*)calloc(6 * Pz, sizeof(float));
    s->conic_opacity = (float*)calloc(4 * Pz, sizeof(float));
    s->rgb = (float*)calloc(3 * Pz, sizeof(float));
    s->clamped = (unsigned char*)calloc(3 * Pz, 1);
    s->tiles_touched = (uint32_t*)calloc(Pz, sizeof(uint32_t));
    s->point_offsets = (uint32_t*)calloc(Pz, sizeof(uint32_t));
    s->ranges = (uint32_t*)calloc(2 * (size_t)T, sizeof(uint32_t));
    s->final_T = (float*)calloc((size_t)W * H, sizeof(float));
    s->n_contrib = (uint32_t*)calloc((size_t)W * H, sizeof(uint32_t));
    float* normals = out_normal ? (float*)calloc(3 * Pz, sizeof(float)) : NULL;

    /* ---- preprocess: forward.cu:144-246 ---- */
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        s->radii[idx] = 0;
        s->tiles_touched[idx] = 0;
        f3 p_orig = mk3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
        f3 p_view = xform_point_4x3(p_orig, view);
        if (p_view.z <= 0.2f) continue;
        float p_hom[4];
        xform_point_4x4(p_orig, proj, p_hom);
        float p_w = 1.0f / (p_hom[3] + 0.0000001f);
        float ppx = p_hom[0] * p_w, ppy = p_hom[1] * p_w;
        const float* cov3D;
        if (cov3D_precomp) {
            cov3D = cov3D_precomp + 6 * (size_t)idx;
        } else {
            compute_cov3d(scales + 3 * (size_t)idx, scale_modifier, rotations + 4 * (size_t)idx, s->cov3D + 6 * (size_t)idx);
            cov3D = s->cov3D + 6 * (size_t)idx;
        }
        cov2d_ctx c;
        cov2d_setup(p_orig, focal_x, focal_y, tanfovx, tanfovy, cov3D, view, &c);
        float ca, cb, cc;
        cov2d_eval(&c, &ca, &cb, &cc);
        ca += low_pass;
        cc += low_pass;
        float det = ca * cc - cb * cb;
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {cc * det_inv, -cb * det_inv, ca * det_inv};
        float mid = 0.5f * (ca + cc);
        float lambda1 = mid + sqrtf(maxf(0.1f, mid * mid - det));
        float lambda2 = mid - sqrtf(maxf(0.1f, mid * mid - det));
        float my_radius = ceilf(3.f * sqrtf(maxf(lambda1, lambda2)));
        float pix_x = ndc2pix(ppx, W), pix_y = ndc2pix(ppy, H);
        int rminx, rminy, rmaxx, rmaxy;
        get_rect(pix_x, pix_y, (int)my_radius, gx, gy, &rminx, &rminy, &rmaxx, &rmaxy);
        if ((rmaxx - rminx) * (rmaxy - rminy) == 0) continue;
        if (!colors_precomp) {
            f3 rgb = color_from_sh(D, M, p_orig, mk3(campos[0], campos[1], campos[2]), shs + (size_t)idx * M * 3,
                                   s->clamped + 3 * (size_t)idx);
            s->rgb[3 * idx + 0] = rgb.x; s->rgb[3 * idx + 1] = rgb.y; s->rgb[3 * idx + 2] = rgb.z;
        }
        s->depths[idx] = p_view.z;
        s->radii[idx] = (int)my_radius;
        s->xy[2 * idx] = pix_x; s->xy[2 * idx + 1] = pix_y;
        s->conic_opacity[4 * idx + 0] = conic[0];
        s->conic_opacity[4 * idx + 1] = conic[1];
        s->conic_opacity[4 * idx + 2] = conic[2];
        s->conic_opacity[4 * idx + 3] = opacities[idx];
        s->tiles_touched[idx] = (uint32_t)((rmaxy - rminy) * (rmaxx - rminx));
        if (normals) {
            f3 nv = gaussian_normal(scales + 3 * (size_t)idx, rotations + 4 * (size_t)idx, view, p_view);
            normals[3 * idx] = nv.x; normals[3 * idx + 1] = nv.y; normals[3 * idx + 2] = nv.z;
        }
    }
    if (radii_out) memcpy(radii_out, s->radii, sizeof(int) * (size_t)P);

    /* ---- inclusive scan (rasterizer_impl.cu:269) ---- */
    uint64_t acc = 0;
    for (int i = 0; i < P; i++) {
        acc += s->tiles_touched[i];
        s->point_offsets[i] = (uint32_t)acc;
    }
    size_t L = (size_t)acc;
    s->num_rendered = (int)L;
    if (num_rendered_out) *num_rendered_out = (int)L;

    /* ---- duplicateWithKeys (rasterizer_impl.cu:59-100) ---- */
    s->keys = (uint64_t*)malloc((L ? L : 1) * sizeof(uint64_t));
    s->point_list = (uint32_t*)malloc((L ? L : 1) * sizeof(uint32_t));
#pragma omp parallel for schedule(dynamic, 256)
    for (int idx = 0; idx < P; idx++) {
        if (s->radii[idx] > 0) {
            size_t off = idx == 0 ? 0 : s->point_offsets[idx - 1];
            int rminx, rminy, rmaxx, rmaxy;
            get_rect(s->xy[2 * idx], s->xy[2 * idx + 1], s->radii[idx], gx, gy, &rminx, &rminy, &rmaxx, &rmaxy);
            uint32_t dbits;
            memcpy(&dbits, &s->depths[idx], 4);
            for (int y = rminy; y < rmaxy; y++)
                for (int x = rminx; x < rmaxx; x++) {
                    uint64_t key = (uint64_t)(y * gx + x);
                    key <<= 32;
                    key |= dbits;
                    s->keys[off] = key;
                    s->point_list[off] = (uint32_t)idx;
                    off++;
                }
        }
    }

    /* ---- stable radix sort on 32+msb(T) bits (rasterizer_impl.cu:292-300) ---- */
    int bit = (int)get_higher_msb((uint32_t)T);
    radix_sort_pairs_u64(s->keys, s->point_list, L, 32 + bit);

    /* ---- identifyTileRanges (rasterizer_impl.cu:105-127) ---- */
    for (size_t i = 0; i < L; i++) {
        uint32_t cur = (uint32_t)(s->keys[i] >> 32);
        if (i == 0) s->ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(s->keys[i - 1] >> 32);
            if (cur != prev) {
                s->ranges[2 * prev + 1] = (uint32_t)i;
                s->ranges[2 * cur] = (uint32_t)i;
            }
        }
        if (i == L - 1) s->ranges[2 * cur + 1] = (uint32_t)L;
    }

    /* ---- blend forward (forward.cu:251-369) ---- */
    const float* features = colors_precomp ? colors_precomp : s->rgb;
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < T; tile++) {
        int tx = tile % gx, ty = tile / gx;
        uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
        for (int ly = 0; ly < BLOCK_Y; ly++)
            for (int lx = 0; lx < BLOCK_X; lx++) {
                int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                if (px >= W || py >= H) continue;
                size_t pix_id = (size_t)W * py + px;
                float pfx = (float)px, pfy = (float)py;
                float Tr = 1.0f;
                uint32_t contributor = 0, last_contributor = 0;
                float C[3] = {0, 0, 0}, Dp = 0, Nm[3] = {0, 0, 0};
                for (uint32_t k = rs; k < re; k++) {
                    contributor++;
                    uint32_t g = s->point_list[k];
                    float dx = s->xy[2 * g] - pfx, dy = s->xy[2 * g + 1] - pfy;
                    const float* co = s->conic_opacity + 4 * (size_t)g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    float alpha = minf(0.99f, co[3] * expf(power));
                    if (alpha < 1.0f / 255.0f) continue;
                    float test_T = Tr * (1 - alpha);
                    if (test_T < 0.0001f) break; /* done = true */
                    for (int ch = 0; ch < 3; ch++) C[ch] += features[3 * (size_t)g + ch] * alpha * Tr;
                    Dp += s->depths[g] * alpha * Tr;
                    if (normals)
                        for (int ch = 0; ch < 3; ch++) Nm[ch] += normals[3 * (size_t)g + ch] * alpha * Tr;
                    Tr = test_T;
                    last_contributor = contributor;
                }
                s->final_T[pix_id] = Tr;
                s->n_contrib[pix_id] = last_contributor;
                for (int ch = 0; ch < 3; ch++) out_color[(size_t)ch * H * W + pix_id] = C[ch] + Tr * bg[ch];
                out_depth[pix_id] = Dp;
                if (out_normal)
                    for (int ch = 0; ch < 3; ch++) out_normal[(size_t)ch * H * W + pix_id] = Nm[ch];
            }
    }
    free(normals);
    return s;
}

/* atomic float add for the backward blend (backward.cu:513,535-544 use atomicAdd) */
static inline void fadd(float* p, float v) {
#pragma omp atomic
    *p += v;
}

/*
 * Full backward (rasterizer_impl.cu:334-430).  All gradient outputs must be zero-filled
 * by the caller (rasterize_points.cu:145-153 allocates them with torch::zeros).
 * dL_dconic is [P,4] (the reference's [P,2,2]; entries 0,1,3 used).
 */
int orc_backward(orc_state* s, const float* bg, const float* means3D, const int* radii, const float* colors_precomp,
                 const float* scales, float scale_modifier, const float* rotations, const float* cov3D_precomp,
                 const float* view, const float* proj, const float* campos, float tanfovx, float tanfovy,
                 const float* shs, const float* dL_dpix, float low_pass, float* dL_dmeans2D, float* dL_dcolors,
                 float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                 float* dL_drot, float* dL_dconic, int nthreads) {
    set_threads(nthreads);
    const int P = s->P, W = s->W, H = s->H, gx = s->gx, gy = s->gy, T = gx * gy, D = s->D, M = s->M;
    if (!radii) radii = s->radii;
    const float focal_y = H / (2.0f * tanfovy);
    const float focal_x = W / (2.0f * tanfovx);
    const float* colors = colors_precomp ? colors_precomp : s->rgb;

    /* ---- blend backward (backward.cu:389-547) ---- */
    const float ddelx_dx = (float)(0.5 * W);
    const float ddely_dy = (float)(0.5 * H);
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < T; tile++) {
        int tx = tile % gx, ty = tile / gx;
        uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
        for (int ly = 0; ly < BLOCK_Y; ly++)
            for (int lx = 0; lx < BLOCK_X; lx++) {
                int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                if (px >= W || py >= H) continue;
                size_t pix_id = (size_t)W * py + px;
                float pfx = (float)px, pfy = (float)py;
                const float T_final = s->final_T[pix_id];
                float Tr = T_final;
                const uint32_t last_contributor = s->n_contrib[pix_id];
                float accum_rec[3] = {0, 0, 0}, dL_dpixel[3], last_color[3] = {0, 0, 0}, last_alpha = 0;
                for (int i = 0; i < 3; i++) dL_dpixel[i] = dL_dpix[(size_t)i * H * W + pix_id];
                uint32_t len = re - rs;
                for (uint32_t k = len; k-- > 0;) { /* contributor-- ; contributor == k */
                    if (k >= last_contributor) continue;
                    uint32_t g = s->point_list[rs + k];
                    float dx = s->xy[2 * g] - pfx, dy = s->xy[2 * g + 1] - pfy;
                    const float* co = s->conic_opacity + 4 * (size_t)g;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    float G = expf(power);
                    float alpha = minf(0.99f, co[3] * G);
                    if (alpha < 1.0f / 255.0f) continue;
                    Tr = Tr / (1.f - alpha);
                    float dchannel_dcolor = alpha * Tr;
                    float dL_dalpha = 0.0f;
                    for (int ch = 0; ch < 3; ch++) {
                        float c = colors[3 * (size_t)g + ch];
                        accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                        last_color[ch] = c;
                        float dL_dchannel = dL_dpixel[ch];
                        dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
                        fadd(&dL_dcolors[3 * (size_t)g + ch], dchannel_dcolor * dL_dchannel);
                    }
                    dL_dalpha *= Tr;
                    last_alpha = alpha;
                    float bg_dot_dpixel = 0;
                    for (int i = 0; i < 3; i++) bg_dot_dpixel += bg[i] * dL_dpixel[i];
                    dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
                    float dL_dG = co[3] * dL_dalpha;
                    float gdx = G * dx, gdy = G * dy;
                    float dG_ddelx = -gdx * co[0] - gdy * co[1];
                    float dG_ddely = -gdy * co[2] - gdx * co[1];
                    fadd(&dL_dmeans2D[3 * (size_t)g + 0], dL_dG * dG_ddelx * ddelx_dx);
                    fadd(&dL_dmeans2D[3 * (size_t)g + 1], dL_dG * dG_ddely * ddely_dy);
                    fadd(&dL_dconic[4 * (size_t)g + 0], -0.5f * gdx * dx * dL_dG);
                    fadd(&dL_dconic[4 * (size_t)g + 1], -0.5f * gdx * dy * dL_dG);
                    fadd(&dL_dconic[4 * (size_t)g + 3], -0.5f * gdy * dy * dL_dG);
                    fadd(&dL_dopacity[g], G * dL_dalpha);
                }
            }
    }

    const float* cov3Ds = cov3D_precomp ? cov3D_precomp : s->cov3D;

    /* ---- computeCov2DCUDA (backward.cu:133-264) ---- */
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        const float* cov3D = cov3Ds + 6 * (size_t)idx;
        f3 mean = mk3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
        float dcx = dL_dconic[4 * (size_t)idx], dcy = dL_dconic[4 * (size_t)idx + 1], dcz = dL_dconic[4 * (size_t)idx + 3];
        cov2d_ctx c;
        cov2d_setup(mean, focal_x, focal_y, tanfovx, tanfovy, cov3D, view, &c);
        const float x_grad_mul = c.txtz < -c.limx || c.txtz > c.limx ? 0 : 1;
        const float y_grad_mul = c.tytz < -c.limy || c.tytz > c.limy ? 0 : 1;
        float a, b, cc;
        cov2d_eval(&c, &a, &b, &cc);
        a += low_pass;
        cc += low_pass;
        float denom = a * cc - b * b;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float* dcov = dL_dcov3D + 6 * (size_t)idx;
        const float (*Tm)[3] = c.A; /* glm T[i][j] == A[i][j] */
        if (denom2inv != 0) {
            dL_da = denom2inv * (-cc * cc * dcx + 2 * b * cc * dcy + (denom - a * cc) * dcz);
            dL_dc = denom2inv * (-a * a * dcz + 2 * a * b * dcy + (denom - a * cc) * dcx);
            dL_db = denom2inv * 2 * (b * cc * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
            dcov[0] = (Tm[0][0] * Tm[0][0] * dL_da + Tm[0][0] * Tm[1][0] * dL_db + Tm[1][0] * Tm[1][0] * dL_dc);
            dcov[3] = (Tm[0][1] * Tm[0][1] * dL_da + Tm[0][1] * Tm[1][1] * dL_db + Tm[1][1] * Tm[1][1] * dL_dc);
            dcov[5] = (Tm[0][2] * Tm[0][2] * dL_da + Tm[0][2] * Tm[1][2] * dL_db + Tm[1][2] * Tm[1][2] * dL_dc);
            dcov[1] = 2 * Tm[0][0] * Tm[0][1] * dL_da + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_db + 2 * Tm[1][0] * Tm[1][1] * dL_dc;
            dcov[2] = 2 * Tm[0][0] * Tm[0][2] * dL_da + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_db + 2 * Tm[1][0] * Tm[1][2] * dL_dc;
            dcov[4] = 2 * Tm[0][2] * Tm[0][1] * dL_da + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_db + 2 * Tm[1][1] * Tm[1][2] * dL_dc;
        } else {
            for (int i = 0; i < 6; i++) dcov[i] = 0;
        }
        const float (*Vr)[3] = c.V;
        float dL_dT00 = 2 * (Tm[0][0] * Vr[0][0] + Tm[0][1] * Vr[0][1] + Tm[0][2] * Vr[0][2]) * dL_da +
                        (Tm[1][0] * Vr[0][0] + Tm[1][1] * Vr[0][1] + Tm[1][2] * Vr[0][2]) * dL_db;
        float dL_dT01 = 2 * (Tm[0][0] * Vr[1][0] + Tm[0][1] * Vr[1][1] + Tm[0][2] * Vr[1][2]) * dL_da +
                        (Tm[1][0] * Vr[1][0] + Tm[1][1] * Vr[1][1] + Tm[1][2] * Vr[1][2]) * dL_db;
        float dL_dT02 = 2 * (Tm[0][0] * Vr[2][0] + Tm[0][1] * Vr[2][1] + Tm[0][2] * Vr[2][2]) * dL_da +
                        (Tm[1][0] * Vr[2][0] + Tm[1][1] * Vr[2][1] + Tm[1][2] * Vr[2][2]) * dL_db;
        float dL_dT10 = 2 * (Tm[1][0] * Vr[0][0] + Tm[1][1] * Vr[0][1] + Tm[1][2] * Vr[0][2]) * dL_dc +
                        (Tm[0][0] * Vr[0][0] + Tm[0][1] * Vr[0][1] + Tm[0][2] * Vr[0][2]) * dL_db;
        float dL_dT11 = 2 * (Tm[1][0] * Vr[1][0] + Tm[1][1] * Vr[1][1] + Tm[1][2] * Vr[1][2]) * dL_dc +
                        (Tm[0][0] * Vr[1][0] + Tm[0][1] * Vr[1][1] + Tm[0][2] * Vr[1][2]) * dL_db;
        float dL_dT12 = 2 * (Tm[1][0] * Vr[2][0] + Tm[1][1] * Vr[2][1] + Tm[1][2] * Vr[2][2]) * dL_dc +
                        (Tm[0][0] * Vr[2][0] + Tm[0][1] * Vr[2][1] + Tm[0][2] * Vr[2][2]) * dL_db;
        /* glm W[i][j] == R_w2c[i][j] == view[4j+i] */
#define WM(i, j) view[4 * (j) + (i)]
        float dL_dJ00 = WM(0, 0) * dL_dT00 + WM(0, 1) * dL_dT01 + WM(0, 2) * dL_dT02;
        float dL_dJ02 = WM(2, 0) * dL_dT00 + WM(2, 1) * dL_dT01 + WM(2, 2) * dL_dT02;
        float dL_dJ11 = WM(1, 0) * dL_dT10 + WM(1, 1) * dL_dT11 + WM(1, 2) * dL_dT12;
        float dL_dJ12 = WM(2, 0) * dL_dT10 + WM(2, 1) * dL_dT11 + WM(2, 2) * dL_dT12;
#undef WM
        f3 t = c.t;
        float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        float dL_dtx = x_grad_mul * -focal_x * tz2 * dL_dJ02;
        float dL_dty = y_grad_mul * -focal_y * tz2 * dL_dJ12;
        float dL_dtz = -focal_x * tz2 * dL_dJ00 - focal_y * tz2 * dL_dJ11 + (2 * focal_x * t.x) * tz3 * dL_dJ02 +
                       (2 * focal_y * t.y) * tz3 * dL_dJ12;
        f3 dm = xform_vec_4x3_T(mk3(dL_dtx, dL_dty, dL_dtz), view);
        dL_dmeans3D[3 * idx] = dm.x; dL_dmeans3D[3 * idx + 1] = dm.y; dL_dmeans3D[3 * idx + 2] = dm.z;
    }

    /* ---- preprocessCUDA backward (backward.cu:336-386) ---- */
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        f3 m = mk3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
        float m_hom[4];
        xform_point_4x4(m, proj, m_hom);
        float m_w = 1.0f / (m_hom[3] + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        float gx2 = dL_dmeans2D[3 * idx], gy2 = dL_dmeans2D[3 * idx + 1];
        f3 dmean;
        dmean.x = (proj[0] * m_w - proj[3] * mul1) * gx2 + (proj[1] * m_w - proj[3] * mul2) * gy2;
        dmean.y = (proj[4] * m_w - proj[7] * mul1) * gx2 + (proj[5] * m_w - proj[7] * mul2) * gy2;
        dmean.z = (proj[8] * m_w - proj[11] * mul1) * gx2 + (proj[9] * m_w - proj[11] * mul2) * gy2;
        dL_dmeans3D[3 * idx] += dmean.x; dL_dmeans3D[3 * idx + 1] += dmean.y; dL_dmeans3D[3 * idx + 2] += dmean.z;

        if (shs) { /* backward.cu:9-128 */
            f3 campos3 = mk3(campos[0], campos[1], campos[2]);
            f3 dir_orig = sub3(m, campos3);
            float len = sqrtf(dot3(dir_orig, dir_orig));
            f3 dir = mk3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
            const float* sh = shs + (size_t)idx * M * 3;
            float* dsh = dL_dsh + (size_t)idx * M * 3;
#define SH(k) mk3(sh[3 * (k) + 0], sh[3 * (k) + 1], sh[3 * (k) + 2])
#define DSH(k, v) do { f3 _v = (v); dsh[3 * (k)] = _v.x; dsh[3 * (k) + 1] = _v.y; dsh[3 * (k) + 2] = _v.z; } while (0)
            f3 dL_dRGB = mk3(dL_dcolors[3 * idx], dL_dcolors[3 * idx + 1], dL_dcolors[3 * idx + 2]);
            dL_dRGB.x *= s->clamped[3 * idx + 0] ? 0 : 1;
            dL_dRGB.y *= s->clamped[3 * idx + 1] ? 0 : 1;
            dL_dRGB.z *= s->clamped[3 * idx + 2] ? 0 : 1;
            f3 dRGBdx = mk3(0, 0, 0), dRGBdy = mk3(0, 0, 0), dRGBdz = mk3(0, 0, 0);
            float x = dir.x, y = dir.y, z = dir.z;
            DSH(0, scl3(SH_C0, dL_dRGB));
            if (D > 0) {
                DSH(1, scl3(-SH_C1 * y, dL_dRGB));
                DSH(2, scl3(SH_C1 * z, dL_dRGB));
                DSH(3, scl3(-SH_C1 * x, dL_dRGB));
                dRGBdx = scl3(-SH_C1, SH(3));
                dRGBdy = scl3(-SH_C1, SH(1));
                dRGBdz = scl3(SH_C1, SH(2));
                if (D > 1) {
                    float xx = x * x, yy = y * y, zz = z * z;
                    float xy = x * y, yz = y * z, xz = x * z;
                    DSH(4, scl3(SH_C2[0] * xy, dL_dRGB));
                    DSH(5, scl3(SH_C2[1] * yz, dL_dRGB));
                    DSH(6, scl3(SH_C2[2] * (2.f * zz - xx - yy), dL_dRGB));
                    DSH(7, scl3(SH_C2[3] * xz, dL_dRGB));
                    DSH(8, scl3(SH_C2[4] * (xx - yy), dL_dRGB));
                    dRGBdx = add3(dRGBdx, add3(add3(add3(scl3(SH_C2[0] * y, SH(4)), scl3(SH_C2[2] * 2.f * -x, SH(6))),
                                                    scl3(SH_C2[3] * z, SH(7))), scl3(SH_C2[4] * 2.f * x, SH(8))));
                    dRGBdy = add3(dRGBdy, add3(add3(add3(scl3(SH_C2[0] * x, SH(4)), scl3(SH_C2[1] * z, SH(5))),
                                                    scl3(SH_C2[2] * 2.f * -y, SH(6))), scl3(SH_C2[4] * 2.f * -y, SH(8))));
                    dRGBdz = add3(dRGBdz, add3(add3(scl3(SH_C2[1] * y, SH(5)), scl3(SH_C2[2] * 2.f * 2.f * z, SH(6))),
                                               scl3(SH_C2[3] * x, SH(7))));
                    if (D > 2) {
                        DSH(9, scl3(SH_C3[0] * y * (3.f * xx - yy), dL_dRGB));
                        DSH(10, scl3(SH_C3[1] * xy * z, dL_dRGB));
                        DSH(11, scl3(SH_C3[2] * y * (4.f * zz - xx - yy), dL_dRGB));
                        DSH(12, scl3(SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy), dL_dRGB));
                        DSH(13, scl3(SH_C3[4] * x * (4.f * zz - xx - yy), dL_dRGB));
                        DSH(14, scl3(SH_C3[5] * z * (xx - yy), dL_dRGB));
                        DSH(15, scl3(SH_C3[6] * x * (xx - 3.f * yy), dL_dRGB));
                        f3 tx = scl3(SH_C3[0] * 3.f * 2.f * xy, SH(9));
                        tx = add3(tx, scl3(SH_C3[1] * yz, SH(10)));
                        tx = add3(tx, scl3(SH_C3[2] * -2.f * xy, SH(11)));
                        tx = add3(tx, scl3(SH_C3[3] * -3.f * 2.f * xz, SH(12)));
                        tx = add3(tx, scl3(SH_C3[4] * (-3.f * xx + 4.f * zz - yy), SH(13)));
                        tx = add3(tx, scl3(SH_C3[5] * 2.f * xz, SH(14)));
                        tx = add3(tx, scl3(SH_C3[6] * 3.f * (xx - yy), SH(15)));
                        dRGBdx = add3(dRGBdx, tx);
                        f3 ty = scl3(SH_C3[0] * 3.f * (xx - yy), SH(9));
                        ty = add3(ty, scl3(SH_C3[1] * xz, SH(10)));
                        ty = add3(ty, scl3(SH_C3[2] * (-3.f * yy + 4.f * zz - xx), SH(11)));
                        ty = add3(ty, scl3(SH_C3[3] * -3.f * 2.f * yz, SH(12)));
                        ty = add3(ty, scl3(SH_C3[4] * -2.f * xy, SH(13)));
                        ty = add3(ty, scl3(SH_C3[5] * -2.f * yz, SH(14)));
                        ty = add3(ty, scl3(SH_C3[6] * -3.f * 2.f * xy, SH(15)));
                        dRGBdy = add3(dRGBdy, ty);
                        f3 tz_ = scl3(SH_C3[1] * xy, SH(10));
                        tz_ = add3(tz_, scl3(SH_C3[2] * 4.f * 2.f * yz, SH(11)));
                        tz_ = add3(tz_, scl3(SH_C3[3] * 3.f * (2.f * zz - xx - yy), SH(12)));
                        tz_ = add3(tz_, scl3(SH_C3[4] * 4.f * 2.f * xz, SH(13)));
                        tz_ = add3(tz_, scl3(SH_C3[5] * (xx - yy), SH(14)));
                        dRGBdz = add3(dRGBdz, tz_);
                    }
                }
            }
#undef SH
#undef DSH
            f3 dL_ddir = mk3(dot3(dRGBdx, dL_dRGB), dot3(dRGBdy, dL_dRGB), dot3(dRGBdz, dL_dRGB));
            f3 dmd = dnormvdv(dir_orig, dL_ddir);
            dL_dmeans3D[3 * idx] += dmd.x; dL_dmeans3D[3 * idx + 1] += dmd.y; dL_dmeans3D[3 * idx + 2] += dmd.z;
        }

        if (scales) { /* backward.cu:268-331 */
            const float* q = rotations + 4 * (size_t)idx;
            float r = q[0], x = q[1], y = q[2], z = q[3];
            float Rs[3][3];
            quat_to_rot(q, Rs);
            float sv[3] = {scale_modifier * scales[3 * idx], scale_modifier * scales[3 * idx + 1],
                           scale_modifier * scales[3 * idx + 2]};
            float Mm[3][3];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) Mm[i][j] = sv[i] * Rs[j][i];
            const float* dc = dL_dcov3D + 6 * (size_t)idx;
            float dS[3][3] = {{dc[0], 0.5f * dc[1], 0.5f * dc[2]},
                              {0.5f * dc[1], dc[3], 0.5f * dc[4]},
                              {0.5f * dc[2], 0.5f * dc[4], dc[5]}};
            float dM[3][3]; /* math 2·M·dSigma */
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++)
                    dM[i][j] = 2.0f * Mm[i][0] * dS[0][j] + 2.0f * Mm[i][1] * dS[1][j] + 2.0f * Mm[i][2] * dS[2][j];
            for (int i = 0; i < 3; i++)
                dL_dscales[3 * idx + i] = Rs[0][i] * dM[i][0] + Rs[1][i] * dM[i][1] + Rs[2][i] * dM[i][2];
            float G[3][3]; /* glm dL_dMt[a][b] after the per-column s scaling */
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) G[i][j] = dM[i][j] * sv[i];
            float* dq = dL_drot + 4 * (size_t)idx;
            dq[0] = 2 * z * (G[0][1] - G[1][0]) + 2 * y * (G[2][0] - G[0][2]) + 2 * x * (G[1][2] - G[2][1]);
            dq[1] = 2 * y * (G[1][0] + G[0][1]) + 2 * z * (G[2][0] + G[0][2]) + 2 * r * (G[1][2] - G[2][1]) - 4 * x * (G[2][2] + G[1][1]);
            dq[2] = 2 * x * (G[1][0] + G[0][1]) + 2 * r * (G[2][0] - G[0][2]) + 2 * z * (G[1][2] + G[2][1]) - 4 * y * (G[2][2] + G[0][0]);
            dq[3] = 2 * r * (G[0][1] - G[1][0]) + 2 * x * (G[2][0] + G[0][2]) + 2 * y * (G[1][2] + G[2][1]) - 4 * z * (G[1][1] + G[0][0]);
        }
    }
    return 0;
}

/* Ordered Gaussian ids actually blended into pixel (px, py) by the forward (the discrete
 * decisions of forward.cu:318-356 replayed on the stored state).  Returns the count. */
int orc_pixel_blend_list(const orc_state* s, int px, int py, uint32_t* out_ids, int cap) {
    int tile = (py / BLOCK_Y) * s->gx + (px / BLOCK_X);
    uint32_t rs = s->ranges[2 * tile], re = s->ranges[2 * tile + 1];
    float pfx = (float)px, pfy = (float)py, Tr = 1.0f;
    int n = 0;
    for (uint32_t k = rs; k < re; k++) {
        uint32_t g = s->point_list[k];
        float dx = s->xy[2 * g] - pfx, dy = s->xy[2 * g + 1] - pfy;
        const float* co = s->conic_opacity + 4 * (size_t)g;
        float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        if (power > 0.0f) continue;
        float alpha = minf(0.99f, co[3] * expf(power));
        if (alpha < 1.0f / 255.0f) continue;
        float test_T = Tr * (1 - alpha);
        if (test_T < 0.0001f) break;
        if (n < cap) out_ids[n] = g;
        n++;
        Tr = test_T;
    }
    return n;
}

/* ---- state accessors for tests ---- */
int orc_num_rendered(const orc_state* s) { return s->num_rendered; }
const uint32_t* orc_point_list(const orc_state* s) { return s->point_list; }
const uint32_t* orc_ranges(const orc_state* s) { return s->ranges; }
const float* orc_final_T(const orc_state* s) { return s->final_T; }
const uint32_t* orc_n_contrib(const orc_state* s) { return s->n_contrib; }
const float* orc_xy(const orc_state* s) { return s->xy; }
const float* orc_depths(const orc_state* s) { return s->depths; }
const float* orc_conic_opacity(const orc_state* s) { return s->conic_opacity; }
const float* orc_rgb(const orc_state* s) { return s->rgb; }
const float* orc_cov3D(const orc_state* s) { return s->cov3D; }
const unsigned char* orc_clamped(const orc_state* s) { return s->clamped; }
const uint32_t* orc_tiles_touched(const orc_state* s) { return s->tiles_touched; }
int orc_threads(void) { return set_threads(0); }
