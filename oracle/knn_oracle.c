/*
 * knn_oracle.c — CPU restatement of simple-knn's distCUDA2 (TEST INFRASTRUCTURE ONLY: used by
 * tests/ as the checker of rain_amd/csrc/knn.hip; never linked into the product).
 *
 * Follows /root/reference/submodules/simple-knn:
 *   spatial.cu:4-13        distCUDA2: means = full({P}, 0) then SimpleKNN::knn
 *   simple_knn.cu:164-207  SimpleKNN::knn
 *     :172-181  bbox = CUB Reduce(min / max) with init {0,0,0}  -> the origin is always inside
 *     :183-198  30-bit Morton codes over that bbox, stable radix sort of (code, index)
 *     :200-203  boxes of BOX_SIZE=1024 consecutive sorted points, per-box AABB (boxMinMax :64-100)
 *     :125-157  boxMeanDist: reject = 3rd best over sorted neighbours idx-3..idx+3, then every box
 *               whose point distance (distBoxPoint :102-112) is <= reject and <= best[2] is scanned
 *               exhaustively; result (best0 + best1 + best2) / 3
 *     :114-124  updateKBest<3>: insertion with strict '>' (values end up ascending)
 * Squared distances are dx*dx + dy*dy + dz*dz without FMA contraction (-ffp-contract=off); the
 * HIP kernel evaluates the same expression with contraction disabled, so results are bitwise equal.
 * Fewer than 4 points leave FLT_MAX entries (mean FLT_MAX/3 for P = 3, +inf for P < 3), exactly as
 * in the reference.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KNN_BOX 1024

static uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

/* float -> uint32 as CUDA's cvt.rzi.u32.f32 does it: truncation, NaN and negatives -> 0, saturating */
static uint32_t f2u(float v) {
    if (!(v > 0.0f)) return 0u;
    if (v >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)v;
}

static uint32_t morton(const float* p, const float* mn, const float* mx) {
    uint32_t c[3];
    for (int a = 0; a < 3; a++) c[a] = prep_morton(f2u(((p[a] - mn[a]) / (mx[a] - mn[a])) * (float)((1 << 10) - 1)));
    return c[0] | (c[1] << 1) | (c[2] << 2);
}

static float sqdist(const float* a, const float* b) {
    const float dx = b[0] - a[0], dy = b[1] - a[1], dz = b[2] - a[2];
    return dx * dx + dy * dy + dz * dz;
}

static void update3(const float* ref, const float* pt, float* best) {
    float d = sqdist(ref, pt);
    for (int j = 0; j < 3; j++)
        if (best[j] > d) {
            const float t = best[j];
            best[j] = d;
            d = t;
        }
}

static float box_dist(const float* mn, const float* mx, const float* p) {
    float diff[3] = {0.f, 0.f, 0.f};
    for (int a = 0; a < 3; a++)
        if (p[a] < mn[a] || p[a] > mx[a]) diff[a] = fminf(fabsf(p[a] - mn[a]), fabsf(p[a] - mx[a]));
    return diff[0] * diff[0] + diff[1] * diff[1] + diff[2] * diff[2];
}

/* stable LSD radix sort of (key, value) pairs, 8-bit digits */
static void radix_sort_u32(uint32_t* keys, uint32_t* vals, int n) {
    uint32_t* k2 = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    uint32_t* v2 = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    for (int shift = 0; shift < 32; shift += 8) {
        size_t cnt[257] = {0};
        for (int i = 0; i < n; i++) cnt[((keys[i] >> shift) & 0xffu) + 1]++;
        for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
        for (int i = 0; i < n; i++) {
            const size_t o = cnt[(keys[i] >> shift) & 0xffu]++;
            k2[o] = keys[i];
            v2[o] = vals[i];
        }
        memcpy(keys, k2, sizeof(uint32_t) * (size_t)n);
        memcpy(vals, v2, sizeof(uint32_t) * (size_t)n);
    }
    free(k2);
    free(v2);
}

/* points [P,3] -> mean_dists [P]; also exposes the sorted order and bbox for tests. */
void orc_dist_knn3(int P, const float* points, float* mean_dists, uint32_t* out_sorted_idx, float* out_bbox6) {
    if (P <= 0) return;
    float mn[3] = {0.f, 0.f, 0.f}, mx[3] = {0.f, 0.f, 0.f}; /* CUB Reduce init {0,0,0} */
    for (int i = 0; i < P; i++)
        for (int a = 0; a < 3; a++) {
            mn[a] = fminf(mn[a], points[3 * i + a]);
            mx[a] = fmaxf(mx[a], points[3 * i + a]);
        }
    uint32_t* codes = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)P);
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)P);
    for (int i = 0; i < P; i++) {
        codes[i] = morton(points + 3 * i, mn, mx);
        idx[i] = (uint32_t)i;
    }
    radix_sort_u32(codes, idx, P);
    const int nb = (P + KNN_BOX - 1) / KNN_BOX;
    float* boxes = (float*)malloc(sizeof(float) * 6 * (size_t)nb);
    for (int b = 0; b < nb; b++) {
        float* B = boxes + 6 * b;
        for (int a = 0; a < 3; a++) {
            B[a] = FLT_MAX;
            B[3 + a] = -FLT_MAX;
        }
        const int e = (b + 1) * KNN_BOX < P ? (b + 1) * KNN_BOX : P;
        for (int s = b * KNN_BOX; s < e; s++)
            for (int a = 0; a < 3; a++) {
                const float v = points[3 * idx[s] + a];
                B[a] = fminf(B[a], v);
                B[3 + a] = fmaxf(B[3 + a], v);
            }
    }
#pragma omp parallel for schedule(dynamic, 256)
    for (int s = 0; s < P; s++) {
        const float* pt = points + 3 * idx[s];
        float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        const int lo = s - 3 > 0 ? s - 3 : 0, hi = s + 3 < P - 1 ? s + 3 : P - 1;
        for (int i = lo; i <= hi; i++)
            if (i != s) update3(pt, points + 3 * idx[i], best);
        const float reject = best[2];
        best[0] = best[1] = best[2] = FLT_MAX;
        for (int b = 0; b < nb; b++) {
            const float d = box_dist(boxes + 6 * b, boxes + 6 * b + 3, pt);
            if (d > reject || d > best[2]) continue;
            const int e = (b + 1) * KNN_BOX < P ? (b + 1) * KNN_BOX : P;
            for (int i = b * KNN_BOX; i < e; i++)
                if (i != s) update3(pt, points + 3 * idx[i], best);
        }
        mean_dists[idx[s]] = (best[0] + best[1] + best[2]) / 3.0f;
    }
    if (out_sorted_idx) memcpy(out_sorted_idx, idx, sizeof(uint32_t) * (size_t)P);
    if (out_bbox6) {
        for (int a = 0; a < 3; a++) {
            out_bbox6[a] = mn[a];
            out_bbox6[3 + a] = mx[a];
        }
    }
    free(codes);
    free(idx);
    free(boxes);
}
