/*
 * rain_knn.h — C ABI of the MI355X simple-knn replacement.
 *
 * sk_dist_cuda2 replaces distCUDA2 (sharonal10/rain submodules/simple-knn/spatial.cu:4-13,
 * simple_knn.cu:164-207), which scene/gaussian_model.py:124 calls once per scene to initialise
 * scales: for every point, the mean of the squared distances to its 3 nearest other points.
 * The result is the exact 3-NN mean (as the reference's box-pruned search is), and keeps the
 * reference's edge behaviour: the Morton bbox always includes the origin (CUB Reduce with init
 * {0,0,0}, simple_knn.cu:172-181) and with fewer than 4 points the missing neighbours count as
 * FLT_MAX (mean FLT_MAX/3 for P = 3, +inf for P < 3).  No host synchronisation.
 */
#ifndef RAIN_KNN_H
#define RAIN_KNN_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* device workspace bytes sk_dist_cuda2 needs for P points */
size_t sk_workspace_bytes(int P);

/* points: [P,3] fp32 device array; mean_dists: [P] fp32 device output (fully written). */
int sk_dist_cuda2(int P, const float* points, float* mean_dists, void* workspace, size_t workspace_bytes,
                  void* stream);

const char* sk_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RAIN_KNN_H */
