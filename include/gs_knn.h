/* gs_knn.h -- C ABI of the exact k-nearest-neighbour search (SURVEY.md 8(f)
 * rank 4), exported by libgsplat_hip.so next to gsplat_hip.h.
 *
 * Replaces the reference's neighbour searches:
 *   o3d_knn(pts, num_knn)    helpers.py:135-146 (Open3D KDTreeFlann,
 *                            search_knn_vector_3d(p, k + 1), self dropped),
 *                            used for the initial scales (train.py:95, k = 3)
 *                            and the neighbour graph (train.py:316-326, k = 20);
 *   distCUDA2(points)        submodules_fsgs/simple-knn/spatial.cu:14-27
 *                            (mean squared distance of the 3 nearest + their
 *                            indices; scene/gaussian_model.py:162).
 *
 * For every point i of points [N, 3] (fp32, device): the K nearest other
 * points by squared Euclidean distance, computed in double from the fp32
 * coordinates (as Open3D does on the float64 copy the reference makes),
 * ascending by (distance, index) -- ties resolve to the lower index.
 * sq_dist [N, K] double, index [N, K] int64 (device).  When fewer than K
 * other points exist the tail is (+inf, -1).  1 <= K <= 32. */
#ifndef GS_KNN_H
#define GS_KNN_H

#include <stdint.h>

#include "gsplat_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GS_KNN_MAX_K 32

size_t gs_knn_workspace_bytes(int64_t N);
int gs_knn(int64_t N, int32_t K, const float *points, double *sq_dist, int64_t *index, void *workspace,
           gs_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GS_KNN_H */
