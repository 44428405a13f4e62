/* gs_neighbor.h -- C ABI of the local-rigidity / rotation / isometry
 * neighbour losses, exported by the same
 * libgsplat_hip.so as gsplat_hip.h.
 *
 * Replaces the PyTorch loss block of the reference's per-step loss
 * (train.py:253-273, identical in cvpr_dyn.py:302-322):
 *
 *   rel_rot = quat_mult(fg_rot, prev_inv_rot_fg)                 helpers.py:124-132
 *   rot     = build_rotation(rel_rot)                            external.py:61-78
 *   off     = fg_pts[nbr] - fg_pts[:, None]
 *   rigid   = weighted_l2_loss_v2(rot^T off, prev_offset, w)     helpers.py:121-122
 *   rot     = weighted_l2_loss_v2(rel_rot[nbr], rel_rot[:, None], w)
 *   iso     = weighted_l2_loss_v1(|off|, nbr_dist, w)            helpers.py:117-118
 *
 * with nbr = neighbor_indices [N, K] (int64, as the reference stores them,
 * train.py:324), w = neighbor_weight [N, K], nbr_dist [N, K],
 * prev_offset [N, K, 3], prev_inv_rot_fg [N, 4], fg_pts [N, 3], fg_rot [N, 4]
 * (all fp32, contiguous, device memory).  The backward needs the reverse
 * adjacency (which (i, k) pairs name each Gaussian as a neighbour) as a CSR
 * ordered by pair index within each row (deterministic sums): rev_ptr [N + 1]
 * and rev_pos [N * K] = the slot of pair i * K + k in that order (the
 * backward writes each pair's neighbour share straight into its slot, so the
 * per-Gaussian sums read contiguous rows).  The neighbour graph is fixed
 * after the first timestep (train.py:316-326), so this is built once
 * (gs_neighbor_reverse).
 *
 * Workspaces are caller-allocated device memory of the size the _bytes()
 * queries return.  All calls are asynchronous on `stream`; return 0 or an
 * error code with gs_last_error() set (as gsplat_hip.h). */
#ifndef GS_NEIGHBOR_H
#define GS_NEIGHBOR_H

#include <stdint.h>

#include "gsplat_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gs_neighbor_graph {
  int64_t N;                    /* foreground Gaussians */
  int32_t K;                    /* neighbours per Gaussian (train.py:316 num_knn=20) */
  int32_t _pad;
  const int64_t *nbr;           /* [N, K] neighbor_indices */
  const float *weight;          /* [N, K] neighbor_weight = exp(-2000 d^2) */
  const float *dist;            /* [N, K] neighbor_dist = sqrt(d^2) */
  const float *prev_offset;     /* [N, K, 3] */
  const float *prev_inv_rot;    /* [N, 4]  conjugate of the previous rotation */
  const int32_t *rev_ptr;       /* [N + 1] reverse CSR row starts (backward only) */
  const int32_t *rev_pos;       /* [N * K] slot of each pair in the reverse order */
} gs_neighbor_graph;

/* Workspace bytes for forward / backward at this N, K. */
size_t gs_neighbor_workspace_bytes(int64_t N, int32_t K, int backward);

/* losses[3] (device) = (rigid, rot, iso), each the mean over N*K pairs
 * (the reference's .mean(); N*K == 0 gives NaN like torch's empty mean).
 * Deterministic: fixed-order block sums. */
int gs_neighbor_loss_forward(const gs_neighbor_graph *g, const float *fg_pts, const float *fg_rot,
                             float *losses, void *workspace, gs_stream_t stream);

/* d_fg_pts [N, 3], d_fg_rot [N, 4] (written, not accumulated) for upstream
 * gradients dL_dlosses[3] (device; the autograd grad_outputs of the three
 * losses).  Deterministic (no atomics). */
int gs_neighbor_loss_backward(const gs_neighbor_graph *g, const float *fg_pts, const float *fg_rot,
                              const float *dL_dlosses, float *d_fg_pts, float *d_fg_rot,
                              void *workspace, gs_stream_t stream);

/* Reverse CSR of the neighbour graph (setup, once per sequence): rev_ptr
 * [N + 1]; rev_pair [N * K] (optional, may be NULL) = the pair indices of
 * each row in ascending order; rev_pos [N * K] = its inverse permutation.
 * Workspace of gs_neighbor_reverse_workspace_bytes(N, K).  Out-of-range
 * indices are an error (status read back; synchronises the stream once). */
size_t gs_neighbor_reverse_workspace_bytes(int64_t N, int32_t K);
int gs_neighbor_reverse(int64_t N, int32_t K, const int64_t *nbr, int32_t *rev_ptr, int32_t *rev_pair,
                        int32_t *rev_pos, void *workspace, gs_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GS_NEIGHBOR_H */
