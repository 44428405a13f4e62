/* gs_optim.h -- C ABI of the fused Adam + densification-statistics step
 * (SURVEY.md 8(f) rank 3), exported by libgsplat_hip.so next to
 * gsplat_hip.h.
 *
 * Replaces, per training iteration of the reference (train.py:422-433):
 *   variables['max_2D_radius'][seen] = max(radius[seen], ...)        train.py:288-290
 *   accumulate_mean2d_gradient(variables)                           external.py:136-140
 *     means2D_gradient_accum[seen] += |means2D.grad[seen, :2]|;  denom[seen] += 1
 *   optimizer.step()   torch.optim.Adam(param_groups, lr=0, eps=1e-15)  train.py:119-135
 * with ONE launch over every parameter tensor and the statistics.
 *
 * Adam follows torch.optim.Adam (amsgrad=False, weight_decay=0,
 * maximize=False): per element
 *   m = m + (1 - b1) (g - m);  v = b2 v + (1 - b2) g^2
 *   p = p + step_size * m / (sqrt(v) / bc2_sqrt + eps)
 * with step_size = -lr / (1 - b1^t) and bc2_sqrt = sqrt(1 - b2^t) computed by
 * the caller in double (as torch does on the host).  Tensors whose grad is
 * absent are simply not listed.  Deterministic, elementwise, HBM-bound. */
#ifndef GS_OPTIM_H
#define GS_OPTIM_H

#include <stdint.h>

#include "gsplat_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ADAM_MAX_TENSORS 16

typedef struct gs_adam_tensor {
  float *param;
  const float *grad;
  float *exp_avg;
  float *exp_avg_sq;
  int64_t numel;
  float step_size;   /* -lr / (1 - beta1^t) */
  float bc2_sqrt;    /* sqrt(1 - beta2^t) */
} gs_adam_tensor;

typedef struct gs_adam_args {
  int32_t n_tensors;            /* <= GS_ADAM_MAX_TENSORS */
  int32_t _pad;
  double beta1, beta2, eps;     /* rounded to fp32 as torch's scalar ops do */
  gs_adam_tensor t[GS_ADAM_MAX_TENSORS];
} gs_adam_args;

/* Densification statistics of one rendered view (all device, length P):
 * seen = radii > 0; max_radius[seen] = max(radii, max_radius);
 * grad_accum[seen] += sqrt(gx^2 + gy^2) of means2D_grad[:, :2]
 * (row stride 3 floats, the reference's means2D [P, 3]); denom[seen] += 1.
 * Any of max_radius / (grad_accum, denom, means2D_grad) may be NULL to skip
 * that half. */
typedef struct gs_densify_stats {
  int64_t P;
  const int32_t *radii;
  const float *means2D_grad;
  float *max_radius;
  float *grad_accum;
  float *denom;
} gs_densify_stats;

/* One launch: the statistics (if stats != NULL and stats->P > 0) and the
 * Adam update of every listed tensor. */
int gs_adam_step(const gs_adam_args *args, const gs_densify_stats *stats, gs_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GS_OPTIM_H */
