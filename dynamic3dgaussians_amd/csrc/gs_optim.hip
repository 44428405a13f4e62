// gs_optim.hip -- fused Adam + densification statistics (SURVEY.md 8(f)
// rank 3; include/gs_optim.h).  One launch per training iteration replaces
// torch.optim.Adam's multi-tensor kernels over the reference's parameter
// groups (train.py:119-135, 432) and the statistics updates of
// train.py:288-290 / external.py:136-140.
//
// Block mapping: blocks [0, stats_blocks) update the per-Gaussian
// statistics; the rest walk a flattened chunk space over the tensor table
// (kernel argument, <= 16 entries), CHUNK elements per block, float4 where
// the tensor allows.  Every element is touched once: p, m, v read + written,
// g read -> 28 B per element, the HBM roof.
#include <hip/hip_runtime.h>

#include "../../include/gs_optim.h"
#include "gs_kernels.h"

namespace gs {

namespace {

constexpr int OPT_THREADS = 256;
constexpr int OPT_CHUNK = OPT_THREADS * 4 * 4;  // 4 float4 per thread

struct AdamTable {
  gs_adam_args a;
  float w1, b2, om_b2, eps;  // (float)(1 - beta1), (float)beta2, (float)(1 - beta2), (float)eps
  int64_t chunk_start[GS_ADAM_MAX_TENSORS + 1];  // prefix of per-tensor chunk counts
  int stats_blocks;
  gs_densify_stats st;
};

// torch's lerp (exp_avg.lerp_(grad, 1 - beta1), weight < 0.5), mul,
// addcmul, sqrt, div, add and addcdiv of _multi_tensor_adam, in the same
// order and with the multiply-adds torch's ROCm build contracts written as
// explicit fmas (this file is built with -ffp-contract=off, so nothing else
// is fused).
__device__ inline void adam1(float& p, float g, float& m, float& v, float w1, float b2, float om_b2, float eps,
                             float step_size, float bc2s) {
  m = fmaf(w1, g - m, m);
  v = fmaf(om_b2, g * g, v * b2);
  const float denom = sqrtf(v) / bc2s + eps;
  p = fmaf(step_size, m / denom, p);
}

__global__ void __launch_bounds__(OPT_THREADS) adam_stats_kernel(const AdamTable T) {
  if ((int)blockIdx.x < T.stats_blocks) {
    const gs_densify_stats& s = T.st;
    const int64_t i = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x;
    if (i >= s.P) return;
    const int32_t r = s.radii[i];
    if (r <= 0) return;  // seen = radius > 0
    if (s.max_radius) s.max_radius[i] = fmaxf((float)r, s.max_radius[i]);
    if (s.grad_accum) {
      const float gx = s.means2D_grad[3 * i], gy = s.means2D_grad[3 * i + 1];
      s.grad_accum[i] += sqrtf(gx * gx + gy * gy);
      s.denom[i] += 1.0f;
    }
    return;
  }
  const int64_t c = (int64_t)blockIdx.x - T.stats_blocks;
  int t = 0;
  while (t + 1 < T.a.n_tensors && c >= T.chunk_start[t + 1]) ++t;
  const gs_adam_tensor& A = T.a.t[t];
  const int64_t base = (c - T.chunk_start[t]) * OPT_CHUNK;
  const int64_t end = base + OPT_CHUNK < A.numel ? base + OPT_CHUNK : A.numel;
  const float w1 = T.w1, b2 = T.b2, om_b2 = T.om_b2, eps = T.eps;
  const bool vec = ((reinterpret_cast<uintptr_t>(A.param) | reinterpret_cast<uintptr_t>(A.grad) |
                     reinterpret_cast<uintptr_t>(A.exp_avg) | reinterpret_cast<uintptr_t>(A.exp_avg_sq)) &
                    15) == 0;
  if (vec && end - base == OPT_CHUNK) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = base + 4 * ((int64_t)u * OPT_THREADS + threadIdx.x);
      float4 p = *reinterpret_cast<const float4*>(A.param + e);
      const float4 g = *reinterpret_cast<const float4*>(A.grad + e);
      float4 m = *reinterpret_cast<const float4*>(A.exp_avg + e);
      float4 v = *reinterpret_cast<const float4*>(A.exp_avg_sq + e);
      adam1(p.x, g.x, m.x, v.x, w1, b2, om_b2, eps, A.step_size, A.bc2_sqrt);
      adam1(p.y, g.y, m.y, v.y, w1, b2, om_b2, eps, A.step_size, A.bc2_sqrt);
      adam1(p.z, g.z, m.z, v.z, w1, b2, om_b2, eps, A.step_size, A.bc2_sqrt);
      adam1(p.w, g.w, m.w, v.w, w1, b2, om_b2, eps, A.step_size, A.bc2_sqrt);
      *reinterpret_cast<float4*>(A.param + e) = p;
      *reinterpret_cast<float4*>(A.exp_avg + e) = m;
      *reinterpret_cast<float4*>(A.exp_avg_sq + e) = v;
    }
  } else {
    for (int64_t e = base + threadIdx.x; e < end; e += OPT_THREADS) {
      float p = A.param[e], m = A.exp_avg[e], v = A.exp_avg_sq[e];
      adam1(p, A.grad[e], m, v, w1, b2, om_b2, eps, A.step_size, A.bc2_sqrt);
      A.param[e] = p;
      A.exp_avg[e] = m;
      A.exp_avg_sq[e] = v;
    }
  }
}

}  // namespace

bool launch_adam_step(const gs_adam_args& a, const gs_densify_stats* st, hipStream_t s) {
  AdamTable T{};
  T.a = a;
  // torch passes these as double scalars to fp32 kernels: round once, here
  T.w1 = (float)(1.0 - a.beta1);
  T.b2 = (float)a.beta2;
  T.om_b2 = (float)(1.0 - a.beta2);
  T.eps = (float)a.eps;
  int64_t c = 0;
  for (int t = 0; t < a.n_tensors; ++t) {
    T.chunk_start[t] = c;
    c += (a.t[t].numel + OPT_CHUNK - 1) / OPT_CHUNK;
  }
  T.chunk_start[a.n_tensors] = c;
  if (st && st->P > 0) {
    T.st = *st;
    T.stats_blocks = (int)((st->P + OPT_THREADS - 1) / OPT_THREADS);
  }
  const int64_t blocks = c + T.stats_blocks;
  if (blocks == 0) return true;
  if (blocks > 0x7FFFFFFF) return false;
  hipLaunchKernelGGL(adam_stats_kernel, dim3((unsigned)blocks), dim3(OPT_THREADS), 0, s, T);
  return true;
}

}  // namespace gs
