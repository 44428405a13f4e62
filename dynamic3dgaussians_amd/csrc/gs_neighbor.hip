// gs_neighbor.hip -- local-rigidity / rotation / isometry neighbour losses
// (reference: train.py:253-273, helpers.py:117-133,
// external.py:61-78), forward and hand-derived backward.
//
// The reference evaluates these as ~30 PyTorch ops over [N, K, *] tensors
// (gathers, a batched 3x3 matmul, sqrt/mean) and as many again in autograd,
// with the neighbour gathers turned into scatter-adds.  Here:
//   prep     one thread per Gaussian: rel_rot = fg_rot (x) prev_inv_rot
//            (16 B, gathered by the neighbours) and the rotation matrix of
//            rel_rot / |rel_rot| (48 B, read by the Gaussian's own pairs);
//   forward  one lane per (Gaussian, neighbour) pair for K <= 64 (a wave
//            holds 64 / K whole Gaussians, so every [N, K] array is read
//            coalesced; one thread per Gaussian walking its K pairs above
//            that); grid-stride, block partial sums reduced in a fixed order
//            (deterministic losses);
//   backward the same mapping computes the per-pair gradients, writes the
//            neighbour's share (32 B) straight into its slot of the reverse
//            CSR order (rev_pos), and sums the Gaussian's own share over its
//            lanes through LDS; a gather then reads each Gaussian's reverse
//            row contiguously -- no atomics, deterministic.
// All HBM-bound (tens of bytes per pair), no matrix work.
#include <hip/hip_runtime.h>

#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

namespace {

constexpr int NB_THREADS = 256;
constexpr int NB_WAVES = NB_THREADS / 64;
constexpr int NB_MAX_BLOCKS = 1024;  // grid-stride cap of the forward walks

// quat_mult (helpers.py:124-132): (w, x, y, z) Hamilton product
__device__ inline float4 quat_mult(float4 a, float4 b) {
  return make_float4(a.x * b.x - a.y * b.y - a.z * b.z - a.w * b.w,
                     a.x * b.y + a.y * b.x + a.z * b.w - a.w * b.z,
                     a.x * b.z - a.y * b.w + a.z * b.x + a.w * b.y,
                     a.x * b.w + a.y * b.z - a.z * b.y + a.w * b.x);
}

// dL/da of quat_mult(a, b) for fixed b, given g = dL/d(a (x) b)
__device__ inline float4 quat_mult_bwd_a(float4 g, float4 b) {
  return make_float4(g.x * b.x + g.y * b.y + g.z * b.z + g.w * b.w,
                     -g.x * b.y + g.y * b.x - g.z * b.w + g.w * b.z,
                     -g.x * b.z + g.y * b.w + g.z * b.x - g.w * b.y,
                     -g.x * b.w - g.y * b.z + g.z * b.y + g.w * b.x);
}

__device__ inline float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ inline float3 ld3(const float* p) { return make_float3(p[0], p[1], p[2]); }

// Rotation record per Gaussian: R (row-major, 9) of rel_rot / |rel_rot|,
// 1/|rel_rot|, 2 pad.
constexpr int RM = 12;

__global__ void __launch_bounds__(NB_THREADS) nb_prep_kernel(int64_t N, const float* __restrict__ fg_rot,
                                                             const float* __restrict__ pinv,
                                                             float4* __restrict__ qv, float* __restrict__ Rm) {
  const int64_t i = (int64_t)blockIdx.x * NB_THREADS + threadIdx.x;
  if (i >= N) return;
  const float4 q = quat_mult(ld4(fg_rot + 4 * i), ld4(pinv + 4 * i));
  // build_rotation (external.py:61-78): normalise, then the usual matrix
  const float nrm = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  const float r = q.x / nrm, x = q.y / nrm, y = q.z / nrm, z = q.w / nrm;
  qv[i] = q;
  float4* o = reinterpret_cast<float4*>(Rm + RM * i);
  o[0] = make_float4(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                     2.f * (x * y + r * z));
  o[1] = make_float4(1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x), 2.f * (x * z - r * y),
                     2.f * (y * z + r * x));
  o[2] = make_float4(1.f - 2.f * (x * x + y * y), 1.f / nrm, 0.f, 0.f);
}

struct Rec {
  float4 q;
  float R[9];
  float invn;
};
__device__ inline Rec load_rec(const float4* qv, const float* Rm, int64_t i) {
  const float4* p = reinterpret_cast<const float4*>(Rm + RM * i);
  const float4 b = p[0], c = p[1], d = p[2];
  Rec r;
  r.q = qv[i];
  r.R[0] = b.x; r.R[1] = b.y; r.R[2] = b.z; r.R[3] = b.w;
  r.R[4] = c.x; r.R[5] = c.y; r.R[6] = c.z; r.R[7] = c.w;
  r.R[8] = d.x;
  r.invn = d.y;
  return r;
}

// Per pair (i, k): the three loss terms.
struct PairTerms {
  float3 o;       // neighbour offset fg_pts[n] - fg_pts[i]
  float3 dc;      // rotated offset minus prev_offset
  float4 dq;      // rel_rot[n] - rel_rot[i]
  float mag, e;   // |o| (with the reference's 1e-20), |o| - dist
  float rigid, rot, iso;
};
__device__ inline PairTerms pair_terms(const Rec& ri, float3 pi, float3 pn, float4 qn, float w, float dist,
                                       float3 po) {
  PairTerms t;
  t.o = make_float3(pn.x - pi.x, pn.y - pi.y, pn.z - pi.z);
  // rot^T @ off (train.py:263): c_b = sum_a R[a][b] o_a
  const float c0 = ri.R[0] * t.o.x + ri.R[3] * t.o.y + ri.R[6] * t.o.z;
  const float c1 = ri.R[1] * t.o.x + ri.R[4] * t.o.y + ri.R[7] * t.o.z;
  const float c2 = ri.R[2] * t.o.x + ri.R[5] * t.o.y + ri.R[8] * t.o.z;
  t.dc = make_float3(c0 - po.x, c1 - po.y, c2 - po.z);
  t.rigid = sqrtf((t.dc.x * t.dc.x + t.dc.y * t.dc.y + t.dc.z * t.dc.z) * w + 1e-20f);
  t.dq = make_float4(qn.x - ri.q.x, qn.y - ri.q.y, qn.z - ri.q.z, qn.w - ri.q.w);
  t.rot = sqrtf((t.dq.x * t.dq.x + t.dq.y * t.dq.y + t.dq.z * t.dq.z + t.dq.w * t.dq.w) * w + 1e-20f);
  t.mag = sqrtf(t.o.x * t.o.x + t.o.y * t.o.y + t.o.z * t.o.z + 1e-20f);
  t.e = t.mag - dist;
  t.iso = sqrtf(t.e * t.e * w + 1e-20f);
  return t;
}

// Per-pair gradients: go = dL/d offset (the neighbour gets +go, the Gaussian
// -go), gq = dL/d(rel_rot[n] - rel_rot[i]), gc = dL/d(rot^T off) (for dL/dR).
struct PairGrads {
  float3 go, gc;
  float4 gq;
};
__device__ inline PairGrads pair_grads(const PairTerms& t, const Rec& ri, float w, float g_rigid, float g_rot,
                                       float g_iso) {
  PairGrads d;
  // rigid: d sqrt(|dc|^2 w + eps) / d dc = w dc / rigid
  const float sr = g_rigid * w / t.rigid;
  d.gc = make_float3(sr * t.dc.x, sr * t.dc.y, sr * t.dc.z);
  // c = R^T o: dL/do = R gc
  d.go = make_float3(ri.R[0] * d.gc.x + ri.R[1] * d.gc.y + ri.R[2] * d.gc.z,
                     ri.R[3] * d.gc.x + ri.R[4] * d.gc.y + ri.R[5] * d.gc.z,
                     ri.R[6] * d.gc.x + ri.R[7] * d.gc.y + ri.R[8] * d.gc.z);
  // iso: d/d|o| = w e / iso, d|o|/do = o / |o|
  const float sm = g_iso * w * t.e / t.iso / t.mag;
  d.go.x += sm * t.o.x;
  d.go.y += sm * t.o.y;
  d.go.z += sm * t.o.z;
  // rot: d/d(q_n - q_i) = w dq / rot
  const float sq = g_rot * w / t.rot;
  d.gq = make_float4(sq * t.dq.x, sq * t.dq.y, sq * t.dq.z, sq * t.dq.w);
  return d;
}

// dL/dR (G[a][b] = sum_k o_a gc_b) -> dL/d rel_rot through build_rotation's
// matrix and its normalisation: (d - qn (qn . d)) / |q|.
__device__ inline float4 rotation_bwd(const float (&G)[9], float4 q, float invn) {
  const float r = q.x * invn, x = q.y * invn, y = q.z * invn, z = q.w * invn;
  const float dr = 2.f * (-z * G[1] + y * G[2] + z * G[3] - x * G[5] - y * G[6] + x * G[7]);
  const float dx = 2.f * (y * G[1] + z * G[2] + y * G[3] - 2.f * x * G[4] - r * G[5] + z * G[6] + r * G[7] -
                          2.f * x * G[8]);
  const float dy = 2.f * (-2.f * y * G[0] + x * G[1] + r * G[2] + x * G[3] + z * G[5] - r * G[6] + z * G[7] -
                          2.f * y * G[8]);
  const float dz = 2.f * (-2.f * z * G[0] - r * G[1] + x * G[2] + r * G[3] - 2.f * z * G[4] + y * G[5] +
                          x * G[6] + y * G[7]);
  const float proj = r * dr + x * dx + y * dy + z * dz;
  return make_float4((dr - r * proj) * invn, (dx - x * proj) * invn, (dy - y * proj) * invn,
                     (dz - z * proj) * invn);
}

__device__ inline float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// Block sums of three per-lane values -> partial[block] (fixed order).
__device__ inline void block_partial(float a, float b, float c, double* __restrict__ partial) {
  __shared__ float red[3][NB_WAVES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  if (lane == 0) {
    red[0][wave] = a;
    red[1][wave] = b;
    red[2][wave] = c;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    double s = 0.0;
    for (int w = 0; w < NB_WAVES; ++w) s += red[threadIdx.x][w];
    partial[3 * (int64_t)blockIdx.x + threadIdx.x] = s;
  }
}

// ---- forward

// Lane per pair (K <= 64): wave-group wg holds Gaussians [wg G, wg G + G).
__global__ void __launch_bounds__(NB_THREADS) nb_fwd_lanes_kernel(int64_t N, int K, int G, int64_t n_groups,
                                                                  const float* __restrict__ pts,
                                                                  const float4* __restrict__ qv,
                                                                  const float* __restrict__ Rm,
                                                                  const int64_t* __restrict__ nbr,
                                                                  const float* __restrict__ wgt,
                                                                  const float* __restrict__ dist,
                                                                  const float* __restrict__ poff,
                                                                  double* __restrict__ partial) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane / K, k = lane - g * K;
  float s_rigid = 0.f, s_rot = 0.f, s_iso = 0.f;
  for (int64_t wg = (int64_t)blockIdx.x * NB_WAVES + wave; wg < n_groups; wg += (int64_t)gridDim.x * NB_WAVES) {
    const int64_t i = wg * G + g;
    if (g < G && i < N) {
      const int64_t pk = i * K + k;
      const int64_t n = nbr[pk];
      const PairTerms t = pair_terms(load_rec(qv, Rm, i), ld3(pts + 3 * i), ld3(pts + 3 * n), qv[n], wgt[pk],
                                     dist[pk], ld3(poff + 3 * pk));
      s_rigid += t.rigid;
      s_rot += t.rot;
      s_iso += t.iso;
    }
  }
  block_partial(s_rigid, s_rot, s_iso, partial);
}

// Thread per Gaussian (K > 64).
__global__ void __launch_bounds__(NB_THREADS) nb_fwd_kernel(int64_t N, int K, const float* __restrict__ pts,
                                                            const float4* __restrict__ qv,
                                                            const float* __restrict__ Rm,
                                                            const int64_t* __restrict__ nbr,
                                                            const float* __restrict__ wgt,
                                                            const float* __restrict__ dist,
                                                            const float* __restrict__ poff,
                                                            double* __restrict__ partial) {
  float s_rigid = 0.f, s_rot = 0.f, s_iso = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * NB_THREADS + threadIdx.x; i < N; i += (int64_t)gridDim.x * NB_THREADS) {
    const Rec ri = load_rec(qv, Rm, i);
    const float3 pi = ld3(pts + 3 * i);
    for (int k = 0; k < K; ++k) {
      const int64_t pk = i * K + k;
      const int64_t n = nbr[pk];
      const PairTerms t = pair_terms(ri, pi, ld3(pts + 3 * n), qv[n], wgt[pk], dist[pk], ld3(poff + 3 * pk));
      s_rigid += t.rigid;
      s_rot += t.rot;
      s_iso += t.iso;
    }
  }
  block_partial(s_rigid, s_rot, s_iso, partial);
}

// Fixed-order sum of the block partials -> the three means.
__global__ void __launch_bounds__(NB_THREADS) nb_final_kernel(int nblocks, const double* __restrict__ partial,
                                                              double inv_count, float* __restrict__ out) {
  __shared__ double red[3][NB_THREADS];
  double s[3] = {0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nblocks; b += NB_THREADS)
    for (int c = 0; c < 3; ++c) s[c] += partial[3 * b + c];
  for (int c = 0; c < 3; ++c) red[c][threadIdx.x] = s[c];
  __syncthreads();
  for (int st = NB_THREADS / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st)
      for (int c = 0; c < 3; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x < 3) out[threadIdx.x] = (float)(red[threadIdx.x][0] * inv_count);
}

// ---- backward.  revbuf[rev_pos[pk]] = (go (3), -, gq (4)): the neighbour's
// share, in reverse-CSR order; selfbuf[i] = (-sum go (3), -, -sum gq +
// rotation_bwd (4)): the Gaussian's own share.

__global__ void __launch_bounds__(NB_THREADS) nb_bwd_lanes_kernel(int64_t N, int K, int G,
                                                                  const float* __restrict__ pts,
                                                                  const float4* __restrict__ qv,
                                                                  const float* __restrict__ Rm,
                                                                  const int64_t* __restrict__ nbr,
                                                                  const float* __restrict__ wgt,
                                                                  const float* __restrict__ dist,
                                                                  const float* __restrict__ poff,
                                                                  const int32_t* __restrict__ rev_pos,
                                                                  const float* __restrict__ dL, float inv_count,
                                                                  float4* __restrict__ revbuf,
                                                                  float4* __restrict__ selfbuf) {
  constexpr int NC = 16;  // -go (3), -gq (4), dL/dR (9)
  __shared__ float s_v[NB_WAVES][NC][65];
  __shared__ float s_sum[NB_WAVES][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t wg = (int64_t)blockIdx.x * NB_WAVES + wave;
  const int g = lane / K, k = lane - g * K;
  const int64_t i = wg * G + g;
  float v[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) v[c] = 0.f;
  if (g < G && i < N) {
    const int64_t pk = i * K + k;
    const int64_t n = nbr[pk];
    const float w = wgt[pk];
    const Rec ri = load_rec(qv, Rm, i);
    const PairTerms t = pair_terms(ri, ld3(pts + 3 * i), ld3(pts + 3 * n), qv[n], w, dist[pk], ld3(poff + 3 * pk));
    const PairGrads d = pair_grads(t, ri, w, dL[0] * inv_count, dL[1] * inv_count, dL[2] * inv_count);
    const int64_t slot = rev_pos[pk];
    revbuf[2 * slot] = make_float4(d.go.x, d.go.y, d.go.z, 0.f);
    revbuf[2 * slot + 1] = d.gq;
    v[0] = -d.go.x; v[1] = -d.go.y; v[2] = -d.go.z;
    v[3] = -d.gq.x; v[4] = -d.gq.y; v[5] = -d.gq.z; v[6] = -d.gq.w;
    v[7] = t.o.x * d.gc.x;  v[8] = t.o.x * d.gc.y;  v[9] = t.o.x * d.gc.z;
    v[10] = t.o.y * d.gc.x; v[11] = t.o.y * d.gc.y; v[12] = t.o.y * d.gc.z;
    v[13] = t.o.z * d.gc.x; v[14] = t.o.z * d.gc.y; v[15] = t.o.z * d.gc.z;
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) s_v[wave][c][lane] = v[c];
  __syncthreads();
  // rounds of 4 Gaussians: lane (g2, c) = (lane / 16, lane % 16) sums
  // component c of Gaussian gb + g2 over its K lanes, then lane gi < 4
  // finishes Gaussian gb + gi
  const int g2 = lane >> 4, c = lane & 15;
  for (int gb = 0; gb < G; gb += 4) {
    if (gb + g2 < G) {
      float a = 0.f;
      for (int kk = 0; kk < K; ++kk) a += s_v[wave][c][(gb + g2) * K + kk];
      s_sum[wave][g2 * 16 + c] = a;
    }
    __syncthreads();
    const int64_t ii = wg * G + gb + lane;
    if (lane < 4 && gb + lane < G && ii < N) {
      const float* S = &s_sum[wave][lane * 16];
      float Gm[9];
#pragma unroll
      for (int m = 0; m < 9; ++m) Gm[m] = S[7 + m];
      const float4 dqr = rotation_bwd(Gm, qv[ii], Rm[RM * ii + 9]);
      selfbuf[2 * ii] = make_float4(S[0], S[1], S[2], 0.f);
      selfbuf[2 * ii + 1] = make_float4(S[3] + dqr.x, S[4] + dqr.y, S[5] + dqr.z, S[6] + dqr.w);
    }
    __syncthreads();
  }
}

// Thread per Gaussian (K > 64).
__global__ void __launch_bounds__(NB_THREADS) nb_bwd_kernel(int64_t N, int K, const float* __restrict__ pts,
                                                            const float4* __restrict__ qv,
                                                            const float* __restrict__ Rm,
                                                            const int64_t* __restrict__ nbr,
                                                            const float* __restrict__ wgt,
                                                            const float* __restrict__ dist,
                                                            const float* __restrict__ poff,
                                                            const int32_t* __restrict__ rev_pos,
                                                            const float* __restrict__ dL, float inv_count,
                                                            float4* __restrict__ revbuf,
                                                            float4* __restrict__ selfbuf) {
  const int64_t i = (int64_t)blockIdx.x * NB_THREADS + threadIdx.x;
  if (i >= N) return;
  const float g_rigid = dL[0] * inv_count, g_rot = dL[1] * inv_count, g_iso = dL[2] * inv_count;
  const Rec ri = load_rec(qv, Rm, i);
  const float3 pi = ld3(pts + 3 * i);
  float G[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float3 dpi = make_float3(0.f, 0.f, 0.f);
  float4 dqi = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k = 0; k < K; ++k) {
    const int64_t pk = i * K + k;
    const int64_t n = nbr[pk];
    const float w = wgt[pk];
    const PairTerms t = pair_terms(ri, pi, ld3(pts + 3 * n), qv[n], w, dist[pk], ld3(poff + 3 * pk));
    const PairGrads d = pair_grads(t, ri, w, g_rigid, g_rot, g_iso);
    G[0] += t.o.x * d.gc.x; G[1] += t.o.x * d.gc.y; G[2] += t.o.x * d.gc.z;
    G[3] += t.o.y * d.gc.x; G[4] += t.o.y * d.gc.y; G[5] += t.o.y * d.gc.z;
    G[6] += t.o.z * d.gc.x; G[7] += t.o.z * d.gc.y; G[8] += t.o.z * d.gc.z;
    const int64_t slot = rev_pos[pk];
    revbuf[2 * slot] = make_float4(d.go.x, d.go.y, d.go.z, 0.f);
    revbuf[2 * slot + 1] = d.gq;
    dpi.x -= d.go.x; dpi.y -= d.go.y; dpi.z -= d.go.z;
    dqi.x -= d.gq.x; dqi.y -= d.gq.y; dqi.z -= d.gq.z; dqi.w -= d.gq.w;
  }
  const float4 dqr = rotation_bwd(G, ri.q, ri.invn);
  selfbuf[2 * i] = make_float4(dpi.x, dpi.y, dpi.z, 0.f);
  selfbuf[2 * i + 1] = make_float4(dqi.x + dqr.x, dqi.y + dqr.y, dqi.z + dqr.z, dqi.w + dqr.w);
}

// Per Gaussian: own share + its reverse row (contiguous in revbuf), then
// rel_rot -> fg_rot through quat_mult.  GL lanes per Gaussian stride the row,
// a fixed-order butterfly combines them: deterministic.
__global__ void __launch_bounds__(NB_THREADS) nb_gather_kernel(int64_t N, const int32_t* __restrict__ rev_ptr,
                                                               const float4* __restrict__ revbuf,
                                                               const float4* __restrict__ selfbuf,
                                                               const float* __restrict__ pinv,
                                                               float* __restrict__ d_pts,
                                                               float* __restrict__ d_rot) {
  constexpr int GL = 4;
  const int64_t t = (int64_t)blockIdx.x * NB_THREADS + threadIdx.x;
  const int64_t i = t / GL;
  const int sub = (int)(t % GL);
  const bool act = i < N;
  float4 dp = make_float4(0.f, 0.f, 0.f, 0.f), dq = dp;
  if (act) {
    const int32_t b = rev_ptr[i], e = rev_ptr[i + 1];
    for (int32_t j = b + sub; j < e; j += GL) {
      const float4 a = revbuf[2 * (int64_t)j], c = revbuf[2 * (int64_t)j + 1];
      dp.x += a.x; dp.y += a.y; dp.z += a.z;
      dq.x += c.x; dq.y += c.y; dq.z += c.z; dq.w += c.w;
    }
  }
#pragma unroll
  for (int o = 1; o < GL; o <<= 1) {
    dp.x += __shfl_xor(dp.x, o, 64); dp.y += __shfl_xor(dp.y, o, 64); dp.z += __shfl_xor(dp.z, o, 64);
    dq.x += __shfl_xor(dq.x, o, 64); dq.y += __shfl_xor(dq.y, o, 64);
    dq.z += __shfl_xor(dq.z, o, 64); dq.w += __shfl_xor(dq.w, o, 64);
  }
  if (!act || sub != 0) return;
  const float4 sp = selfbuf[2 * i], sq = selfbuf[2 * i + 1];
  d_pts[3 * i] = sp.x + dp.x;
  d_pts[3 * i + 1] = sp.y + dp.y;
  d_pts[3 * i + 2] = sp.z + dp.z;
  const float4 g = quat_mult_bwd_a(make_float4(sq.x + dq.x, sq.y + dq.y, sq.z + dq.z, sq.w + dq.w),
                                   ld4(pinv + 4 * i));
  *reinterpret_cast<float4*>(d_rot + 4 * i) = g;
}

// ---- reverse CSR: keys = neighbour id (invalid -> status), values = pair
// index; after a stable sort, row starts from the key boundaries and the
// inverse permutation (pair -> slot).
__global__ void nb_rev_keys_kernel(int64_t NK, int64_t N, const int64_t* __restrict__ nbr,
                                   uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                   int* __restrict__ status) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= NK) return;
  int64_t n = nbr[p];
  if (n < 0 || n >= N) {
    atomicOr(status, 1);
    n = N;  // sorts past every valid row
  }
  keys[p] = (uint64_t)n;
  vals[p] = (uint32_t)p;
}

__global__ void nb_rev_ptr_kernel(int64_t NK, int64_t N, const uint64_t* __restrict__ keys,
                                  const uint32_t* __restrict__ vals, int32_t* __restrict__ rev_ptr,
                                  int32_t* __restrict__ rev_pair, int32_t* __restrict__ rev_pos) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p > NK) return;
  const int64_t prev = p > 0 ? (int64_t)keys[p - 1] : -1;
  const int64_t cur = p < NK ? (int64_t)keys[p] : N;
  const int64_t hi = cur < N ? cur : N;
  for (int64_t n = prev + 1; n <= hi; ++n) rev_ptr[n] = (int32_t)p;
  if (p < NK) {
    if (rev_pair) rev_pair[p] = (int32_t)vals[p];
    rev_pos[vals[p]] = (int32_t)p;
  }
}

inline unsigned blocks_for(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }
inline unsigned capped(int64_t b) { return (unsigned)(b < NB_MAX_BLOCKS ? (b > 0 ? b : 1) : NB_MAX_BLOCKS); }

struct Work {
  float4* qv;
  float* Rm;
  double* partial;
  float4* revbuf;
  float4* selfbuf;
};
Work carve(const NeighborLayout& L, void* ws) {
  char* w = static_cast<char*>(ws);
  return Work{reinterpret_cast<float4*>(w + L.qv), reinterpret_cast<float*>(w + L.Rm),
              reinterpret_cast<double*>(w + L.partial), reinterpret_cast<float4*>(w + L.revbuf),
              reinterpret_cast<float4*>(w + L.selfbuf)};
}

}  // namespace

NeighborLayout::NeighborLayout(int64_t N, int K, bool backward) {
  size_t o = 0;
  qv = o; o = align_up(o + 16 * (size_t)N, 256);
  Rm = o; o = align_up(o + sizeof(float) * RM * (size_t)N, 256);
  partial = o; o = align_up(o + sizeof(double) * 3 * NB_MAX_BLOCKS, 256);
  revbuf = selfbuf = o;
  if (backward) {
    revbuf = o; o = align_up(o + 32 * (size_t)N * K, 256);
    selfbuf = o; o = align_up(o + 32 * (size_t)N, 256);
  }
  total = o;
}

void launch_neighbor_forward(const NeighborArgs& a, float* losses, void* ws, hipStream_t s) {
  const Work w = carve(NeighborLayout(a.N, a.K, false), ws);
  unsigned nb = 0;
  if (a.N > 0) {
    hipLaunchKernelGGL(nb_prep_kernel, dim3(blocks_for(a.N, NB_THREADS)), dim3(NB_THREADS), 0, s, a.N, a.fg_rot,
                       a.prev_inv_rot, w.qv, w.Rm);
    if (a.K >= 1 && a.K <= 64) {
      const int G = 64 / a.K;
      const int64_t groups = (a.N + G - 1) / G;
      nb = capped(blocks_for(groups, NB_WAVES));
      hipLaunchKernelGGL(nb_fwd_lanes_kernel, dim3(nb), dim3(NB_THREADS), 0, s, a.N, a.K, G, groups, a.fg_pts,
                         w.qv, w.Rm, a.nbr, a.weight, a.dist, a.prev_offset, w.partial);
    } else if (a.K > 64) {
      nb = capped(blocks_for(a.N, NB_THREADS));
      hipLaunchKernelGGL(nb_fwd_kernel, dim3(nb), dim3(NB_THREADS), 0, s, a.N, a.K, a.fg_pts, w.qv, w.Rm, a.nbr,
                         a.weight, a.dist, a.prev_offset, w.partial);
    }
  }
  const double cnt = (double)a.N * (double)a.K;
  hipLaunchKernelGGL(nb_final_kernel, dim3(1), dim3(NB_THREADS), 0, s, (int)nb, w.partial,
                     cnt > 0 ? 1.0 / cnt : __builtin_nan(""), losses);
}

void launch_neighbor_backward(const NeighborArgs& a, const float* dL, float* d_pts, float* d_rot, void* ws,
                              hipStream_t s) {
  if (a.N <= 0) return;
  const Work w = carve(NeighborLayout(a.N, a.K, true), ws);
  const float inv = a.K > 0 ? (float)(1.0 / ((double)a.N * (double)a.K)) : 0.f;
  hipLaunchKernelGGL(nb_prep_kernel, dim3(blocks_for(a.N, NB_THREADS)), dim3(NB_THREADS), 0, s, a.N, a.fg_rot,
                     a.prev_inv_rot, w.qv, w.Rm);
  if (a.K >= 1 && a.K <= 64) {
    const int G = 64 / a.K;
    hipLaunchKernelGGL(nb_bwd_lanes_kernel, dim3(blocks_for((a.N + G - 1) / G, NB_WAVES)), dim3(NB_THREADS), 0, s,
                       a.N, a.K, G, a.fg_pts, w.qv, w.Rm, a.nbr, a.weight, a.dist, a.prev_offset, a.rev_pos, dL,
                       inv, w.revbuf, w.selfbuf);
  } else {
    // K == 0 walks nothing and leaves the own share zero
    hipLaunchKernelGGL(nb_bwd_kernel, dim3(blocks_for(a.N, NB_THREADS)), dim3(NB_THREADS), 0, s, a.N, a.K,
                       a.fg_pts, w.qv, w.Rm, a.nbr, a.weight, a.dist, a.prev_offset, a.rev_pos, dL, inv, w.revbuf,
                       w.selfbuf);
  }
  hipLaunchKernelGGL(nb_gather_kernel, dim3(blocks_for(a.N * 4, NB_THREADS)), dim3(NB_THREADS), 0, s, a.N,
                     a.rev_ptr, w.revbuf, w.selfbuf, a.prev_inv_rot, d_pts, d_rot);
}

void launch_neighbor_rev_keys(int64_t NK, int64_t N, const int64_t* nbr, uint64_t* keys, uint32_t* vals,
                              int* status, hipStream_t s) {
  if (NK > 0)
    hipLaunchKernelGGL(nb_rev_keys_kernel, dim3(blocks_for(NK, 256)), dim3(256), 0, s, NK, N, nbr, keys, vals,
                       status);
}

void launch_neighbor_rev_ptr(int64_t NK, int64_t N, const uint64_t* keys, const uint32_t* vals, int32_t* rev_ptr,
                             int32_t* rev_pair, int32_t* rev_pos, hipStream_t s) {
  hipLaunchKernelGGL(nb_rev_ptr_kernel, dim3(blocks_for(NK + 1, 256)), dim3(256), 0, s, NK, N, keys, vals, rev_ptr,
                     rev_pair, rev_pos);
}

}  // namespace gs
