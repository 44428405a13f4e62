// gs_render.hip -- tile-ordered alpha blending, forward and backward.
//
// Reference: DGR/cuda_rasterizer/forward.cu:274-408 (renderCUDA) and
// backward.cu:432-652 (renderCUDA backward).
//
// MI355X design:
//  * A 16x16 binning tile is one 256-thread workgroup; each of its 4 waves
//    owns a 16x4 pixel strip and walks the tile's depth-sorted list on its
//    own -- no block barriers, every wave exits when its own pixels are done.
//  * The list is consumed in chunks of 64: lane j gathers the 48-B render
//    record of the chunk's j-th Gaussian (prefetched one chunk ahead), tests
//    it against the wave's strip (the Gaussian's alpha >= 1/255 extent) and
//    parks it in a wave-private LDS slot.  A ballot leaves the Gaussians the
//    strip can see; the inner loop visits only those, reading each record
//    back with broadcast ds_read_b128.  Culled Gaussians are exactly the ones
//    every pixel of the strip skips in the reference loop.
//  * Semantic features (F = 32/64) are a dense contraction and go to the fp32
//    matrix cores (v_mfma_f32_32x32x2_f32, an exact k-ordered fma chain):
//      forward   out_feat^T[ch][pix] += f[g][ch] * w[g][pix]  over Gaussian pairs
//      backward  dL/df[g][ch]        += w[g][pix] * dL/dfeat[pix][ch] over 32-Gaussian batches
//    Colour, depth and the geometric gradients stay on the VALU.
//  * Backward per-Gaussian sums (mean2D, conic, opacity, colour, depth) are
//    reduced over the wave with permlane32/16 swaps + DPP and committed with
//    ONE atomic wave-instruction; feature gradients leave the MFMA
//    accumulator as 2 x 128-B rows per atomic instruction.
#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

constexpr float ALPHA_MIN = 1.0f / 255.0f;
constexpr int CHUNK = 64;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float float4_t __attribute__((ext_vector_type(4)));

__device__ inline bool wave_any(bool p) { return __ballot(p) != 0ull; }

// Work counters for kernel tuning (tools/render_stats.py); compiled only into
// the "stats" build variant (-DGS_STATS), never into the product library.
#ifdef GS_STATS
__device__ unsigned long long g_stats[32];
#define STAT(i, n)                                                               \
  do {                                                                           \
    const unsigned long long n_ = (unsigned long long)(n);                       \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_stats[i], n_);                     \
  } while (0)
#define STAT_DECL(v) unsigned long long v = 0
#define STAT_INC(v) (++v)
#define STAT_WAVE(i_max, i_hist, v)                                              \
  do {                                                                           \
    if ((threadIdx.x & 63) == 0) {                                               \
      atomicMax(&g_stats[i_max], v);                                             \
      const int b_ = v < 256 ? 0 : v < 512 ? 1 : v < 1024 ? 2 : v < 2048 ? 3 : 4; \
      atomicAdd(&g_stats[i_hist + b_], 1ull);                                    \
    }                                                                            \
  } while (0)
#else
#define STAT(i, n) ((void)0)
#define STAT_DECL(v) ((void)0)
#define STAT_INC(v) ((void)0)
#define STAT_WAVE(i_max, i_hist, v) ((void)0)
#endif

// exp(x) as one v_exp_f32 (2^x) on x*log2(e): ~3 ulp instead of libm's
// correctly-rounded-ish 14-instruction sequence.  Forward and backward use
// the same function, so their alpha decisions agree bit for bit.
__device__ inline float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
// 1/x as one v_rcp_f32 (1 ulp).
__device__ inline float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ inline f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Swap the upper half of `a` with the lower half of `b`:
// lo = [a_lo, b_lo], hi = [a_hi, b_hi].
__device__ inline void swap32(float a, float b, float& lo, float& hi) {
  auto r = __builtin_amdgcn_permlane32_swap(f_bits(a), f_bits(b), false, false);
  lo = bits_f(r[0]);
  hi = bits_f(r[1]);
}

// Gather the record of list entry i (all 16 fields).  The index is clamped
// to the last entry of the (non-empty) range, so the loads are unconditional:
// lanes past the end re-read a valid record and are masked out by the caller.
// (A conditional update of a register struct made the compiler keep it in
// scratch memory.)
struct RecRegs {
  float4 q0, q1, q2, q3;
  uint32_t gid;
};
__device__ inline RecRegs load_rec(const uint32_t* __restrict__ point_list, const float* __restrict__ rec,
                                   uint32_t i, uint32_t last_valid) {
  RecRegs r;
  r.gid = point_list[i < last_valid ? i : last_valid];
  const float4* p = reinterpret_cast<const float4*>(rec + (size_t)r.gid * REC);
  r.q0 = p[0];  // x, y, conic a, conic b
  r.q1 = p[1];  // conic c, opacity, r, g
  r.q2 = p[2];  // b, depth, ext x, ext y
  r.q3 = p[3];  // radius, cull threshold tq, -, -
  return r;
}

// Gaussian exponent at pixel offset (dx, dy) from the conic scaled once per
// record: h = (-a/2, -b, -c/2).  power = -1/2 (a dx^2 + c dy^2) - b dx dy
// (CR/forward.cu:353-355) in a fixed fma order shared by the forward and the
// backward kernel, so both make bit-identical alpha decisions.
__device__ inline float4 half_conic(const float4& q0, const float4& q1) {
  return make_float4(-0.5f * q0.z, -q0.w, -0.5f * q1.x, 0.0f);
}
__device__ inline float gauss_power(float dx, float dy, const float4& h) {
  return fmaf(h.x * dx, dx, fmaf(h.z * dy, dy, (h.y * dx) * dy));
}

// Can the Gaussian reach alpha >= 1/255 at any pixel centre of the strip
// [sx0, sx1] x [sy0, sy1]?  rect_culled (gs_common.h) on the record's mean,
// conic and threshold tq: exact up to tq's margin, so it culls the Gaussians
// whose bounding box touches the strip but whose ellipse does not.
__device__ inline bool strip_culled(const RecRegs& q, float sx0, float sx1, float sy0, float sy1) {
#ifdef GS_EXP_BOX_CULL
  return q.q0.x + q.q2.z < sx0 || q.q0.x - q.q2.z > sx1 || q.q0.y + q.q2.w < sy0 || q.q0.y - q.q2.w > sy1;
#endif
  return rect_culled(q.q0.x, q.q0.y, q.q0.z, q.q0.w, q.q1.x, q.q3.y, sx0, sx1, sy0, sy1);
}

// ------------------------------------------------------------------ forward

#ifdef GS_FWD_WPE  // occupancy experiment: request GS_FWD_WPE waves per SIMD
#define GS_FWD_ATTR __attribute__((amdgpu_waves_per_eu(GS_FWD_WPE, 8)))
#else
#define GS_FWD_ATTR
#endif
template <int F, int COMPAT>
__global__ __launch_bounds__(256) GS_FWD_ATTR void render_fwd_kernel(
    int W, int H, int grid_x, int num_tiles, const uint2* __restrict__ ranges,
    const uint32_t* __restrict__ point_list, const float* __restrict__ rec,
    const float* __restrict__ feats, const float* __restrict__ bg, float* __restrict__ out_color,
    float* __restrict__ out_feature, float* __restrict__ out_depth, float* __restrict__ out_alpha,
    uint32_t* __restrict__ n_contrib) {
  // Features: 8 / 16 channels on the VALU (v_pk_fma_f32 with the Gaussian's
  // row in SGPRs, requested at the top of the iteration); 32 / 64 channels on
  // the matrix cores (measured faster at 32: 223 vs 227 us on the bench scene).
  constexpr bool MF = (F == 32 || F == 64);
  constexpr int FB = MF ? F / 32 : 1;        // 32-channel blocks
  constexpr int NSF = (!MF && F > 0) ? F : 1;
  // per record: (x, y, -a/2, -b) (-c/2, opacity, r, g) (b, depth, -, -)
  __shared__ float4 s_rec[4][CHUNK][3];

  const int tile = xcd_remap(blockIdx.x, num_tiles);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tx = tile % grid_x, ty = tile / grid_x;
  const int px = tx * TILE + (lane & 15), py = ty * TILE + wave * WAVE_ROWS + (lane >> 4);
  const bool inside = px < W && py < H;
  const float pfx = (float)px, pfy = (float)py;
  const float sx0 = (float)(tx * TILE), sx1 = sx0 + 15.0f;
  const float sy0 = (float)(ty * TILE + wave * WAVE_ROWS), sy1 = sy0 + 3.0f;
  const uint2 range = ranges[tile];

  float T = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f, Dp = 0.f;
  float SF[NSF];
#pragma unroll
  for (int c = 0; c < NSF; ++c) SF[c] = 0.f;
  f32x16 acc[2 * FB];
#pragma unroll
  for (int i = 0; i < 2 * FB; ++i) acc[i] = f32x16{0};
  uint32_t last = 0;
  // lane still blending (the reference's !done); an integer, not a bool, so
  // that it lives in a VGPR instead of exec-mask bookkeeping across the loops
  uint32_t live = inside ? 1u : 0u;
  // MFMA pairing: a blended Gaussian waits for a partner; a completed pair's
  // feature rows are loaded one pair ahead of its MFMAs (latency hiding).
  int pend = 0;
  uint32_t pend_gid = 0;
  float pend_w = 0.f;
  int have_prev = 0;
  float pa[FB], pb0 = 0.f, pb1 = 0.f;
#pragma unroll
  for (int fb = 0; fb < FB; ++fb) pa[fb] = 0.f;
  auto push_pair = [&](float b0, float b1, const float (&an)[FB]) {
    if (have_prev) {
#ifndef GS_EXP_FWD_NO_MFMA
#pragma unroll
      for (int fb = 0; fb < FB; ++fb) {
        acc[2 * fb] = mfma32(pa[fb], pb0, acc[2 * fb]);
        acc[2 * fb + 1] = mfma32(pa[fb], pb1, acc[2 * fb + 1]);
      }
#endif
    }
#pragma unroll
    for (int fb = 0; fb < FB; ++fb) pa[fb] = an[fb];
    pb0 = b0;
    pb1 = b1;
    have_prev = 1;
  };

  const uint32_t lastv = range.y > range.x ? range.y - 1 : range.x;
  RecRegs q;
  if (range.y > range.x) q = load_rec(point_list, rec, range.x + lane, lastv);
  STAT_DECL(st_it);
  STAT(6, 1);
  STAT(7, range.y - range.x);
  if (!wave_any(live != 0u)) goto blend_done;
  for (uint32_t c0 = range.x; c0 < range.y; c0 += CHUNK) {
    const bool keep = (c0 + lane < range.y) && !strip_culled(q, sx0, sx1, sy0, sy1);
    {
      const float4 h = half_conic(q.q0, q.q1);
      s_rec[wave][lane][0] = make_float4(q.q0.x, q.q0.y, h.x, h.y);
      s_rec[wave][lane][1] = make_float4(h.z, q.q1.y, q.q1.z, q.q1.w);
      s_rec[wave][lane][2] = q.q2;
    }
    const uint32_t chunk_gid = q.gid;  // lane j: id of the chunk's j-th record
    uint64_t mask = __ballot(keep);
    STAT(0, 1);
    STAT(1, range.y - c0 < CHUNK ? range.y - c0 : CHUNK);
    STAT(2, __builtin_popcountll(mask));
    q = load_rec(point_list, rec, c0 + CHUNK + lane, lastv);  // prefetch (clamped)
    while (mask) {
      const int j = __builtin_ctzll(mask);
      mask &= ~(1ull << j);
      // the survivor's feature row, requested before its alpha is computed so
      // the scalar loads overlap that work
      float fcur[NSF];
      if constexpr (!MF && F > 0) {
        const uint32_t g = __builtin_amdgcn_readlane(chunk_gid, j);
#pragma unroll
        for (int c = 0; c < NSF; ++c) fcur[c] = feats[(size_t)g * F + c];
      }
      STAT(3, 1);
      STAT_INC(st_it);
      const float4 r0 = s_rec[wave][j][0];
      const float4 r1 = s_rec[wave][j][1];
      const float4 r2 = s_rec[wave][j][2];
      const float dx = r0.x - pfx, dy = r0.y - pfy;
      const float power = gauss_power(dx, dy, make_float4(r0.z, r0.w, r1.x, 0.f));
      const float alpha = fminf(0.99f, r1.y * fast_exp(power));
      const float test_T = T * (1 - alpha);
      // Branch-free blend (CR/forward.cu:350-380): non-blending lanes add
      // zero-weighted terms, and T / last / live are selected, so the loop
      // body has no exec-mask juggling.
      const bool cand = live != 0u && !(power > 0.0f) && !(alpha < ALPHA_MIN);
      const bool fin = cand && test_T < 0.0001f;  // saturated: not blended, lane done
      const bool blend = cand && !fin;
      live = fin ? 0u : live;
      const float w = blend ? alpha * T : 0.0f;
      C0 = fmaf(r1.z, w, C0);
      C1 = fmaf(r1.w, w, C1);
      C2 = fmaf(r2.x, w, C2);
      Dp = fmaf(r2.y, w, Dp);
      T = blend ? test_T : T;
      last = blend ? c0 + j - range.x + 1 : last;
      STAT(4, wave_any(blend));
      STAT(5, __builtin_popcountll(__ballot(blend)));
      STAT(18, wave_any(blend) && ((__ballot(blend) & 0xFFFFFFFFull) == 0 || (__ballot(blend) >> 32) == 0));
      if constexpr (!MF && F > 0) {
        // keep the row loads above the blend decision (issued early, used late)
#pragma unroll
        for (int c = 0; c < NSF; ++c) asm volatile("" ::"s"(fcur[c]));
      }
      if (F > 0 && wave_any(blend)) {
        {
          const uint32_t gid = __builtin_amdgcn_readlane(chunk_gid, j);
          if constexpr (MF) {
            if (pend == 0) {
              pend = 1;
              pend_gid = gid;
              pend_w = w;
            } else {
              const uint32_t ga = lane < 32 ? pend_gid : gid;
              float b0, b1, an[FB];
              swap32(pend_w, w, b0, b1);
#pragma unroll
#ifdef GS_EXP_FWD_NO_FEAT_LOAD
              for (int fb = 0; fb < FB; ++fb) an[fb] = (float)(ga & 7);
#else
              for (int fb = 0; fb < FB; ++fb) an[fb] = feats[(size_t)ga * F + fb * 32 + (lane & 31)];
#endif
              push_pair(b0, b1, an);
              pend = 0;
            }
          } else {
            (void)gid;
#pragma unroll
            for (int c = 0; c < NSF; ++c) SF[c] = fmaf(fcur[c], w, SF[c]);
          }
        }
      }
      if (!wave_any(live != 0u)) goto blend_done;
    }
  }
blend_done:
  STAT_WAVE(16, 20, st_it);
  if constexpr (MF) {
    if (pend) {
      float b0, b1, an[FB];
      swap32(pend_w, 0.0f, b0, b1);
#pragma unroll
      for (int fb = 0; fb < FB; ++fb) an[fb] = lane < 32 ? feats[(size_t)pend_gid * F + fb * 32 + lane] : 0.0f;
      push_pair(b0, b1, an);
    }
    if (have_prev) {
#pragma unroll
      for (int fb = 0; fb < FB; ++fb) {
        acc[2 * fb] = mfma32(pa[fb], pb0, acc[2 * fb]);
        acc[2 * fb + 1] = mfma32(pa[fb], pb1, acc[2 * fb + 1]);
      }
    }
  }
  const size_t HW = (size_t)H * W;
  if (inside) {
    const size_t pix = (size_t)py * W + px;
    n_contrib[pix] = last;
    out_color[pix] = C0 + T * bg[0];
    out_color[HW + pix] = C1 + T * bg[1];
    out_color[2 * HW + pix] = C2 + T * bg[2];
    out_depth[pix] = Dp;
    if constexpr (!MF && F > 0) {
#pragma unroll
      for (int c = 0; c < F; ++c) {
        // Q4: the reference adds bg[ch] (an out-of-bounds read for ch >= 3;
        // zero here); the fixed mode adds no background to features.
        const float b = (COMPAT == COMPAT_REFERENCE && c < 3) ? bg[c] : 0.0f;
        out_feature[c * HW + pix] = SF[c] + T * b;
      }
    }
    // Q1: the reference never writes out_alpha (torch::full -> 0 stays 0);
    // we store that 0 here instead of a separate fill launch.
    if (COMPAT != COMPAT_REFERENCE) out_alpha[pix] = 1.0f - T;
    else if (out_alpha) out_alpha[pix] = 0.0f;
  }
  if constexpr (MF) {
    // acc[2*fb + blk] holds out_feat^T: lane l, register r ->
    // channel fb*32 + (r&3) + 8(r>>2) + 4(l>>5), strip pixel (l&31) + 32 blk.
    float t_lo, t_hi;
    swap32(T, T, t_lo, t_hi);  // T of strip pixel (l&31) and (l&31)+32
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      const int p = (lane & 31) + 32 * blk;
      const int qx = tx * TILE + (p & 15), qy = ty * TILE + wave * WAVE_ROWS + (p >> 4);
      if (qx < W && qy < H) {
        const size_t pix = (size_t)qy * W + qx;
        const float Tp = blk ? t_hi : t_lo;
#pragma unroll
        for (int fb = 0; fb < FB; ++fb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ch = fb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const float b = (COMPAT == COMPAT_REFERENCE && ch < 3) ? bg[ch < 3 ? ch : 0] : 0.0f;
            out_feature[ch * HW + pix] = acc[2 * fb + blk][r] + Tp * b;
          }
      }
    }
  }
}

// ------------------------------------------------------------------ backward

// Reduce N per-lane components over the wave and add them with one atomic
// wave-instruction per 64 components: components [0, A_FEAT) go to the
// per-Gaussian record acc[g][0..A_FEAT), features to dsem[g][0..F).
template <int N, int OFF = 0>
__device__ inline void commit(const float (&v)[N], float* __restrict__ acc_g, float* __restrict__ dsem_g,
                              int lane) {
  constexpr int n = (N - OFF) < 64 ? (N - OFF) : 64;
  float t[64];
#pragma unroll
  for (int c = 0; c < n; ++c) t[c] = v[OFF + c];
  const float s = wave_reduce_transposed<n>(t, lane);
  const int comp = OFF + bitrev6(lane);
#ifdef GS_EXP_NO_ACC_ATOMIC
  if (comp < OFF + n && s == 12345.f) acc_g[comp] = s;
#else
  if (comp < OFF + n) atomicAdd(comp < A_FEAT ? acc_g + comp : dsem_g + (comp - A_FEAT), s);
#endif
  if constexpr (OFF + 64 < N) commit<N, OFF + 64>(v, acc_g, dsem_g, lane);
}

// dL/dsemantic of a batch of WB (<= 16) Gaussians: C[g][ch] = sum over the
// wave's 64 pixels of w[g][pix] * dLf[pix][ch] on v_mfma_f32_16x16x4_f32
// (A[g = l&15][k = l>>4] from the batch weights in LDS, B from registers,
// C row (l>>4)*4 + r, column l&15), then one atomic per (Gaussian, channel).
__device__ inline float4_t mfma16(float a, float b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
template <int F, int WB>
__device__ inline void flush_feature_batch(const float (*w)[68], const uint32_t* bgid, const float (&Bs)[F / 16][16],
                                           float* __restrict__ dsem, int lane, int rows) {
  float a[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) a[s] = w[lane & 15][4 * s + (lane >> 4)];
#pragma unroll
  for (int cb = 0; cb < F / 16; ++cb) {
    float4_t c = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) c = mfma16(a[s], Bs[cb][s], c);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = (lane >> 4) * 4 + r;
      if (row < rows) {
#ifdef GS_EXP_NO_FEAT_ATOMIC
        if (c[r] == 12345.f) dsem[(size_t)bgid[row] * F + cb * 16 + (lane & 15)] = c[r];
#else
        atomicAdd(dsem + (size_t)bgid[row] * F + cb * 16 + (lane & 15), c[r]);
#endif
      }
    }
  }
}

template <int F, int COMPAT>
__global__ __launch_bounds__(256) void render_bwd_kernel(
    int W, int H, int grid_x, int num_tiles, const uint2* __restrict__ ranges,
    const uint32_t* __restrict__ point_list, const float* __restrict__ rec,
    const float* __restrict__ feats, const float* __restrict__ bg, const float* __restrict__ alphas,
    const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpix,
    const float* __restrict__ dL_dfeat, const float* __restrict__ dL_ddepth,
    const float* __restrict__ dL_dalpha, float* __restrict__ acc, float* __restrict__ dsem) {
#ifdef GS_EXP_BWD_VALU_FEAT
  constexpr bool MF = false;
#else
  constexpr bool MF = (F == 32 || F == 64);
#endif
  constexpr int FB = MF ? F / 32 : 1;
  constexpr int NV = MF ? A_FEAT : A_FEAT + F;  // components reduced on the VALU
  constexpr int WB = 16;                        // Gaussians per MFMA batch
  constexpr int CB = MF ? F / 16 : 1;           // 16-channel blocks
  constexpr bool FIXED_FEAT = (COMPAT != COMPAT_REFERENCE) && F > 0;
  constexpr int NF_REG = (!MF && F > 0) ? F : 1;
  __shared__ float4 s_rec[4][CHUNK][4];  // the record's 3 float4 + half conic
  // batch weights w[g][pixel] (row pad 4: the 16x16x4 A reads are conflict-free)
  __shared__ float s_w[MF ? 4 : 1][MF ? WB : 1][68];
  __shared__ uint32_t s_bgid[MF ? 4 : 1][WB];

  const int tile = xcd_remap(blockIdx.x, num_tiles);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tx = tile % grid_x, ty = tile / grid_x;
  const int px = tx * TILE + (lane & 15), py = ty * TILE + wave * WAVE_ROWS + (lane >> 4);
  const bool inside = px < W && py < H;
  const float pfx = (float)px, pfy = (float)py;
  const float sx0 = (float)(tx * TILE), sx1 = sx0 + 15.0f;
  const float sy0 = (float)(ty * TILE + wave * WAVE_ROWS), sy1 = sy0 + 3.0f;
  const uint2 range = ranges[tile];
  const size_t HW = (size_t)H * W, pix = inside ? (size_t)py * W + px : 0;

  const float T_final = inside ? 1 - alphas[pix] : 0.0f;
  float T = T_final;
  const uint32_t last = inside ? n_contrib[pix] : 0u;
  float dLp[3];
  // absent upstream gradients (NULL) are zeros
  dLp[0] = inside && dL_dpix ? dL_dpix[pix] : 0.f;
  dLp[1] = inside && dL_dpix ? dL_dpix[HW + pix] : 0.f;
  dLp[2] = inside && dL_dpix ? dL_dpix[2 * HW + pix] : 0.f;
  const float dLd = inside && dL_ddepth ? dL_ddepth[pix] : 0.f;
  const float dLa = inside && dL_dalpha ? dL_dalpha[pix] : 0.f;
  const float bg_dot = bg[0] * dLp[0] + bg[1] * dLp[1] + bg[2] * dLp[2];

  // Upstream feature gradients.  VALU path: one register per channel.
  // MFMA path (v_mfma_f32_16x16x4_f32, K = pixels): the B operands of
  // dL/df = W . dLf, lane l / step s / block cb holding
  // dLf[pixel 4s + (l>>4)][channel 16cb + (l&15)], transposed through LDS.
  float dLf[NF_REG];
  float Bs[MF ? CB : 1][MF ? 16 : 1];
  float dLf_own[FIXED_FEAT && MF ? F : 1];  // fixed mode also needs f . dLf per pixel
  if constexpr (MF) {
    // B operands straight from the CHW image: lane l, step s reads channel
    // 16cb + (l&15) at strip pixel 4s + (l>>4) (4 lanes share a 16-B run of
    // one row); the loads are first needed at the first batch flush.
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int p = 4 * s + (lane >> 4);
      const int qx = tx * TILE + (p & 15), qy = ty * TILE + wave * WAVE_ROWS + (p >> 4);
      const bool qin = qx < W && qy < H;
      const size_t qpix = qin ? (size_t)qy * W + qx : 0;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
#ifdef GS_EXP_BWD_NO_DLF
        Bs[cb][s] = (float)cb;
#else
        Bs[cb][s] = qin && dL_dfeat ? dL_dfeat[(size_t)(cb * 16 + (lane & 15)) * HW + qpix] : 0.f;
#endif
      }
    }
    if constexpr (FIXED_FEAT) {
#pragma unroll
      for (int c = 0; c < F; ++c) dLf_own[c] = inside && dL_dfeat ? dL_dfeat[(size_t)c * HW + pix] : 0.f;
    }
  } else {
#pragma unroll
    for (int c = 0; c < NF_REG; ++c) dLf[c] = (F > 0 && inside && dL_dfeat) ? dL_dfeat[c * HW + pix] : 0.f;
  }

  // The reference carries per-channel "accum_rec" recurrences
  // (CR/backward.cu:560-615): for every channel k with colour c_k and upstream
  // gradient g_k,  rec_k <- la*last_k + (1-la)*rec_k  and  dL/dalpha += (c_k -
  // rec_k)*g_k.  Since g_k is fixed per pixel, only the dot products matter:
  // with  cdot = sum_k c_k g_k  (colour, depth, alpha with c = 1, and in fixed
  // mode the features) and  Q = sum_k rec_k g_k  the recurrence is
  //   Q <- Q + la*(last_cdot - Q),   dL/dalpha = cdot - Q  -- the same value
  // with fewer operations (fp32 reassociation only).
  float Q = 0.f, lcd = 0.f, la = 0.f;
  int nb = 0;  // MFMA batch fill

  const uint32_t wmax = __builtin_amdgcn_readfirstlane(wave_max_u(last));
  const uint32_t top = range.x + wmax;  // exclusive end of this wave's walk
  STAT(14, 1);
  STAT(15, wmax);
  STAT_DECL(st_it);
  RecRegs q;
  if (top > range.x) {
    const uint32_t c0 = top > range.x + CHUNK ? top - CHUNK : range.x;
    q = load_rec(point_list, rec, c0 + lane, top - 1);
  }
  for (uint32_t hi = top; hi > range.x;) {
    const uint32_t c0 = hi > range.x + CHUNK ? hi - CHUNK : range.x;
    const bool keep = (c0 + lane < hi) && !strip_culled(q, sx0, sx1, sy0, sy1);
    s_rec[wave][lane][0] = q.q0;
    s_rec[wave][lane][1] = q.q1;
    s_rec[wave][lane][2] = q.q2;
    s_rec[wave][lane][3] = half_conic(q.q0, q.q1);
    const uint32_t chunk_gid = q.gid;  // lane j: id of the chunk's j-th record
    uint64_t mask = __ballot(keep);
    STAT(8, 1);
    STAT(9, hi - c0);
    STAT(10, __builtin_popcountll(mask));
    {
      const uint32_t n0 = c0 > range.x + CHUNK ? c0 - CHUNK : range.x;
      q = load_rec(point_list, rec, n0 + lane, top - 1);  // prefetch the next (lower) chunk
    }
    while (mask) {
      const int j = 63 - __builtin_clzll(mask);
      mask &= ~(1ull << j);
      const uint32_t k = c0 + j - range.x;  // position in the tile list
      const float4 r0 = s_rec[wave][j][0];
      const float4 r1 = s_rec[wave][j][1];
      const float4 r2 = s_rec[wave][j][2];
      const float dx = r0.x - pfx, dy = r0.y - pfy;
      const float op = r1.y;
      const float power = gauss_power(dx, dy, s_rec[wave][j][3]);
      const float G = fast_exp(power);
      const float alpha = fminf(0.99f, op * G);
      const bool valid = (k < last) && !(power > 0.0f) && !(alpha < ALPHA_MIN);
      STAT(11, 1);
      STAT_INC(st_it);
      STAT(12, wave_any(valid));
      STAT(13, __builtin_popcountll(__ballot(valid)));
      if (!wave_any(valid)) continue;
      const uint32_t gid = __builtin_amdgcn_readlane(chunk_gid, j);
      // Invalid lanes keep dch = dL_dopa = Gv = 0, which zeroes every
      // contribution below without per-component selects.
      float dch = 0.f, dL_dopa = 0.f, Gv = 0.f;
      if (valid) {
        const float rinv = fast_rcp(1.f - alpha);
        T = T * rinv;
        dch = alpha * T;
        float cdot = fmaf(r2.y, dLd, fmaf(r2.x, dLp[2], fmaf(r1.w, dLp[1], r1.z * dLp[0]))) + dLa;
        if constexpr (FIXED_FEAT) {
          // fixed mode: the features feed dL/dalpha (Q5 fixed)
          const float* f = feats + (size_t)gid * F;
          float fd = 0.f;
          if constexpr (MF) {
#pragma unroll
            for (int c = 0; c < F; ++c) fd = fmaf(f[c], dLf_own[c], fd);
          } else {
#pragma unroll
            for (int c = 0; c < NF_REG; ++c) fd = fmaf(f[c], dLf[c], fd);
          }
          cdot += fd;
        }
        Q = fmaf(la, lcd - Q, Q);
        dL_dopa = fmaf(-T_final * rinv, bg_dot, (cdot - Q) * T);
        lcd = cdot;
        la = alpha;
        Gv = G;
      }
      float v[NV];
      v[A_R] = dch * dLp[0];
      v[A_G] = dch * dLp[1];
      v[A_B] = dch * dLp[2];
      v[A_DEPTH] = dch * dLd;
      if constexpr (!MF) {
#pragma unroll
        for (int c = 0; c < NF_REG; ++c) if (A_FEAT + c < NV) v[A_FEAT + c] = dch * dLf[c];
      }
      // dL/dG -> mean2D and conic (CR/backward.cu:616-630).  Those are linear
      // in e = dL/dG * G times dx, dy, dx^2, dx dy, dy^2 with per-Gaussian
      // factors (conic, -1/2, ndc scale), so the wave sums only the five
      // basis terms; preprocess_bwd applies the factors once per Gaussian.
      const float e = (op * dL_dopa) * Gv;
      const float ex = e * dx, ey = e * dy;
      v[A_MX] = ex;
      v[A_MY] = ey;
      v[A_CA] = ex * dx;
      v[A_CB] = ex * dy;
      v[A_CC] = ey * dy;
      v[A_OP] = Gv * dL_dopa;
      commit<NV>(v, acc + (size_t)A_FEAT * gid, dsem + (size_t)F * gid, lane);
      if constexpr (MF) {
        s_w[wave][nb][lane] = dch;
        if (lane == 0) s_bgid[wave][nb] = gid;
        if (++nb == WB) {
#ifndef GS_EXP_BWD_NO_MFMA
          flush_feature_batch<F, WB>(s_w[wave], s_bgid[wave], Bs, dsem, lane, WB);
#endif
          nb = 0;
        }
      }
    }
    hi = c0;
  }
  STAT_WAVE(17, 25, st_it);
  if constexpr (MF) {
    // rows >= nb hold stale weights; MFMA rows are independent, so they only
    // produce results that are not committed
    if (nb > 0) flush_feature_batch<F, WB>(s_w[wave], s_bgid[wave], Bs, dsem, lane, nb);
  }
}

// ------------------------------------------------------------------ dispatch

template <int F>
static void fwd_f(const RenderArgs& a, hipStream_t s) {
  dim3 grid(a.num_tiles), block(256);
#ifdef GS_EXP_FWD_LDS_PAD
  const size_t pad = GS_EXP_FWD_LDS_PAD;  // occupancy experiment: unused dynamic LDS
#else
  const size_t pad = 0;
#endif
  if (a.compat == COMPAT_REFERENCE)
    hipLaunchKernelGGL((render_fwd_kernel<F, COMPAT_REFERENCE>), grid, block, pad, s, a.W, a.H, a.grid_x,
                       a.num_tiles, a.ranges, a.point_list, a.rec, a.feats, a.bg, a.out_color,
                       a.out_feature, a.out_depth, a.out_alpha, a.n_contrib);
  else
    hipLaunchKernelGGL((render_fwd_kernel<F, COMPAT_FIXED>), grid, block, 0, s, a.W, a.H, a.grid_x,
                       a.num_tiles, a.ranges, a.point_list, a.rec, a.feats, a.bg, a.out_color,
                       a.out_feature, a.out_depth, a.out_alpha, a.n_contrib);
}

template <int F>
static void bwd_f(const RenderBwdArgs& a, hipStream_t s) {
  dim3 grid(a.num_tiles), block(256);
  if (a.compat == COMPAT_REFERENCE)
    hipLaunchKernelGGL((render_bwd_kernel<F, COMPAT_REFERENCE>), grid, block, 0, s, a.W, a.H, a.grid_x,
                       a.num_tiles, a.ranges, a.point_list, a.rec, a.feats, a.bg, a.alphas, a.n_contrib,
                       a.dL_dpix, a.dL_dfeat, a.dL_ddepth, a.dL_dalpha, a.acc, a.dsem);
  else
    hipLaunchKernelGGL((render_bwd_kernel<F, COMPAT_FIXED>), grid, block, 0, s, a.W, a.H, a.grid_x,
                       a.num_tiles, a.ranges, a.point_list, a.rec, a.feats, a.bg, a.alphas, a.n_contrib,
                       a.dL_dpix, a.dL_dfeat, a.dL_ddepth, a.dL_dalpha, a.acc, a.dsem);
}

bool launch_render_fwd(const RenderArgs& a, hipStream_t s) {
  if (a.num_tiles <= 0) return true;
  switch (a.F) {
    case 0: fwd_f<0>(a, s); return true;
    case 4: fwd_f<4>(a, s); return true;
    case 8: fwd_f<8>(a, s); return true;
    case 16: fwd_f<16>(a, s); return true;
    case 32: fwd_f<32>(a, s); return true;
    case 64: fwd_f<64>(a, s); return true;
    default: return false;
  }
}

bool launch_render_bwd(const RenderBwdArgs& a, hipStream_t s) {
  if (a.num_tiles <= 0) return true;
  switch (a.F) {
    case 0: bwd_f<0>(a, s); return true;
    case 4: bwd_f<4>(a, s); return true;
    case 8: bwd_f<8>(a, s); return true;
    case 16: bwd_f<16>(a, s); return true;
    case 32: bwd_f<32>(a, s); return true;
    case 64: bwd_f<64>(a, s); return true;
    default: return false;
  }
}

#ifdef GS_STATS
extern "C" int gs_stats_read(unsigned long long* out, int n) {
  if (n > 32) n = 32;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stats), sizeof(unsigned long long) * n, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int gs_stats_reset(void) {
  static const unsigned long long z[32] = {0};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#endif

// ------------------------------------------------------------------ self-test

template <int N>
__global__ void test_wave_reduce_kernel(const float* __restrict__ in, float* __restrict__ out) {
  const int lane = threadIdx.x;
  float v[64];
#pragma unroll
  for (int c = 0; c < N; ++c) v[c] = in[c * 64 + lane];
  const float s = wave_reduce_transposed<N>(v, lane);
  const int comp = bitrev6(lane);
  if (comp < N) out[comp] = s;
}

void launch_test_wave_reduce(int n, const float* in, float* out, hipStream_t s) {
#define CASE(K) case K: hipLaunchKernelGGL(test_wave_reduce_kernel<K>, dim3(1), dim3(64), 0, s, in, out); break;
  switch (n) {
    CASE(1) CASE(2) CASE(3) CASE(10) CASE(13) CASE(18) CASE(26) CASE(42) CASE(64)
    default: break;
  }
#undef CASE
}

}  // namespace gs
