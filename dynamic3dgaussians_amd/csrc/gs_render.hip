// gs_render.hip -- tile-ordered alpha blending, forward and backward.
//
// Reference: DGR/cuda_rasterizer/forward.cu:274-408 (renderCUDA) and
// backward.cu:432-652 (renderCUDA backward).
//
// MI355X design (no LDS staging, no block barriers):
//  * A 16x16 binning tile is one 256-thread workgroup; each of its 4 waves
//    owns a 16x4 pixel strip and walks the tile's depth-sorted list on its
//    own.  The Gaussian index and its 64-B render record are wave-uniform,
//    so they arrive through the scalar unit (s_load_dwordx16) and feed the
//    VALU as SGPR operands -- no per-lane gather, no LDS round trip.
//  * Wave-level culling: a wave skips a Gaussian whose alpha >= 1/255 region
//    (precomputed half extents) misses its 16x4 strip -- exactly the
//    Gaussians every one of its pixels would skip in the reference loop.
//  * Forward early exit is a wave vote (the reference votes per 256-thread
//    block); the backward starts each wave at its own max n_contrib.
//  * Backward: per-pixel contributions are summed over the wave with a
//    transposed reduction (permlane32/16 swaps + DPP), then ONE atomic
//    wave-instruction commits all 10+F per-Gaussian sums, instead of the
//    reference's 10+F atomics per pixel.
#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

constexpr float ALPHA_MIN = 1.0f / 255.0f;

__device__ inline bool wave_any(bool p) { return __ballot(p) != 0ull; }

// ------------------------------------------------------------------ forward

template <int F, int COMPAT>
__global__ __launch_bounds__(256) void render_fwd_kernel(
    int W, int H, int grid_x, int num_tiles, const uint2* __restrict__ ranges,
    const uint32_t* __restrict__ point_list, const float* __restrict__ rec,
    const float* __restrict__ feats, const float* __restrict__ bg, float* __restrict__ out_color,
    float* __restrict__ out_feature, float* __restrict__ out_depth, float* __restrict__ out_alpha,
    uint32_t* __restrict__ n_contrib) {
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
  float SF[F > 0 ? F : 1];
#pragma unroll
  for (int c = 0; c < F; ++c) SF[c] = 0.f;
  uint32_t last = 0;
  bool done = !inside;

  for (uint32_t i = range.x; i < range.y; ++i) {
    if (!wave_any(!done)) break;
    const uint32_t g = point_list[i];
    const float* r = rec + (size_t)g * REC;
    const float gx = r[R_X], gy = r[R_Y], ex = r[R_EX], ey = r[R_EY];
    if (gx + ex < sx0 || gx - ex > sx1 || gy + ey < sy0 || gy - ey > sy1) continue;
    const float ca = r[R_CA], cb = r[R_CB], cc = r[R_CC], op = r[R_OP];
    const float dx = gx - pfx, dy = gy - pfy;
    const float power = -0.5f * (ca * dx * dx + cc * dy * dy) - cb * dx * dy;
    const float alpha = fminf(0.99f, op * expf(power));
    const float test_T = T * (1 - alpha);
    bool blend = !done && !(power > 0.0f) && !(alpha < ALPHA_MIN);
    if (blend && test_T < 0.0001f) { done = true; blend = false; }
    if (!wave_any(blend)) continue;
    if (blend) {
      const float w = alpha * T;
      C0 += r[R_R] * w;
      C1 += r[R_G] * w;
      C2 += r[R_B] * w;
      Dp += r[R_DEPTH] * w;
      if constexpr (F > 0) {
        const float* f = feats + (size_t)g * F;
#pragma unroll
        for (int c = 0; c < F; ++c) SF[c] += f[c] * w;
      }
      T = test_T;
      last = i - range.x + 1;
    }
  }
  if (inside) {
    const size_t HW = (size_t)H * W, pix = (size_t)py * W + px;
    n_contrib[pix] = last;
    out_color[pix] = C0 + T * bg[0];
    out_color[HW + pix] = C1 + T * bg[1];
    out_color[2 * HW + pix] = C2 + T * bg[2];
    out_depth[pix] = Dp;
#pragma unroll
    for (int c = 0; c < F; ++c) {
      // Q4: the reference adds bg[ch] (an out-of-bounds read for ch >= 3;
      // zero here); the fixed mode adds no background to features.
      const float b = (COMPAT == COMPAT_REFERENCE && c < 3) ? bg[c] : 0.0f;
      out_feature[c * HW + pix] = SF[c] + T * b;
    }
    if (COMPAT != COMPAT_REFERENCE) out_alpha[pix] = 1.0f - T;  // Q1
  }
}

// ------------------------------------------------------------------ backward

// Reduce N per-lane components over the wave and add them to dst[0..N) with
// one atomic wave-instruction per 64 components.
template <int N, int OFF = 0>
__device__ inline void commit(const float (&v)[N], float* __restrict__ dst, int lane) {
  constexpr int n = (N - OFF) < 64 ? (N - OFF) : 64;
  float t[64];
#pragma unroll
  for (int c = 0; c < n; ++c) t[c] = v[OFF + c];
  const float s = wave_reduce_transposed<n>(t, lane);
  const int comp = bitrev6(lane);
  if (comp < n) atomicAdd(dst + OFF + comp, s);
  if constexpr (OFF + 64 < N) commit<N, OFF + 64>(v, dst, lane);
}

template <int F, int COMPAT>
__global__ __launch_bounds__(256) void render_bwd_kernel(
    int W, int H, int grid_x, int num_tiles, const uint2* __restrict__ ranges,
    const uint32_t* __restrict__ point_list, const float* __restrict__ rec,
    const float* __restrict__ feats, const float* __restrict__ bg, const float* __restrict__ alphas,
    const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpix,
    const float* __restrict__ dL_dfeat, const float* __restrict__ dL_ddepth,
    const float* __restrict__ dL_dalpha, float* __restrict__ acc) {
  constexpr int N = A_FEAT + F;
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
  float dLp[3], dLf[F > 0 ? F : 1];
  dLp[0] = inside ? dL_dpix[pix] : 0.f;
  dLp[1] = inside ? dL_dpix[HW + pix] : 0.f;
  dLp[2] = inside ? dL_dpix[2 * HW + pix] : 0.f;
#pragma unroll
  for (int c = 0; c < F; ++c) dLf[c] = inside ? dL_dfeat[c * HW + pix] : 0.f;
  const float dLd = inside ? dL_ddepth[pix] : 0.f;
  const float dLa = inside ? dL_dalpha[pix] : 0.f;
  const float bg_dot = bg[0] * dLp[0] + bg[1] * dLp[1] + bg[2] * dLp[2];
  const float ddelx_dx = 0.5f * (float)W, ddely_dy = 0.5f * (float)H;

  float ar0 = 0.f, ar1 = 0.f, ar2 = 0.f, lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;
  float ad = 0.f, ld = 0.f, aa = 0.f, la = 0.f;
  float af = 0.f, lfd = 0.f;  // fixed mode: feature accum . dL/dfeature

  const uint32_t wmax = __builtin_amdgcn_readfirstlane(wave_max_u(last));
  for (uint32_t k = wmax; k-- > 0;) {
    const uint32_t g = point_list[range.x + k];
    const float* r = rec + (size_t)g * REC;
    const float gx = r[R_X], gy = r[R_Y], ex = r[R_EX], ey = r[R_EY];
    if (gx + ex < sx0 || gx - ex > sx1 || gy + ey < sy0 || gy - ey > sy1) continue;
    const float ca = r[R_CA], cb = r[R_CB], cc = r[R_CC], op = r[R_OP];
    const float dx = gx - pfx, dy = gy - pfy;
    const float power = -0.5f * (ca * dx * dx + cc * dy * dy) - cb * dx * dy;
    const float G = expf(power);
    const float alpha = fminf(0.99f, op * G);
    const bool valid = (k < last) && !(power > 0.0f) && !(alpha < ALPHA_MIN);
    if (!wave_any(valid)) continue;
    float v[N];
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] = 0.f;
    if (valid) {
      T = T / (1.f - alpha);
      const float dch = alpha * T;
      float dL_dopa = 0.f;
      const float c0 = r[R_R], c1 = r[R_G], c2 = r[R_B];
      ar0 = la * lc0 + (1.f - la) * ar0; lc0 = c0; dL_dopa += (c0 - ar0) * dLp[0];
      ar1 = la * lc1 + (1.f - la) * ar1; lc1 = c1; dL_dopa += (c1 - ar1) * dLp[1];
      ar2 = la * lc2 + (1.f - la) * ar2; lc2 = c2; dL_dopa += (c2 - ar2) * dLp[2];
      v[A_R] = dch * dLp[0]; v[A_G] = dch * dLp[1]; v[A_B] = dch * dLp[2];
      const float cd = r[R_DEPTH];
      ad = la * ld + (1.f - la) * ad; ld = cd; dL_dopa += (cd - ad) * dLd;
      if constexpr (F > 0) {
        const float* f = feats + (size_t)g * F;
        float fd = 0.f;
#pragma unroll
        for (int c = 0; c < F; ++c) {
          v[A_FEAT + c] = dch * dLf[c];
          if constexpr (COMPAT != COMPAT_REFERENCE) fd += f[c] * dLf[c];
        }
        // Q5: in the reference the feature term reads a never-written
        // (zero) scratch and contributes nothing to dL/dalpha.
        if constexpr (COMPAT != COMPAT_REFERENCE) {
          af = la * lfd + (1.f - la) * af;
          lfd = fd;
          dL_dopa += fd - af;
        }
      }
      v[A_DEPTH] = dch * dLd;
      aa = la + (1.f - la) * aa;
      dL_dopa += (1 - aa) * dLa;
      dL_dopa *= T;
      la = alpha;
      dL_dopa += (-T_final / (1.f - alpha)) * bg_dot;
      const float dL_dG = op * dL_dopa;
      const float gdx = G * dx, gdy = G * dy;
      const float dG_ddelx = -gdx * ca - gdy * cb;
      const float dG_ddely = -gdy * cc - gdx * cb;
      v[A_MX] = dL_dG * dG_ddelx * ddelx_dx;
      v[A_MY] = dL_dG * dG_ddely * ddely_dy;
      v[A_CA] = -0.5f * gdx * dx * dL_dG;
      v[A_CB] = -0.5f * gdx * dy * dL_dG;
      v[A_CC] = -0.5f * gdy * dy * dL_dG;
      v[A_OP] = G * dL_dopa;
    }
    commit<N>(v, acc + (size_t)N * g, lane);
  }
}

// ------------------------------------------------------------------ dispatch

template <int F>
static void fwd_f(const RenderArgs& a, hipStream_t s) {
  dim3 grid(a.num_tiles), block(256);
  if (a.compat == COMPAT_REFERENCE)
    hipLaunchKernelGGL((render_fwd_kernel<F, COMPAT_REFERENCE>), grid, block, 0, s, a.W, a.H, a.grid_x,
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
                       a.dL_dpix, a.dL_dfeat, a.dL_ddepth, a.dL_dalpha, a.acc);
  else
    hipLaunchKernelGGL((render_bwd_kernel<F, COMPAT_FIXED>), grid, block, 0, s, a.W, a.H, a.grid_x,
                       a.num_tiles, a.ranges, a.point_list, a.rec, a.feats, a.bg, a.alphas, a.n_contrib,
                       a.dL_dpix, a.dL_dfeat, a.dL_ddepth, a.dL_dalpha, a.acc);
}

bool launch_render_fwd(const RenderArgs& a, hipStream_t s) {
  if (a.num_tiles <= 0) return true;
  switch (a.F) {
    case 0: fwd_f<0>(a, s); return true;
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
    case 8: bwd_f<8>(a, s); return true;
    case 16: bwd_f<16>(a, s); return true;
    case 32: bwd_f<32>(a, s); return true;
    case 64: bwd_f<64>(a, s); return true;
    default: return false;
  }
}

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
