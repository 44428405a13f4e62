// gs_preprocess.hip -- per-Gaussian forward projection and its backward
// chain rule, plus frustum marking.  One thread per Gaussian; these kernels
// are HBM-bound (~80 B in / ~90 B out per Gaussian forward).
//
// Compiled with -ffp-contract=off: every expression follows the same
// operation order as the CPU oracle (oracle/gs_oracle.c), so preprocess
// outputs match it bit for bit on identical inputs.
//
// Reference: DGR/cuda_rasterizer/forward.cu:20-269 (computeColorFromSH,
// computeCov2D, computeCov3D, preprocessCUDA), backward.cu:20-429
// (computeColorFromSH, computeCov2DCUDA, computeCov3D, preprocessCUDA),
// auxiliary.h:41-170, rasterizer_impl.cu:54-66 (checkFrustum).
#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f,
                SH_C2_2 = 0.31539156525252005f, SH_C2_3 = -1.0925484305920792f,
                SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f,
                SH_C3_2 = -0.4570457994644658f, SH_C3_3 = 0.3731763325901154f,
                SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                SH_C3_6 = -0.5900435899266435f;

struct V3 { float x, y, z; };

__device__ inline V3 ld3(const float* p) { return V3{p[0], p[1], p[2]}; }

// transformPoint4x3 (auxiliary.h:58-66); m = column-major 4x4.
__device__ inline V3 xf43(const float* __restrict__ m, V3 p) {
  return V3{m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
            m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}
__device__ inline float4 xf44(const float* __restrict__ m, V3 p) {
  return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                     m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                     m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
                     m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

// ndc2Pix in double (double literals at auxiliary.h:43).
__device__ inline float ndc_to_pix(float v, int S) {
  return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

// getRect (auxiliary.h:46-56).
__device__ inline void tile_rect(float px, float py, int r, int gx, int gy, int2& rmin, int2& rmax) {
  int a;
  a = (int)((px - (float)r) / (float)TILE); a = a > 0 ? a : 0; rmin.x = a < gx ? a : gx;
  a = (int)((py - (float)r) / (float)TILE); a = a > 0 ? a : 0; rmin.y = a < gy ? a : gy;
  a = (int)((((px + (float)r) + (float)TILE) - 1.0f) / (float)TILE); a = a > 0 ? a : 0; rmax.x = a < gx ? a : gx;
  a = (int)((((py + (float)r) + (float)TILE) - 1.0f) / (float)TILE); a = a > 0 ? a : 0; rmax.y = a < gy ? a : gy;
}

// glm columns of the (unnormalised, Q7) quaternion rotation, forward.cu:137-149.
__device__ inline void quat_cols(float4 q, float rc[3][3]) {
  const float r = q.x, x = q.y, y = q.z, z = q.w;
  rc[0][0] = 1.f - 2.f * (y * y + z * z); rc[0][1] = 2.f * (x * y - r * z); rc[0][2] = 2.f * (x * z + r * y);
  rc[1][0] = 2.f * (x * y + r * z); rc[1][1] = 1.f - 2.f * (x * x + z * z); rc[1][2] = 2.f * (y * z - r * x);
  rc[2][0] = 2.f * (x * z - r * y); rc[2][1] = 2.f * (y * z + r * x); rc[2][2] = 1.f - 2.f * (x * x + y * y);
}

// Shared EWA setup (forward.cu:75-118 / backward.cu:166-211).
struct Ewa {
  float t[3], txtz, tytz, lxp, lxn, lyp, lyn;
  float a[2][3];
};
__device__ inline void ewa_setup(V3 mean, const float* __restrict__ view, int W, int H, float cx,
                                 float cy, float fx, float fy, float tfx, float tfy, Ewa& e) {
  V3 t = xf43(view, mean);
  e.lxp = ((float)W - cx) / fx + 0.3f * tfx;
  e.lxn = cx / fx + 0.3f * tfx;
  e.lyp = ((float)H - cy) / fy + 0.3f * tfy;
  e.lyn = cy / fy + 0.3f * tfy;
  e.txtz = t.x / t.z;
  e.tytz = t.y / t.z;
  t.x = fminf(e.lxp, fmaxf(-e.lxn, e.txtz)) * t.z;
  t.y = fminf(e.lyp, fmaxf(-e.lyn, e.tytz)) * t.z;
  e.t[0] = t.x; e.t[1] = t.y; e.t[2] = t.z;
  const float j00 = fx / t.z, j02 = -(fx * t.x) / (t.z * t.z);
  const float j11 = fy / t.z, j12 = -(fy * t.y) / (t.z * t.z);
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    e.a[0][r] = view[4 * r] * j00 + view[1 + 4 * r] * 0.0f + view[2 + 4 * r] * j02;
    e.a[1][r] = view[4 * r] * 0.0f + view[1 + 4 * r] * j11 + view[2 + 4 * r] * j12;
  }
}
__device__ inline void ewa_cov2d(const Ewa& e, const float c3[6], float out[3]) {
  const float v[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
  float u[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      u[i][k] = e.a[i][0] * v[0][k] + e.a[i][1] * v[1][k] + e.a[i][2] * v[2][k];
  const float a = u[0][0] * e.a[0][0] + u[0][1] * e.a[0][1] + u[0][2] * e.a[0][2];
  const float b = u[1][0] * e.a[0][0] + u[1][1] * e.a[0][1] + u[1][2] * e.a[0][2];
  const float c = u[1][0] * e.a[1][0] + u[1][1] * e.a[1][1] + u[1][2] * e.a[1][2];
  out[0] = a + 0.3f; out[1] = b; out[2] = c + 0.3f;
}

// Half extents of the region where a pixel can still pass the reference's
// blend test (power <= 0 and alpha >= 1/255): outside it every pixel is
// skipped by the reference too, so a wave whose 16x4 pixels all lie outside
// skips the Gaussian as a whole.  Conservative: tau is inflated by the
// rounding error the fp32 power evaluation can make on this conic.
// Also returns `tq`, the same inflated threshold on the quadratic form
// q(d) = a dx^2 + 2 b dx dy + c dy^2 (alpha >= 1/255 needs q <= tq), used by
// the blend kernels' exact ellipse-vs-strip test; +inf = never cull,
// -inf = never blends.
__device__ inline void alpha_extent(float ca, float cb, float cc, float op, float& ex, float& ey, float& tq) {
  const float thr = 1.0f / 255.0f;
  if (!(op >= thr)) { ex = -INFINITY; ey = -INFINITY; tq = -INFINITY; return; }  // never blends
  const double a = ca, b = cb, c = cc;
  const double det = a * c - b * b;
  const double tr = a + c;
  if (!(a > 0.0 && c > 0.0 && det > 0.0)) { ex = INFINITY; ey = INFINITY; tq = INFINITY; return; }
  const double disc = sqrt(fmax(tr * tr - 4.0 * det, 0.0));
  const double lmin = 0.5 * (tr - disc), lmax = 0.5 * (tr + disc);
  const double cond = lmin > 0.0 ? lmax / lmin : 1e30;
  if (!(cond < 5.0e5)) { ex = INFINITY; ey = INFINITY; tq = INFINITY; return; }
  // fp32 log: its rounding is far inside the 2 % + 1e-3 inflation below
  const double tau = 2.0 * (double)logf(op * 255.0f);
  const double taup = tau * (1.02 + 32.0 * 6.0e-8 * cond) + 1e-3;
  ex = (float)(sqrt(taup * c / det) + 0.01);
  ey = (float)(sqrt(taup * a / det) + 0.01);
  tq = (float)(taup * 1.0001 + 1e-4);
}

// computeColorFromSH forward (forward.cu:20-71), one colour channel at a time.
__device__ inline void sh_fwd(int deg, int M, V3 p, V3 cp, const float* __restrict__ shs, int g,
                              float rgb[3], uint8_t& clampbits) {
  float dx = p.x - cp.x, dy = p.y - cp.y, dz = p.z - cp.z;
  const float len = sqrtf(dx * dx + dy * dy + dz * dz);
  const float x = dx / len, y = dy / len, z = dz / len;
  const float* sh = shs + (size_t)g * M * 3;
  clampbits = 0;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
#define S(i) sh[3 * (i) + ch]
    float res = SH_C0 * S(0);
    if (deg > 0) {
      res = res - SH_C1 * y * S(1) + SH_C1 * z * S(2) - SH_C1 * x * S(3);
      if (deg > 1) {
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        res = res + SH_C2_0 * xy * S(4) + SH_C2_1 * yz * S(5) + SH_C2_2 * (2.0f * zz - xx - yy) * S(6) +
              SH_C2_3 * xz * S(7) + SH_C2_4 * (xx - yy) * S(8);
        if (deg > 2) {
          res = res + SH_C3_0 * y * (3.0f * xx - yy) * S(9) + SH_C3_1 * xy * z * S(10) +
                SH_C3_2 * y * (4.0f * zz - xx - yy) * S(11) +
                SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                SH_C3_4 * x * (4.0f * zz - xx - yy) * S(13) + SH_C3_5 * z * (xx - yy) * S(14) +
                SH_C3_6 * x * (xx - 3.0f * yy) * S(15);
        }
      }
    }
#undef S
    res += 0.5f;
    if (res < 0.0f) clampbits |= (uint8_t)(1u << ch);
    rgb[ch] = res > 0.0f ? res : 0.0f;
  }
}

// ------------------------------------------------------------------ activations
// GS_FLAG_ACTIVATE: the Dynamic3DGaussians parameterisation of
// helpers.py:98-107 (params2rendervar) applied in the kernels, in the
// operation order of torch's kernels for the same ops (this file is compiled
// without fma contraction): sigmoid = 1 / (1 + exp(-x)), exp, and
// F.normalize = q / max(|q|, 1e-12) (torch.nn.functional.normalize, p = 2,
// dim = 1).  Their backward follows autograd's formulas: sigmoid_backward
// g (1 - y) y, exp's g y, and normalize's div / clamp_min / norm chain.
// The squared norm is summed pairwise, (x^2 + y^2) + (z^2 + w^2): the order
// that reproduces torch's GPU reduction bit for bit (tools/act_probe.py on an
// MI355X: 100 % of 400k quaternions vs 88 % for the sequential sum,
// profiles/r04b/act_probe.txt).
constexpr float NORMALIZE_EPS = 1e-12f;
__device__ inline float act_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ inline float act_norm(float4 q) { return sqrtf((q.x * q.x + q.y * q.y) + (q.z * q.z + q.w * q.w)); }
__device__ inline float4 act_normalize(float4 q) {
  const float d = fmaxf(act_norm(q), NORMALIZE_EPS);
  return make_float4(q.x / d, q.y / d, q.z / d, q.w / d);
}
// dL/dq of q_hat = q / max(|q|, eps) for the upstream gradient gq of q_hat:
// DivBackward (g / d for q, -g (q / d) / d summed for the denominator),
// ClampMinBackward (passes where |q| >= eps), NormBackward (q (g_n / |q|)).
__device__ inline float4 act_normalize_bwd(float4 q, float4 gq) {
  const float n = act_norm(q);
  const float d = fmaxf(n, NORMALIZE_EPS);
  const float gd = (-gq.x * ((q.x / d) / d) + -gq.y * ((q.y / d) / d)) +
                   (-gq.z * ((q.z / d) / d) + -gq.w * ((q.w / d) / d));
  const float gn = (n >= NORMALIZE_EPS && n != 0.0f) ? gd / n : 0.0f;
  return make_float4(gq.x / d + q.x * gn, gq.y / d + q.y * gn, gq.z / d + q.z * gn, gq.w / d + q.w * gn);
}
// The activated rotation / scale of Gaussian g.
__device__ inline float4 rotation_of(const float* __restrict__ rotations, int g, int activate) {
  const float4 q = reinterpret_cast<const float4*>(rotations)[g];
  return activate ? act_normalize(q) : q;
}
__device__ inline V3 scale_of(const float* __restrict__ scales, int g, int activate) {
  const V3 s = ld3(scales + 3 * g);
  return activate ? V3{expf(s.x), expf(s.y), expf(s.z)} : s;
}

// ------------------------------------------------------------------ forward

// Camera c (blockIdx.y) of a batch: its parameters and per-camera outputs.
__device__ inline PreprocessArgs cam_args(const PreprocessArgs& a0, const CamBatch& cb, int c) {
  PreprocessArgs a = a0;
  a.view = cb.view + 16 * c;
  a.proj = cb.proj + 16 * c;
  a.campos = cb.campos + 3 * c;
  a.c_x = cb.c_x[c];
  a.c_y = cb.c_y[c];
  a.tan_fovx = cb.tanx[c];
  a.tan_fovy = cb.tany[c];
  a.focal_y = (float)a.H / (2.0f * a.tan_fovy);  // CR/rasterizer_impl.cu:227-228
  a.focal_x = (float)a.W / (2.0f * a.tan_fovx);
  const int64_t go = c * cb.geom_stride;
  a.radii = a0.radii + (size_t)c * a0.P;
  a.rec = shift_bytes(a0.rec, go);
  a.cov3D = shift_bytes(a0.cov3D, go);
  a.clamped = shift_bytes(a0.clamped, go);
  a.tiles = shift_bytes(a0.tiles, go);
  a.rect = shift_bytes(a0.rect, go);
  a.status = shift_bytes(a0.status, c * cb.img_stride);
  return a;
}

__global__ __launch_bounds__(256) void preprocess_fwd_kernel(PreprocessArgs a0, CamBatch batch) {
  // camera-major dispatch (blockIdx.y = camera): each camera's output arrays
  // are written as one stream.  Dispatching a Gaussian slice's cameras
  // together cut the kernel's reads 0.45 -> 0.14 GB per 27-camera launch but
  // ran 0.27 vs 0.22 ms: the kernel is bound by its per-camera writes
  // (profiles/r04t/).
  const int cam = blockIdx.y, g = blockIdx.x * 256 + threadIdx.x;
  if (g >= a0.P) return;
  const PreprocessArgs a = cam_args(a0, batch, cam);
  // a culled Gaussian's outputs (a visible one's are written once, at the end)
  auto culled = [&]() {
    a.radii[g] = 0;
    a.tiles[g] = 0;
    a.rect[g] = make_uint4(0u, 0u, 0u, 0u);
  };
  const V3 p = ld3(a.means3D + 3 * g);
  // The 3D covariance does not depend on the camera: the batch's camera 0
  // stores it for every Gaussian (before the frustum test, so a Gaussian
  // camera 0 does not see still has it) and preprocess_bwd reads it there
  // once per Gaussian; the other cameras compute it without storing.
  float c3[6];
  if (a.cov3D_precomp) {
#pragma unroll
    for (int i = 0; i < 6; ++i) c3[i] = a.cov3D_precomp[6 * g + i];
  } else {
    float rc[3][3];
    const float4 q = rotation_of(a.rotations, g, a.activate);
    quat_cols(q, rc);
    const V3 s = scale_of(a.scales, g, a.activate);
    const float sx = a.scale_modifier * s.x, sy = a.scale_modifier * s.y, sz = a.scale_modifier * s.z;
    float m[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { m[c][0] = sx * rc[c][0]; m[c][1] = sy * rc[c][1]; m[c][2] = sz * rc[c][2]; }
#define DOT3(i, j) (m[i][0] * m[j][0] + m[i][1] * m[j][1] + m[i][2] * m[j][2])
    c3[0] = DOT3(0, 0); c3[1] = DOT3(0, 1); c3[2] = DOT3(0, 2);
    c3[3] = DOT3(1, 1); c3[4] = DOT3(1, 2); c3[5] = DOT3(2, 2);
#undef DOT3
    if (cam == 0) {
#pragma unroll
      for (int i = 0; i < 6; ++i) a.cov3D[6 * g + i] = c3[i];
    }
  }
  const V3 pv = xf43(a.view, p);
  if (pv.z <= 0.0f) {  // in_frustum, Q8
    if (a.prefiltered) atomicOr(a.status, 1);
    culled();
    return;
  }
  const float4 ph = xf44(a.proj, p);
  const float pw = 1.0f / (ph.w + 0.0000001f);
  const float ppx = ph.x * pw, ppy = ph.y * pw;
  Ewa e;
  ewa_setup(p, a.view, a.W, a.H, a.c_x, a.c_y, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy, e);
  float cov[3];
  ewa_cov2d(e, c3, cov);
  const float det = cov[0] * cov[2] - cov[1] * cov[1];
  if (det == 0.0f) {
    culled();
    return;
  }
  const float det_inv = 1.f / det;
  const float ca = cov[2] * det_inv, cb = -cov[1] * det_inv, cc = cov[0] * det_inv;
  const float mid = 0.5f * (cov[0] + cov[2]);
  const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
  const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
  const float rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
  const float px = ndc_to_pix(ppx, a.W), py = ndc_to_pix(ppy, a.H);
  int2 rmin, rmax;
  tile_rect(px, py, (int)rad, a.grid_x, a.grid_y, rmin, rmax);
  if ((rmax.x - rmin.x) * (rmax.y - rmin.y) == 0) {
    culled();
    return;
  }

  float rgb[3];
  if (a.colors_precomp) {
    rgb[0] = a.colors_precomp[3 * g]; rgb[1] = a.colors_precomp[3 * g + 1]; rgb[2] = a.colors_precomp[3 * g + 2];
  } else {
    uint8_t cl;
    sh_fwd(a.D, a.M, p, ld3(a.campos), a.shs, g, rgb, cl);
    a.clamped[g] = cl;
  }
  const float op = a.activate ? act_sigmoid(a.opacities[g]) : a.opacities[g];
  float ex, ey, tq;
  alpha_extent(ca, cb, cc, op, ex, ey, tq);
  float4* rec = reinterpret_cast<float4*>(a.rec + (size_t)REC * g);
  rec[0] = make_float4(px, py, ca, cb);
  rec[1] = make_float4(cc, op, rgb[0], rgb[1]);
  rec[2] = make_float4(rgb[2], pv.z, ex, ey);
  rec[3] = make_float4((float)rad, tq, 0.f, 0.f);
  a.radii[g] = (int)rad;
  a.tiles[g] = (uint32_t)((rmax.y - rmin.y) * (rmax.x - rmin.x));  // the reference's tiles_touched
  // The binning rect: the reference's rect cut down to the tiles whose pixel
  // centres the alpha >= 1/255 ellipse's bounding box (half extents ex, ey,
  // margins included) reaches -- the other instances blend at no pixel.
  // +inf extents keep the reference rect; -inf (never blends) empties it.
  const float fx0 = fminf(fmaxf(ceilf((px - ex - (TILE - 1)) / TILE), (float)rmin.x), (float)rmax.x);
  const float fx1 = fminf(fmaxf(floorf((px + ex) / TILE) + 1.f, (float)rmin.x), (float)rmax.x);
  const float fy0 = fminf(fmaxf(ceilf((py - ey - (TILE - 1)) / TILE), (float)rmin.y), (float)rmax.y);
  const float fy1 = fminf(fmaxf(floorf((py + ey) / TILE) + 1.f, (float)rmin.y), (float)rmax.y);
  // ... and to the camera's tile window (gs_camera tile_*: image sharding)
  const uint16_t* win = batch.win[cam];
  const int bx0 = max((int)fx0, (int)win[0]), by0 = max((int)fy0, (int)win[1]);
  const int bx1 = max(min((int)fx1, (int)win[2]), bx0), by1 = max(min((int)fy1, (int)win[3]), by0);
  a.rect[g] = make_uint4((uint32_t)bx0 | ((uint32_t)by0 << 16), (uint32_t)bx1 | ((uint32_t)by1 << 16),
                         __float_as_uint(pv.z), (uint32_t)((rmax.y - rmin.y) * (rmax.x - rmin.x)));
}

void launch_preprocess_fwd(const PreprocessArgs& a, const CamBatch& cb, hipStream_t s) {
  if (a.P <= 0) return;
  hipLaunchKernelGGL(preprocess_fwd_kernel, dim3((a.P + 255) / 256, cb.C), dim3(256), 0, s, a, cb);
}

__global__ __launch_bounds__(256) void mark_visible_kernel(int P, const float* __restrict__ means3D,
                                                           const float* __restrict__ view,
                                                           uint8_t* __restrict__ present) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= P) return;
  const V3 pv = xf43(view, ld3(means3D + 3 * g));
  present[g] = !(pv.z <= 0.0f);
}

void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t s) {
  if (P <= 0) return;
  hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, view, present);
}

// ------------------------------------------------------------------ backward

// computeColorFromSH backward (backward.cu:20-139): writes dL/dsh (all M
// coefficients, zero beyond the active degree) and adds the view-direction
// term to dmean.
// Gradient store of preprocess_bwd: overwrite, or add to the caller's sums
// (GS_FLAG_ACCUMULATE).
__device__ inline void gput(float* p, float v, int accumulate) { *p = accumulate ? *p + v : v; }

// SH backward; dsh is stored as (value * dRGB) * mk -- the reference's
// `grad * label` rounding (DGR/__init__.py:159-173) -- written or added.
__device__ inline void sh_bwd(int deg, int M, V3 mean, V3 cp, const float* __restrict__ shs, int g,
                              uint8_t clampbits, const float dcolor[3], float* __restrict__ dsh_out,
                              float dmean[3], float mk, int accumulate) {
  const float dox = mean.x - cp.x, doy = mean.y - cp.y, doz = mean.z - cp.z;
  const float len = sqrtf(dox * dox + doy * doy + doz * doz);
  const float x = dox / len, y = doy / len, z = doz / len;
  const float* sh = shs + (size_t)g * M * 3;
  float* ds = dsh_out + (size_t)g * M * 3;
  float dRGB[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) dRGB[ch] = dcolor[ch] * (((clampbits >> ch) & 1) ? 0.0f : 1.0f);
  float ddx[3] = {0, 0, 0}, ddy[3] = {0, 0, 0}, ddz[3] = {0, 0, 0};
  const int ncoef = (deg + 1) * (deg + 1);
  if (!accumulate)
    for (int i = ncoef; i < M; ++i) { ds[3 * i] = 0.f * mk; ds[3 * i + 1] = 0.f * mk; ds[3 * i + 2] = 0.f * mk; }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
#define S(i) sh[3 * (i) + ch]
#define WR(i, v) gput(ds + 3 * (i) + ch, ((v) * dRGB[ch]) * mk, accumulate)
    WR(0, SH_C0);
    if (deg > 0) {
      WR(1, -SH_C1 * y); WR(2, SH_C1 * z); WR(3, -SH_C1 * x);
      ddx[ch] = -SH_C1 * S(3); ddy[ch] = -SH_C1 * S(1); ddz[ch] = SH_C1 * S(2);
      if (deg > 1) {
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        WR(4, SH_C2_0 * xy); WR(5, SH_C2_1 * yz); WR(6, SH_C2_2 * (2.f * zz - xx - yy));
        WR(7, SH_C2_3 * xz); WR(8, SH_C2_4 * (xx - yy));
        ddx[ch] += SH_C2_0 * y * S(4) + SH_C2_2 * 2.f * -x * S(6) + SH_C2_3 * z * S(7) + SH_C2_4 * 2.f * x * S(8);
        ddy[ch] += SH_C2_0 * x * S(4) + SH_C2_1 * z * S(5) + SH_C2_2 * 2.f * -y * S(6) + SH_C2_4 * 2.f * -y * S(8);
        ddz[ch] += SH_C2_1 * y * S(5) + SH_C2_2 * 2.f * 2.f * z * S(6) + SH_C2_3 * x * S(7);
        if (deg > 2) {
          WR(9, SH_C3_0 * y * (3.f * xx - yy)); WR(10, SH_C3_1 * xy * z);
          WR(11, SH_C3_2 * y * (4.f * zz - xx - yy)); WR(12, SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy));
          WR(13, SH_C3_4 * x * (4.f * zz - xx - yy)); WR(14, SH_C3_5 * z * (xx - yy));
          WR(15, SH_C3_6 * x * (xx - 3.f * yy));
          ddx[ch] += (SH_C3_0 * S(9) * 3.f * 2.f * xy + SH_C3_1 * S(10) * yz + SH_C3_2 * S(11) * -2.f * xy +
                      SH_C3_3 * S(12) * -3.f * 2.f * xz + SH_C3_4 * S(13) * (-3.f * xx + 4.f * zz - yy) +
                      SH_C3_5 * S(14) * 2.f * xz + SH_C3_6 * S(15) * 3.f * (xx - yy));
          ddy[ch] += (SH_C3_0 * S(9) * 3.f * (xx - yy) + SH_C3_1 * S(10) * xz +
                      SH_C3_2 * S(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3_3 * S(12) * -3.f * 2.f * yz +
                      SH_C3_4 * S(13) * -2.f * xy + SH_C3_5 * S(14) * -2.f * yz + SH_C3_6 * S(15) * -3.f * 2.f * xy);
          ddz[ch] += (SH_C3_1 * S(10) * xy + SH_C3_2 * S(11) * 4.f * 2.f * yz +
                      SH_C3_3 * S(12) * 3.f * (2.f * zz - xx - yy) + SH_C3_4 * S(13) * 4.f * 2.f * xz +
                      SH_C3_5 * S(14) * (xx - yy));
        }
      }
    }
#undef S
#undef WR
  }
  const float dd0 = ddx[0] * dRGB[0] + ddx[1] * dRGB[1] + ddx[2] * dRGB[2];
  const float dd1 = ddy[0] * dRGB[0] + ddy[1] * dRGB[1] + ddy[2] * dRGB[2];
  const float dd2 = ddz[0] * dRGB[0] + ddz[1] * dRGB[1] + ddz[2] * dRGB[2];
  // dnormvdv (auxiliary.h:107-117)
  const float s2 = dox * dox + doy * doy + doz * doz;
  const float inv = 1.0f / sqrtf(s2 * s2 * s2);
  dmean[0] += ((s2 - dox * dox) * dd0 - doy * dox * dd1 - doz * dox * dd2) * inv;
  dmean[1] += (-dox * doy * dd0 + (s2 - doy * doy) * dd1 - doz * doy * dd2) * inv;
  dmean[2] += (-dox * doz * dd0 - doy * doz * dd1 + (s2 - doz * doz) * dd2) * inv;
}

// computeCov3D backward (backward.cu:295-358).
__device__ inline void cov3d_bwd(V3 scale, float mod, float4 rot, const float d[6], float dscale[3],
                                 float drot[4]) {
  float rc[3][3];
  quat_cols(rot, rc);
  const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
  const float s[3] = {mod * scale.x, mod * scale.y, mod * scale.z};
  float m[3][3];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int k = 0; k < 3; ++k) m[c][k] = s[k] * rc[c][k];
  const float sg[3][3] = {{d[0], 0.5f * d[1], 0.5f * d[2]},
                          {0.5f * d[1], d[3], 0.5f * d[4]},
                          {0.5f * d[2], 0.5f * d[4], d[5]}};
  float dmt[3][3];  // transpose(dL_dM), dL_dM = 2 M dL_dSigma
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int rr = 0; rr < 3; ++rr)
      dmt[rr][c] = 2.0f * (m[0][rr] * sg[c][0] + m[1][rr] * sg[c][1] + m[2][rr] * sg[c][2]);
#pragma unroll
  for (int i = 0; i < 3; ++i) dscale[i] = rc[0][i] * dmt[i][0] + rc[1][i] * dmt[i][1] + rc[2][i] * dmt[i][2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k) dmt[i][k] *= s[i];
  drot[0] = 2 * z * (dmt[0][1] - dmt[1][0]) + 2 * y * (dmt[2][0] - dmt[0][2]) + 2 * x * (dmt[1][2] - dmt[2][1]);
  drot[1] = 2 * y * (dmt[1][0] + dmt[0][1]) + 2 * z * (dmt[2][0] + dmt[0][2]) + 2 * r * (dmt[1][2] - dmt[2][1]) - 4 * x * (dmt[2][2] + dmt[1][1]);
  drot[2] = 2 * x * (dmt[1][0] + dmt[0][1]) + 2 * r * (dmt[2][0] - dmt[0][2]) + 2 * z * (dmt[1][2] + dmt[2][1]) - 4 * y * (dmt[2][2] + dmt[0][0]);
  drot[3] = 2 * r * (dmt[0][1] - dmt[1][0]) + 2 * x * (dmt[2][0] + dmt[0][2]) + 2 * y * (dmt[1][2] + dmt[2][1]) - 4 * z * (dmt[1][1] + dmt[0][0]);
}

// Fused computeCov2DCUDA + preprocessCUDA backward + scatter of the blend
// gradients (the per-Gaussian accumulation record) into the output tensors,
// for every camera of the batch: one thread per Gaussian walks the cameras in
// order and sums their contributions in registers (deterministic, one write
// per output), so a batch costs one pass over the Gaussian state instead of
// C read-modify-write passes.  Every output element is written, so outputs
// need no zero-fill.
constexpr int PB_GROUP = 2;  // cameras whose operands are requested together
// SH: the SH-coefficient backward is compiled in (launched when a.shs is set);
// the precomputed-colour instantiation carries none of its registers.
template <bool SH>
__global__ __launch_bounds__(256) void preprocess_bwd_kernel(PreprocessBwdArgs a, CamBatch cb) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= a.P) return;
  const int ac = a.accumulate;
  const bool masked = a.grad_mask != nullptr;
  const float mk = masked ? a.grad_mask[g] : 1.f;
  const V3 mean = ld3(a.means3D + 3 * g);
  // camera sums (the first camera assigns, so C = 1 is the single-view value)
  float am[2] = {0.f, 0.f}, dcol[3] = {0.f, 0.f, 0.f}, dop = 0.f;
  float dm[3] = {0.f, 0.f, 0.f};
  float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float st_acc = 0.f, st_den = 0.f, st_rad = 0.f;
  bool any_vis = false, sh_written = ac != 0;
  // The cameras are walked in groups of PB_GROUP: every operand of a group
  // (radius, accumulation record, conic, 3D covariance of each camera) is
  // requested before the first of them is used, so the group's loads are in
  // flight together instead of one dependent round trip (radius, then the
  // rest) per camera.  The sums still run camera by camera in order.
  // the 3D covariance: precomputed, or stored by camera 0's preprocess
  // (preprocess_fwd_kernel) -- one read per Gaussian for all cameras
  float c3v[6];
  {
    const float* c3 = a.cov3D_precomp ? a.cov3D_precomp + 6 * g : a.cov3D + 6 * g;
#pragma unroll
    for (int i = 0; i < 6; ++i) c3v[i] = c3[i];
  }
  for (int cg = 0; cg < cb.C; cg += PB_GROUP) {
    int radk[PB_GROUP];
    float acck[PB_GROUP][A_FEAT], cck[PB_GROUP];
    float4 conk[PB_GROUP];
#pragma unroll
    for (int k = 0; k < PB_GROUP; ++k) {
      const int c = cg + k < cb.C ? cg + k : cb.C - 1;  // a short last group re-reads a valid camera
      const float* acc = a.acc + ((size_t)c * a.P + g) * ACC_STRIDE;
#pragma unroll
      for (int i = 0; i < A_FEAT; ++i) acck[k][i] = acc[i];
      radk[k] = a.radii[(size_t)c * a.P + g];
      const float* rec = shift_bytes(a.rec, c * cb.geom_stride) + (size_t)REC * g;
      conk[k] = reinterpret_cast<const float4*>(rec)[0];  // x, y, a, b
      cck[k] = rec[R_CC];
    }
#pragma unroll
  for (int k = 0; k < PB_GROUP; ++k) {
    const int c = cg + k;
    if (c >= cb.C) break;
    const bool first = c == 0;
    auto add = [&](float& sum, float v) { sum = first ? v : sum + v; };
    const float* acc = acck[k];
    const int rad = radk[k];
    const bool vis = rad > 0;
    // blend gradients -> output tensors (zero for culled Gaussians: never touched)
    // dL/dmean2D = sum over pixels of dL/dG * dG/d(offset) * ndc scale
    // (CR/backward.cu:616-621): from the blend kernel's basis sums (AccField),
    // the conic and ddelx_dx = 0.5 W, ddely_dy = 0.5 H (:520-521).
    float am0 = 0.f, am1 = 0.f;
    if (vis) {
      const float4 con = conk[k];
      const float cc = cck[k];
      const float sex = acc[A_MX], sey = acc[A_MY];
      am0 = (-con.z * sex - con.w * sey) * (0.5f * (float)a.W);
      am1 = (-cc * sey - con.w * sex) * (0.5f * (float)a.H);
    }
    add(am[0], am0);
    add(am[1], am1);
    // densification statistics of this view (external.py:136-140: the norm of
    // the view's own means2D gradient, as gs_optim.hip's statistics do;
    // train.py:288-290: the max screen radius); unseen Gaussians add nothing
    add(st_acc, vis ? sqrtf(am0 * am0 + am1 * am1) : 0.f);
    add(st_den, vis ? 1.f : 0.f);
    st_rad = fmaxf(st_rad, vis ? (float)rad : 0.f);
    const float dcol_c[3] = {acc[A_R], acc[A_G], acc[A_B]};
    add(dcol[0], dcol_c[0]);
    add(dcol[1], dcol_c[1]);
    add(dcol[2], dcol_c[2]);
    add(dop, acc[A_OP]);
    if (!vis) continue;
    const float* view = cb.view + 16 * c;
    const float* pr = cb.proj + 16 * c;
    // the camera scalars exactly as the binding passed them (Q2 in reference
    // mode: the Python wrapper's swapped order, DGR/__init__.py:130-133)
    const float c_x = cb.c_x[c], c_y = cb.c_y[c], tan_fovx = cb.tanx[c], tan_fovy = cb.tany[c];
    const float focal_y = (float)a.H / (2.0f * tan_fovy);  // CR/rasterizer_impl.cu:398-399
    const float focal_x = (float)a.W / (2.0f * tan_fovx);
    // dL/dconic = -1/2 sum e (dx^2, dx dy, dy^2) (CR/backward.cu:622-624)
    const float dcx = -0.5f * acc[A_CA], dcy = -0.5f * acc[A_CB], dcz = -0.5f * acc[A_CC];
    Ewa e;
    ewa_setup(mean, view, a.W, a.H, c_x, c_y, focal_x, focal_y, tan_fovx, tan_fovy, e);
    float xg, yg;
    if (a.compat == COMPAT_REFERENCE) {  // Q3
      xg = (e.txtz < e.lxn || e.txtz > e.lxp) ? 0.f : 1.f;
      yg = (e.tytz < e.lyn || e.tytz > e.lyp) ? 0.f : 1.f;
    } else {
      xg = (e.txtz < -e.lxn || e.txtz > e.lxp) ? 0.f : 1.f;
      yg = (e.tytz < -e.lyn || e.tytz > e.lyp) ? 0.f : 1.f;
    }
    float cov[3];
    ewa_cov2d(e, c3v, cov);
    const float ca = cov[0], cb2 = cov[1], cc = cov[2];
    const float denom = ca * cc - cb2 * cb2;
    float da = 0, db = 0, dc = 0;
    float dcv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float d2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float(&A)[2][3] = e.a;
    if (d2inv != 0) {
      da = d2inv * (-cc * cc * dcx + 2 * cb2 * cc * dcy + (denom - ca * cc) * dcz);
      dc = d2inv * (-ca * ca * dcz + 2 * ca * cb2 * dcy + (denom - ca * cc) * dcx);
      db = d2inv * 2 * (cb2 * cc * dcx - (denom + 2 * cb2 * cb2) * dcy + ca * cb2 * dcz);
      dcv[0] = (A[0][0] * A[0][0] * da + A[0][0] * A[1][0] * db + A[1][0] * A[1][0] * dc);
      dcv[3] = (A[0][1] * A[0][1] * da + A[0][1] * A[1][1] * db + A[1][1] * A[1][1] * dc);
      dcv[5] = (A[0][2] * A[0][2] * da + A[0][2] * A[1][2] * db + A[1][2] * A[1][2] * dc);
      dcv[1] = 2 * A[0][0] * A[0][1] * da + (A[0][0] * A[1][1] + A[0][1] * A[1][0]) * db + 2 * A[1][0] * A[1][1] * dc;
      dcv[2] = 2 * A[0][0] * A[0][2] * da + (A[0][0] * A[1][2] + A[0][2] * A[1][0]) * db + 2 * A[1][0] * A[1][2] * dc;
      dcv[4] = 2 * A[0][2] * A[0][1] * da + (A[0][1] * A[1][2] + A[0][2] * A[1][1]) * db + 2 * A[1][1] * A[1][2] * dc;
    }
    const float V[3][3] = {{c3v[0], c3v[1], c3v[2]}, {c3v[1], c3v[3], c3v[4]}, {c3v[2], c3v[4], c3v[5]}};
    float dT0[3], dT1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float r0 = A[0][0] * V[k][0] + A[0][1] * V[k][1] + A[0][2] * V[k][2];
      const float r1 = A[1][0] * V[k][0] + A[1][1] * V[k][1] + A[1][2] * V[k][2];
      dT0[k] = 2 * r0 * da + r1 * db;
      dT1[k] = 2 * r1 * dc + r0 * db;
    }
    const float* v = view;
    const float dJ00 = v[0] * dT0[0] + v[4] * dT0[1] + v[8] * dT0[2];
    const float dJ02 = v[2] * dT0[0] + v[6] * dT0[1] + v[10] * dT0[2];
    const float dJ11 = v[1] * dT1[0] + v[5] * dT1[1] + v[9] * dT1[2];
    const float dJ12 = v[2] * dT1[0] + v[6] * dT1[1] + v[10] * dT1[2];
    const float tz = 1.f / e.t[2], tz2 = tz * tz, tz3 = tz2 * tz;
    const float hx = focal_x, hy = focal_y;
    const float dtx = xg * -hx * tz2 * dJ02;
    const float dty = yg * -hy * tz2 * dJ12;
    const float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * e.t[0]) * tz3 * dJ02 + (2 * hy * e.t[1]) * tz3 * dJ12;
    float dmc[3];
    dmc[0] = v[0] * dtx + v[1] * dty + v[2] * dtz;
    dmc[1] = v[4] * dtx + v[5] * dty + v[6] * dtz;
    dmc[2] = v[8] * dtx + v[9] * dty + v[10] * dtz;
    // mean2D and depth contributions (backward.cu:389-420)
    const float4 mh = xf44(pr, mean);
    const float mw = 1.0f / (mh.w + 0.0000001f);
    const float mul1 = (pr[0] * mean.x + pr[4] * mean.y + pr[8] * mean.z + pr[12]) * mw * mw;
    const float mul2 = (pr[1] * mean.x + pr[5] * mean.y + pr[9] * mean.z + pr[13]) * mw * mw;
    dmc[0] += (pr[0] * mw - pr[3] * mul1) * am0 + (pr[1] * mw - pr[3] * mul2) * am1;
    dmc[1] += (pr[4] * mw - pr[7] * mul1) * am0 + (pr[5] * mw - pr[7] * mul2) * am1;
    dmc[2] += (pr[8] * mw - pr[11] * mul1) * am0 + (pr[9] * mw - pr[11] * mul2) * am1;
    const float mul3 = v[2] * mean.x + v[6] * mean.y + v[10] * mean.z + v[14];
    const float dd = acc[A_DEPTH];
    dmc[0] += (v[2] - v[3] * mul3) * dd;
    dmc[1] += (v[6] - v[7] * mul3) * dd;
    dmc[2] += (v[10] - v[11] * mul3) * dd;
    if (SH && a.shs) {
      const uint8_t* clamped = shift_bytes(a.clamped, c * cb.geom_stride);
      sh_bwd(a.D, a.M, mean, ld3(cb.campos + 3 * c), a.shs, g, clamped[g], dcol_c, a.dsh, dmc, mk,
             sh_written ? 1 : 0);
      sh_written = true;
    }
    // the first camera that sees the Gaussian assigns, the later ones add
#pragma unroll
    for (int i = 0; i < 3; ++i) dm[i] = any_vis ? dm[i] + dmc[i] : dmc[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) dcov[i] = any_vis ? dcov[i] + dcv[i] : dcv[i];
    any_vis = true;
  }
  }
  float dscale[3] = {0.f, 0.f, 0.f}, drot[4] = {0.f, 0.f, 0.f, 0.f};
  const int act = a.activate;
  V3 sc{0.f, 0.f, 0.f};
  if (any_vis && a.scales) {
    sc = scale_of(a.scales, g, act);
    cov3d_bwd(sc, a.scale_modifier, rotation_of(a.rotations, g, act), dcov, dscale, drot);
  }
  gput(a.dmeans2D + 3 * g, am[0], ac); gput(a.dmeans2D + 3 * g + 1, am[1], ac);
  if (!ac) a.dmeans2D[3 * g + 2] = 0.f;
  if (a.st_accum) gput(a.st_accum + g, st_acc, ac);
  if (a.st_denom) gput(a.st_denom + g, st_den, ac);
  if (a.st_maxrad) a.st_maxrad[g] = ac ? fmaxf(a.st_maxrad[g], st_rad) : st_rad;
  // Q12 label mask (DGR/__init__.py:159-173), applied at store time exactly as
  // the reference's elementwise `grad * label` (the chain rule uses unmasked dcol).
  gput(a.dcolors + 3 * g, dcol[0] * mk, ac); gput(a.dcolors + 3 * g + 1, dcol[1] * mk, ac);
  gput(a.dcolors + 3 * g + 2, dcol[2] * mk, ac);
  if (act) {
    // through the activations (the label mask applies to the activated
    // gradients, then autograd's backward of params2rendervar)
    const float y = act_sigmoid(a.opacities[g]);
    gput(a.dopacity + g, ((dop * mk) * (1.0f - y)) * y, ac);
  } else {
    gput(a.dopacity + g, dop * mk, ac);
  }
  if (!sh_written && a.M > 0) {  // no SH gradient: zeros (masked like the rest)
    float* ds = a.dsh + (size_t)g * a.M * 3;
    for (int i = 0; i < 3 * a.M; ++i) ds[i] = 0.f * mk;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) gput(a.dmeans3D + 3 * g + i, dm[i] * mk, ac);
#pragma unroll
  for (int i = 0; i < 6; ++i) gput(a.dcov3D + 6 * g + i, dcov[i] * mk, ac);
  if (act && a.scales) {
    const float sv[3] = {sc.x, sc.y, sc.z};
    // an unseen Gaussian keeps zero gradients (sc is never evaluated for it)
#pragma unroll
    for (int i = 0; i < 3; ++i) gput(a.dscales + 3 * g + i, any_vis ? (dscale[i] * mk) * sv[i] : 0.f * mk, ac);
    float4 dq = make_float4(drot[0] * mk, drot[1] * mk, drot[2] * mk, drot[3] * mk);
    if (any_vis) dq = act_normalize_bwd(reinterpret_cast<const float4*>(a.rotations)[g], dq);
    drot[0] = dq.x; drot[1] = dq.y; drot[2] = dq.z; drot[3] = dq.w;
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) gput(a.dscales + 3 * g + i, dscale[i] * mk, ac);
#pragma unroll
    for (int i = 0; i < 4; ++i) drot[i] = drot[i] * mk;
  }
  if (ac) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a.drot[4 * g + i] += drot[i];
  } else {
    reinterpret_cast<float4*>(a.drot)[g] = make_float4(drot[0], drot[1], drot[2], drot[3]);
  }
}

void launch_preprocess_bwd(const PreprocessBwdArgs& a, const CamBatch& cb, hipStream_t s) {
  if (a.P <= 0) return;
  if (a.shs)
    hipLaunchKernelGGL(preprocess_bwd_kernel<true>, dim3((a.P + 255) / 256), dim3(256), 0, s, a, cb);
  else
    hipLaunchKernelGGL(preprocess_bwd_kernel<false>, dim3((a.P + 255) / 256), dim3(256), 0, s, a, cb);
}

}  // namespace gs
