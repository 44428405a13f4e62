/*
 * gs_oracle.c -- CPU restatement of the reference differentiable Gaussian
 * rasterizer.  TEST INFRASTRUCTURE ONLY: it is the checker the HIP kernels are
 * compared against (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline
 * leg).  Nothing in the product package links, loads or calls it.
 *
 * Reference = submodules_fsgs/diff-gaussian-rasterization-confidence/
 *   (abbreviated DGR/, and CR/ = DGR/cuda_rasterizer/).
 *
 * Parity pinning (see DESIGN.md "Oracle"): the reference CUDA path cannot be
 * compiled in this image (it needs cuda_runtime.h / cooperative_groups / cub,
 * and stand-in headers are not allowed), and the reference repository ships no
 * tests or golden vectors.  This restatement is pinned by (a) the reference's
 * own Python SH evaluator utils/sh_utils.py:eval_sh and projection helpers
 * (fixtures in tests/golden/), (b) closed-form known-answer tests derived from
 * the reference formulas, (c) finite-difference gradient checks in the
 * "fixed" compat mode.  Everything else is "parity partially pinned".
 *
 * Arithmetic is plain IEEE fp32 (built with -ffp-contract=off), following the
 * reference's expression order where the reference defines one.  Every
 * function names the reference lines it restates.
 *
 * Compat modes (see DESIGN.md "Quirks"):
 *   GS_COMPAT_REFERENCE (0): reproduce the as-shipped numerics
 *       Q1 out_alpha never written (stays 0)           CR/forward.cu:397-407
 *       Q3 x/y_grad_mul compare against +lim_neg        CR/backward.cu:191-192
 *       Q4 feature background = bg[ch] for ch<3, else 0 CR/forward.cu:405-406
 *       Q5 feature term of dL/dalpha uses a never-written
 *          scratch (zero) -> contributes nothing        CR/backward.cu:596-612
 *   GS_COMPAT_FIXED (1): out_alpha = 1 - T, -lim_neg clamp test, no feature
 *       background, feature channels feed dL/dopacity.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GS_COMPAT_REFERENCE 0
#define GS_COMPAT_FIXED 1
#define TILE 16 /* CR/config.h:18-19 BLOCK_X = BLOCK_Y = 16 */

static const float SH_C0 = 0.28209479177387814f; /* CR/auxiliary.h:22-39 */
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f,
                               0.31539156525252005f, -1.0925484305920792f,
                               0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f,
                               -0.4570457994644658f, 0.3731763325901154f,
                               -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

int or_version(void) { return 1; }

/* ---------------------------------------------------------------- helpers */

/* transformPoint4x3 / transformPoint4x4 / transformVec4x3Transpose,
 * CR/auxiliary.h:58-97.  Matrices are column-major float[16]. */
static void xf43(const float *m, const float p[3], float o[3]) {
  o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
  o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
  o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
static void xf44(const float *m, const float p[3], float o[4]) {
  o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
  o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
  o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
  o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}

/* ndc2Pix, CR/auxiliary.h:41-44: evaluated in double (double literals). */
static float ndc_to_pix(float v, int S) {
  return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

/* getRect, CR/auxiliary.h:46-56. */
static void tile_rect(float px, float py, int r, int gx, int gy, int rmin[2],
                      int rmax[2]) {
  int a;
  a = (int)((px - (float)r) / (float)TILE); a = a > 0 ? a : 0; rmin[0] = a < gx ? a : gx;
  a = (int)((py - (float)r) / (float)TILE); a = a > 0 ? a : 0; rmin[1] = a < gy ? a : gy;
  /* p + r + BLOCK - 1 evaluates as ((p + r) + 16) - 1 in float */
  a = (int)((((px + (float)r) + (float)TILE) - 1.0f) / (float)TILE); a = a > 0 ? a : 0; rmax[0] = a < gx ? a : gx;
  a = (int)((((py + (float)r) + (float)TILE) - 1.0f) / (float)TILE); a = a > 0 ? a : 0; rmax[1] = a < gy ? a : gy;
}

/* Quaternion (r,x,y,z) -> the glm columns of R, CR/forward.cu:137-149
 * (Q7: the quaternion is NOT normalised). rc[c][k] = column c, row k. */
static void quat_cols(const float q[4], float rc[3][3]) {
  float r = q[0], x = q[1], y = q[2], z = q[3];
  rc[0][0] = 1.f - 2.f * (y * y + z * z); rc[0][1] = 2.f * (x * y - r * z); rc[0][2] = 2.f * (x * z + r * y);
  rc[1][0] = 2.f * (x * y + r * z); rc[1][1] = 1.f - 2.f * (x * x + z * z); rc[1][2] = 2.f * (y * z - r * x);
  rc[2][0] = 2.f * (x * z - r * y); rc[2][1] = 2.f * (y * z + r * x); rc[2][2] = 1.f - 2.f * (x * x + y * y);
}

/* computeCov3D (forward), CR/forward.cu:129-163:  Sigma = (S R)^T (S R),
 * M[c][k] = mod*s_k * R[c][k]; Sigma[a][b] = sum_k M[a][k] M[b][k]. */
static void cov3d_fwd(const float s[3], float mod, const float q[4], float out[6]) {
  float rc[3][3], m[3][3];
  quat_cols(q, rc);
  float sx = mod * s[0], sy = mod * s[1], sz = mod * s[2];
  for (int c = 0; c < 3; ++c) {
    m[c][0] = sx * rc[c][0]; m[c][1] = sy * rc[c][1]; m[c][2] = sz * rc[c][2];
  }
#define DOT3(a, b) (m[a][0] * m[b][0] + m[a][1] * m[b][1] + m[a][2] * m[b][2])
  out[0] = DOT3(0, 0); out[1] = DOT3(0, 1); out[2] = DOT3(0, 2);
  out[3] = DOT3(1, 1); out[4] = DOT3(1, 2); out[5] = DOT3(2, 2);
#undef DOT3
}

/* Screen-space limits and the projective Jacobian rows shared by the forward
 * (CR/forward.cu:75-124) and backward (CR/backward.cu:144-211) EWA code.
 * a[0], a[1] = rows of J*R (the glm T columns 0 and 1). */
typedef struct {
  float t[3];        /* view-space mean after clamping */
  float txtz, tytz;  /* unclamped t.x/t.z, t.y/t.z */
  float lxp, lxn, lyp, lyn;
  float j00, j02, j11, j12;
  float a[2][3];
} ewa_t;

static void ewa_setup(const float mean[3], const float *view, int W, int H,
                      float cx, float cy, float fx, float fy, float tfx,
                      float tfy, ewa_t *e) {
  float t[3];
  xf43(view, mean, t);
  /* "added" asymmetric limits (Q9), CR/forward.cu:87-90 */
  e->lxp = ((float)W - cx) / fx + 0.3f * tfx;
  e->lxn = cx / fx + 0.3f * tfx;
  e->lyp = ((float)H - cy) / fy + 0.3f * tfy;
  e->lyn = cy / fy + 0.3f * tfy;
  e->txtz = t[0] / t[2];
  e->tytz = t[1] / t[2];
  /* the symmetric 1.3*tan clamp (CR/forward.cu:95-96) is overwritten: dead */
  t[0] = fminf(e->lxp, fmaxf(-e->lxn, e->txtz)) * t[2];
  t[1] = fminf(e->lyp, fmaxf(-e->lyn, e->tytz)) * t[2];
  e->t[0] = t[0]; e->t[1] = t[1]; e->t[2] = t[2];
  e->j00 = fx / t[2];
  e->j02 = -(fx * t[0]) / (t[2] * t[2]);
  e->j11 = fy / t[2];
  e->j12 = -(fy * t[1]) / (t[2] * t[2]);
  /* T = W * J in glm; T[0][r] = view[4r]*j00 + view[1+4r]*0 + view[2+4r]*j02 */
  for (int r = 0; r < 3; ++r) {
    e->a[0][r] = view[4 * r] * e->j00 + view[1 + 4 * r] * 0.0f + view[2 + 4 * r] * e->j02;
    e->a[1][r] = view[4 * r] * 0.0f + view[1 + 4 * r] * e->j11 + view[2 + 4 * r] * e->j12;
  }
}

/* cov2D = T^T Sigma^T T, upper 2x2, plus the 0.3 low-pass.  Returns (a,b,c). */
static void ewa_cov2d(const ewa_t *e, const float *c3, float out[3]) {
  float v[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
  float u[2][3];
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 3; ++k)
      u[i][k] = e->a[i][0] * v[0][k] + e->a[i][1] * v[1][k] + e->a[i][2] * v[2][k];
  float a = u[0][0] * e->a[0][0] + u[0][1] * e->a[0][1] + u[0][2] * e->a[0][2];
  float b = u[1][0] * e->a[0][0] + u[1][1] * e->a[0][1] + u[1][2] * e->a[0][2];
  float c = u[1][0] * e->a[1][0] + u[1][1] * e->a[1][1] + u[1][2] * e->a[1][2];
  out[0] = a + 0.3f; out[1] = b; out[2] = c + 0.3f;
}

/* computeColorFromSH (forward), CR/forward.cu:20-71. */
static void sh_fwd(int deg, int M, const float *mean, const float *campos,
                   const float *sh_all, int g, float rgb[3], uint8_t cl[3]) {
  float dir[3] = {mean[0] - campos[0], mean[1] - campos[1], mean[2] - campos[2]};
  float len = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
  dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
  const float *sh = sh_all + (size_t)g * M * 3;
  for (int ch = 0; ch < 3; ++ch) {
#define S(i) sh[3 * (i) + ch]
    float x = dir[0], y = dir[1], z = dir[2];
    float res = SH_C0 * S(0);
    if (deg > 0) {
      res = res - SH_C1 * y * S(1) + SH_C1 * z * S(2) - SH_C1 * x * S(3);
      if (deg > 1) {
        float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        res = res + SH_C2[0] * xy * S(4) + SH_C2[1] * yz * S(5) +
              SH_C2[2] * (2.0f * zz - xx - yy) * S(6) + SH_C2[3] * xz * S(7) +
              SH_C2[4] * (xx - yy) * S(8);
        if (deg > 2) {
          res = res + SH_C3[0] * y * (3.0f * xx - yy) * S(9) +
                SH_C3[1] * xy * z * S(10) +
                SH_C3[2] * y * (4.0f * zz - xx - yy) * S(11) +
                SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                SH_C3[4] * x * (4.0f * zz - xx - yy) * S(13) +
                SH_C3[5] * z * (xx - yy) * S(14) +
                SH_C3[6] * x * (xx - 3.0f * yy) * S(15);
        }
      }
    }
#undef S
    res += 0.5f;
    cl[ch] = res < 0.0f;
    rgb[ch] = res > 0.0f ? res : 0.0f; /* glm::max(result, 0) */
  }
}

/* ------------------------------------------------------------- forward */

/* checkFrustum / in_frustum, CR/rasterizer_impl.cu:54-66, CR/auxiliary.h:145-170
 * (Q8: only the p_view.z <= 0 test survives). */
void or_mark_visible(int P, const float *means3D, const float *view,
                     const float *proj, uint8_t *present) {
  (void)proj;
  for (int g = 0; g < P; ++g) {
    float pv[3];
    xf43(view, means3D + 3 * g, pv);
    present[g] = !(pv[2] <= 0.0f);
  }
}

/* preprocessCUDA<3> (forward), CR/forward.cu:166-269.  focal from
 * CR/rasterizer_impl.cu:227-228.  Returns 1 if a point was culled while
 * `prefiltered` was set (the reference traps, CR/auxiliary.h:162-166). */
int or_preprocess(int P, int D, int M, const float *means3D, const float *scales,
                  float scale_modifier, const float *rotations,
                  const float *opacities, const float *shs,
                  const float *cov3D_precomp, const float *colors_precomp,
                  const float *view, const float *proj, const float *campos,
                  int W, int H, float c_x, float c_y, float tan_fovx,
                  float tan_fovy, int prefiltered, int *radii, float *means2D,
                  float *depths, float *cov3D, float *rgb, float *conic_opacity,
                  uint32_t *tiles_touched, uint8_t *clamped) {
  const float fy = (float)H / (2.0f * tan_fovy);
  const float fx = (float)W / (2.0f * tan_fovx);
  const int gx = (W + TILE - 1) / TILE, gy = (H + TILE - 1) / TILE;
  int trapped = 0;
  for (int g = 0; g < P; ++g) {
    radii[g] = 0;
    tiles_touched[g] = 0;
    const float *p = means3D + 3 * g;
    float pv[3];
    xf43(view, p, pv);
    if (pv[2] <= 0.0f) {
      if (prefiltered) trapped = 1;
      continue;
    }
    float ph[4];
    xf44(proj, p, ph);
    float pw = 1.0f / (ph[3] + 0.0000001f);
    float pp[2] = {ph[0] * pw, ph[1] * pw};
    const float *c3;
    if (cov3D_precomp) {
      c3 = cov3D_precomp + 6 * g;
    } else {
      cov3d_fwd(scales + 3 * g, scale_modifier, rotations + 4 * g, cov3D + 6 * g);
      c3 = cov3D + 6 * g;
    }
    ewa_t e;
    ewa_setup(p, view, W, H, c_x, c_y, fx, fy, tan_fovx, tan_fovy, &e);
    float cov[3];
    ewa_cov2d(&e, c3, cov);
    float det = cov[0] * cov[2] - cov[1] * cov[1];
    if (det == 0.0f) continue;
    float det_inv = 1.f / det;
    float conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
    float mid = 0.5f * (cov[0] + cov[2]);
    float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    float rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    float px = ndc_to_pix(pp[0], W), py = ndc_to_pix(pp[1], H);
    int rmin[2], rmax[2];
    tile_rect(px, py, (int)rad, gx, gy, rmin, rmax);
    if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
    if (!colors_precomp) sh_fwd(D, M, p, campos, shs, g, rgb + 3 * g, clamped + 3 * g);
    depths[g] = pv[2];
    radii[g] = (int)rad;
    means2D[2 * g] = px; means2D[2 * g + 1] = py;
    conic_opacity[4 * g + 0] = conic[0];
    conic_opacity[4 * g + 1] = conic[1];
    conic_opacity[4 * g + 2] = conic[2];
    conic_opacity[4 * g + 3] = opacities[g];
    tiles_touched[g] = (uint32_t)((rmax[1] - rmin[1]) * (rmax[0] - rmin[0]));
  }
  return trapped;
}

typedef struct { uint64_t key; uint32_t pos; } kv_t;
static int kv_cmp(const void *a, const void *b) {
  const kv_t *x = (const kv_t *)a, *y = (const kv_t *)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

/* getHigherMsb, CR/rasterizer_impl.cu:35-50. */
uint32_t or_higher_msb(uint32_t n) {
  uint32_t msb = sizeof(n) * 4, step = msb;
  while (step > 1) {
    step /= 2;
    if (n >> msb) msb += step; else msb -= step;
  }
  if (n >> msb) msb++;
  return msb;
}

/* Binning: InclusiveSum (CR/rasterizer_impl.cu:283), duplicateWithKeys
 * (:70-111), stable radix SortPairs on bits [0, 32+msb) (:306-314) -- the
 * stable sort is restated as a sort by (key, unsorted position) -- and
 * identifyTileRanges (:116-138, after the memset at :316).
 * ranges: uint32 pairs, one per tile.  keys_out may be NULL. */
int64_t or_binning(int P, const float *means2D, const float *depths,
                   const int *radii, const uint32_t *tiles_touched, int W, int H,
                   uint32_t *point_list, uint64_t *keys_out, uint32_t *ranges) {
  const int gx = (W + TILE - 1) / TILE, gy = (H + TILE - 1) / TILE;
  uint64_t L = 0;
  for (int g = 0; g < P; ++g) L += tiles_touched[g];
  kv_t *kv = (kv_t *)malloc(sizeof(kv_t) * (L ? L : 1));
  uint32_t *vals = (uint32_t *)malloc(sizeof(uint32_t) * (L ? L : 1));
  uint64_t off = 0;
  for (int g = 0; g < P; ++g) {
    if (radii[g] > 0) {
      int rmin[2], rmax[2];
      tile_rect(means2D[2 * g], means2D[2 * g + 1], radii[g], gx, gy, rmin, rmax);
      uint32_t dbits;
      memcpy(&dbits, depths + g, 4);
      for (int y = rmin[1]; y < rmax[1]; ++y)
        for (int x = rmin[0]; x < rmax[0]; ++x) {
          kv[off].key = ((uint64_t)(uint32_t)(y * gx + x) << 32) | dbits;
          kv[off].pos = (uint32_t)off;
          vals[off] = (uint32_t)g;
          off++;
        }
    }
  }
  qsort(kv, L, sizeof(kv_t), kv_cmp);
  memset(ranges, 0, sizeof(uint32_t) * 2 * (size_t)gx * gy);
  for (uint64_t i = 0; i < L; ++i) {
    point_list[i] = vals[kv[i].pos];
    if (keys_out) keys_out[i] = kv[i].key;
    uint32_t cur = (uint32_t)(kv[i].key >> 32);
    if (i == 0) ranges[2 * cur] = 0;
    else {
      uint32_t prev = (uint32_t)(kv[i - 1].key >> 32);
      if (cur != prev) { ranges[2 * prev + 1] = (uint32_t)i; ranges[2 * cur] = (uint32_t)i; }
    }
    if (i == L - 1) ranges[2 * cur + 1] = (uint32_t)L;
  }
  free(kv);
  free(vals);
  return (int64_t)L;
}

/* renderCUDA<3> (forward), CR/forward.cu:274-408.  One pass per pixel over
 * its tile's sorted list.  colors: P x 3, feats: P x F (may be NULL if F==0). */
void or_render_fwd(int W, int H, const uint32_t *ranges,
                   const uint32_t *point_list, const float *means2D,
                   const float *colors, const float *feats, int F,
                   const float *depths, const float *conic_opacity,
                   const float *bg, int compat, float *out_color,
                   float *out_feature, float *out_depth, float *out_alpha,
                   uint32_t *n_contrib) {
  const int gx = (W + TILE - 1) / TILE, gy = (H + TILE - 1) / TILE;
  const size_t HW = (size_t)H * W;
  float *sf = (float *)calloc(F > 0 ? F : 1, sizeof(float));
  for (int ty = 0; ty < gy; ++ty)
    for (int tx = 0; tx < gx; ++tx) {
      const uint32_t r0 = ranges[2 * (ty * gx + tx)], r1 = ranges[2 * (ty * gx + tx) + 1];
      for (int ly = 0; ly < TILE; ++ly)
        for (int lx = 0; lx < TILE; ++lx) {
          const int px = tx * TILE + lx, py = ty * TILE + ly;
          if (px >= W || py >= H) continue;
          const float pfx = (float)px, pfy = (float)py;
          float T = 1.0f, C[3] = {0, 0, 0}, Dp = 0.0f;
          uint32_t contributor = 0, last = 0;
          for (int ch = 0; ch < F; ++ch) sf[ch] = 0.0f;
          for (uint32_t i = r0; i < r1; ++i) {
            contributor++;
            const uint32_t g = point_list[i];
            const float dx = means2D[2 * g] - pfx, dy = means2D[2 * g + 1] - pfy;
            const float *co = conic_opacity + 4 * g;
            float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
            if (power > 0.0f) continue;
            float alpha = fminf(0.99f, co[3] * expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            float test_T = T * (1 - alpha);
            if (test_T < 0.0001f) break; /* done = true; nothing further blends */
            for (int ch = 0; ch < 3; ++ch) C[ch] += colors[3 * g + ch] * alpha * T;
            Dp += depths[g] * alpha * T;
            for (int ch = 0; ch < F; ++ch) sf[ch] += feats[(size_t)g * F + ch] * alpha * T;
            T = test_T;
            last = contributor;
          }
          const size_t pix = (size_t)py * W + px;
          n_contrib[pix] = last;
          for (int ch = 0; ch < 3; ++ch) out_color[ch * HW + pix] = C[ch] + T * bg[ch];
          out_depth[pix] = Dp;
          for (int ch = 0; ch < F; ++ch) {
            float b = (compat == GS_COMPAT_REFERENCE && ch < 3) ? bg[ch] : 0.0f;
            out_feature[ch * HW + pix] = sf[ch] + T * b;
          }
          if (compat != GS_COMPAT_REFERENCE) out_alpha[pix] = 1.0f - T;
        }
    }
  free(sf);
}

/* Pixel visiting order of or_render_bwd (NULL: tile by tile, row-major inside
 * a tile).  The per-Gaussian gradient sums are fp32 additions in pixel order,
 * as the reference's atomicAdd calls are in arrival order; a permuted order
 * measures how far fp32 summation order alone moves them (the envelope the
 * GPU's differences are judged against, tests/test_gpu_envelope.py). */
static const uint32_t *g_pix_order = NULL;
static int64_t g_pix_order_n = 0;
void or_set_pixel_order(const uint32_t *order, int64_t n) {
  g_pix_order = order;
  g_pix_order_n = order ? n : 0;
}

/* renderCUDA<3> (backward), CR/backward.cu:432-652.  Per-pixel reverse walk.
 * Gradients are accumulated (+=) into caller-zeroed arrays:
 *   dmean2D P x 3 (x,y), dconic P x 4 (x,y,w), dopacity P, dcolors P x 3,
 *   dsemantic P x F, ddepths P. */
void or_render_bwd(int W, int H, const uint32_t *ranges,
                   const uint32_t *point_list, const float *bg,
                   const float *means2D, const float *conic_opacity,
                   const float *colors, const float *feats, int F,
                   const float *depths, const float *alphas,
                   const uint32_t *n_contrib, const float *dL_dpix,
                   const float *dL_dfeat, const float *dL_ddepth_pix,
                   const float *dL_dalpha_pix, int compat, float *dmean2D,
                   float *dconic, float *dopacity, float *dcolors,
                   float *dsemantic, float *ddepths) {
  const int gx = (W + TILE - 1) / TILE, gy = (H + TILE - 1) / TILE;
  const size_t HW = (size_t)H * W;
  const float ddelx_dx = (float)(0.5 * W), ddely_dy = (float)(0.5 * H);
  const int Fa = F > 0 ? F : 1;
  float *acc_f = (float *)malloc(sizeof(float) * Fa);
  float *last_f = (float *)malloc(sizeof(float) * Fa);
  float *dlf = (float *)malloc(sizeof(float) * Fa);
  const int permuted = g_pix_order != NULL && g_pix_order_n == (int64_t)HW;
  for (int ty = 0; ty < gy; ++ty)
    for (int tx = 0; tx < gx; ++tx) {
      for (int ly = 0; ly < TILE; ++ly)
        for (int lx = 0; lx < TILE; ++lx) {
          int px = tx * TILE + lx, py = ty * TILE + ly;
          if (px >= W || py >= H) continue;
          if (permuted) { /* visit the pixels in the caller's order instead */
            const size_t q = g_pix_order[(size_t)py * W + px];
            px = (int)(q % (size_t)W);
            py = (int)(q / (size_t)W);
          }
          const int tile = (py / TILE) * gx + px / TILE;
          const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
          const size_t pix = (size_t)py * W + px;
          const float pfx = (float)px, pfy = (float)py;
          const float T_final = 1 - alphas[pix];
          float T = T_final;
          const uint32_t last_contrib = n_contrib[pix];
          float acc_rec[3] = {0, 0, 0}, last_color[3] = {0, 0, 0}, dLp[3];
          float acc_depth = 0, last_depth = 0, acc_alpha = 0, last_alpha = 0;
          for (int ch = 0; ch < 3; ++ch) dLp[ch] = dL_dpix[ch * HW + pix];
          for (int ch = 0; ch < F; ++ch) { acc_f[ch] = 0; last_f[ch] = 0; dlf[ch] = dL_dfeat[ch * HW + pix]; }
          const float dLd = dL_ddepth_pix[pix];
          float dLa = dL_dalpha_pix[pix];
          for (uint32_t k = r1 - r0; k-- > 0;) {
            if (k >= last_contrib) continue; /* contributor >= last_contributor */
            const uint32_t g = point_list[r0 + k];
            const float dx = means2D[2 * g] - pfx, dy = means2D[2 * g + 1] - pfy;
            const float *co = conic_opacity + 4 * g;
            const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
            if (power > 0.0f) continue;
            const float G = expf(power);
            const float alpha = fminf(0.99f, co[3] * G);
            if (alpha < 1.0f / 255.0f) continue;
            T = T / (1.f - alpha);
            const float dchannel = alpha * T;
            float dL_dopa = 0.0f;
            for (int ch = 0; ch < 3; ++ch) {
              const float c = colors[3 * g + ch];
              acc_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * acc_rec[ch];
              last_color[ch] = c;
              dL_dopa += (c - acc_rec[ch]) * dLp[ch];
              dcolors[3 * g + ch] += dchannel * dLp[ch];
            }
            const float cd = depths[g];
            acc_depth = last_alpha * last_depth + (1.f - last_alpha) * acc_depth;
            last_depth = cd;
            dL_dopa += (cd - acc_depth) * dLd;
            for (int ch = 0; ch < F; ++ch) {
              /* Q5: the reference reads a never-written scratch (zero here) */
              const float f = compat == GS_COMPAT_REFERENCE ? 0.0f : feats[(size_t)g * F + ch];
              acc_f[ch] = last_alpha * last_f[ch] + (1.f - last_alpha) * acc_f[ch];
              last_f[ch] = f;
              if (compat == GS_COMPAT_REFERENCE) dLa += (f - acc_f[ch]) * dlf[ch];
              else dL_dopa += (f - acc_f[ch]) * dlf[ch];
              dsemantic[(size_t)g * F + ch] += dchannel * dlf[ch];
            }
            ddepths[g] += dchannel * dLd;
            acc_alpha = last_alpha + (1.f - last_alpha) * acc_alpha;
            dL_dopa += (1 - acc_alpha) * dLa;
            dL_dopa *= T;
            last_alpha = alpha;
            float bg_dot = 0;
            for (int ch = 0; ch < 3; ++ch) bg_dot += bg[ch] * dLp[ch];
            dL_dopa += (-T_final / (1.f - alpha)) * bg_dot;
            const float dL_dG = co[3] * dL_dopa;
            const float gdx = G * dx, gdy = G * dy;
            const float dG_ddelx = -gdx * co[0] - gdy * co[1];
            const float dG_ddely = -gdy * co[2] - gdx * co[1];
            dmean2D[3 * g + 0] += dL_dG * dG_ddelx * ddelx_dx;
            dmean2D[3 * g + 1] += dL_dG * dG_ddely * ddely_dy;
            dconic[4 * g + 0] += -0.5f * gdx * dx * dL_dG;
            dconic[4 * g + 1] += -0.5f * gdx * dy * dL_dG;
            dconic[4 * g + 3] += -0.5f * gdy * dy * dL_dG;
            dopacity[g] += G * dL_dopa;
          }
        }
    }
  free(acc_f); free(last_f); free(dlf);
}

/* computeColorFromSH (backward), CR/backward.cu:20-139. */
static void sh_bwd(int g, int deg, int M, const float *mean, const float *campos,
                   const float *shs, const uint8_t *clamped, const float *dcolor,
                   float *dmean, float *dsh) {
  const float dor[3] = {mean[0] - campos[0], mean[1] - campos[1], mean[2] - campos[2]};
  const float len = sqrtf(dor[0] * dor[0] + dor[1] * dor[1] + dor[2] * dor[2]);
  const float x = dor[0] / len, y = dor[1] / len, z = dor[2] / len;
  const float *sh = shs + (size_t)g * M * 3;
  float *ds = dsh + (size_t)g * M * 3;
  float dRGB[3];
  for (int ch = 0; ch < 3; ++ch) dRGB[ch] = dcolor[3 * g + ch] * (clamped[3 * g + ch] ? 0.0f : 1.0f);
  float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
#define S(i) sh[3 * (i) + ch]
#define W(i, v) ds[3 * (i) + ch] = (v) * dRGB[ch]
  for (int ch = 0; ch < 3; ++ch) {
    W(0, SH_C0);
    if (deg > 0) {
      W(1, -SH_C1 * y); W(2, SH_C1 * z); W(3, -SH_C1 * x);
      dx[ch] = -SH_C1 * S(3); dy[ch] = -SH_C1 * S(1); dz[ch] = SH_C1 * S(2);
      if (deg > 1) {
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        W(4, SH_C2[0] * xy); W(5, SH_C2[1] * yz); W(6, SH_C2[2] * (2.f * zz - xx - yy));
        W(7, SH_C2[3] * xz); W(8, SH_C2[4] * (xx - yy));
        dx[ch] += SH_C2[0] * y * S(4) + SH_C2[2] * 2.f * -x * S(6) + SH_C2[3] * z * S(7) + SH_C2[4] * 2.f * x * S(8);
        dy[ch] += SH_C2[0] * x * S(4) + SH_C2[1] * z * S(5) + SH_C2[2] * 2.f * -y * S(6) + SH_C2[4] * 2.f * -y * S(8);
        dz[ch] += SH_C2[1] * y * S(5) + SH_C2[2] * 2.f * 2.f * z * S(6) + SH_C2[3] * x * S(7);
        if (deg > 2) {
          W(9, SH_C3[0] * y * (3.f * xx - yy)); W(10, SH_C3[1] * xy * z);
          W(11, SH_C3[2] * y * (4.f * zz - xx - yy)); W(12, SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy));
          W(13, SH_C3[4] * x * (4.f * zz - xx - yy)); W(14, SH_C3[5] * z * (xx - yy));
          W(15, SH_C3[6] * x * (xx - 3.f * yy));
          dx[ch] += (SH_C3[0] * S(9) * 3.f * 2.f * xy + SH_C3[1] * S(10) * yz + SH_C3[2] * S(11) * -2.f * xy +
                     SH_C3[3] * S(12) * -3.f * 2.f * xz + SH_C3[4] * S(13) * (-3.f * xx + 4.f * zz - yy) +
                     SH_C3[5] * S(14) * 2.f * xz + SH_C3[6] * S(15) * 3.f * (xx - yy));
          dy[ch] += (SH_C3[0] * S(9) * 3.f * (xx - yy) + SH_C3[1] * S(10) * xz +
                     SH_C3[2] * S(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3[3] * S(12) * -3.f * 2.f * yz +
                     SH_C3[4] * S(13) * -2.f * xy + SH_C3[5] * S(14) * -2.f * yz + SH_C3[6] * S(15) * -3.f * 2.f * xy);
          dz[ch] += (SH_C3[1] * S(10) * xy + SH_C3[2] * S(11) * 4.f * 2.f * yz +
                     SH_C3[3] * S(12) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * S(13) * 4.f * 2.f * xz +
                     SH_C3[5] * S(14) * (xx - yy));
        }
      }
    }
  }
#undef S
#undef W
  const float ddir[3] = {dx[0] * dRGB[0] + dx[1] * dRGB[1] + dx[2] * dRGB[2],
                         dy[0] * dRGB[0] + dy[1] * dRGB[1] + dy[2] * dRGB[2],
                         dz[0] * dRGB[0] + dz[1] * dRGB[1] + dz[2] * dRGB[2]};
  /* dnormvdv(float3), CR/auxiliary.h:107-117 */
  const float s2 = dor[0] * dor[0] + dor[1] * dor[1] + dor[2] * dor[2];
  const float inv = 1.0f / sqrtf(s2 * s2 * s2);
  dmean[3 * g + 0] += ((s2 - dor[0] * dor[0]) * ddir[0] - dor[1] * dor[0] * ddir[1] - dor[2] * dor[0] * ddir[2]) * inv;
  dmean[3 * g + 1] += (-dor[0] * dor[1] * ddir[0] + (s2 - dor[1] * dor[1]) * ddir[1] - dor[2] * dor[1] * ddir[2]) * inv;
  dmean[3 * g + 2] += (-dor[0] * dor[2] * ddir[0] - dor[1] * dor[2] * ddir[1] + (s2 - dor[2] * dor[2]) * ddir[2]) * inv;
}

/* computeCov3D (backward), CR/backward.cu:295-358 (Q7: no quaternion
 * normalisation, so dL/dq is returned for the raw quaternion). */
static void cov3d_bwd(int g, const float *scale, float mod, const float *rot,
                      const float *dcov, float *dscale, float *drot) {
  float rc[3][3];
  quat_cols(rot, rc);
  const float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
  const float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
  /* M = S*R: M[c][k] = s_k R[c][k] */
  float m[3][3];
  for (int c = 0; c < 3; ++c) for (int k = 0; k < 3; ++k) m[c][k] = s[k] * rc[c][k];
  const float *d = dcov + 6 * g;
  /* dL_dSigma (glm columns), symmetric */
  const float sg[3][3] = {{d[0], 0.5f * d[1], 0.5f * d[2]},
                          {0.5f * d[1], d[3], 0.5f * d[4]},
                          {0.5f * d[2], 0.5f * d[4], d[5]}};
  /* dL_dM = 2 * M * dL_dSigma (glm product): dM[c][r] = 2 * sum_k M[k][r] sg[c][k] */
  float dm[3][3];
  for (int c = 0; c < 3; ++c)
    for (int rr = 0; rr < 3; ++rr)
      dm[c][rr] = 2.0f * (m[0][rr] * sg[c][0] + m[1][rr] * sg[c][1] + m[2][rr] * sg[c][2]);
  /* dL_dMt = transpose(dL_dM): dmt[c][r] = dm[r][c]; Rt[c][r] = rc[r][c] */
  float dmt[3][3];
  for (int c = 0; c < 3; ++c) for (int rr = 0; rr < 3; ++rr) dmt[c][rr] = dm[rr][c];
  for (int i = 0; i < 3; ++i)
    dscale[3 * g + i] = rc[0][i] * dmt[i][0] + rc[1][i] * dmt[i][1] + rc[2][i] * dmt[i][2];
  for (int i = 0; i < 3; ++i) for (int k = 0; k < 3; ++k) dmt[i][k] *= s[i];
  drot[4 * g + 0] = 2 * z * (dmt[0][1] - dmt[1][0]) + 2 * y * (dmt[2][0] - dmt[0][2]) + 2 * x * (dmt[1][2] - dmt[2][1]);
  drot[4 * g + 1] = 2 * y * (dmt[1][0] + dmt[0][1]) + 2 * z * (dmt[2][0] + dmt[0][2]) + 2 * r * (dmt[1][2] - dmt[2][1]) - 4 * x * (dmt[2][2] + dmt[1][1]);
  drot[4 * g + 2] = 2 * x * (dmt[1][0] + dmt[0][1]) + 2 * r * (dmt[2][0] - dmt[0][2]) + 2 * z * (dmt[1][2] + dmt[2][1]) - 4 * y * (dmt[2][2] + dmt[0][0]);
  drot[4 * g + 3] = 2 * r * (dmt[0][1] - dmt[1][0]) + 2 * x * (dmt[2][0] + dmt[0][2]) + 2 * y * (dmt[1][2] + dmt[2][1]) - 4 * z * (dmt[1][1] + dmt[0][0]);
}

/* computeCov2DCUDA (CR/backward.cu:144-291) followed by preprocessCUDA<3>
 * backward (:363-429).  Camera scalars arrive in C++ positional order
 * (rasterize_points.cu:141-144); focal is derived from the received
 * tan_fov values (CR/rasterizer_impl.cu:398-399), so the Python-side
 * argument swap (Q2) flows through unchanged.  dmean3D/dcov3D/dsh/dscale/
 * drot must be zeroed by the caller. */
void or_preprocess_bwd(int P, int D, int M, const float *means3D,
                       const int *radii, const float *shs, const uint8_t *clamped,
                       const float *scales, const float *rotations,
                       float scale_modifier, const float *cov3D,
                       const float *view, const float *proj, int W, int H,
                       float c_x, float c_y, float tan_fovx, float tan_fovy,
                       const float *campos, const float *dmean2D,
                       const float *dconic, const float *dcolor,
                       const float *ddepth, int compat, float *dmean3D,
                       float *dcov3D, float *dsh, float *dscale, float *drot) {
  const float hy = (float)H / (2.0f * tan_fovy);
  const float hx = (float)W / (2.0f * tan_fovx);
  for (int g = 0; g < P; ++g) {
    if (!(radii[g] > 0)) continue;
    const float *mean = means3D + 3 * g;
    const float *c3 = cov3D + 6 * g;
    const float dcx = dconic[4 * g], dcy = dconic[4 * g + 1], dcz = dconic[4 * g + 3];
    ewa_t e;
    ewa_setup(mean, view, W, H, c_x, c_y, hx, hy, tan_fovx, tan_fovy, &e);
    float xg, yg;
    if (compat == GS_COMPAT_REFERENCE) { /* Q3 */
      xg = (e.txtz < e.lxn || e.txtz > e.lxp) ? 0.f : 1.f;
      yg = (e.tytz < e.lyn || e.tytz > e.lyp) ? 0.f : 1.f;
    } else {
      xg = (e.txtz < -e.lxn || e.txtz > e.lxp) ? 0.f : 1.f;
      yg = (e.tytz < -e.lyn || e.tytz > e.lyp) ? 0.f : 1.f;
    }
    float cov[3];
    ewa_cov2d(&e, c3, cov);
    const float a = cov[0], b = cov[1], c = cov[2];
    const float denom = a * c - b * b;
    float da = 0, db = 0, dc = 0;
    const float d2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float (*A)[3] = e.a; /* A[i][r] == glm T[i][r] */
    float *o = dcov3D + 6 * g;
    if (d2inv != 0) {
      da = d2inv * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz);
      dc = d2inv * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx);
      db = d2inv * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
      o[0] = (A[0][0] * A[0][0] * da + A[0][0] * A[1][0] * db + A[1][0] * A[1][0] * dc);
      o[3] = (A[0][1] * A[0][1] * da + A[0][1] * A[1][1] * db + A[1][1] * A[1][1] * dc);
      o[5] = (A[0][2] * A[0][2] * da + A[0][2] * A[1][2] * db + A[1][2] * A[1][2] * dc);
      o[1] = 2 * A[0][0] * A[0][1] * da + (A[0][0] * A[1][1] + A[0][1] * A[1][0]) * db + 2 * A[1][0] * A[1][1] * dc;
      o[2] = 2 * A[0][0] * A[0][2] * da + (A[0][0] * A[1][2] + A[0][2] * A[1][0]) * db + 2 * A[1][0] * A[1][2] * dc;
      o[4] = 2 * A[0][2] * A[0][1] * da + (A[0][1] * A[1][2] + A[0][2] * A[1][1]) * db + 2 * A[1][1] * A[1][2] * dc;
    } else {
      for (int i = 0; i < 6; ++i) o[i] = 0;
    }
    const float V[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float dT[2][3];
    for (int k = 0; k < 3; ++k) {
      const float r0 = A[0][0] * V[k][0] + A[0][1] * V[k][1] + A[0][2] * V[k][2];
      const float r1 = A[1][0] * V[k][0] + A[1][1] * V[k][1] + A[1][2] * V[k][2];
      dT[0][k] = 2 * r0 * da + r1 * db;
      dT[1][k] = 2 * r1 * dc + r0 * db;
    }
    const float dJ00 = view[0] * dT[0][0] + view[4] * dT[0][1] + view[8] * dT[0][2];
    const float dJ02 = view[2] * dT[0][0] + view[6] * dT[0][1] + view[10] * dT[0][2];
    const float dJ11 = view[1] * dT[1][0] + view[5] * dT[1][1] + view[9] * dT[1][2];
    const float dJ12 = view[2] * dT[1][0] + view[6] * dT[1][1] + view[10] * dT[1][2];
    const float tz = 1.f / e.t[2], tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = xg * -hx * tz2 * dJ02;
    const float dty = yg * -hy * tz2 * dJ12;
    const float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * e.t[0]) * tz3 * dJ02 + (2 * hy * e.t[1]) * tz3 * dJ12;
    float *dm = dmean3D + 3 * g;
    dm[0] = view[0] * dtx + view[1] * dty + view[2] * dtz;
    dm[1] = view[4] * dtx + view[5] * dty + view[6] * dtz;
    dm[2] = view[8] * dtx + view[9] * dty + view[10] * dtz;

    /* preprocessCUDA backward: mean2D and depth contributions */
    float mh[4];
    xf44(proj, mean, mh);
    const float mw = 1.0f / (mh[3] + 0.0000001f);
    const float mul1 = (proj[0] * mean[0] + proj[4] * mean[1] + proj[8] * mean[2] + proj[12]) * mw * mw;
    const float mul2 = (proj[1] * mean[0] + proj[5] * mean[1] + proj[9] * mean[2] + proj[13]) * mw * mw;
    const float d2x = dmean2D[3 * g], d2y = dmean2D[3 * g + 1];
    dm[0] += (proj[0] * mw - proj[3] * mul1) * d2x + (proj[1] * mw - proj[3] * mul2) * d2y;
    dm[1] += (proj[4] * mw - proj[7] * mul1) * d2x + (proj[5] * mw - proj[7] * mul2) * d2y;
    dm[2] += (proj[8] * mw - proj[11] * mul1) * d2x + (proj[9] * mw - proj[11] * mul2) * d2y;
    const float mul3 = view[2] * mean[0] + view[6] * mean[1] + view[10] * mean[2] + view[14];
    const float dd = ddepth[g];
    dm[0] += (view[2] - view[3] * mul3) * dd;
    dm[1] += (view[6] - view[7] * mul3) * dd;
    dm[2] += (view[10] - view[11] * mul3) * dd;
    if (shs) sh_bwd(g, D, M, mean, campos, shs, clamped, dcolor, dmean3D, dsh);
    if (scales) cov3d_bwd(g, scales + 3 * g, scale_modifier, rotations + 4 * g, dcov3D, dscale, drot);
  }
}
