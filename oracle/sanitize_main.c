/*
 * sanitize_main.c -- TEST INFRASTRUCTURE: the CPU sanitizer pass (SURVEY.md
 * section 5).  Built by `make -C oracle sanitize` with
 * AddressSanitizer + UndefinedBehaviorSanitizer (-fno-sanitize-recover: the
 * first finding aborts) over
 *   - the C oracle's whole forward and backward chain (or_preprocess ->
 *     or_binning -> or_render_fwd -> or_render_bwd -> or_preprocess_bwd,
 *     or_mark_visible, or_higher_msb, or_set_pixel_order) on seeded scenes:
 *     SH degrees 0 / 3 or precomputed colours, F = 0 / 32, both compat modes,
 *     an off-centre principal point, Gaussians on and beyond the image edges;
 *   - the library's host validators (dynamic3dgaussians_amd/csrc/gs_host.cpp:
 *     gs_check_plan_header / gs_check_ranges / gs_check_point_list / gs_check_walk_order,
 *     gs_last_error) on the oracle's own plan, lists and ranges and on
 *     corrupted copies of them (each must be refused with a message).
 * Prints "sanitize ok" and exits 0 when clean; tests/test_sanitize.py runs it.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gsplat_hip.h"

/* gs_oracle.c (no header: oracle.py binds it through ctypes) */
void or_mark_visible(int P, const float *means3D, const float *view, const float *proj, uint8_t *present);
int or_preprocess(int P, int D, int M, const float *means3D, const float *scales, float scale_modifier,
                  const float *rotations, const float *opacities, const float *shs, const float *cov3D_precomp,
                  const float *colors_precomp, const float *view, const float *proj, const float *campos, int W,
                  int H, float c_x, float c_y, float tan_fovx, float tan_fovy, int prefiltered, int *radii,
                  float *means2D, float *depths, float *cov3D, float *rgb, float *conic_opacity,
                  uint32_t *tiles_touched, uint8_t *clamped);
uint32_t or_higher_msb(uint32_t n);
int64_t or_binning(int P, const float *means2D, const float *depths, const int *radii,
                   const uint32_t *tiles_touched, int W, int H, uint32_t *point_list, uint64_t *keys_out,
                   uint32_t *ranges);
void or_render_fwd(int W, int H, const uint32_t *ranges, const uint32_t *point_list, const float *means2D,
                   const float *colors, const float *feats, int F, const float *depths, const float *conic_opacity,
                   const float *bg, int compat, float *out_color, float *out_feature, float *out_depth,
                   float *out_alpha, uint32_t *n_contrib);
void or_set_pixel_order(const uint32_t *order, int64_t n);
void or_render_bwd(int W, int H, const uint32_t *ranges, const uint32_t *point_list, const float *bg,
                   const float *means2D, const float *conic_opacity, const float *colors, const float *feats, int F,
                   const float *depths, const float *alphas, const uint32_t *n_contrib, const float *dL_dpix,
                   const float *dL_dfeat, const float *dL_ddepth_pix, const float *dL_dalpha_pix, int compat,
                   float *dmean2D, float *dconic, float *dopacity, float *dcolors, float *dsemantic,
                   float *ddepths);
void or_preprocess_bwd(int P, int D, int M, const float *means3D, const int *radii, const float *shs,
                       const uint8_t *clamped, const float *scales, const float *rotations, float scale_modifier,
                       const float *cov3D, const float *view, const float *proj, int W, int H, float c_x, float c_y,
                       float tan_fovx, float tan_fovy, const float *campos, const float *dmean2D, const float *dconic,
                       const float *dcolor, const float *ddepth, int compat, float *dmean3D, float *dcov3D,
                       float *dsh, float *dscale, float *drot);

static uint64_t g_rng = 88172645463325252ull;
static float urand(void) { /* xorshift64, [0, 1) */
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return (float)((g_rng >> 40) & 0xFFFFFF) / 16777216.0f;
}
static float nrand(void) { return (urand() + urand() + urand() + urand() - 2.0f) * 1.7f; }

static void *xcalloc(size_t n, size_t sz) {
  void *p = calloc(n ? n : 1, sz);
  if (!p) {
    fprintf(stderr, "out of memory\n");
    exit(2);
  }
  return p;
}

static int g_fail = 0;
#define EXPECT(cond, ...)                          \
  do {                                             \
    if (!(cond)) {                                 \
      fprintf(stderr, "FAILED %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                \
      fprintf(stderr, "\n");                       \
      g_fail = 1;                                  \
    }                                              \
  } while (0)

/* column-major 4x4 of the row-major product a*b */
static void mat_mul_cm(const double a[4][4], const double b[4][4], float out[16]) {
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      double s = 0;
      for (int k = 0; k < 4; ++k) s += a[r][k] * b[k][c];
      out[c * 4 + r] = (float)s;
    }
}

static void run_case(int P, int W, int H, int D, int F, int compat, int precomp, float cx_off) {
  const int M = D >= 0 ? (D + 1) * (D + 1) : 0;
  const float tanx = 0.55f, tany = tanx * (float)H / (float)W;
  const float cx = 0.5f * W + cx_off, cy = 0.5f * H;
  /* camera 4 units back, looking down +z (utils/graphics_utils.py conventions) */
  double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 4.0}, {0, 0, 0, 1}};
  const double n = 0.01, f = 100.0;
  double Pm[4][4] = {{1.0 / tanx, 0, 0, 0}, {0, 1.0 / tany, 0, 0}, {0, 0, f / (f - n), -f * n / (f - n)},
                     {0, 0, 1, 0}};
  double I[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  float view[16], proj[16];
  mat_mul_cm(V, I, view);
  mat_mul_cm(Pm, V, proj);
  const float campos[3] = {0.f, 0.f, -4.f}, bg[3] = {0.2f, 0.1f, 0.3f};

  float *means = xcalloc((size_t)P * 3, 4), *scales = xcalloc((size_t)P * 3, 4), *rots = xcalloc((size_t)P * 4, 4);
  float *opac = xcalloc(P, 4), *cols = xcalloc((size_t)P * 3, 4), *feats = xcalloc((size_t)P * (F ? F : 1), 4);
  float *shs = xcalloc((size_t)P * (M ? M : 1) * 3, 4);
  for (int g = 0; g < P; ++g) {
    for (int k = 0; k < 3; ++k) {
      means[3 * g + k] = nrand() * (k == 2 ? 0.8f : 1.2f);  /* some beyond the image edges */
      scales[3 * g + k] = 0.01f + 0.12f * urand();
      cols[3 * g + k] = urand();
    }
    if (g % 97 == 0) means[3 * g + 2] = -6.0f;  /* behind the camera */
    for (int k = 0; k < 4; ++k) rots[4 * g + k] = nrand();  /* unnormalised (Q7) */
    opac[g] = 0.05f + 0.9f * urand();
    for (int k = 0; k < F; ++k) feats[(size_t)F * g + k] = nrand();
    for (int k = 0; k < M * 3; ++k) shs[(size_t)M * 3 * g + k] = 0.3f * nrand();
  }
  uint8_t *present = xcalloc(P, 1);
  or_mark_visible(P, means, view, proj, present);

  int *radii = xcalloc(P, 4);
  float *m2 = xcalloc((size_t)P * 2, 4), *depths = xcalloc(P, 4), *cov3 = xcalloc((size_t)P * 6, 4);
  float *rgb = xcalloc((size_t)P * 3, 4), *conic = xcalloc((size_t)P * 4, 4);
  uint32_t *touched = xcalloc(P, 4);
  uint8_t *clamped = xcalloc((size_t)P * 3, 1);
  const int trapped = or_preprocess(P, D < 0 ? 0 : D, M, means, scales, 1.0f, rots, opac, D >= 0 ? shs : NULL, NULL,
                                    precomp ? cols : NULL, view, proj, campos, W, H, cx, cy, tanx, tany, 0, radii,
                                    m2, depths, cov3, rgb, conic, touched, clamped);
  EXPECT(trapped == 0, "preprocess trapped without prefiltered");
  int64_t L = 0;
  int visible = 0;
  for (int g = 0; g < P; ++g) {
    L += touched[g];
    visible += radii[g] > 0;
  }
  EXPECT(visible > P / 4, "only %d of %d Gaussians visible", visible, P);
  const int gx = (W + 15) / 16, gy = (H + 15) / 16, T = gx * gy;
  uint32_t *plist = xcalloc(L, 4), *ranges = xcalloc((size_t)2 * T, 4);
  uint64_t *keys = xcalloc(L, 8);
  const int64_t L2 = or_binning(P, m2, depths, radii, touched, W, H, plist, keys, ranges);
  EXPECT(L2 == L, "binning %lld vs %lld", (long long)L2, (long long)L);
  (void)or_higher_msb((uint32_t)T);

  const size_t HW = (size_t)W * H;
  float *oc = xcalloc(3 * HW, 4), *of = xcalloc((F ? F : 1) * HW, 4), *od = xcalloc(HW, 4), *oa = xcalloc(HW, 4);
  uint32_t *ncon = xcalloc(HW, 4);
  const float *colour_src = precomp ? cols : rgb;
  or_render_fwd(W, H, ranges, plist, m2, colour_src, F ? feats : NULL, F, depths, conic, bg, compat, oc,
                F ? of : NULL, od, oa, ncon);

  /* the library's validators on the oracle's own lists, then corrupted */
  uint32_t maxlen = 0;
  for (int t = 0; t < T; ++t)
    if (ranges[2 * t + 1] - ranges[2 * t] > maxlen) maxlen = ranges[2 * t + 1] - ranges[2 * t];
  uint32_t hdr[8] = {(uint32_t)L, maxlen, (uint32_t)L, 0u, 0u, 0u, 0u, 0u};
  EXPECT(gs_check_plan_header(hdr, T) == 0, "valid header refused: %s", gs_last_error());
  EXPECT(gs_check_ranges(ranges, T, L, maxlen) == 0, "valid ranges refused: %s", gs_last_error());
  EXPECT(gs_check_point_list(plist, L, P) == 0, "valid list refused: %s", gs_last_error());
  uint32_t bad[8];
  memcpy(bad, hdr, sizeof(bad));
  bad[3] = 9u;
  EXPECT(gs_check_plan_header(bad, T) < 0 && strlen(gs_last_error()) > 0, "status bits accepted");
  memcpy(bad, hdr, sizeof(bad));
  bad[1] = (uint32_t)L + 1u;
  EXPECT(gs_check_plan_header(bad, T) < 0, "longest tile > L accepted");
  memcpy(bad, hdr, sizeof(bad));
  bad[4] = (uint32_t)T + 1u;
  EXPECT(gs_check_plan_header(bad, T) < 0, "sort prefix > tiles accepted");
  EXPECT(gs_check_plan_header(NULL, T) < 0, "null header accepted");
  {
    /* a walk order: a permutation passes, a repeated id and an id out of range do not */
    int32_t *wo = xcalloc((size_t)P, 4);
    for (int i = 0; i < P; ++i) wo[i] = P - 1 - i;
    EXPECT(gs_check_walk_order(wo, P) == 0, "valid walk order refused: %s", gs_last_error());
    if (P > 1) {
      wo[0] = wo[1];
      EXPECT(gs_check_walk_order(wo, P) < 0, "repeated id in the walk order accepted");
      wo[0] = P;
      EXPECT(gs_check_walk_order(wo, P) < 0, "out-of-range id in the walk order accepted");
    }
    free(wo);
  }
  if (L > 2) {
    uint32_t *r2 = xcalloc((size_t)2 * T, 4);
    memcpy(r2, ranges, sizeof(uint32_t) * 2 * T);
    for (int t = 0; t < T; ++t)
      if (r2[2 * t + 1] > r2[2 * t]) {
        r2[2 * t] += 1;  /* a gap before this list */
        break;
      }
    EXPECT(gs_check_ranges(r2, T, L, -1) < 0, "non-contiguous ranges accepted");
    EXPECT(gs_check_ranges(ranges, T, L - 1, -1) < 0, "ranges past L accepted");
    EXPECT(maxlen < 1 || gs_check_ranges(ranges, T, L, maxlen - 1) < 0, "a list over max_len accepted");
    plist[L / 2] = (uint32_t)P;
    EXPECT(gs_check_point_list(plist, L, P) < 0, "out-of-range id accepted");
    plist[L / 2] = 0u;
    free(r2);
  }
  /* restore the list the blend used */
  (void)or_binning(P, m2, depths, radii, touched, W, H, plist, keys, ranges);

  /* backward, twice: the plain pixel order and a permuted one (the envelope) */
  float *dLc = xcalloc(3 * HW, 4), *dLf = xcalloc((F ? F : 1) * HW, 4), *dLd = xcalloc(HW, 4), *dLa = xcalloc(HW, 4);
  for (size_t i = 0; i < 3 * HW; ++i) dLc[i] = nrand();
  for (size_t i = 0; i < (size_t)F * HW; ++i) dLf[i] = nrand();
  for (size_t i = 0; i < HW; ++i) {
    dLd[i] = 0.1f * nrand();
    dLa[i] = 0.1f * nrand();
  }
  uint32_t *order = xcalloc(HW, 4);
  for (size_t i = 0; i < HW; ++i) order[i] = (uint32_t)i;
  for (size_t i = HW - 1; i > 0; --i) {
    const size_t j = (size_t)(urand() * (float)(i + 1)) % (i + 1);
    const uint32_t t = order[i];
    order[i] = order[j];
    order[j] = t;
  }
  for (int pass = 0; pass < 2; ++pass) {
    or_set_pixel_order(pass ? order : NULL, (int64_t)HW);
    float *dm2 = xcalloc((size_t)P * 3, 4), *dcon = xcalloc((size_t)P * 4, 4), *dop = xcalloc(P, 4);
    float *dcol = xcalloc((size_t)P * 3, 4), *dsem = xcalloc((size_t)P * (F ? F : 1), 4), *ddep = xcalloc(P, 4);
    or_render_bwd(W, H, ranges, plist, bg, m2, conic, colour_src, F ? feats : NULL, F, depths, oa, ncon, dLc,
                  F ? dLf : NULL, dLd, dLa, compat, dm2, dcon, dop, dcol, F ? dsem : NULL, ddep);
    float *dm3 = xcalloc((size_t)P * 3, 4), *dc3 = xcalloc((size_t)P * 6, 4);
    float *dsh = xcalloc((size_t)P * (M ? M : 1) * 3, 4), *dsc = xcalloc((size_t)P * 3, 4);
    float *drot = xcalloc((size_t)P * 4, 4);
    or_preprocess_bwd(P, D < 0 ? 0 : D, M, means, radii, D >= 0 ? shs : NULL, clamped, scales, rots, 1.0f, cov3, view,
                      proj, W, H, cx, cy, tanx, tany, campos, dm2, dcon, dcol, ddep, compat, dm3, dc3,
                      D >= 0 ? dsh : NULL, dsc, drot);
    double s = 0;
    for (int g = 0; g < 3 * P; ++g) s += fabs((double)dm3[g]);
    EXPECT(isfinite(s) && s > 0, "means3D gradient sum %g", s);
    free(dm2); free(dcon); free(dop); free(dcol); free(dsem); free(ddep);
    free(dm3); free(dc3); free(dsh); free(dsc); free(drot);
  }
  or_set_pixel_order(NULL, 0);
  printf("case P=%d %dx%d D=%d F=%d compat=%d precomp=%d: L=%lld visible=%d\n", P, W, H, D, F, compat, precomp,
         (long long)L, visible);
  free(means); free(scales); free(rots); free(opac); free(cols); free(feats); free(shs); free(present);
  free(radii); free(m2); free(depths); free(cov3); free(rgb); free(conic); free(touched); free(clamped);
  free(plist); free(ranges); free(keys); free(oc); free(of); free(od); free(oa); free(ncon);
  free(dLc); free(dLf); free(dLd); free(dLa); free(order);
}

int main(void) {
  if (getenv("GS_SANITIZE_SELFTEST")) {  /* the negative control: a heap overflow the build must catch */
    volatile int *p = (volatile int *)malloc(4 * sizeof(int));
    p[4] = 1;
    free((void *)p);
    printf("selftest: overflow NOT detected\n");
    return 0;
  }
  run_case(3000, 96, 72, -1, 0, 0, 1, 0.0f);   /* precomputed colours, F = 0, reference numerics */
  run_case(2500, 112, 80, 3, 32, 0, 0, 7.5f);  /* SH degree 3, F = 32, off-centre principal point */
  run_case(2000, 80, 80, 1, 4, 1, 0, -5.0f);   /* fixed numerics (alpha output, dL/dalpha) */
  run_case(1500, 100, 60, -1, 32, 1, 1, 0.0f);  /* odd tile counts, fixed, precomputed colours */
  if (g_fail) return 1;
  printf("sanitize ok\n");
  return 0;
}
