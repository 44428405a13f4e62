// gs_torch_binding.cpp -- native (C++) fast path of the `_C` binding.
//
// The reference binds its rasterizer with a C++ torch extension
// (DGR/rasterize_points.cu:35-246, RasterizeGaussiansCUDA /
// RasterizeGaussiansBackwardCUDA, DGR/ext.cpp:15-19).  This file is our
// counterpart on top of the C ABI (include/gsplat_hip.h): the same argument
// handling as dynamic3dgaussians_amd/_C.py (which remains the documented
// ctypes binding and the fallback for argument errors), without the Python
// per-call work -- tensor checks, output allocation, struct packing and the
// ABI calls are ~0.2 ms of host time per camera in Python, tens of
// microseconds here.  Built with torch.utils.cpp_extension by build.py into
// lib/ next to libgsplat_hip.so (found through rpath $ORIGIN).  No device
// code: every kernel runs through the C ABI.
#include <torch/extension.h>

#include <stdexcept>
#include <string>
#include <tuple>

#include "gsplat_hip.h"

namespace {

using at::Tensor;
using OptT = c10::optional<Tensor>;

const int kSupportedF[] = {0, 4, 8, 16, 32, 36, 64};

bool present(const OptT& t) { return t.has_value() && t->defined() && t->numel() > 0; }

Tensor dev_f32(const Tensor& t, const at::Device& dev, const char* name) {
  if (t.device() != dev)
    throw std::runtime_error(std::string(name) + " must be on the rasterizer's HIP device");
  Tensor u = t.scalar_type() == at::kFloat ? t : t.to(at::kFloat);
  return u.contiguous();
}

void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + ": " + gs_last_error() + " (code " + std::to_string(rc) + ")");
}

int feature_width(int64_t F) {
  for (int k : kSupportedF)
    if (k >= F) return k;
  throw std::runtime_error("semantic feature width " + std::to_string(F) + " exceeds the largest compiled width 64");
}

struct Inputs {
  at::Device dev{at::kCUDA};
  int64_t P = 0, M = 0, F = 0, F_user = 0;
  int D = 0;
  float scale_modifier = 1.f;
  Tensor means3D, colors, opacity, scales, rotations, cov3D, sh, sem;
  gs_gaussians g{};

  Inputs(const Tensor& means3D_, const OptT& colors_, const OptT& sem_, const OptT& opacity_, const OptT& scales_,
         const OptT& rotations_, double scale_mod, const OptT& cov3D_, const OptT& sh_, int64_t degree) {
    if (means3D_.dim() != 2 || means3D_.size(1) != 3)
      throw std::runtime_error("means3D must have dimensions (num_points, 3)");  // rasterize_points.cu:60-62
    dev = means3D_.device();
    P = means3D_.size(0);
    means3D = dev_f32(means3D_, dev, "means3D");
    if (present(colors_)) colors = dev_f32(*colors_, dev, "colors_precomp");
    if (present(opacity_)) opacity = dev_f32(*opacity_, dev, "opacities");
    if (present(scales_)) scales = dev_f32(*scales_, dev, "scales");
    if (present(rotations_)) rotations = dev_f32(*rotations_, dev, "rotations");
    if (present(cov3D_)) cov3D = dev_f32(*cov3D_, dev, "cov3D_precomp");
    if (present(sh_)) {
      sh = dev_f32(*sh_, dev, "sh");
      M = sh.size(1);
    }
    D = (int)degree;
    scale_modifier = (float)scale_mod;
    if (present(sem_)) {
      sem = dev_f32(*sem_, dev, "semantic_feature").reshape({P, -1});
      F_user = sem.size(1);
      F = feature_width(F_user);
      if (F != F_user) sem = at::constant_pad_nd(sem, {0, F - F_user}, 0.0);
      sem = sem.contiguous();
    }
    auto ptr = [](const Tensor& t) -> const float* { return t.defined() ? t.data_ptr<float>() : nullptr; };
    g.P = (int32_t)P;
    g.D = D;
    g.M = (int32_t)M;
    g.F = (int32_t)F;
    g.means3D = ptr(means3D);
    g.shs = ptr(sh);
    g.colors_precomp = ptr(colors);
    g.semantic_feature = ptr(sem);
    g.opacities = ptr(opacity);
    g.scales = ptr(scales);
    g.rotations = ptr(rotations);
    g.cov3D_precomp = ptr(cov3D);
    g.scale_modifier = scale_modifier;
    g.flags = 0;
    g.grad_mask = nullptr;
    g.densify_accum = g.densify_denom = g.max_radius = nullptr;
    g.feature_ready = nullptr;
    g.walk_order = nullptr;
  }
};

struct Camera {
  Tensor keep[4];
  gs_camera cam{};
  Camera(const at::Device& dev, const Tensor& bg, const Tensor& view, const Tensor& proj, const Tensor& campos,
         double c_x, double c_y, double tanx, double tany, int64_t W, int64_t H) {
    keep[0] = dev_f32(bg, dev, "bg").reshape({-1});
    keep[1] = dev_f32(view, dev, "viewmatrix").reshape({-1});
    keep[2] = dev_f32(proj, dev, "projmatrix").reshape({-1});
    keep[3] = dev_f32(campos, dev, "campos").reshape({-1});
    cam.background = keep[0].data_ptr<float>();
    cam.viewmatrix = keep[1].data_ptr<float>();
    cam.projmatrix = keep[2].data_ptr<float>();
    cam.campos = keep[3].data_ptr<float>();
    cam.c_x = (float)c_x;
    cam.c_y = (float)c_y;
    cam.tan_fovx = (float)tanx;
    cam.tan_fovy = (float)tany;
    cam.image_width = (int32_t)W;
    cam.image_height = (int32_t)H;
  }
};

void* nz(const Tensor& t) { return (t.defined() && t.numel()) ? t.data_ptr() : nullptr; }

// RasterizeGaussiansCUDA (DGR/rasterize_points.cu:35-126), positional order of
// _C.rasterize_gaussians + compat code + stream handle.  P > 0 (the Python
// layer answers P == 0).
std::tuple<int64_t, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> forward(
    const Tensor& bg, const Tensor& means3D, const OptT& colors, const OptT& sem, const OptT& opacity,
    const OptT& scales, const OptT& rotations, double scale_modifier, const OptT& cov3D, const Tensor& view,
    const Tensor& proj, double c_x, double c_y, double tanx, double tany, int64_t H, int64_t W, const OptT& sh,
    int64_t degree, const Tensor& campos, bool prefiltered, bool debug, int64_t compat, int64_t stream) {
  Inputs in(means3D, colors, sem, opacity, scales, rotations, scale_modifier, cov3D, sh, degree);
  Camera c(in.dev, bg, view, proj, campos, c_x, c_y, tanx, tany, W, H);
  const auto f32 = at::TensorOptions().dtype(at::kFloat).device(in.dev);
  const auto u8 = at::TensorOptions().dtype(at::kByte).device(in.dev);
  Tensor out_color = at::empty({3, H, W}, f32);
  Tensor out_feature = at::empty({in.F, H, W}, f32);
  Tensor out_depth = at::empty({1, H, W}, f32);
  Tensor out_alpha = at::empty({1, H, W}, f32);
  Tensor radii = at::empty({in.P}, f32.dtype(at::kInt));
  Tensor geom = at::empty({(int64_t)gs_geom_buffer_bytes(in.P)}, u8);
  Tensor img = at::empty({(int64_t)gs_image_buffer_bytes((int32_t)W, (int32_t)H)}, u8);
  int64_t L = 0, NI = 0;
  gs_stream_t s = reinterpret_cast<gs_stream_t>(stream);
  check(gs_forward_plan(&in.g, &c.cam, prefiltered ? 1 : 0, debug ? 1 : 0, (int)compat, geom.data_ptr(),
                        img.data_ptr(), radii.data_ptr<int32_t>(), &L, &NI, s),
        "rasterize_gaussians (preprocess)");
  Tensor binning = at::empty({(int64_t)gs_binning_buffer_bytes(NI)}, u8);
  check(gs_forward_render(&in.g, &c.cam, debug ? 1 : 0, (int)compat, geom.data_ptr(), binning.data_ptr(),
                          img.data_ptr(), NI, radii.data_ptr<int32_t>(), out_color.data_ptr<float>(),
                          in.F ? out_feature.data_ptr<float>() : nullptr, out_depth.data_ptr<float>(),
                          out_alpha.data_ptr<float>(), s),
        "rasterize_gaussians (render)");
  Tensor feature_map = in.F_user != in.F ? out_feature.narrow(0, 0, in.F_user) : out_feature;
  return {L, out_color, feature_map, out_depth, out_alpha, radii, geom, binning, img};
}

// RasterizeGaussiansBackwardCUDA (DGR/rasterize_points.cu:128-225), positional
// order of _C.rasterize_gaussians_backward + compat code, optional label mask,
// optional caller-owned buffers (9, in the output order) with the accumulate
// flag, optional densification statistics (accum, denom, max_radius), and the
// stream handle.
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> backward(
    const Tensor& bg, const Tensor& means3D, const Tensor& radii, const OptT& colors, const OptT& sem,
    const OptT& scales, const OptT& rotations, double scale_modifier, const OptT& cov3D, const Tensor& view,
    const Tensor& proj, double c_x, double c_y, double tanx, double tany, const OptT& dL_color,
    const OptT& dL_feature, const OptT& dL_depth, const OptT& dL_alpha, const OptT& sh, int64_t degree,
    const Tensor& campos, const Tensor& geom, int64_t R, const OptT& binning, const Tensor& img,
    const Tensor& alphas, bool debug, int64_t compat, const OptT& grad_mask, c10::optional<std::vector<Tensor>> out,
    bool accumulate, c10::optional<std::vector<Tensor>> densify, int64_t stream) {
  Inputs in(means3D, colors, sem, c10::nullopt, scales, rotations, scale_modifier, cov3D, sh, degree);
  const Tensor& img_ref = present(dL_color) ? *dL_color : alphas;
  const int64_t H = img_ref.size(-2), W = img_ref.size(-1);
  Camera c(in.dev, bg, view, proj, campos, c_x, c_y, tanx, tany, W, H);
  const auto f32 = at::TensorOptions().dtype(at::kFloat).device(in.dev);
  const int64_t P = in.P;
  Tensor gm;
  if (grad_mask.has_value() && grad_mask->defined()) {
    gm = grad_mask->to(in.dev, at::kFloat).reshape({-1}).contiguous();
    if (gm.numel() != P) throw std::runtime_error("grad_mask must have P elements");
    in.g.grad_mask = gm.data_ptr<float>();
  }
  Tensor dLc = present(dL_color) ? dev_f32(*dL_color, in.dev, "dL_dout_color") : Tensor();
  Tensor dLd = present(dL_depth) ? dev_f32(*dL_depth, in.dev, "dL_dout_depth") : Tensor();
  Tensor dLa = present(dL_alpha) ? dev_f32(*dL_alpha, in.dev, "dL_dout_alpha") : Tensor();
  Tensor alphas_c = dev_f32(alphas, in.dev, "alpha");
  Tensor dLf;
  if (in.F && present(dL_feature)) {
    dLf = dev_f32(*dL_feature, in.dev, "dL_dout_feature").reshape({-1, H, W});
    if (dLf.size(0) < in.F) dLf = at::cat({dLf, at::zeros({in.F - dLf.size(0), H, W}, f32)}).contiguous();
  }
  Tensor radii_c = radii.to(in.dev, at::kInt).contiguous();
  const std::vector<std::vector<int64_t>> shapes = {{P, 3}, {P, 3}, {P, in.F}, {P, 1}, {P, 3},
                                                    {P, 6}, {P, in.M, 3}, {P, 3}, {P, 4}};
  std::vector<Tensor> o;
  if (out.has_value()) {
    o = *out;
    if (o.size() != 9) throw std::runtime_error("out must hold the 9 gradient buffers");
    for (int i = 0; i < 9; ++i)
      if (o[i].sizes() != at::IntArrayRef(shapes[i]) || o[i].scalar_type() != at::kFloat || o[i].device() != in.dev ||
          !o[i].is_contiguous())
        throw std::runtime_error("gradient buffer " + std::to_string(i) + " has the wrong shape/dtype/device");
    if (accumulate) in.g.flags = GS_FLAG_ACCUMULATE;
  } else {
    if (accumulate) throw std::runtime_error("accumulate needs the caller's gradient buffers");
    for (int i = 0; i < 9; ++i) o.push_back(at::empty(shapes[i], f32));
  }
  if (densify.has_value()) {
    const auto& d = *densify;
    if (d.size() != 3) throw std::runtime_error("densify must hold (accum, denom, max_radius)");
    for (const auto& t : d)
      if (t.dim() != 1 || t.size(0) != P || t.scalar_type() != at::kFloat || t.device() != in.dev || !t.is_contiguous())
        throw std::runtime_error("densify statistics must be contiguous fp32 (P,) tensors on the device");
    in.g.densify_accum = d[0].data_ptr<float>();
    in.g.densify_denom = d[1].data_ptr<float>();
    in.g.max_radius = d[2].data_ptr<float>();
  }
  Tensor scratch = at::empty({(int64_t)gs_backward_scratch_bytes(P, (int32_t)in.F)},
                             f32.dtype(at::kByte));
  const Tensor bin = binning.has_value() ? *binning : Tensor();
  check(gs_backward(&in.g, &c.cam, radii_c.data_ptr<int32_t>(), debug ? 1 : 0, (int)compat, geom.data_ptr(),
                    nz(bin), img.data_ptr(), R, alphas_c.data_ptr<float>(),
                    dLc.defined() ? dLc.data_ptr<float>() : nullptr, dLf.defined() ? dLf.data_ptr<float>() : nullptr,
                    dLd.defined() ? dLd.data_ptr<float>() : nullptr, dLa.defined() ? dLa.data_ptr<float>() : nullptr,
                    scratch.data_ptr(), o[0].data_ptr<float>(), o[1].data_ptr<float>(),
                    static_cast<float*>(nz(o[2])), o[3].data_ptr<float>(), o[4].data_ptr<float>(),
                    o[5].data_ptr<float>(), static_cast<float*>(nz(o[6])), o[7].data_ptr<float>(),
                    o[8].data_ptr<float>(), reinterpret_cast<gs_stream_t>(stream)),
        "rasterize_gaussians_backward");
  Tensor dsem = in.F_user != in.F ? o[2].narrow(1, 0, in.F_user) : o[2];
  return {o[0], o[1], dsem, o[3], o[4], o[5], o[6], o[7], o[8]};
}

// ---- camera batches (gs_*_batch): the C++ counterpart of
// _C.rasterize_gaussians_batch / rasterize_gaussians_batch_backward.  The
// forward's one host round trip (the plan header) sits between the two ABI
// calls, so the host work around it is on the step's critical path.

struct Cameras {
  Tensor view, proj, cpos, bg;
  std::vector<gs_camera> cams;
  Cameras(const at::Device& dev, const Tensor& bg_, const Tensor& views, const Tensor& projs, const Tensor& campos,
          const std::vector<double>& cx, const std::vector<double>& cy, const std::vector<double>& tx,
          const std::vector<double>& ty, int64_t W, int64_t H, const std::vector<std::vector<int64_t>>& windows) {
    const int64_t C = (int64_t)cx.size();
    if (C < 1 || C > 64) throw std::runtime_error("camera batch size " + std::to_string(C) + " outside 1..64");
    if ((int64_t)cy.size() != C || (int64_t)tx.size() != C || (int64_t)ty.size() != C)
      throw std::runtime_error("per-camera scalars must all have C entries");
    view = dev_f32(views, dev, "viewmatrices").reshape({C, 16}).contiguous();
    proj = dev_f32(projs, dev, "projmatrices").reshape({C, 16}).contiguous();
    cpos = dev_f32(campos, dev, "campos").reshape({C, 3}).contiguous();
    bg = dev_f32(bg_, dev, "bg").reshape({-1});
    if (!windows.empty() && (int64_t)windows.size() != C)
      throw std::runtime_error("tile windows: one (x0, y0, x1, y1) per camera");
    cams.assign(C, gs_camera{});
    for (int64_t c = 0; c < C; ++c) {
      gs_camera& k = cams[c];
      if (!windows.empty()) {
        if (windows[c].size() != 4) throw std::runtime_error("a tile window is (x0, y0, x1, y1)");
        k.tile_x0 = (int32_t)windows[c][0];
        k.tile_y0 = (int32_t)windows[c][1];
        k.tile_x1 = (int32_t)windows[c][2];
        k.tile_y1 = (int32_t)windows[c][3];
      }
      k.viewmatrix = view.data_ptr<float>() + 16 * c;
      k.projmatrix = proj.data_ptr<float>() + 16 * c;
      k.campos = cpos.data_ptr<float>() + 3 * c;
      k.background = bg.data_ptr<float>();
      k.c_x = (float)cx[c];
      k.c_y = (float)cy[c];
      k.tan_fovx = (float)tx[c];
      k.tan_fovy = (float)ty[c];
      k.image_width = (int32_t)W;
      k.image_height = (int32_t)H;
    }
  }
};

// capacity: empty = the two-phase path (plan, host read, render); else the
// sync-free gs_forward_batch with a binning buffer of capacity[c] instances
// per camera and `hint` (gs_batch_hint as {valid, p1, q1, p2, max_len,
// total}), retried with the exact lengths when they do not fit.  Returns the
// reference's counts, the images and state, the exact num_instances, the
// per-camera lengths the binning buffer is laid out with (what the backward
// takes), the updated hint and whether the first attempt fitted.
std::tuple<std::vector<int64_t>, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, std::vector<int64_t>,
           std::vector<int64_t>, std::vector<int64_t>, bool>
forward_batch(const Tensor& bg, const Tensor& means3D, const OptT& colors, const OptT& sem, const OptT& opacity,
              const OptT& scales, const OptT& rotations, double scale_modifier, const OptT& cov3D, const Tensor& views,
              const Tensor& projs, const std::vector<double>& cx, const std::vector<double>& cy,
              const std::vector<double>& tx, const std::vector<double>& ty, int64_t H, int64_t W, const OptT& sh,
              int64_t degree, const Tensor& campos, bool prefiltered, bool debug, int64_t compat, bool activate,
              const std::vector<std::vector<int64_t>>& windows, int64_t feature_ready,
              const std::vector<int64_t>& capacity, const std::vector<int64_t>& hint, const OptT& walk_order,
              const OptT& zero_fill, int64_t stream) {
  Inputs in(means3D, colors, sem, opacity, scales, rotations, scale_modifier, cov3D, sh, degree);
  if (activate) in.g.flags |= GS_FLAG_ACTIVATE;
  in.g.feature_ready = reinterpret_cast<gs_event_t>(feature_ready);
  if (present(zero_fill)) {  // the backward's scratch, zeroed by the blend (gs_gaussians.zero_fill)
    const Tensor& z = *zero_fill;
    if (z.device() != in.dev || !z.is_contiguous())
      throw std::runtime_error("zero_fill must be a contiguous device tensor");
    in.g.zero_fill = z.data_ptr();
    in.g.zero_fill_bytes = (int64_t)(z.numel() * z.element_size()) & ~(int64_t)15;
  }
  if (present(walk_order)) {
    const Tensor& w = *walk_order;
    if (w.scalar_type() != at::kInt || w.device() != in.dev || !w.is_contiguous() || w.numel() != in.P)
      throw std::runtime_error("walk_order must be a contiguous int32 device tensor of P ids");
    in.g.walk_order = w.data_ptr<int32_t>();
  }
  Cameras k(in.dev, bg, views, projs, campos, cx, cy, tx, ty, W, H, windows);
  const int32_t C = (int32_t)k.cams.size();
  const auto f32 = at::TensorOptions().dtype(at::kFloat).device(in.dev);
  const auto u8 = at::TensorOptions().dtype(at::kByte).device(in.dev);
  Tensor out_color = at::empty({C, 3, H, W}, f32);
  Tensor out_feature = at::empty({C, in.F, H, W}, f32);
  Tensor out_depth = at::empty({C, 1, H, W}, f32);
  Tensor out_alpha = at::empty({C, 1, H, W}, f32);
  Tensor radii = at::empty({C, in.P}, f32.dtype(at::kInt));
  Tensor geom = at::empty({(int64_t)gs_batch_geom_buffer_bytes(in.P, C)}, u8);
  Tensor img = at::empty({(int64_t)gs_batch_image_buffer_bytes((int32_t)W, (int32_t)H, C)}, u8);
  std::vector<int64_t> NR(C, 0), NI(C, 0);
  gs_stream_t s = reinterpret_cast<gs_stream_t>(stream);
  float* oc = out_color.data_ptr<float>();
  float* of = in.F ? out_feature.data_ptr<float>() : nullptr;
  float* od = out_depth.data_ptr<float>();
  float* oa = out_alpha.data_ptr<float>();
  Tensor binning;
  bool fitted = false;
  gs_batch_hint h{};
  if (!capacity.empty() && !debug) {
    if ((int64_t)capacity.size() != C) throw std::runtime_error("capacity must have C entries");
    if (hint.size() == 6) {
      h.valid = (int32_t)hint[0];
      h.p1 = (int32_t)hint[1];
      h.q1 = (int32_t)hint[2];
      h.p2 = (int32_t)hint[3];
      h.max_len = hint[4];
      h.total = hint[5];
    }
    const int64_t nb = (int64_t)gs_batch_binning_buffer_bytes(C, capacity.data());
    binning = at::empty({nb > 1 ? nb : 1}, u8);
    int32_t fits = 0;
    check(gs_forward_batch(&in.g, k.cams.data(), C, prefiltered ? 1 : 0, (int)compat, geom.data_ptr(),
                           img.data_ptr(), binning.data_ptr(), capacity.data(), &h, radii.data_ptr<int32_t>(),
                           NR.data(), NI.data(), &fits, oc, of, od, oa, s),
          "rasterize_gaussians_batch (sync-free forward)");
    fitted = fits != 0;
  } else {
    check(gs_forward_plan_batch(&in.g, k.cams.data(), C, prefiltered ? 1 : 0, debug ? 1 : 0, (int)compat,
                                geom.data_ptr(), img.data_ptr(), radii.data_ptr<int32_t>(), NR.data(), NI.data(), s),
          "rasterize_gaussians_batch (preprocess)");
  }
  std::vector<int64_t> layout = NI;
  if (fitted) {
    layout = capacity;
  } else {
    // two-phase, or the sync-free attempt's retry with the exact lengths
    const int64_t nb = (int64_t)gs_batch_binning_buffer_bytes(C, NI.data());
    binning = at::empty({nb > 1 ? nb : 1}, u8);
    check(gs_forward_render_batch(&in.g, k.cams.data(), C, debug ? 1 : 0, (int)compat, geom.data_ptr(),
                                  binning.data_ptr(), img.data_ptr(), NI.data(), radii.data_ptr<int32_t>(), oc, of, od,
                                  oa, s),
          "rasterize_gaussians_batch (render)");
  }
  Tensor feature_map = in.F_user != in.F ? out_feature.narrow(1, 0, in.F_user) : out_feature;
  std::vector<int64_t> hint_out = {h.valid, h.p1, h.q1, h.p2, h.max_len, h.total};
  return {NR, out_color, feature_map, out_depth, out_alpha, radii, geom, binning, img, NI, layout, hint_out, fitted};
}

// [C, ch, H, W] fp32 of an upstream gradient (channels zero-padded to ch), or undefined
Tensor batch_image(const OptT& t, int64_t C, int64_t ch, int64_t H, int64_t W, const at::Device& dev,
                   const char* name) {
  if (!present(t)) return Tensor();
  Tensor u = dev_f32(*t, dev, name).reshape({C, -1, H, W});
  if (u.size(1) < ch)
    u = at::cat({u, at::zeros({C, ch - u.size(1), H, W}, u.options())}, 1);
  return u.contiguous();
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> backward_batch(
    const Tensor& bg, const Tensor& means3D, const Tensor& radii, const OptT& colors, const OptT& sem,
    const OptT& scales, const OptT& rotations, double scale_modifier, const OptT& cov3D, const Tensor& views,
    const Tensor& projs, const std::vector<double>& cx, const std::vector<double>& cy, const std::vector<double>& tx,
    const std::vector<double>& ty, const OptT& dL_color, const OptT& dL_feature, const OptT& dL_depth,
    const OptT& dL_alpha, const OptT& sh, int64_t degree, const Tensor& campos, const Tensor& geom,
    const std::vector<int64_t>& num_instances, const OptT& binning, const Tensor& img, const Tensor& alphas,
    bool debug, int64_t compat, const OptT& grad_mask, c10::optional<std::vector<Tensor>> densify,
    const OptT& opacity, bool activate, const std::vector<std::vector<int64_t>>& windows,
    const std::vector<Tensor>& out, const OptT& scratch_in, bool scratch_zeroed, int64_t stream) {
  if (activate && !present(opacity)) throw std::runtime_error("activate=True needs the raw opacities");
  Inputs in(means3D, colors, sem, activate ? opacity : c10::nullopt, scales, rotations, scale_modifier, cov3D, sh,
            degree);
  if (activate) in.g.flags |= GS_FLAG_ACTIVATE;
  const int64_t C = (int64_t)cx.size();
  if (!out.empty() && out.size() != 9) throw std::runtime_error("out must hold the 9 gradient destinations");
  const Tensor& img_ref = present(dL_color) ? *dL_color : alphas;
  const int64_t H = img_ref.size(-2), W = img_ref.size(-1);
  Cameras k(in.dev, bg, views, projs, campos, cx, cy, tx, ty, W, H, windows);
  const auto f32 = at::TensorOptions().dtype(at::kFloat).device(in.dev);
  const int64_t P = in.P;
  Tensor gm;
  if (grad_mask.has_value() && grad_mask->defined()) {
    gm = grad_mask->to(in.dev, at::kFloat).reshape({-1}).contiguous();
    if (gm.numel() != P) throw std::runtime_error("grad_mask must have " + std::to_string(P) + " elements");
    in.g.grad_mask = gm.data_ptr<float>();
  }
  Tensor dLc = batch_image(dL_color, C, 3, H, W, in.dev, "dL_dout_color");
  Tensor dLd = batch_image(dL_depth, C, 1, H, W, in.dev, "dL_dout_depth");
  Tensor dLa = batch_image(dL_alpha, C, 1, H, W, in.dev, "dL_dout_alpha");
  Tensor dLf = in.F ? batch_image(dL_feature, C, in.F, H, W, in.dev, "dL_dout_feature") : Tensor();
  Tensor alphas_c = dev_f32(alphas, in.dev, "alpha");
  Tensor radii_c = radii.to(in.dev, at::kInt).contiguous();
  if (radii_c.dim() != 2 || radii_c.size(0) != C || radii_c.size(1) != P)
    throw std::runtime_error("radii must be [C=" + std::to_string(C) + ", P=" + std::to_string(P) + "]");
  if ((int64_t)num_instances.size() != C) throw std::runtime_error("num_instances must have C entries");
  const std::vector<std::vector<int64_t>> shapes = {{P, 3}, {P, 3}, {P, in.F}, {P, 1}, {P, 3},
                                                    {P, 6}, {P, in.M, 3}, {P, 3}, {P, 4}};
  // Caller-owned destinations (a gradient bucket's views): written, not
  // accumulated; an empty tensor = allocate.
  std::vector<Tensor> o;
  for (int i = 0; i < 9; ++i) {
    if (out.empty() || out[i].numel() == 0) {
      o.push_back(at::empty(shapes[i], f32));
      continue;
    }
    const Tensor& d = out[i];
    int64_t n = 1;
    for (int64_t e : shapes[i]) n *= e;
    if (d.scalar_type() != at::kFloat || d.device() != in.dev || !d.is_contiguous() || d.numel() != n)
      throw std::runtime_error("out[" + std::to_string(i) + "] must be a contiguous fp32 device tensor of " +
                               std::to_string(n) + " elements");
    o.push_back(d.view(shapes[i]));
  }
  if (densify.has_value()) {
    const auto& d = *densify;
    if (d.size() != 3) throw std::runtime_error("densify must hold (accum, denom, max_radius)");
    for (const auto& t : d)
      if (t.dim() != 1 || t.size(0) != P || t.scalar_type() != at::kFloat || t.device() != in.dev || !t.is_contiguous())
        throw std::runtime_error("densify statistics must be contiguous fp32 (P,) tensors on the device");
    in.g.densify_accum = d[0].data_ptr<float>();
    in.g.densify_denom = d[1].data_ptr<float>();
    in.g.max_radius = d[2].data_ptr<float>();
  }
  // the scratch: the caller's (kept from the forward, which may have zeroed
  // it: scratch_zeroed -> GS_FLAG_SCRATCH_ZEROED) or a fresh one
  const int64_t nscr = (int64_t)gs_batch_backward_scratch_bytes(P, (int32_t)in.F, (int32_t)C);
  Tensor scratch;
  if (present(scratch_in)) {
    scratch = *scratch_in;
    if (scratch.device() != in.dev || !scratch.is_contiguous() || scratch.numel() * scratch.element_size() < nscr)
      throw std::runtime_error("scratch must be a contiguous device tensor of " + std::to_string(nscr) + " bytes");
    if (scratch_zeroed) in.g.flags |= GS_FLAG_SCRATCH_ZEROED;
  } else {
    scratch = at::empty({nscr}, f32.dtype(at::kByte));
  }
  const Tensor bin = binning.has_value() ? *binning : Tensor();
  auto fp = [](const Tensor& t) -> const float* { return t.defined() ? t.data_ptr<float>() : nullptr; };
  check(gs_backward_batch(&in.g, k.cams.data(), (int32_t)C, radii_c.data_ptr<int32_t>(), debug ? 1 : 0, (int)compat,
                          geom.data_ptr(), nz(bin), img.data_ptr(), num_instances.data(), alphas_c.data_ptr<float>(),
                          fp(dLc), fp(dLf), fp(dLd), fp(dLa), scratch.data_ptr(), o[0].data_ptr<float>(),
                          o[1].data_ptr<float>(), static_cast<float*>(nz(o[2])), o[3].data_ptr<float>(),
                          o[4].data_ptr<float>(), o[5].data_ptr<float>(), static_cast<float*>(nz(o[6])),
                          o[7].data_ptr<float>(), o[8].data_ptr<float>(), reinterpret_cast<gs_stream_t>(stream)),
        "rasterize_gaussians_batch_backward");
  Tensor dsem = in.F_user != in.F ? o[2].narrow(1, 0, in.F_user) : o[2];
  return {o[0], o[1], dsem, o[3], o[4], o[5], o[6], o[7], o[8]};
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "native fast path of dynamic3dgaussians_amd._C (C++ over the gsplat_hip C ABI)";
  m.def("abi_version", []() { return gs_version(); });
  m.def("forward", &forward);
  m.def("backward", &backward);
  m.def("forward_batch", &forward_batch);
  m.def("backward_batch", &backward_batch);
}
