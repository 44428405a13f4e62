// gs_api.hip -- the C ABI (include/gsplat_hip.h): argument checks, opaque
// state-buffer carving, launch order and error reporting.  Host code only.
//
// Launch order mirrors CudaRasterizer::Rasterizer::forward/backward
// (DGR/cuda_rasterizer/rasterizer_impl.cu:198-467), but everything goes to
// the caller's stream, nothing is allocated inside the library, and the
// backward's per-call cudaMalloc/cudaFree (:408-409, :436) is gone.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gs_knn.h"
#include "../../include/gs_neighbor.h"
#include "../../include/gs_optim.h"
#include "../../include/gsplat_hip.h"
#include "gs_common.h"
#include "gs_kernels.h"

using namespace gs;

namespace {
// the thread's error message (gs_host.cpp: gs_last_error)
#define fail gs_set_error

// Post-launch check: always catch launch errors; with `debug`, also
// synchronise and surface asynchronous faults (the reference's CHECK_CUDA
// debug mode, CR/auxiliary.h:172-179).
int check(const char* what, int debug, hipStream_t s) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && debug) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail((int)e, "%s: %s", what, hipGetErrorString(e));
  return 0;
}

int higher_msb(uint32_t n) {  // getHigherMsb, CR/rasterizer_impl.cu:35-50
  uint32_t msb = sizeof(n) * 4, step = msb;
  while (step > 1) {
    step /= 2;
    if (n >> msb) msb += step; else msb -= step;
  }
  if (n >> msb) msb++;
  return (int)msb;
}

template <class T>
T* at(void* base, size_t off) { return reinterpret_cast<T*>(static_cast<char*>(base) + off); }
template <class T>
const T* at(const void* base, size_t off) { return reinterpret_cast<const T*>(static_cast<const char*>(base) + off); }

bool feature_supported(int F) { return F == 0 || F == 4 || F == 8 || F == 16 || F == 32 || F == 36 || F == 64; }

int check_gaussians(const gs_gaussians* g, const gs_camera* c, bool forward) {
  if (!g || !c) return fail(-1, "null argument block");
  if (g->P < 0) return fail(-1, "P must be >= 0 (got %d)", g->P);
  if (c->image_width <= 0 || c->image_height <= 0)
    return fail(-1, "image size must be positive (got %dx%d)", c->image_width, c->image_height);
  if (!feature_supported(g->F))
    return fail(-1, "semantic feature width %d not instantiated (0, 4, 8, 16, 32, 36, 64)", g->F);
  if (g->P > 0) {
    if (!g->means3D || (forward && !g->opacities)) return fail(-1, "means3D and opacities are required");
    if (!c->viewmatrix || !c->projmatrix || !c->campos || !c->background)
      return fail(-1, "camera matrices, campos and background are required");
    if (!g->colors_precomp && !g->shs) return fail(-1, "provide SHs or precomputed colors");
    if (!g->cov3D_precomp && (!g->scales || !g->rotations))
      return fail(-1, "provide scales+rotations or a precomputed 3D covariance");
    if (g->shs && (g->D < 0 || g->D > 3 || g->M < (g->D + 1) * (g->D + 1)))
      return fail(-1, "SH degree %d needs M >= %d coefficients (got M=%d)", g->D, (g->D + 1) * (g->D + 1), g->M);
    if (g->F > 0 && !g->semantic_feature) return fail(-1, "F > 0 but semantic_feature is null");
  }
  return 0;
}
// ---- optional live kernel timing (bench instrumentation) ------------------
// When enabled, an event pair is recorded on the launch stream around each
// timed stage; gs_timing_read() resolves them.  Off by default (zero cost).
struct TimedEvent {
  hipEvent_t a, b;
  int kind;
};
std::mutex g_tmu;
bool g_timing = false;
uint32_t g_timing_mask = 0xFFFFFFFFu;  // stages timed while enabled
std::vector<TimedEvent> g_events;
std::vector<hipEvent_t> g_pool;

hipEvent_t pool_get() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  // device-scope release: no system-scope cache writeback when the stream
  // reaches the event (hipEventReleaseToDevice), so timing a kernel does not
  // add that to the step it is timed in
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventReleaseToDevice) != hipSuccess) (void)hipEventCreate(&e);
  return e;
}

// attach = true: a one-kernel stage whose launch goes through timed_launch
// (gs_kernels.h): the events ride on the dispatch instead of marker packets.
struct StageTimer {
  hipStream_t s;
  int kind;
  bool attach;
  hipEvent_t a = nullptr, b = nullptr;
  StageTimer(hipStream_t s_, int kind_, bool attach_ = false) : s(s_), kind(kind_), attach(attach_) {
    std::lock_guard<std::mutex> lk(g_tmu);
    if (!g_timing || !((g_timing_mask >> kind) & 1u)) return;
    a = pool_get();
    b = pool_get();
    if (attach) launch_events() = LaunchEvents{a, b};
    else (void)hipEventRecord(a, s);
  }
  ~StageTimer() {
    if (!a) return;
    if (!attach) {
      (void)hipEventRecord(b, s);
    } else if (launch_events().start) {  // nothing was launched: an empty interval
      launch_events() = LaunchEvents{};
      (void)hipEventRecord(a, s);
      (void)hipEventRecord(b, s);
    }
    std::lock_guard<std::mutex> lk(g_tmu);
    g_events.push_back({a, b, kind});
  }
};
}  // namespace
namespace gs {
LaunchEvents& launch_events() {
  thread_local LaunchEvents e;
  return e;
}
}  // namespace gs
namespace {

// The plan's header as read back by gs_forward_plan, remembered per thread so
// that gs_forward_render can size its sort launch without another readback.
struct PlanInfo {
  const void* image = nullptr;
  int C = 0;
  int64_t L = -1;        // the batch's total list instances
  int64_t max_len = -1;  // its longest tile
  SortClasses sort;       // where the sort's length classes sit in the dispatch order
};
thread_local PlanInfo g_plan;

// Host landing areas of the plan headers (GS_MAX_CAMS x M_WORDS words each):
// page-locked, device-mapped, coherent host memory that tile_offsets_kernel
// writes directly (the host polls a sentinel word, publish_wait).  Leased
// per call from a process-wide pool, so the number of buffers is bounded by
// the number of concurrent callers (not by the threads that ever called:
// thread pools and autograd workers would otherwise each pin one for good).
// Never freed: a pool destructor could run after the HIP runtime is gone.
// A slot belongs to the device that was current when it was made (its
// device-side mapping is that device's): a lease only takes a free
// slot of the calling thread's current device.
struct HeaderSlot {
  uint32_t* host = nullptr;  // host pointer
  uint32_t* dev = nullptr;   // the same memory as the kernels address it
  int device = -1;
};
std::mutex g_hmu;
std::vector<HeaderSlot> g_hfree;

struct HeaderLease {
  HeaderSlot s;
  // set once a plan kernel that writes this slot may have been enqueued (on
  // `stream`); cleared when the caller has seen every header written.  A
  // lease dropped in between (an error path after the launch) synchronizes
  // that stream before the slot goes back to the pool, so the next caller's
  // sentinel cannot be overwritten by a stale kernel.
  bool in_flight = false;
  hipStream_t stream = nullptr;
  void launched(hipStream_t s_) {
    in_flight = true;
    stream = s_;
  }
  HeaderLease() {
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) return;
    {
      std::lock_guard<std::mutex> lk(g_hmu);
      for (size_t i = g_hfree.size(); i-- > 0;) {
        if (g_hfree[i].device != device) continue;
        s = g_hfree[i];
        g_hfree.erase(g_hfree.begin() + (std::ptrdiff_t)i);
        return;
      }
    }
    s.device = device;
    void* h = nullptr;
    if (hipHostMalloc(&h, sizeof(uint32_t) * GS_MAX_CAMS * M_WORDS,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      s = HeaderSlot{};
      return;
    }
    s.host = static_cast<uint32_t*>(h);
    s.dev = static_cast<uint32_t*>(d);
  }
  ~HeaderLease() {
    if (!s.host) return;
    // a kernel that may still write the slot: wait for it, or (the device
    // failed) keep the slot out of the pool for good
    if (in_flight && hipStreamSynchronize(stream) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(g_hmu);
    g_hfree.push_back(s);
  }
  bool ok() const { return s.host != nullptr; }
};

// The tile sort's launch extents: the plan's longest tile and class prefixes
// (exact, from the header; or a previous plan's with margins, whose coverage
// the caller checks against the header afterwards), or unknown (every class
// launch covers all tiles).
struct SortPlan {
  int64_t max_len = -1;  // -1: unknown
  int64_t total = -1;    // instances of the batch (the short class's workgroup size)
  SortClasses sc;
  bool hinted = false;   // extents from an earlier plan (gs_batch_hint): coverage checked
};

// What launch_tile_sort(max_len, sc) covers (tile_sort_launches' class
// decisions): nothing to check with unknown extents (every class launch
// covers all tiles) or when exact (they came from this very plan).
SortCover sort_cover(const SortPlan& sp, int64_t tiles) {
  SortCover cv;
  if (sp.max_len < 0 || !sp.sc.valid || !sp.hinted) return cv;
  cv.on = 1;
  cv.q1 = sp.sc.q1;
  cv.p1 = sp.sc.p1;
  cv.p2 = sp.sc.p2;
  cv.mid = sp.max_len > SORT_SMALL;
  cv.lng = sp.max_len > TS_CAP;
  (void)tiles;
  return cv;
}

TileArgs tile_args(int P, int W, int H, void* geom, void* image, const int32_t* walk = nullptr) {
  TileArgs t{};
  t.walk = walk;
  const GeomLayout gl(P);
  const ImgLayout il(W, H);
  t.P = P; t.W = W; t.H = H;
  t.grid_x = (W + TILE - 1) / TILE; t.grid_y = (H + TILE - 1) / TILE;
  t.num_tiles = (int)il.tiles;
  t.rect = at<uint4>(geom, gl.rect);
  t.tiles = at<uint32_t>(geom, gl.tiles);
  t.rec = at<float>(geom, gl.rec);
  t.thist = at<uint32_t>(image, il.thist);
  t.ttotal = at<uint32_t>(image, il.ttotal);
  t.bsum = at<uint32_t>(image, il.bsum);
  t.meta = at<uint32_t>(image, il.meta);
  t.ranges = at<uint2>(image, il.ranges);
  t.order = at<uint4>(image, il.order);
  t.fmax = at<uint32_t>(image, il.fmax);
  return t;
}
}  // namespace

extern "C" {

int gs_timing_enable(int enable) {
  std::lock_guard<std::mutex> lk(g_tmu);
  for (auto& e : g_events) { g_pool.push_back(e.a); g_pool.push_back(e.b); }
  g_events.clear();
  g_timing = enable != 0;
  return 0;
}

int gs_timing_select(uint32_t stage_mask) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_timing_mask = stage_mask;
  return 0;
}

int gs_timing_read(double* ms, int64_t* count, int n_kinds) {
  std::lock_guard<std::mutex> lk(g_tmu);
  for (int k = 0; k < n_kinds; ++k) { ms[k] = 0.0; count[k] = 0; }
  for (auto& e : g_events) {
    if (e.kind < 0 || e.kind >= n_kinds) continue;
    hipError_t r = hipEventSynchronize(e.b);
    float t = 0.f;
    if (r == hipSuccess) r = hipEventElapsedTime(&t, e.a, e.b);
    if (r != hipSuccess) return fail((int)r, "timing read: %s", hipGetErrorString(r));
    ms[e.kind] += t;
    count[e.kind] += 1;
  }
  return 0;
}

int gs_version(void) { return GS_ABI_VERSION; }

size_t gs_geom_buffer_bytes(int64_t P) { return GeomLayout(P > 0 ? P : 0).total; }
size_t gs_binning_buffer_bytes(int64_t L) { return BinLayout(L > 0 ? L : 0).total; }
size_t gs_image_buffer_bytes(int32_t W, int32_t H) { return ImgLayout(W, H).total; }
size_t gs_backward_scratch_bytes(int64_t P, int32_t F) { return gs_batch_backward_scratch_bytes(P, F, 1); }

// ---- forward / backward: camera batches (C = 1: the reference's entry points)

// The batch's CamBatch from C gs_camera blocks: matrices contiguous per
// camera (camera c's at camera 0's + 16 c / + 3 c), one shared background.
static int make_batch(const gs_camera* cams, int C, int P, int W, int H, CamBatch& cb) {
  if (C < 1 || C > GS_MAX_CAMS) return fail(-1, "camera batch size %d outside 1..%d", C, GS_MAX_CAMS);
  cb = CamBatch{};
  cb.C = C;
  cb.geom_stride = (int64_t)GeomLayout(P).total;
  cb.img_stride = (int64_t)ImgLayout(W, H).total;
  cb.view = cams[0].viewmatrix;
  cb.proj = cams[0].projmatrix;
  cb.campos = cams[0].campos;
  for (int c = 0; c < C; ++c) {
    const gs_camera& k = cams[c];
    if (k.image_width != W || k.image_height != H)
      return fail(-1, "camera %d: every camera of a batch has the image size of camera 0", c);
    if (k.viewmatrix != cb.view + 16 * c || k.projmatrix != cb.proj + 16 * c || k.campos != cb.campos + 3 * c)
      return fail(-1, "camera %d: batch camera matrices must be contiguous ([C,16], [C,16], [C,3])", c);
    if (k.background != cams[0].background)
      return fail(-1, "camera %d: the cameras of a batch share one background", c);
    const int gx = (W + TILE - 1) / TILE, gy = (H + TILE - 1) / TILE;
    if (k.tile_x0 == 0 && k.tile_y0 == 0 && k.tile_x1 == 0 && k.tile_y1 == 0) {
      cb.win[c][0] = 0; cb.win[c][1] = 0; cb.win[c][2] = (uint16_t)gx; cb.win[c][3] = (uint16_t)gy;
    } else {
      if (k.tile_x0 < 0 || k.tile_y0 < 0 || k.tile_x0 >= k.tile_x1 || k.tile_y0 >= k.tile_y1 || k.tile_x1 > gx ||
          k.tile_y1 > gy)
        return fail(-1, "camera %d: tile window [%d, %d) x [%d, %d) outside the %d x %d tile grid", c, k.tile_x0,
                    k.tile_x1, k.tile_y0, k.tile_y1, gx, gy);
      cb.win[c][0] = (uint16_t)k.tile_x0; cb.win[c][1] = (uint16_t)k.tile_y0;
      cb.win[c][2] = (uint16_t)k.tile_x1; cb.win[c][3] = (uint16_t)k.tile_y1;
    }
    cb.c_x[c] = k.c_x;
    cb.c_y[c] = k.c_y;
    cb.tanx[c] = k.tan_fovx;
    cb.tany[c] = k.tan_fovy;
  }
  return 0;
}

// Binning buffer offsets of the cameras (each a BinLayout of its own length).
static int64_t batch_bin_offsets(int C, const int64_t* L, CamBatch* cb) {
  int64_t o = 0;
  for (int c = 0; c < C; ++c) {
    const int64_t l = L ? (L[c] > 0 ? L[c] : 0) : 0;
    if (cb) {
      cb->bin_off[c] = o;
      cb->bin_L[c] = l;
    }
    o += (int64_t)BinLayout(l).total;
  }
  return o;
}

// backward scratch: the per-camera accumulation records, then (feature widths
// whose gradient rows are not 64-B multiples, F = 36) a padded-stride feature
// gradient area
static size_t acc_bytes(int64_t P, int32_t C) {
  return align_up(sizeof(float) * (size_t)ACC_STRIDE * (size_t)(P > 0 ? P : 0) * (C > 0 ? C : 0), 256);
}
static size_t feat_pad_bytes(int64_t P, int32_t F) {
  const int FS = feature_grad_stride(F);
  return FS == F ? 0 : align_up(sizeof(float) * (size_t)FS * (size_t)(P > 0 ? P : 0), 256);
}

// ---------------------------------------------------------------- debug checks
// Host-side validation of the forward's state under `debug` (gsplat_hip.h):
// gs_check_plan_header / gs_check_ranges / gs_check_point_list, gs_host.cpp.

// debug mode, after the sort: every camera's ranges and list ids, read back
static int debug_check_lists(const TileArgs& ta, const CamBatch& cb, const void* binning, const int64_t* L,
                             int64_t P, int64_t tiles, int64_t max_len, hipStream_t s) {
  std::vector<uint32_t> rg((size_t)2 * (tiles > 0 ? tiles : 1)), ids;
  for (int c = 0; c < cb.C; ++c) {
    hipError_t e = hipMemcpyAsync(rg.data(), shift_bytes(ta.ranges, c * cb.img_stride), 8 * (size_t)tiles,
                                  hipMemcpyDeviceToHost, s);
    const int64_t l = L[c] > 0 ? L[c] : 0;
    ids.resize((size_t)(l > 0 ? l : 1));
    if (e == hipSuccess && l > 0)
      e = hipMemcpyAsync(ids.data(), static_cast<const char*>(binning) + cb.bin_off[c], 4 * (size_t)l,
                         hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail((int)e, "debug readback: %s", hipGetErrorString(e));
    if (int r = gs_check_ranges(rg.data(), tiles, l, max_len)) return r;
    if (int r = gs_check_point_list(ids.data(), l, P)) return r;
  }
  return 0;
}

// The plan's kernels (preprocess, tile histogram, column scan, offsets), the
// headers published to hdr_dev (mapped host memory) by the last of them.
static int plan_enqueue(const gs_gaussians* g, const gs_camera* cams, int C, int prefiltered, int debug, void* geom,
                        void* image, int32_t* radii, uint32_t* hdr_dev, CamBatch& cb, hipStream_t s) {
  const int P = g->P;
  const int W = cams[0].image_width, H = cams[0].image_height;
  if (int e = make_batch(cams, C, P, W, H, cb)) return e;
  const GeomLayout gl(P);
  if (debug && g->walk_order && P > 0) {
    // debug mode: the walk order must be a permutation of the ids (a
    // repeated or missing id would bin a Gaussian twice or not at all)
    std::vector<int32_t> w(P);
    const hipError_t e = hipMemcpyAsync(w.data(), g->walk_order, 4 * (size_t)P, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return fail((int)e, "walk_order: cannot read it back");
    if (int r = gs_check_walk_order(w.data(), P)) return r;
  }
  const TileArgs ta = tile_args(P, W, H, geom, image, g->walk_order);
  PreprocessArgs a{};
  a.P = P; a.D = g->D; a.M = g->M; a.W = W; a.H = H;
  a.grid_x = ta.grid_x; a.grid_y = ta.grid_y;
  a.prefiltered = prefiltered;
  a.activate = (g->flags & GS_FLAG_ACTIVATE) != 0;
  a.means3D = g->means3D; a.scales = g->scales; a.rotations = g->rotations; a.opacities = g->opacities;
  a.shs = g->shs; a.cov3D_precomp = g->cov3D_precomp; a.colors_precomp = g->colors_precomp;
  a.scale_modifier = g->scale_modifier;
  a.radii = radii;
  a.rec = at<float>(geom, gl.rec);
  a.cov3D = at<float>(geom, gl.cov3D);
  a.clamped = at<uint8_t>(geom, gl.clamped);
  a.tiles = at<uint32_t>(geom, gl.tiles);
  a.rect = at<uint4>(geom, gl.rect);
  a.status = reinterpret_cast<int*>(ta.meta + M_STATUS);
  if (prefiltered)  // culled-but-prefiltered flags
    for (int c = 0; c < C; ++c) (void)hipMemsetAsync(shift_bytes(a.status, c * cb.img_stride), 0, 4, s);
  {
    StageTimer t(s, GS_STAGE_PREPROCESS);
    launch_preprocess_fwd(a, cb, s);
  }
  if (int e = check("preprocess", debug, s)) return e;
  {
    StageTimer t(s, GS_STAGE_SCAN);
    launch_tile_plan(ta, cb, prefiltered, hdr_dev, s);
  }
  return check("tile plan", debug, s);
}

// The host's reading of the C plan headers: the reference's counts, the list
// instances, the sort extents (PlanInfo), status checks.
static int plan_read(const uint32_t (*host)[M_WORDS], int C, int prefiltered, int debug, int64_t tiles,
                     int64_t* num_rendered, int64_t* num_instances, PlanInfo& info) {
  int64_t max_len = 0, total = 0;
  SortClasses sc;
  sc.valid = true;
  sc.q1 = 0x7FFFFFFF;
  for (int c = 0; c < C; ++c) {
    if (debug)
      if (int e = gs_check_plan_header(host[c], tiles)) return e;
    sc.p1 = (int)host[c][M_SORT_P1] > sc.p1 ? (int)host[c][M_SORT_P1] : sc.p1;
    sc.p2 = (int)host[c][M_SORT_P2] > sc.p2 ? (int)host[c][M_SORT_P2] : sc.p2;
    sc.q1 = (int)host[c][M_SORT_Q1] < sc.q1 ? (int)host[c][M_SORT_Q1] : sc.q1;
    if (prefiltered && (host[c][M_STATUS] & 1u))
      return fail(-2, "Point is filtered although prefiltered is set. This shouldn't happen!");
    if (host[c][M_STATUS] & 2u) return fail(-1, "more than 2^32 tile instances");
    num_rendered[c] = host[c][M_LREF];
    if (num_instances) num_instances[c] = host[c][M_L];
    max_len = host[c][M_MAXN] > max_len ? host[c][M_MAXN] : max_len;
    total += host[c][M_L];
  }
  info.C = C;
  info.L = total;
  info.max_len = max_len;
  info.sort = C > 0 ? sc : SortClasses{};
  return 0;
}

// The headers' way to the host after plan_enqueue: tile_offsets_kernel
// stores them to the mapped buffer (an in-stream copy of the device headers
// instead measured slower).
// Wait until the plan kernel has written every camera's header: the host
// polls each header's last word (header_sentinel: 0 once written, stored by
// tile_offsets_kernel after the rest and a system fence), yielding the core
// between reads.  Every few thousand reads it asks whether the stream has
// drained: a stream done or failed with a header still unwritten is an error,
// not a hang.  No event rides on the plan kernel (its completion signal idled
// the GPU 15-27 us behind it, profiles/r06gaps3/).
static int publish_wait(HeaderLease& hl, int C, hipStream_t s) {
  auto written = [&]() {
    for (int c = 0; c < C; ++c)
      if (__atomic_load_n(&hl.s.host[c * M_WORDS + M_WORDS - 1], __ATOMIC_ACQUIRE) != 0u) return false;
    return true;
  };
  for (uint32_t spin = 1; !written(); ++spin) {
    if ((spin & 4095u) == 0u) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) {
        if (written()) break;
        for (int c = 0; c < C; ++c)
          if (__atomic_load_n(&hl.s.host[c * M_WORDS + M_WORDS - 1], __ATOMIC_ACQUIRE) != 0u)
            return fail(-4, "plan header of camera %d was not written (header path)", c);
      } else if (q != hipErrorNotReady) {
        return fail((int)q, "num_rendered readback: %s", hipGetErrorString(q));
      }
    }
    std::this_thread::yield();
  }
  hl.in_flight = false;
  return 0;
}

// Mark the leased header words unwritten before the plan that fills them.
static void header_sentinel(HeaderLease& hl, int C) {
  for (int c = 0; c < C; ++c) hl.s.host[c * M_WORDS + M_WORDS - 1] = 0xFFFFFFFFu;
}

static int plan_impl(const gs_gaussians* g, const gs_camera* cams, int C, int prefiltered, int debug, int compat,
                     void* geom, void* image, int32_t* radii, int64_t* num_rendered, int64_t* num_instances,
                     hipStream_t s) {
  if (int e = check_gaussians(g, cams, true)) return e;
  if (!num_rendered) return fail(-1, "num_rendered is null");
  for (int c = 0; c < C; ++c) {
    num_rendered[c] = 0;
    if (num_instances) num_instances[c] = 0;
  }
  g_plan = PlanInfo{};
  const int P = g->P;
  if (P == 0) return 0;
  if (!geom || !image || !radii) return fail(-1, "geom buffer, image buffer and radii are required");
  HeaderLease hl;
  if (!hl.ok()) return fail((int)hipErrorOutOfMemory, "cannot allocate the page-locked plan header buffer");
  header_sentinel(hl, C);
  CamBatch cb;
  hl.launched(s);
  if (int e = plan_enqueue(g, cams, C, prefiltered, debug, geom, image, radii, hl.s.dev, cb, s))
    return e;
  // The one host read of the forward (CR/rasterizer_impl.cu:287), one for
  // the whole batch: the list instance counts size the binning buffer; the
  // reference's counts and the rest of the headers ride along.
  const TileArgs ta = tile_args(P, cams[0].image_width, cams[0].image_height, geom, image);
  if (int e = publish_wait(hl, C, s)) return e;
  PlanInfo info;
  if (int e = plan_read(reinterpret_cast<const uint32_t(*)[M_WORDS]>(hl.s.host), C, prefiltered, debug,
                        (int64_t)ta.grid_x * ta.grid_y, num_rendered, num_instances, info))
    return e;
  info.image = image;
  g_plan = info;
  (void)compat;
  return 0;
}

// L[c]: the instances camera c's binning buffer is laid out for (its list
// length, or gs_forward_batch's capacity); sp: the sort launch extents.
static int render_impl(const gs_gaussians* g, const gs_camera* cams, int C, int debug, int compat, void* geom,
                       void* binning, void* image, const int64_t* L, const int32_t* radii, float* out_color,
                       float* out_feature, float* out_depth, float* out_alpha, const SortPlan& sp, hipStream_t s) {
  if (int e = check_gaussians(g, cams, true)) return e;
  const int P = g->P;
  if (P == 0) return 0;  // the reference leaves the zero-filled outputs untouched
  int64_t total = 0;
  for (int c = 0; c < C; ++c) total += L[c] > 0 ? L[c] : 0;
  if (!geom || !image || (total > 0 && !binning) || !radii) return fail(-1, "state buffers are required");
  if (!out_color || !out_depth || (g->F > 0 && !out_feature) || (compat != COMPAT_REFERENCE && !out_alpha))
    return fail(-1, "output image pointers are required");
  const int W = cams[0].image_width, H = cams[0].image_height;
  CamBatch cb;
  if (int e = make_batch(cams, C, P, W, H, cb)) return e;
  batch_bin_offsets(C, L, &cb);
  const int gx = (W + TILE - 1) / TILE, gy = (H + TILE - 1) / TILE;
  const GeomLayout gl(P);
  const ImgLayout il(W, H);
  const float* rec = at<float>(geom, gl.rec);
  TileArgs ta = tile_args(P, W, H, geom, image, g->walk_order);
  ta.binning = total > 0 ? binning : nullptr;
  {
    // the dispatch order (longest list first) from the ranges: the stage the
    // reference's identifyTileRanges occupies
    StageTimer t(s, GS_STAGE_RANGES);
    launch_tile_order(ta, cb, sort_cover(sp, gx * gy), s);
  }
  if (total > 0) {
    {
      StageTimer t(s, GS_STAGE_DUPLICATE);
      launch_tile_bucket(ta, cb, s);
    }
    if (int e = check("duplicateWithKeys", debug, s)) return e;
    {
      StageTimer t(s, GS_STAGE_SORT);
      launch_tile_sort(ta, cb, sp.max_len, sp.total >= 0 ? sp.total : total,
                       sp.max_len >= 0 ? sp.sc : SortClasses{}, s);
    }
    if (int e = check("tile sort", debug, s)) return e;
    if (debug)
      if (int e = debug_check_lists(ta, cb, binning, L, P, (int64_t)gx * gy, sp.max_len, s))
        return e;
  }
  RenderArgs ra{};
  // the matrix-core feature widths gather rows by 32-bit byte offsets
  if (g->F >= 32 && (uint64_t)g->P * (uint64_t)g->F * 4u > 0xFFFFFFFFull)
    return fail(-1, "semantic feature table of %lld x %d floats exceeds 4 GiB", (long long)g->P, g->F);
  ra.W = W; ra.H = H; ra.grid_x = gx; ra.num_tiles = gx * gy; ra.F = g->F; ra.compat = compat; ra.P = g->P;
  ra.order = ta.order;
  ra.smax = at<uint32_t>(image, il.smax);
  ra.ranges = ta.ranges; ra.point_list = total > 0 ? static_cast<const uint32_t*>(binning) : nullptr;
  ra.rec = rec; ra.feats = g->semantic_feature;
  ra.bg = cams[0].background;
  ra.out_color = out_color; ra.out_feature = out_feature; ra.out_depth = out_depth; ra.out_alpha = out_alpha;
  ra.n_contrib = at<uint32_t>(image, il.n_contrib);
  ra.fmax = at<uint32_t>(image, il.fmax);
  if (g->zero_fill) {
    if ((reinterpret_cast<uintptr_t>(g->zero_fill) & 15) || g->zero_fill_bytes < 0 || (g->zero_fill_bytes & 15))
      return fail(-1, "zero_fill must be 16-B aligned and a multiple of 16 bytes long");
    ra.zero = static_cast<float4*>(g->zero_fill);
    ra.zero_n = g->zero_fill_bytes / 16;
    if (ra.num_tiles <= 0) {  // no blend launch to carry it
      (void)hipMemsetAsync(g->zero_fill, 0, (size_t)g->zero_fill_bytes, s);
      ra.zero = nullptr;
      ra.zero_n = 0;
    }
  }
  if (g->feature_ready) {
    const hipError_t e = hipStreamWaitEvent(s, (hipEvent_t)g->feature_ready, 0);
    if (e != hipSuccess) return fail((int)e, "waiting for feature_ready: %s", hipGetErrorString(e));
  }
  {
    // the matrix-core widths first take the features' per-channel range
    // (after the wait: the features may just have been updated); the stage
    // then holds both launches
    const bool mf = g->F >= 32;
    StageTimer t(s, GS_STAGE_RENDER_FWD, !mf);
    if (mf) launch_feature_absmax(g->semantic_feature, g->P, g->F, at<uint32_t>(image, il.fmax), s);
    if (!launch_render_fwd(ra, cb, s)) return fail(-1, "unsupported feature width %d", g->F);
  }
  return check("render", debug, s);
}

static int backward_impl(const gs_gaussians* g, const gs_camera* cams, int C, const int32_t* radii, int debug,
                         int compat, const void* geom, const void* binning, const void* image, const int64_t* L,
                         const float* alphas, const float* dL_dout_color, const float* dL_dout_feature,
                         const float* dL_dout_depth, const float* dL_dout_alpha, void* scratch, float* dL_dmeans2D,
                         float* dL_dcolors, float* dL_dsemantic, float* dL_dopacity, float* dL_dmeans3D,
                         float* dL_dcov3D, float* dL_dsh, float* dL_dscales, float* dL_drotations, hipStream_t s) {
  if (int e = check_gaussians(g, cams, false)) return e;
  const int P = g->P;
  if (P == 0) return 0;
  if (!geom || !image || !scratch || !radii) return fail(-1, "state buffers are required");
  if (!alphas) return fail(-1, "the forward's alpha image is required");
  if ((g->flags & GS_FLAG_ACTIVATE) && !g->opacities)
    return fail(-1, "GS_FLAG_ACTIVATE: the backward needs the raw opacities");
  if (!dL_dmeans2D || !dL_dcolors || !dL_dopacity || !dL_dmeans3D || !dL_dcov3D || !dL_dscales ||
      !dL_drotations || (g->F > 0 && !dL_dsemantic) || (g->M > 0 && !dL_dsh))
    return fail(-1, "gradient outputs are required");
  const int W = cams[0].image_width, H = cams[0].image_height;
  CamBatch cb;
  if (int e = make_batch(cams, C, P, W, H, cb)) return e;
  // the tile lists sit at the start of each camera's binning buffer and the
  // ranges say how long they are (an empty binning buffer: every list empty)
  batch_bin_offsets(C, L, &cb);
  const int gx = (W + TILE - 1) / TILE, gy = (H + TILE - 1) / TILE;
  const GeomLayout gl(P);
  const ImgLayout il(W, H);
  float* acc = static_cast<float*>(scratch);
  // the accumulation records start at zero: filled here, or already zeroed by
  // the forward's blend (gs_gaussians.zero_fill + GS_FLAG_SCRATCH_ZEROED)
  if (!(g->flags & GS_FLAG_SCRATCH_ZEROED)) (void)hipMemsetAsync(acc, 0, sizeof(float) * (size_t)ACC_STRIDE * P * C, s);
  const bool accumulate = (g->flags & GS_FLAG_ACCUMULATE) != 0;
  // the blend kernel adds the feature gradients atomically: zero first unless
  // the output already holds the sums to add to; a padded-stride width adds
  // into a zeroed scratch, copied (added) into the output after the blend
  float* dsem_pad = feat_pad_bytes(P, g->F) ? reinterpret_cast<float*>(static_cast<char*>(scratch) + acc_bytes(P, C))
                                            : nullptr;
  if (dsem_pad)
    (void)hipMemsetAsync(dsem_pad, 0, feat_pad_bytes(P, g->F), s);
  else if (g->F > 0 && !accumulate)
    (void)hipMemsetAsync(dL_dsemantic, 0, sizeof(float) * (size_t)g->F * P, s);
  RenderBwdArgs ra{};
  ra.W = W; ra.H = H; ra.grid_x = gx; ra.num_tiles = gx * gy; ra.F = g->F; ra.compat = compat; ra.P = P;
  ra.order = at<uint4>(image, il.order);
  ra.ranges = at<uint2>(image, il.ranges);
  ra.smax = at<uint32_t>(image, il.smax);
  ra.point_list = static_cast<const uint32_t*>(binning);
  ra.rec = at<float>(geom, gl.rec);
  ra.feats = g->semantic_feature;
  ra.bg = cams[0].background;
  ra.alphas = alphas;
  ra.n_contrib = at<uint32_t>(image, il.n_contrib);
  ra.dL_dpix = dL_dout_color; ra.dL_dfeat = dL_dout_feature; ra.dL_ddepth = dL_dout_depth;
  ra.dL_dalpha = dL_dout_alpha; ra.acc = acc; ra.dsem = dsem_pad ? dsem_pad : dL_dsemantic;
  {
    // with a padded feature width the stage also holds the feature-row copy:
    // marker events around both launches instead of the blend's dispatch
    StageTimer t(s, GS_STAGE_RENDER_BWD, dsem_pad == nullptr);
    if (!launch_render_bwd(ra, cb, s)) return fail(-1, "unsupported feature width %d", g->F);
    if (dsem_pad) launch_feature_grad_rows(dsem_pad, dL_dsemantic, P, g->F, accumulate ? 1 : 0, s);
  }
  if (int e = check("render backward", debug, s)) return e;
  PreprocessBwdArgs b{};
  b.P = P; b.D = g->D; b.M = g->M; b.F = g->F; b.W = W; b.H = H; b.compat = compat;
  b.accumulate = accumulate ? 1 : 0;
  b.activate = (g->flags & GS_FLAG_ACTIVATE) != 0;
  b.opacities = g->opacities;
  b.means3D = g->means3D; b.radii = radii; b.shs = g->shs; b.clamped = at<uint8_t>(geom, gl.clamped);
  b.scales = g->scales; b.rotations = g->rotations;
  b.cov3D = at<float>(geom, gl.cov3D);
  b.cov3D_precomp = g->cov3D_precomp;
  b.scale_modifier = g->scale_modifier;
  b.acc = acc;
  b.rec = at<float>(geom, gl.rec);
  b.grad_mask = g->grad_mask;
  b.st_accum = g->densify_accum; b.st_denom = g->densify_denom; b.st_maxrad = g->max_radius;
  b.dmeans2D = dL_dmeans2D; b.dcolors = dL_dcolors; b.dsemantic = dL_dsemantic; b.dopacity = dL_dopacity;
  b.dmeans3D = dL_dmeans3D; b.dcov3D = dL_dcov3D; b.dsh = dL_dsh; b.dscales = dL_dscales;
  b.drot = dL_drotations;
  {
    StageTimer t(s, GS_STAGE_PREPROCESS_BWD);
    launch_preprocess_bwd(b, cb, s);
  }
  return check("preprocess backward", debug, s);
}

// The sort extents of the last plan of this thread when the render belongs
// to it (same image buffer, cameras and list lengths), else unknown.
static SortPlan exact_sort_plan(const void* image, int C, const int64_t* L) {
  SortPlan sp;
  int64_t total = 0;
  for (int c = 0; c < C; ++c) total += L[c] > 0 ? L[c] : 0;
  if (g_plan.image == image && g_plan.C == C && g_plan.L == total) {
    sp.max_len = g_plan.max_len;
    sp.total = total;
    sp.sc = g_plan.sort;
  }
  return sp;
}

int gs_forward_plan(const gs_gaussians* g, const gs_camera* cam, int prefiltered, int debug, int compat,
                    void* geom, void* image, int32_t* radii, int64_t* num_rendered, int64_t* num_instances,
                    gs_stream_t stream) {
  if (!cam) return fail(-1, "null argument block");
  return plan_impl(g, cam, 1, prefiltered, debug, compat, geom, image, radii, num_rendered, num_instances,
                   (hipStream_t)stream);
}

int gs_forward_render(const gs_gaussians* g, const gs_camera* cam, int debug, int compat, void* geom,
                      void* binning, void* image, int64_t L, const int32_t* radii, float* out_color,
                      float* out_feature, float* out_depth, float* out_alpha, gs_stream_t stream) {
  if (!cam) return fail(-1, "null argument block");
  return render_impl(g, cam, 1, debug, compat, geom, binning, image, &L, radii, out_color, out_feature, out_depth,
                     out_alpha, exact_sort_plan(image, 1, &L), (hipStream_t)stream);
}

int gs_backward(const gs_gaussians* g, const gs_camera* cam, const int32_t* radii, int debug, int compat,
                const void* geom, const void* binning, const void* image, int64_t L, const float* alphas,
                const float* dL_dout_color, const float* dL_dout_feature, const float* dL_dout_depth,
                const float* dL_dout_alpha, void* scratch, float* dL_dmeans2D, float* dL_dcolors,
                float* dL_dsemantic, float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh,
                float* dL_dscales, float* dL_drotations, gs_stream_t stream) {
  if (!cam) return fail(-1, "null argument block");
  // L (num_rendered) is not needed: one camera's tile lists start the binning buffer
  (void)L;
  const int64_t L0 = 0;
  return backward_impl(g, cam, 1, radii, debug, compat, geom, binning, image, &L0, alphas, dL_dout_color,
                       dL_dout_feature, dL_dout_depth, dL_dout_alpha, scratch, dL_dmeans2D, dL_dcolors,
                       dL_dsemantic, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations,
                       (hipStream_t)stream);
}

size_t gs_batch_geom_buffer_bytes(int64_t P, int32_t C) { return GeomLayout(P > 0 ? P : 0).total * (C > 0 ? C : 0); }
size_t gs_batch_image_buffer_bytes(int32_t W, int32_t H, int32_t C) { return ImgLayout(W, H).total * (C > 0 ? C : 0); }
size_t gs_batch_binning_buffer_bytes(int32_t C, const int64_t* num_instances) {
  if (C < 1 || C > GS_MAX_CAMS || !num_instances) return 0;
  return (size_t)batch_bin_offsets(C, num_instances, nullptr);
}
size_t gs_batch_backward_scratch_bytes(int64_t P, int32_t F, int32_t C) {
  return acc_bytes(P, C) + feat_pad_bytes(P, F) + 256;
}

int gs_forward_plan_batch(const gs_gaussians* g, const gs_camera* cams, int32_t C, int prefiltered, int debug,
                          int compat, void* geom, void* image, int32_t* radii, int64_t* num_rendered,
                          int64_t* num_instances, gs_stream_t stream) {
  if (!cams) return fail(-1, "null argument block");
  if (C < 1 || C > GS_MAX_CAMS) return fail(-1, "camera batch size %d outside 1..%d", C, GS_MAX_CAMS);
  return plan_impl(g, cams, C, prefiltered, debug, compat, geom, image, radii, num_rendered, num_instances,
                   (hipStream_t)stream);
}

int gs_forward_render_batch(const gs_gaussians* g, const gs_camera* cams, int32_t C, int debug, int compat,
                            void* geom, void* binning, void* image, const int64_t* num_instances,
                            const int32_t* radii, float* out_color, float* out_feature, float* out_depth,
                            float* out_alpha, gs_stream_t stream) {
  if (!cams || !num_instances) return fail(-1, "null argument block");
  if (C < 1 || C > GS_MAX_CAMS) return fail(-1, "camera batch size %d outside 1..%d", C, GS_MAX_CAMS);
  return render_impl(g, cams, C, debug, compat, geom, binning, image, num_instances, radii, out_color,
                     out_feature, out_depth, out_alpha, exact_sort_plan(image, C, num_instances),
                     (hipStream_t)stream);
}

// ---- sync-free batch forward (ABI 11)

// Launch extents from a previous plan (gs_batch_hint), widened by margins;
// tile_sort_launches launches the class above SORT_SMALL keys when max_len
// exceeds it and the one above TS_CAP likewise.
static SortPlan hinted_sort_plan(const gs_batch_hint* h, int64_t tiles) {
  SortPlan sp;
  if (!h || !h->valid) return sp;  // unknown: every class launch covers all tiles
  auto grow = [&](int64_t v) { return v + (v / 8 > 16 ? v / 8 : 16); };
  sp.max_len = grow(h->max_len > 0 ? h->max_len : 1);
  sp.total = h->total > 0 ? h->total : 0;
  sp.sc.valid = true;
  const int64_t q = h->q1 - (h->q1 / 8 > 16 ? h->q1 / 8 : 16);
  sp.sc.q1 = (int)(q < 0 ? 0 : (q > tiles ? tiles : q));
  sp.hinted = true;
  sp.sc.p1 = (int)(grow(h->p1) < tiles ? grow(h->p1) : tiles);
  sp.sc.p2 = (int)(grow(h->p2) < tiles ? grow(h->p2) : tiles);
  return sp;
}

// Did the sort launches of `sp` cover every tile of the plan `a`?  (Class
// extents are positions in the dispatch order: the short class [q1, T), the
// classes above SORT_SMALL / TS_CAP keys [0, p1) / [0, p2).)
// The batch-wide form of tile_order_kernel's per-camera test (q1 the least
// over the cameras, p1 / p2 / max_len the largest): false iff some camera
// was rendered empty.
static bool sort_covered(const SortCover& cv, const PlanInfo& a) {
  if (!cv.on) return true;
  if (a.sort.q1 < cv.q1) return false;
  if (a.max_len > SORT_SMALL && (!cv.mid || a.sort.p1 > cv.p1)) return false;
  if (a.max_len > TS_CAP && (!cv.lng || a.sort.p2 > cv.p2)) return false;
  return true;
}

int gs_forward_batch(const gs_gaussians* g, const gs_camera* cams, int32_t C, int prefiltered, int compat,
                     void* geom, void* image, void* binning, const int64_t* capacity, gs_batch_hint* hint,
                     int32_t* radii, int64_t* num_rendered, int64_t* num_instances, int32_t* fits,
                     float* out_color, float* out_feature, float* out_depth, float* out_alpha, gs_stream_t stream) {
  if (!cams || !capacity || !num_rendered || !num_instances || !fits) return fail(-1, "null argument block");
  if (C < 1 || C > GS_MAX_CAMS) return fail(-1, "camera batch size %d outside 1..%d", C, GS_MAX_CAMS);
  if (int e = check_gaussians(g, cams, true)) return e;
  *fits = 1;
  for (int c = 0; c < C; ++c) {
    num_rendered[c] = 0;
    num_instances[c] = 0;
    if (capacity[c] < 0) return fail(-1, "capacity[%d] = %lld < 0", c, (long long)capacity[c]);
  }
  g_plan = PlanInfo{};
  const int P = g->P;
  if (P == 0) return 0;  // the reference leaves the zero-filled outputs untouched
  if (!geom || !image || !radii) return fail(-1, "geom buffer, image buffer and radii are required");
  int64_t cap_total = 0;
  for (int c = 0; c < C; ++c) cap_total += capacity[c];
  if (cap_total > 0 && !binning) return fail(-1, "binning buffer is null");
  if (!out_color || !out_depth || (g->F > 0 && !out_feature) || (compat != COMPAT_REFERENCE && !out_alpha))
    return fail(-1, "output image pointers are required");
  HeaderLease hl;
  if (!hl.ok()) return fail((int)hipErrorOutOfMemory, "cannot allocate the page-locked plan header buffer");
  header_sentinel(hl, C);
  hipStream_t s = (hipStream_t)stream;
  CamBatch cb;
  hl.launched(s);
  if (int e = plan_enqueue(g, cams, C, prefiltered, 0, geom, image, radii, hl.s.dev, cb, s))
    return e;
  const int W = cams[0].image_width, H = cams[0].image_height;
  const TileArgs ta = tile_args(P, W, H, geom, image);
  const int64_t tiles = (int64_t)ta.grid_x * ta.grid_y;
  // Every stage behind the plan is enqueued before the host looks at the
  // headers: the GPU goes on from the plan to the bucket, sort and blend
  // launches while the host polls the headers.
  const SortPlan sp = hinted_sort_plan(hint, tiles);
  if (int e = render_impl(g, cams, C, 0, compat, geom, binning, image, capacity, radii, out_color, out_feature,
                          out_depth, out_alpha, sp, s))
    return e;
  // the same wait and sentinel check as the two-phase plan (gs_forward_plan)
  if (int e = publish_wait(hl, C, s)) return e;
  PlanInfo info;
  if (int e = plan_read(reinterpret_cast<const uint32_t(*)[M_WORDS]>(hl.s.host), C, prefiltered, 0, tiles,
                        num_rendered, num_instances, info))
    return e;
  info.image = image;
  g_plan = info;  // a follow-up gs_forward_render_batch with the exact lengths uses the exact extents
  bool ok = sort_covered(sort_cover(sp, tiles), info);
  for (int c = 0; c < C; ++c) ok = ok && num_instances[c] <= capacity[c];
  *fits = ok ? 1 : 0;
  if (hint) {
    hint->valid = 1;
    hint->max_len = info.max_len;
    hint->total = info.L;
    hint->p1 = info.sort.p1;
    hint->q1 = info.sort.q1;
    hint->p2 = info.sort.p2;
  }
  return 0;
}

int gs_backward_batch(const gs_gaussians* g, const gs_camera* cams, int32_t C, const int32_t* radii, int debug,
                      int compat, const void* geom, const void* binning, const void* image,
                      const int64_t* num_instances, const float* alphas, const float* dL_dout_color,
                      const float* dL_dout_feature, const float* dL_dout_depth, const float* dL_dout_alpha,
                      void* scratch, float* dL_dmeans2D, float* dL_dcolors, float* dL_dsemantic,
                      float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                      float* dL_drotations, gs_stream_t stream) {
  if (!cams || !num_instances) return fail(-1, "null argument block");
  if (C < 1 || C > GS_MAX_CAMS) return fail(-1, "camera batch size %d outside 1..%d", C, GS_MAX_CAMS);
  return backward_impl(g, cams, C, radii, debug, compat, geom, binning, image, num_instances, alphas,
                       dL_dout_color, dL_dout_feature, dL_dout_depth, dL_dout_alpha, scratch, dL_dmeans2D,
                       dL_dcolors, dL_dsemantic, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                       dL_drotations, (hipStream_t)stream);
}

int gs_mark_visible(int64_t P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                    uint8_t* present, gs_stream_t stream) {
  (void)projmatrix;
  if (P < 0) return fail(-1, "P must be >= 0");
  if (P == 0) return 0;
  if (!means3D || !viewmatrix || !present) return fail(-1, "null argument");
  hipStream_t s = (hipStream_t)stream;
  launch_mark_visible((int)P, means3D, viewmatrix, present, s);
  return check("markVisible", 0, s);
}

int gs_debug_export(int64_t P, int32_t W, int32_t H, const void* geom, const void* binning, const void* image,
                    int64_t L, float* means2D, float* depths, float* conic_opacity, float* rgb,
                    uint32_t* tiles_touched, uint32_t* point_list, uint32_t* ranges, uint32_t* n_contrib,
                    gs_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const GeomLayout gl(P);
  const BinLayout bl(L);
  const ImgLayout il(W, H);
  const float* rec = at<float>(geom, gl.rec);
  hipError_t e = hipSuccess;
  auto cp2d = [&](float* dst, int cols, int first) {
    if (dst && P > 0 && e == hipSuccess)
      e = hipMemcpy2DAsync(dst, sizeof(float) * cols, rec + first, sizeof(float) * REC, sizeof(float) * cols,
                           (size_t)P, hipMemcpyDeviceToDevice, s);
  };
  cp2d(means2D, 2, R_X);
  cp2d(depths, 1, R_DEPTH);
  if (conic_opacity && P > 0 && e == hipSuccess)
    e = hipMemcpy2DAsync(conic_opacity, sizeof(float) * 4, rec + R_CA, sizeof(float) * REC, sizeof(float) * 4,
                         (size_t)P, hipMemcpyDeviceToDevice, s);
  cp2d(rgb, 3, R_R);
  if (tiles_touched && P > 0 && e == hipSuccess)
    e = hipMemcpyAsync(tiles_touched, at<uint32_t>(geom, gl.tiles), 4 * P, hipMemcpyDeviceToDevice, s);
  if (point_list && L > 0 && e == hipSuccess)
    e = hipMemcpyAsync(point_list, at<uint32_t>(binning, bl.plist), 4 * L,
                       hipMemcpyDeviceToDevice, s);
  const int64_t tiles = (int64_t)((W + TILE - 1) / TILE) * ((H + TILE - 1) / TILE);
  if (ranges && e == hipSuccess)
    e = hipMemcpyAsync(ranges, at<uint32_t>(image, il.ranges), 8 * tiles, hipMemcpyDeviceToDevice, s);
  if (n_contrib && e == hipSuccess)
    e = hipMemcpyAsync(n_contrib, at<uint32_t>(image, il.n_contrib), 4 * (size_t)W * H, hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return fail((int)e, "debug export: %s", hipGetErrorString(e));
  return 0;
}

size_t gs_sort_scratch_bytes(int64_t n) { return SortLayout(n > 0 ? n : 0).total; }

int gs_sort_pairs(int64_t n, uint64_t* keys, uint32_t* vals, int end_bit, void* scratch, gs_stream_t stream) {
  if (n < 0 || end_bit < 0 || end_bit > 64) return fail(-1, "bad sort arguments");
  if (n <= 1) return 0;
  hipStream_t s = (hipStream_t)stream;
  const SortLayout sl(n);
  uint64_t* k1 = at<uint64_t>(scratch, sl.keys1);
  uint32_t* v1 = at<uint32_t>(scratch, sl.vals1);
  const int which = launch_radix_sort(n, keys, vals, k1, v1, at<uint32_t>(scratch, sl.hist),
                                      at<uint32_t>(scratch, sl.rowtot), end_bit, s);
  if (which) {
    (void)hipMemcpyAsync(keys, k1, 8 * n, hipMemcpyDeviceToDevice, s);
    (void)hipMemcpyAsync(vals, v1, 4 * n, hipMemcpyDeviceToDevice, s);
  }
  return check("sort", 0, s);
}

// ---- the binning passes' spatial walk order (gs_gaussians.walk_order) ----

size_t gs_spatial_order_scratch_bytes(int64_t P) { return SpatialLayout(P < 0 ? 0 : P).total; }

int gs_spatial_order(int64_t P, const float* means3D, int32_t* order, void* scratch, gs_stream_t stream) {
  if (P < 0 || P > 0x7FFFFFFF) return fail(-1, "spatial order: P = %lld out of range", (long long)P);
  if (P > 0 && (!means3D || !order || !scratch)) return fail(-1, "spatial order: null pointer");
  launch_spatial_order(P, means3D, order, scratch, (hipStream_t)stream);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail((int)e, "spatial order: %s", hipGetErrorString(e));
}

// ---- exact k-nearest neighbours (include/gs_knn.h) ----

size_t gs_knn_workspace_bytes(int64_t N) { return KnnLayout(N < 0 ? 0 : N).total; }

int gs_knn(int64_t N, int32_t K, const float* points, double* sq_dist, int64_t* index, void* workspace,
           gs_stream_t stream) {
  if (N < 0) return fail(-1, "N must be >= 0");
  if (K < 1 || K > GS_KNN_MAX_K) return fail(-1, "K must be in [1, %d] (got %d)", GS_KNN_MAX_K, K);
  if (N >= (int64_t)1 << 31) return fail(-1, "N must fit in int32");
  if (N == 0) return 0;
  if (!points || !sq_dist || !index || !workspace) return fail(-1, "knn: null argument");
  hipStream_t s = (hipStream_t)stream;
  if (!launch_knn(N, K, points, sq_dist, index, workspace, s)) return fail(-1, "knn: unsupported K %d", K);
  return check("knn", 0, s);
}

// ---- fused Adam + densification statistics (include/gs_optim.h) ----

int gs_adam_step(const gs_adam_args* a, const gs_densify_stats* st, gs_stream_t stream) {
  if (!a) return fail(-1, "null Adam arguments");
  if (a->n_tensors < 0 || a->n_tensors > GS_ADAM_MAX_TENSORS)
    return fail(-1, "n_tensors must be in [0, %d] (got %d)", GS_ADAM_MAX_TENSORS, a->n_tensors);
  for (int t = 0; t < a->n_tensors; ++t) {
    const gs_adam_tensor& x = a->t[t];
    if (x.numel < 0) return fail(-1, "tensor %d: numel < 0", t);
    if (x.numel > 0 && (!x.param || !x.grad || !x.exp_avg || !x.exp_avg_sq))
      return fail(-1, "tensor %d: param, grad, exp_avg and exp_avg_sq are required", t);
    if (!(x.bc2_sqrt > 0.f)) return fail(-1, "tensor %d: bc2_sqrt must be > 0 (step >= 1)", t);
  }
  if (st && st->P > 0) {
    if (!st->radii) return fail(-1, "densify stats: radii are required");
    if (st->grad_accum && (!st->denom || !st->means2D_grad))
      return fail(-1, "densify stats: grad_accum needs denom and means2D_grad");
  }
  hipStream_t s = (hipStream_t)stream;
  if (!launch_adam_step(*a, st, s)) return fail(-1, "Adam step: too many blocks");
  return check("adam step", 0, s);
}

// ---- neighbour losses (include/gs_neighbor.h) ----

static int check_graph(const gs_neighbor_graph* g, bool backward, NeighborArgs* a) {
  if (!g) return fail(-1, "null neighbour graph");
  if (g->N < 0 || g->K < 0) return fail(-1, "N and K must be >= 0 (got N=%lld K=%d)", (long long)g->N, g->K);
  if ((double)g->N * g->K >= 2147483647.0) return fail(-1, "N*K must fit in int32 (got N=%lld K=%d)", (long long)g->N, g->K);
  if (g->N > 0 && (!g->prev_inv_rot || (g->K > 0 && (!g->nbr || !g->weight || !g->dist || !g->prev_offset))))
    return fail(-1, "neighbour graph arrays are required");
  if (backward && g->N > 0 && (!g->rev_ptr || (g->K > 0 && !g->rev_pos)))
    return fail(-1, "the backward needs the reverse CSR (gs_neighbor_reverse)");
  *a = NeighborArgs{g->N, g->K, nullptr, nullptr, g->nbr, g->weight, g->dist, g->prev_offset, g->prev_inv_rot,
                    g->rev_ptr, g->rev_pos};
  return 0;
}

size_t gs_neighbor_workspace_bytes(int64_t N, int32_t K, int backward) {
  return NeighborLayout(N < 0 ? 0 : N, K < 0 ? 0 : K, backward != 0).total;
}

int gs_neighbor_loss_forward(const gs_neighbor_graph* g, const float* fg_pts, const float* fg_rot, float* losses,
                             void* workspace, gs_stream_t stream) {
  NeighborArgs a;
  if (int e = check_graph(g, false, &a)) return e;
  if (!losses || !workspace) return fail(-1, "losses and workspace are required");
  if (a.N > 0 && (!fg_pts || !fg_rot)) return fail(-1, "fg_pts and fg_rot are required");
  a.fg_pts = fg_pts;
  a.fg_rot = fg_rot;
  hipStream_t s = (hipStream_t)stream;
  launch_neighbor_forward(a, losses, workspace, s);
  return check("neighbour loss forward", 0, s);
}

int gs_neighbor_loss_backward(const gs_neighbor_graph* g, const float* fg_pts, const float* fg_rot,
                              const float* dL_dlosses, float* d_fg_pts, float* d_fg_rot, void* workspace,
                              gs_stream_t stream) {
  NeighborArgs a;
  if (int e = check_graph(g, true, &a)) return e;
  if (a.N == 0) return 0;
  if (!fg_pts || !fg_rot || !dL_dlosses || !d_fg_pts || !d_fg_rot || !workspace)
    return fail(-1, "neighbour loss backward: null argument");
  a.fg_pts = fg_pts;
  a.fg_rot = fg_rot;
  hipStream_t s = (hipStream_t)stream;
  launch_neighbor_backward(a, dL_dlosses, d_fg_pts, d_fg_rot, workspace, s);
  return check("neighbour loss backward", 0, s);
}

namespace {
struct RevLayout {
  size_t keys, vals, status, sort, total;
  explicit RevLayout(int64_t NK) {
    size_t o = 0;
    keys = o; o = align_up(o + 8 * (size_t)NK, 256);
    vals = o; o = align_up(o + 4 * (size_t)NK, 256);
    status = o; o = align_up(o + 4, 256);
    sort = o; o = align_up(o + SortLayout(NK).total, 256);
    total = o;
  }
};
}  // namespace

size_t gs_neighbor_reverse_workspace_bytes(int64_t N, int32_t K) {
  return RevLayout((N < 0 ? 0 : N) * (K < 0 ? 0 : K)).total;
}

int gs_neighbor_reverse(int64_t N, int32_t K, const int64_t* nbr, int32_t* rev_ptr, int32_t* rev_pair,
                        int32_t* rev_pos, void* workspace, gs_stream_t stream) {
  if (N < 0 || K < 0) return fail(-1, "N and K must be >= 0");
  if ((double)N * K >= 2147483647.0) return fail(-1, "N*K must fit in int32");
  const int64_t NK = N * K;
  if (!rev_ptr || !workspace || (NK > 0 && (!nbr || !rev_pos))) return fail(-1, "neighbour reverse: null argument");
  hipStream_t s = (hipStream_t)stream;
  const RevLayout L(NK);
  uint64_t* keys = at<uint64_t>(workspace, L.keys);
  uint32_t* vals = at<uint32_t>(workspace, L.vals);
  int* status = at<int>(workspace, L.status);
  (void)hipMemsetAsync(status, 0, 4, s);
  launch_neighbor_rev_keys(NK, N, nbr, keys, vals, status, s);
  if (NK > 1) {
    const SortLayout sl(NK);
    void* sc = at<char>(workspace, L.sort);
    uint64_t* k1 = at<uint64_t>(sc, sl.keys1);
    uint32_t* v1 = at<uint32_t>(sc, sl.vals1);
    int end_bit = 1;  // keys <= N (N marks invalid ids)
    while (end_bit < 63 && ((uint64_t)N >> end_bit)) ++end_bit;
    if (launch_radix_sort(NK, keys, vals, k1, v1, at<uint32_t>(sc, sl.hist), at<uint32_t>(sc, sl.rowtot),
                          end_bit, s)) {
      keys = k1;
      vals = v1;
    }
  }
  launch_neighbor_rev_ptr(NK, N, keys, vals, rev_ptr, rev_pair, rev_pos, s);
  int host_status = 0;
  (void)hipMemcpyAsync(&host_status, status, 4, hipMemcpyDeviceToHost, s);
  if (int e = check("neighbour reverse", 1, s)) return e;
  if (host_status) return fail(-1, "neighbor_indices out of range [0, %lld)", (long long)N);
  return 0;
}

int gs_test_wave_reduce(int n_comp, const float* in, float* out, gs_stream_t stream) {
  if (n_comp < 1 || n_comp > 64) return fail(-1, "n_comp must be in [1, 64]");
  launch_test_wave_reduce(n_comp, in, out, (hipStream_t)stream);
  return check("wave reduce test", 1, (hipStream_t)stream);
}

}  // extern "C"
