// gs_kernels.h -- kernel argument blocks and host launchers (internal).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "../../include/gs_optim.h"
#include <stdint.h>

#include "gs_common.h"

namespace gs {

struct PreprocessArgs {
  int P, D, M, W, H, grid_x, grid_y, prefiltered;
  int activate;  // GS_FLAG_ACTIVATE: opacities / scales / rotations are raw parameters
  const float* means3D;
  const float* scales;
  const float* rotations;
  const float* opacities;
  const float* shs;
  const float* cov3D_precomp;
  const float* colors_precomp;
  const float* view;
  const float* proj;
  const float* campos;
  float scale_modifier, c_x, c_y, tan_fovx, tan_fovy, focal_x, focal_y;
  int* radii;
  float* rec;
  float* cov3D;
  uint8_t* clamped;
  uint32_t* tiles;
  uint4* rect;     // P: binning record {x0 | y0 << 16, x1 | y1 << 16, depth bits, tiles_touched} (rect [x0, x1) x [y0, y1), empty when culled)
  int* status;
};

struct PreprocessBwdArgs {
  int P, D, M, F, W, H, compat;
  int accumulate;  // add into the gradient outputs (GS_FLAG_ACCUMULATE)
  int activate;    // GS_FLAG_ACTIVATE: gradients of the raw opacity / scale / rotation parameters
  const float* opacities;  // read with `activate` only
  const float* means3D;
  const int* radii;
  const float* shs;
  const uint8_t* clamped;
  const float* scales;
  const float* rotations;
  const float* cov3D;          // the forward's (geometry buffer of camera 0; per camera at geom_stride)
  const float* cov3D_precomp;  // the caller's, or null
  const float* view;
  const float* proj;
  const float* campos;
  float scale_modifier, c_x, c_y, tan_fovx, tan_fovy, focal_x, focal_y;
  const float* rec;  // P x REC render records (conic)
  const float* acc;  // P x 10 blend gradient sums (AccField)
  const float* grad_mask;  // P or null (Q12 label)
  float* st_accum;   // P or null: densification statistics of this view (gs_gaussians.densify_accum)
  float* st_denom;   // P or null
  float* st_maxrad;  // P or null
  float* dmeans2D;
  float* dcolors;
  float* dsemantic;
  float* dopacity;
  float* dmeans3D;
  float* dcov3D;
  float* dsh;
  float* dscales;
  float* drot;
};

struct RenderArgs {
  int W, H, grid_x, num_tiles, F, compat, P;
  const uint4* order;  // num_tiles: dispatch records {tile, range.x, range.y, 0}, longest list first
  const uint2* ranges;
  const uint32_t* point_list;
  const float* rec;
  const float* feats;  // P x F
  uint32_t* smax;      // 4 x num_tiles: per strip item (dispatch order) the longest pixel walk (max n_contrib)
  const float* bg;     // 3
  float* out_color;
  float* out_feature;
  float* out_depth;
  float* out_alpha;
  uint32_t* n_contrib;
  // F >= 32: per channel the largest |feature| of the table (float bits,
  // launch_feature_absmax; the whole batch's, camera 0's image buffer)
  const uint32_t* fmax;
  // a region the launch zeroes alongside (gs_gaussians.zero_fill), zero_n
  // 16-B words; each workgroup its 1/gridDim share
  float4* zero;
  int64_t zero_n;
};

// Row stride (floats) of the feature gradients the backward blend adds into:
// F when its 16-channel blocks are 64-B aligned (F % 16 == 0 or F < 16),
// else F rounded up to 16 (F = 36 -> 48, through a scratch copy) -- float
// atomics execute per 64-B segment, and a straddling 16-channel block costs
// two requests.
__host__ __device__ constexpr int feature_grad_stride(int F) {
  return (F < 16 || F % 16 == 0) ? F : (F + 15) / 16 * 16;
}
void launch_feature_grad_rows(const float* pad, float* out, int64_t P, int F, int accumulate, hipStream_t s);
// out[c] = bits of max_g |feats[g][c]| (c < F <= 64), into a table the
// caller zeroed (tile_order_kernel, earlier on the stream): the scales of the
// forward's fp16 feature contraction (render_fwd, F >= 32)
void launch_feature_absmax(const float* feats, int64_t P, int F, uint32_t* out, hipStream_t s);

struct RenderBwdArgs {
  int W, H, grid_x, num_tiles, F, compat, P;
  const uint4* order;  // num_tiles: dispatch records {tile, range.x, range.y, 0}, longest list first
  const uint2* ranges;
  const uint32_t* point_list;
  const float* rec;
  const float* feats;
  const float* bg;
  const uint32_t* smax;  // 4 x num_tiles: the forward's per-strip walk lengths
  const float* alphas;
  const uint32_t* n_contrib;
  const float* dL_dpix;
  const float* dL_dfeat;
  const float* dL_ddepth;
  const float* dL_dalpha;
  float* acc;   // P x 10 blend gradients, zeroed by the caller
  float* dsem;  // P x F semantic-feature gradients (the output), zeroed (or holding earlier sums) by the caller
};

// Live stage timing of a one-kernel stage (gs_timing_*, gs_api.hip): the
// stage's event pair travels to its kernel launch (thread-local, consumed by
// timed_launch) and is attached to the dispatch itself through
// hipExtLaunchKernel -- the kernel's own start / end timestamps, no marker
// packets in the stream between it and its neighbours (a marker pair cost the
// timed step ~12 us of idle GPU: profiles/r05sf2, tools/step_gaps.py).
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents& launch_events();
template <class K, class... A>
inline void timed_launch(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, A... args) {
  LaunchEvents& e = launch_events();
  if (e.start) {
    const LaunchEvents ev = e;
    e = LaunchEvents{};
    hipExtLaunchKernelGGL(kernel, grid, block, lds, s, ev.start, ev.stop, 0u, args...);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
  }
}

void launch_preprocess_fwd(const PreprocessArgs& a, const CamBatch& cb, hipStream_t s);
void launch_preprocess_bwd(const PreprocessBwdArgs& a, const CamBatch& cb, hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t s);

// Stable LSD radix sort on bits [0, end_bit) (the standalone gs_sort_pairs
// entry point); the result ends in keys0/vals0 or keys1/vals1 -- returns 0
// or 1 for which (passes of 8 bits swap slots).
int launch_radix_sort(int64_t n, uint64_t* keys0, uint32_t* vals0, uint64_t* keys1, uint32_t* vals1,
                      uint32_t* hist, uint32_t* rowtot, int end_bit, hipStream_t s);

// Tile binning (gs_tiles.hip).
struct TileArgs {
  int P, W, H, grid_x, grid_y, num_tiles;
  const uint4* rect;     // P: binning record (PreprocessArgs::rect)
  const uint32_t* tiles; // P: the reference's tiles_touched
  const float* rec;      // P x REC (depth)
  uint32_t* thist;       // TB_BLOCKS x num_tiles
  uint32_t* ttotal;      // num_tiles
  uint32_t* bsum;        // TB_BLOCKS: bounding-rect instances per block (the reference's count)
  uint32_t* meta;        // 4
  uint2* ranges;         // num_tiles
  uint4* order;          // num_tiles: dispatch records {tile, range.x, range.y, 0}, longest list first
  uint32_t* fmax;        // 64: the forward's feature-range table (camera 0's), zeroed by tile_order_kernel
  uint64_t* keys;        // L
  uint64_t* keys2;       // L (sort twin for long tiles)
  uint32_t* plist;       // L
  void* binning;         // binning buffer base (batch: camera c at CamBatch::bin_off[c]), or null
  const int32_t* walk;   // P: the binning passes' walk order (a permutation of the ids), or null (id order)
};
// TileArgs of camera c of a batch (pointers of camera 0 -> camera c).
__host__ __device__ inline TileArgs cam_tile_args(const TileArgs& a0, const CamBatch& cb, int c) {
  TileArgs a = a0;
  const int64_t go = c * cb.geom_stride, io = c * cb.img_stride;
  a.rect = shift_bytes(a0.rect, go);
  a.tiles = shift_bytes(a0.tiles, go);
  a.rec = shift_bytes(a0.rec, go);
  a.thist = shift_bytes(a0.thist, io);
  a.ttotal = shift_bytes(a0.ttotal, io);
  a.bsum = shift_bytes(a0.bsum, io);
  a.meta = shift_bytes(a0.meta, io);
  a.ranges = shift_bytes(a0.ranges, io);
  a.order = shift_bytes(a0.order, io);
  if (a0.binning) {
    char* b = static_cast<char*>(a0.binning) + cb.bin_off[c];
    const BinLayout bl(cb.bin_L[c]);
    a.plist = reinterpret_cast<uint32_t*>(b + bl.plist);
    a.keys = reinterpret_cast<uint64_t*>(b + bl.keys);
    a.keys2 = reinterpret_cast<uint64_t*>(b + bl.keys2);
  }
  return a;
}
// plan: per-block tile histograms, tile totals and offsets, ranges, header
// (also stored to hdr_host[c * M_WORDS ..] when non-null: mapped host memory,
// its last word stored last, after a system fence -- the host polls it)
void launch_tile_plan(const TileArgs& a, const CamBatch& cb, int prefiltered, uint32_t* hdr_host, hipStream_t s);
// render: bucket the instances by tile, then sort every tile by (depth, id).
// max_len = the plan header's longest tile (host copy), or -1 if unknown.
void launch_tile_bucket(const TileArgs& a, const CamBatch& cb, hipStream_t s);
// What the tile sort launches of a render cover (tile_sort_launches): on = 0
// every tile (the exact or unknown extents); else the short class the
// dispatch positions [q1, T), the class above SORT_SMALL keys (if mid) [0,
// p1), the one above TS_CAP (if lng) [0, p2).  A camera whose plan puts a
// tile outside them (gs_forward_batch's hinted extents gone stale) gets empty
// dispatch records, like one over its binning capacity: its lists are never
// read unsorted, and the host, checking the same condition on the headers,
// renders it again.
struct SortCover {
  int on = 0;
  int q1 = 0, p1 = 0, p2 = 0;
  int mid = 0, lng = 0;
};
// dispatch order of the blend / sort kernels (tiles by descending list length)
void launch_tile_order(const TileArgs& a, const CamBatch& cb, const SortCover& cv, hipStream_t s);
// max_len: the longest tile over the batch (-1: unknown); L: the batch's total instances
// Dispatch-order extents of the sort's length classes over the batch (plan
// header M_SORT_*: p1 / p2 = max over cameras of the prefixes holding every
// tile longer than SORT_SMALL / TS_CAP, q1 = min over cameras of the
// prefix of tiles known to be longer than SORT_SMALL); valid = false:
// every class launch covers all tiles.
struct SortClasses {
  bool valid = false;
  int p1 = 0, q1 = 0, p2 = 0;
};
void launch_tile_sort(const TileArgs& a, const CamBatch& cb, int64_t max_len, int64_t L, const SortClasses& sc,
                      hipStream_t s);

// Camera c of a batch: image-buffer, geometry, binning and image pointers of
// camera 0 -> camera c (point_list = the batch's binning base).
__host__ __device__ inline RenderArgs cam_render_args(const RenderArgs& a0, const CamBatch& cb, int c) {
  RenderArgs a = a0;
  const int64_t go = c * cb.geom_stride, io = c * cb.img_stride, hw = (int64_t)a0.W * a0.H;
  a.order = shift_bytes(a0.order, io);
  a.ranges = shift_bytes(a0.ranges, io);
  a.smax = shift_bytes(a0.smax, io);
  a.n_contrib = shift_bytes(a0.n_contrib, io);
  a.rec = shift_bytes(a0.rec, go);
  a.point_list = shift_bytes(a0.point_list, cb.bin_off[c]);
  a.out_color = a0.out_color ? a0.out_color + c * 3 * hw : nullptr;
  a.out_feature = a0.out_feature ? a0.out_feature + c * a0.F * hw : nullptr;
  a.out_depth = a0.out_depth ? a0.out_depth + c * hw : nullptr;
  a.out_alpha = a0.out_alpha ? a0.out_alpha + c * hw : nullptr;
  return a;
}
__host__ __device__ inline RenderBwdArgs cam_render_bwd_args(const RenderBwdArgs& a0, const CamBatch& cb, int c) {
  RenderBwdArgs a = a0;
  const int64_t go = c * cb.geom_stride, io = c * cb.img_stride, hw = (int64_t)a0.W * a0.H;
  a.order = shift_bytes(a0.order, io);
  a.ranges = shift_bytes(a0.ranges, io);
  a.smax = shift_bytes(a0.smax, io);
  a.n_contrib = shift_bytes(a0.n_contrib, io);
  a.rec = shift_bytes(a0.rec, go);
  a.point_list = shift_bytes(a0.point_list, cb.bin_off[c]);
  a.alphas = a0.alphas ? a0.alphas + c * hw : nullptr;
  a.dL_dpix = a0.dL_dpix ? a0.dL_dpix + c * 3 * hw : nullptr;
  a.dL_dfeat = a0.dL_dfeat ? a0.dL_dfeat + c * a0.F * hw : nullptr;
  a.dL_ddepth = a0.dL_ddepth ? a0.dL_ddepth + c * hw : nullptr;
  a.dL_dalpha = a0.dL_dalpha ? a0.dL_dalpha + c * hw : nullptr;
  a.acc = a0.acc + (size_t)c * a0.P * ACC_STRIDE;
  return a;
}
bool launch_render_fwd(const RenderArgs& a, const CamBatch& cb, hipStream_t s);
bool launch_render_bwd(const RenderBwdArgs& a, const CamBatch& cb, hipStream_t s);

void launch_test_wave_reduce(int n, const float* in, float* out, hipStream_t s);

// Fused Adam + densification statistics (gs_optim.hip, include/gs_optim.h).
bool launch_adam_step(const gs_adam_args& a, const gs_densify_stats* st, hipStream_t s);

// Exact k-nearest neighbours (gs_knn.hip, include/gs_knn.h).
struct KnnLayout {
  size_t bbox, keys, vals, sort, spts, boxes, total;
  explicit KnnLayout(int64_t N);
};
bool launch_knn(int64_t N, int K, const float* pts, double* out_d, int64_t* out_i, void* ws, hipStream_t s);
// Spatial walk order of the binning passes (gs_spatial_order): the ids in 3-D
// Morton order of the points (the kNN's bounding box, codes and radix sort).
struct SpatialLayout {
  size_t bbox, keys, vals, sort, total;
  explicit SpatialLayout(int64_t N);
};
void launch_spatial_order(int64_t N, const float* pts, int32_t* order, void* ws, hipStream_t s);

// Neighbour losses (gs_neighbor.hip, include/gs_neighbor.h).
struct NeighborArgs {
  int64_t N;
  int K;
  const float* fg_pts;        // N x 3
  const float* fg_rot;        // N x 4
  const int64_t* nbr;         // N x K
  const float* weight;        // N x K
  const float* dist;          // N x K
  const float* prev_offset;   // N x K x 3
  const float* prev_inv_rot;  // N x 4
  const int32_t* rev_ptr;     // N + 1
  const int32_t* rev_pos;     // N x K: slot of pair i*K+k in the reverse order
};
struct NeighborLayout {
  size_t qv, Rm, partial, revbuf, selfbuf, total;
  NeighborLayout(int64_t N, int K, bool backward);
};
void launch_neighbor_forward(const NeighborArgs& a, float* losses, void* ws, hipStream_t s);
void launch_neighbor_backward(const NeighborArgs& a, const float* dL, float* d_pts, float* d_rot, void* ws,
                              hipStream_t s);
void launch_neighbor_rev_keys(int64_t NK, int64_t N, const int64_t* nbr, uint64_t* keys, uint32_t* vals,
                              int* status, hipStream_t s);
void launch_neighbor_rev_ptr(int64_t NK, int64_t N, const uint64_t* keys, const uint32_t* vals, int32_t* rev_ptr,
                             int32_t* rev_pair, int32_t* rev_pos, hipStream_t s);

}  // namespace gs
