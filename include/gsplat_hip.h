/*
 * gsplat_hip.h -- C ABI of the MI355X-native differentiable Gaussian
 * rasterizer (libgsplat_hip.so, hand-written HIP kernels for gfx950).
 *
 * This is the drop-in boundary for the reference's pybind module
 * `diff_gaussian_rasterization._C` (DGR/ext.cpp:15-19), where
 * DGR = submodules_fsgs/diff-gaussian-rasterization-confidence and
 * CR = DGR/cuda_rasterizer.  Each entry point names the reference interface
 * it replaces.  No torch types cross this boundary: plain device pointers,
 * sizes, camera scalars and an explicit hipStream_t.
 *
 * Conventions (all entry points):
 *  - Return 0 on success, <0 on an invalid argument, >0 = a hipError_t code.
 *    The message is in gs_last_error() (thread-local).
 *  - The library never allocates device memory: the caller supplies the three
 *    opaque state buffers (sized by gs_*_buffer_bytes) and the backward
 *    scratch, normally from torch's caching allocator.
 *  - "Absent" optional inputs are NULL pointers (the reference passes empty
 *    tensors whose data_ptr is null, DGR/diff_gaussian_rasterization/
 *    __init__.py:220-230).
 *  - Camera scalars are in the reference's C++ positional semantics
 *    (DGR/rasterize_points.h); the Python layer decides what it passes.
 *  - All work is enqueued on `stream`; gs_forward_plan performs the one
 *    device->host read the reference also performs (num_rendered,
 *    CR/rasterizer_impl.cu:287).  gs_forward_batch (ABI 11) performs it after
 *    every forward stage is enqueued, so the GPU does not wait for the host.
 */
#ifndef GSPLAT_HIP_H
#define GSPLAT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 13

/* compat modes: numerics of the as-shipped reference vs corrected ones */
#define GS_COMPAT_REFERENCE 0
#define GS_COMPAT_FIXED 1

typedef void *gs_stream_t;
typedef void *gs_event_t; /* a hipEvent_t */

/* gs_gaussians.flags.  GS_FLAG_ACCUMULATE (gs_backward only; no reference
 * analogue): ADD this call's gradients into the dL_d* outputs instead of
 * overwriting them, so the cameras of a multi-camera step sum into one set
 * of buffers without an elementwise add per camera and parameter.  The
 * outputs must hold valid sums (e.g. the first camera's, written without the
 * flag); calls accumulating into the same outputs must be ordered on one
 * stream (the non-atomic read-modify-write of the per-Gaussian outputs is
 * not safe across concurrent streams). */
#define GS_FLAG_ACCUMULATE 1u
/* GS_FLAG_ACTIVATE (ABI 8; no reference analogue): opacities, scales and
 * rotations are the Dynamic3DGaussians raw parameters -- logit_opacities,
 * log_scales, unnorm_rotations -- and the kernels apply the activations of
 * helpers.py:98-107 (params2rendervar) themselves: sigmoid, exp and
 * F.normalize (q / max(|q|, 1e-12)).  The backward's dL_dopacity,
 * dL_dscales and dL_drotations are then the gradients of the raw parameters
 * (through the activations, with grad_mask applied to the activated
 * gradients first, as the reference's label mask precedes autograd through
 * params2rendervar).  Replaces ~20 elementwise launches of the caller's
 * activations and their backward per step. */
#define GS_FLAG_ACTIVATE 2u
/* GS_FLAG_SCRATCH_ZEROED (ABI 13, gs_backward / gs_backward_batch only; no
 * reference analogue): the scratch buffer is already zero -- a forward zeroed
 * it through gs_gaussians.zero_fill and nothing has written it since -- so the
 * backward skips its zero fill of the accumulation records.  Set it for the
 * first backward of a forward only. */
#define GS_FLAG_SCRATCH_ZEROED 4u

/* Per-Gaussian inputs (device pointers, fp32, row-major/contiguous).
 * Mirrors the tensor arguments of RasterizeGaussiansCUDA
 * (DGR/rasterize_points.cu:36-58). */
typedef struct gs_gaussians {
  int32_t P;                      /* number of Gaussians */
  int32_t D;                      /* active SH degree (0..3) */
  int32_t M;                      /* SH coefficients per Gaussian (shs is P x M x 3) */
  int32_t F;                      /* semantic feature channels (0 = none) */
  const float *means3D;           /* P x 3 */
  const float *shs;               /* P x M x 3 or NULL */
  const float *colors_precomp;    /* P x 3 or NULL */
  const float *semantic_feature;  /* P x F or NULL */
  const float *opacities;         /* P */
  const float *scales;            /* P x 3 or NULL */
  const float *rotations;         /* P x 4 (r,x,y,z) or NULL */
  const float *cov3D_precomp;     /* P x 6 or NULL */
  float scale_modifier;
  uint32_t flags;                 /* GS_FLAG_* (0 = the reference's semantics) */
  /* Optional per-Gaussian gradient mask (P floats or NULL), used by
   * gs_backward only: dL/d{means3D, sh, colors, opacity, scales, rotations,
   * cov3D} are multiplied by it, exactly as the reference's Python autograd
   * wrapper does with `label` after the binding returns
   * (DGR/diff_gaussian_rasterization/__init__.py:159-173).  dL/dmeans2D and
   * dL/dsemantic are not masked (Q12). */
  const float *grad_mask;
  /* Optional densification statistics of this view (gs_backward only; P
   * floats each or NULL), the reference's per-camera bookkeeping after the
   * backward (external.py:136-140 accumulate_mean2d_gradient, train.py:288-290):
   * for seen = radii > 0,
   *   densify_accum[seen] += |dL/dmeans2D[seen, :2]|   (this view's gradient)
   *   densify_denom[seen] += 1
   *   max_radius[seen]     = max(max_radius[seen], radii[seen])
   * With GS_FLAG_ACCUMULATE clear they are written instead (unseen -> 0), so
   * a multi-camera step can sum per-view norms while dL_dmeans2D itself
   * holds the sum of the views' gradients. */
  float *densify_accum;
  float *densify_denom;
  float *max_radius;
  /* Optional (ABI 10; no reference analogue): an event the forward's blend
   * launch -- the first reader of semantic_feature -- waits for on the launch
   * stream (hipStreamWaitEvent), or NULL.  A caller that updates the features
   * on another stream (an optimizer step behind an overlapped gradient
   * all-reduce) orders that update before the blend without ordering the
   * projection and binning behind it. */
  gs_event_t feature_ready;
  /* Optional (ABI 12; no reference analogue): the order in which the
   * binning passes (tile histogram and bucket) walk the Gaussians -- P ids,
   * a permutation of [0, P) -- or NULL (id order).  Outputs do not depend
   * on it: every tile list is sorted by its unique (depth bits, id) keys.  A
   * spatially coherent order (gs_spatial_order) gives each binning
   * workgroup's slice a compact footprint on every camera's screen, so its
   * per-tile runs are long and its key stores coalesce.  Debug mode checks
   * that it is a permutation (gs_check_walk_order). */
  const int32_t *walk_order;
  /* Optional (ABI 13; no reference analogue): a device region the forward's
   * blend launch zeroes (zero_fill_bytes, a multiple of 16, 16-B aligned), or
   * NULL.  A caller that keeps the backward's scratch from the forward
   * (gs_batch_backward_scratch_bytes) hands it here and to the backward with
   * GS_FLAG_SCRATCH_ZEROED: the zeroing then rides in the VALU-bound blend,
   * whose HBM is mostly idle, instead of a fill launch before the backward
   * blend (0.5 GB at the 27-camera bench step). */
  void *zero_fill;
  int64_t zero_fill_bytes;
} gs_gaussians;

/* Camera / raster settings (GaussianRasterizationSettings,
 * DGR/diff_gaussian_rasterization/__init__.py:176-192).
 *
 * Tile window (ABI 9; no reference analogue): render only the 16x16 tiles
 * [tile_x0, tile_x1) x [tile_y0, tile_y1) of the camera's tile grid -- image
 * sharding of one camera over several calls or ranks.  All
 * four 0 = the whole image.  Projection, culling, radii and num_rendered are
 * the whole camera's; only the window's tiles are binned, blended and
 * back-propagated, so a window's pixels are bit-identical to the whole
 * render's and the gradients of windows that partition the grid sum to the
 * whole camera's.  Pixels outside the window are written as zeros (colour,
 * features, depth, alpha, n_contrib) and their upstream gradients are
 * ignored.  The densification statistics (gs_gaussians.densify_*) count a
 * projected Gaussian in every window call: keep them to whole-image calls. */
typedef struct gs_camera {
  const float *viewmatrix; /* 16 floats, column-major (device) */
  const float *projmatrix; /* 16 floats, column-major (device) */
  const float *campos;     /* 3 floats (device) */
  const float *background; /* 3 floats (device) */
  float c_x, c_y, tan_fovx, tan_fovy;
  int32_t image_width, image_height;
  int32_t tile_x0, tile_y0, tile_x1, tile_y1; /* tile window; all 0 = whole image */
} gs_camera;

int gs_version(void);
const char *gs_last_error(void);

/* Opaque state buffer sizes (replace GeometryState/BinningState/ImageState
 * ::fromChunk + required<>, CR/rasterizer_impl.cu:155-194,
 * CR/rasterizer_impl.h:67-73). */
size_t gs_geom_buffer_bytes(int64_t P);
size_t gs_binning_buffer_bytes(int64_t num_instances);
size_t gs_image_buffer_bytes(int32_t W, int32_t H);
size_t gs_backward_scratch_bytes(int64_t P, int32_t F);

/* Forward, phase 1 -- replaces CR/rasterizer_impl.cu:198-287 (preprocess,
 * inclusive scan of tiles_touched, D2H of num_rendered).  Writes radii[P]
 * and the binning plan (per-tile counts and ranges) into the image buffer,
 * which must be the one later passed to gs_forward_render.
 * *num_rendered = the reference's count (sum of the Gaussians' bounding-rect
 * tiles, tiles_touched); *num_instances (may be NULL) = the tile-list length
 * actually binned: the bounding-rect tiles that the Gaussian's alpha >= 1/255
 * ellipse reaches (an exact test -- a dropped instance is one the reference's
 * blend loop skips at every pixel of the tile).  Size the binning buffer and
 * call gs_forward_render / gs_debug_export with num_instances. */
int gs_forward_plan(const gs_gaussians *g, const gs_camera *cam, int prefiltered,
                    int debug, int compat, void *geom_buffer, void *image_buffer,
                    int32_t *radii, int64_t *num_rendered, int64_t *num_instances,
                    gs_stream_t stream);

/* Forward, phase 2 -- replaces CR/rasterizer_impl.cu:289-345 (duplicateWithKeys,
 * radix sort, identifyTileRanges, render): instances are bucketed by tile and
 * each tile's list sorted by (depth, index) -- the reference's order.  Outputs are planar CHW:
 * out_color 3xHxW, out_feature FxHxW (may be NULL if F==0), out_depth HxW,
 * out_alpha HxW.  Every output pixel is written.  In GS_COMPAT_REFERENCE mode
 * out_alpha receives zeros (the reference never writes it, Q1) and may be NULL;
 * in GS_COMPAT_FIXED mode it receives 1 - T_final. */
int gs_forward_render(const gs_gaussians *g, const gs_camera *cam, int debug,
                      int compat, void *geom_buffer, void *binning_buffer,
                      void *image_buffer, int64_t num_instances, const int32_t *radii,
                      float *out_color, float *out_feature, float *out_depth,
                      float *out_alpha, gs_stream_t stream);

/* Backward -- replaces RasterizeGaussiansBackwardCUDA / Rasterizer::backward
 * (DGR/rasterize_points.cu:128-225, CR/rasterizer_impl.cu:350-467).
 * Every element of every gradient output is written (no pre-zeroing needed).
 * Upstream gradients (dL_dout_*) may be NULL: an output that received no
 * gradient counts as zeros (autograd's unmaterialized grads).
 * dL_dmeans2D P x 3, dL_dcolors P x 3, dL_dsemantic P x F, dL_dopacity P,
 * dL_dmeans3D P x 3, dL_dcov3D P x 6, dL_dsh P x M x 3, dL_dscales P x 3,
 * dL_drotations P x 4. */
int gs_backward(const gs_gaussians *g, const gs_camera *cam, const int32_t *radii,
                int debug, int compat, const void *geom_buffer,
                const void *binning_buffer, const void *image_buffer,
                int64_t num_rendered, const float *alphas,  /* num_rendered: either count; unused */
                const float *dL_dout_color, const float *dL_dout_feature,
                const float *dL_dout_depth, const float *dL_dout_alpha,
                void *scratch, float *dL_dmeans2D, float *dL_dcolors,
                float *dL_dsemantic, float *dL_dopacity, float *dL_dmeans3D,
                float *dL_dcov3D, float *dL_dsh, float *dL_dscales,
                float *dL_drotations, gs_stream_t stream);

/* ---- camera batches (no reference analogue): the C cameras of one
 * multi-camera training step (the per-timestep camera rig)
 * rendered by ONE launch per stage instead of C per-camera call sequences --
 * no per-camera tails in the blend kernels, one host read of the plan for
 * the whole batch.  The per-camera semantics are exactly those of
 * gs_forward_plan / gs_forward_render / gs_backward (which are the C = 1
 * case), except that the backward SUMS the per-Gaussian gradients over the
 * cameras (and the densification statistics, gs_gaussians.densify_*).
 *
 *  - cams[C] (host array, 1 <= C <= 64): one image size; the device
 *    matrices of camera c are rows c of [C,16] view / [C,16] proj / [C,3]
 *    campos arrays (cams[c].viewmatrix == cams[0].viewmatrix + 16 c, ...);
 *    one shared background.  Camera scalars per camera, in the reference's
 *    positional semantics as for the single-camera calls (Q2 included).
 *  - State buffers: gs_batch_*_bytes; radii C x P; images C x (3|F|1|1) x H x W.
 *  - num_instances[C] from the plan is passed back to the render and the
 *    backward (each camera's binning buffer has its own length).
 *  - Memory: the state scales with C.  Geometry 121 B x P per camera (the
 *    64-B render record, 24-B covariance, rect, counts); backward scratch
 *    64 B x P per camera (one accumulation record per Gaussian and camera,
 *    zero-filled by every backward; + 4 B x 48 x P at F = 36); binning
 *    24 B per tile instance.  At P = 300k, C = 27 the scratch is 518 MB and
 *    the fill ~0.1 ms per step; at P = 1M, C = 64 it is 4.1 GB -- split
 *    larger rigs into camera groups of one batch call each (the gradients
 *    of successive calls add with GS_FLAG_ACCUMULATE). */
size_t gs_batch_geom_buffer_bytes(int64_t P, int32_t C);
size_t gs_batch_image_buffer_bytes(int32_t W, int32_t H, int32_t C);
size_t gs_batch_binning_buffer_bytes(int32_t C, const int64_t *num_instances);
size_t gs_batch_backward_scratch_bytes(int64_t P, int32_t F, int32_t C);

int gs_forward_plan_batch(const gs_gaussians *g, const gs_camera *cams, int32_t C,
                          int prefiltered, int debug, int compat, void *geom_buffer,
                          void *image_buffer, int32_t *radii, int64_t *num_rendered,
                          int64_t *num_instances, gs_stream_t stream);

int gs_forward_render_batch(const gs_gaussians *g, const gs_camera *cams, int32_t C,
                            int debug, int compat, void *geom_buffer, void *binning_buffer,
                            void *image_buffer, const int64_t *num_instances,
                            const int32_t *radii, float *out_color, float *out_feature,
                            float *out_depth, float *out_alpha, gs_stream_t stream);

int gs_backward_batch(const gs_gaussians *g, const gs_camera *cams, int32_t C,
                      const int32_t *radii, int debug, int compat, const void *geom_buffer,
                      const void *binning_buffer, const void *image_buffer,
                      const int64_t *num_instances, const float *alphas,
                      const float *dL_dout_color, const float *dL_dout_feature,
                      const float *dL_dout_depth, const float *dL_dout_alpha, void *scratch,
                      float *dL_dmeans2D, float *dL_dcolors, float *dL_dsemantic,
                      float *dL_dopacity, float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh,
                      float *dL_dscales, float *dL_drotations, gs_stream_t stream);

/* ---- sync-free batch forward (ABI 11; no reference analogue).
 * gs_forward_plan_batch + gs_forward_render_batch in one call without the
 * host round trip between them (the reference reads num_rendered back before
 * it can size the binning buffer, CR/rasterizer_impl.cu:283-287, and the GPU
 * idles while the host does):
 *  - the binning buffer is laid out for capacity[c] instances of camera c
 *    (gs_batch_binning_buffer_bytes(C, capacity)), e.g. the previous step's
 *    num_instances with a margin;
 *  - the tile sort's launches are sized from *hint (the previous call's plan,
 *    written back by this call; hint->valid = 0 or hint = NULL: launches
 *    that cover every tile);
 *  - the plan headers reach page-locked host memory behind the plan kernels
 *    and the call waits for them only after the bucket, sort and blend
 *    launches are enqueued.
 * On return *fits = 1: every camera's lists fit its capacity and every tile
 * was sorted -- the outputs are complete and bit-identical to the two-phase
 * path's, num_rendered / num_instances as from gs_forward_plan_batch.
 * *fits = 0: some camera's lists exceed its capacity (or a tile lay outside
 * the hinted sort launches); the kernels stored nothing into the binning
 * buffer beyond it and the outputs are NOT valid.  num_instances holds the
 * exact counts and the plan stays valid: size a binning buffer with
 * gs_batch_binning_buffer_bytes(C, num_instances) and call
 * gs_forward_render_batch with it and num_instances (the retry; its outputs
 * are those of the two-phase path).  The backward takes the per-camera
 * lengths the binning buffer of the forward it follows was laid out with
 * (capacity when *fits = 1, num_instances after a retry). */
typedef struct gs_batch_hint {
  int32_t valid;                /* 0 until a call wrote it */
  int32_t p1, q1, p2;           /* the plan's sort-class extents (opaque) */
  int64_t max_len;              /* the longest tile list */
  int64_t total;                /* the batch's list instances */
} gs_batch_hint;

int gs_forward_batch(const gs_gaussians *g, const gs_camera *cams, int32_t C, int prefiltered,
                     int compat, void *geom_buffer, void *image_buffer, void *binning_buffer,
                     const int64_t *capacity, gs_batch_hint *hint, int32_t *radii,
                     int64_t *num_rendered, int64_t *num_instances, int32_t *fits,
                     float *out_color, float *out_feature, float *out_depth, float *out_alpha,
                     gs_stream_t stream);

/* markVisible -- replaces DGR/rasterize_points.cu:227-246 and
 * CR/rasterizer_impl.cu:141-153 (checkFrustum).  present[P] is 0/1 bytes. */
int gs_mark_visible(int64_t P, const float *means3D, const float *viewmatrix,
                    const float *projmatrix, uint8_t *present, gs_stream_t stream);

/* ---- live stage timing (benchmark instrumentation; no reference analogue).
 * When enabled, a hipEvent pair is recorded on the launch stream around each
 * stage below; gs_timing_read() waits for them and returns, per stage, the
 * summed elapsed milliseconds and the number of launches since the last
 * gs_timing_enable().  Disabled by default. */
#define GS_STAGE_PREPROCESS 0
#define GS_STAGE_SCAN 1
#define GS_STAGE_DUPLICATE 2
#define GS_STAGE_SORT 3
#define GS_STAGE_RANGES 4
#define GS_STAGE_RENDER_FWD 5
#define GS_STAGE_RENDER_BWD 6
#define GS_STAGE_PREPROCESS_BWD 7
#define GS_NUM_STAGES 8
int gs_timing_enable(int enable);
/* Restrict timing to the stages whose bit (1 << GS_STAGE_x) is set (default:
 * all).  Each timed stage adds an event pair -- a few microseconds of stream
 * time -- so a benchmark times only the kernel it reports on. */
int gs_timing_select(uint32_t stage_mask);
int gs_timing_read(double *ms, int64_t *count, int n_stages);

/* ---- inspection entry points (tests and benchmarks; no reference analogue) */

/* Copy the internal per-stage state of the last forward into host-visible
 * device arrays for stage-level parity checks:
 *   means2D P x 2, depths P, conic_opacity P x 4, rgb P x 3, tiles_touched P,
 *   point_list num_rendered, ranges (tiles x 2), n_contrib H x W.
 * Any output pointer may be NULL. */
int gs_debug_export(int64_t P, int32_t W, int32_t H, const void *geom_buffer,
                    const void *binning_buffer, const void *image_buffer,
                    int64_t num_instances, float *means2D, float *depths,
                    float *conic_opacity, float *rgb, uint32_t *tiles_touched,
                    uint32_t *point_list, uint32_t *ranges, uint32_t *n_contrib,
                    gs_stream_t stream);

/* ---- debug-mode state validation (host functions, no device access)
 *
 * With `debug` set the forward checks the state it built before the blend
 * kernels dereference it (the reference's debug mode only synchronises and
 * reports launch errors, CR/auxiliary.h:172-179): the plan header after the
 * one host read of the forward, then the per-tile ranges and the tile lists
 * after the sort.  A violation returns a negative status with the message in
 * gs_last_error() (GsplatError in Python) instead of launching.  Exported so
 * the checks themselves are testable on the host with corrupted inputs.
 *
 * gs_check_plan_header: hdr = the 8-word plan header of one camera
 *   {list instances L, longest tile, reference num_rendered, status, sort-class
 *   prefixes p1, q1, p2, -}; tiles = the camera's tile count.  Requires
 *   L <= num_rendered, longest tile <= L, status bits <= 3 and
 *   q1 <= p1, p2 <= p1 <= tiles.
 * gs_check_ranges: ranges = tiles x [begin, end) of one camera's lists;
 *   every range in [0, L], begin <= end, the non-empty ranges contiguous in
 *   tile order and covering exactly [0, L); longest range <= max_len (< 0: no
 *   bound).
 * gs_check_point_list: every id of a camera's L list entries < P.
 * gs_check_walk_order: the P entries are a permutation of [0, P). */
int gs_check_plan_header(const uint32_t *hdr, int64_t tiles);
int gs_check_ranges(const uint32_t *ranges, int64_t tiles, int64_t L, int64_t max_len);
int gs_check_point_list(const uint32_t *ids, int64_t L, int64_t P);
int gs_check_walk_order(const int32_t *order, int64_t P);

/* A spatially coherent walk order for gs_gaussians.walk_order (ABI 12): the
 * ids 0..P-1 sorted by the 30-bit Morton code of means3D (P x 3) in its
 * bounding box (the stable radix sort below; ties keep id order).  scratch
 * is gs_spatial_order_scratch_bytes(P) bytes.  Any later change of the means
 * only makes the order less coherent, never wrong. */
size_t gs_spatial_order_scratch_bytes(int64_t P);
int gs_spatial_order(int64_t P, const float *means3D, int32_t *order, void *scratch, gs_stream_t stream);

/* Stable LSD radix sort of (u64 key, u32 value) pairs on bits [0, end_bit)
 * -- the standalone form of the binning sort (cub::DeviceRadixSort::SortPairs
 * at CR/rasterizer_impl.cu:309).  keys/vals are sorted in place; scratch is
 * gs_sort_scratch_bytes(n) bytes. */
size_t gs_sort_scratch_bytes(int64_t n);
int gs_sort_pairs(int64_t n, uint64_t *keys, uint32_t *vals, int end_bit,
                  void *scratch, gs_stream_t stream);

/* Self-test of the wave64 transposed reduction used by the backward blend:
 * in[n_comp][64] -> out[n_comp] (sums over the 64 lanes).  n_comp <= 64. */
int gs_test_wave_reduce(int n_comp, const float *in, float *out, gs_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GSPLAT_HIP_H */
