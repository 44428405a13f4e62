// gs_common.h -- shared constants, layouts and device helpers of the
// MI355X-native Gaussian rasterizer (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "gs_meta.h"

namespace gs {

// Binning tile = 16x16 pixels, identical to the reference (CR/config.h:18-19)
// so that tiles_touched / num_rendered / sort keys agree with it.  Inside a
// tile the blend kernels use 4 waves of 64 pixels each ("strips").
constexpr int TILE = 16;
constexpr int TILE_PIX = TILE * TILE;
constexpr int WAVE = 64;
// Strip shape: 8 x 8.  A square strip has the shortest perimeter, so fewer
// Gaussians reach it: on the bench camera 3.43 M (Gaussian, strip) survivors
// at 8 x 8 vs 3.81 M at 16 x 4 for the same 115 M blended (Gaussian, pixel)
// pairs (tools/strip_survey.py; 16 x 4 strips measured slower).
constexpr int STRIP_W = 8, STRIP_H = 8;
constexpr int STRIPS_X = TILE / STRIP_W;  // strips per tile row
// top-left pixel of strip `s` (0..3) of tile (tx, ty)
__host__ __device__ inline int strip_x0(int tx, int s) { return tx * TILE + (s % STRIPS_X) * STRIP_W; }
__host__ __device__ inline int strip_y0(int ty, int s) { return ty * TILE + (s / STRIPS_X) * STRIP_H; }

// Per-Gaussian render record written by preprocess: one 64-B line, read by
// the blend kernels with a single wave-uniform s_load_dwordx16.
constexpr int REC = 16;
enum RecField {
  R_X = 0, R_Y = 1,           // pixel-space mean (ndc2Pix)
  R_CA = 2, R_CB = 3, R_CC = 4,  // conic (inverse 2D covariance)
  R_OP = 5,                   // opacity
  R_R = 6, R_G = 7, R_B = 8,  // colour (SH-evaluated or precomputed)
  R_DEPTH = 9,                // view-space z
  R_EX = 10, R_EY = 11,       // half extents of the alpha >= 1/255 region (box-cull experiment only; 0)
  R_RAD = 12,                 // screen radius (ceil(3 sqrt(lambda_max)))
  R_TQ = 13,                  // cull threshold on a dx^2 + 2b dx dy + c dy^2
};

// Gradient accumulation record per Gaussian (backward scratch), sums over
// the Gaussian's pixels with e = dL/dG * G:  A_MX = sum e dx, A_MY = sum e dy,
// A_CA = sum e dx^2, A_CB = sum e dx dy, A_CC = sum e dy^2 (turned into
// dL/dmean2D and dL/dconic by preprocess_bwd), A_OP = dL/dopacity,
// A_R..A_B = dL/dcolour, A_DEPTH = dL/ddepth.
enum AccField {
  A_MX = 0, A_MY = 1, A_CA = 2, A_CB = 3, A_CC = 4, A_OP = 5,
  A_R = 6, A_G = 7, A_B = 8, A_DEPTH = 9, A_FEAT = 10,
};
// A Gaussian's accumulation record occupies one aligned 64-B segment: float
// atomics execute at the memory side per 64-B segment, so a record that
// straddles two segments costs two requests per commit.
constexpr int ACC_STRIDE = 16;

constexpr int COMPAT_REFERENCE = 0;
constexpr int COMPAT_FIXED = 1;

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------- layouts
// Radix-sort geometry: 256 threads per block, `rounds` items per thread,
// chosen so that a pass has ~2048 blocks (>= 8 per CU) for any n; small
// sorts (the per-Gaussian depth sort) would otherwise run on a few dozen
// latency-bound blocks.
constexpr int SORT_THREADS = 256;
__host__ __device__ inline int sort_rounds(int64_t n) {
  int64_t r = (n + (int64_t)SORT_THREADS * 2048 - 1) / ((int64_t)SORT_THREADS * 2048);
  return (int)(r < 1 ? 1 : (r > 16 ? 16 : r));
}
__host__ __device__ inline int64_t sort_blocks(int64_t n) {
  const int64_t tile = (int64_t)SORT_THREADS * sort_rounds(n);
  return (n + tile - 1) / tile;
}
// Tile bucketing geometry (gs_tiles.hip): TB_BLOCKS workgroups each own a
// contiguous slice of the Gaussians and histogram their instances over (a
// range of at most TB_BINS) tiles in LDS.  128 per camera: with the bucket
// pass staging a workgroup's keys in LDS (tile_bucket_kernel), longer per-tile
// runs make longer coalesced stores -- bench step duplicate 0.253-0.260 vs
// 0.341-0.343 ms and scan 0.091 vs 0.121 at 256 (profiles/r03w_ab_tbb128.log);
// the bench camera's ~13 k keys per workgroup fit the LDS.
constexpr int TB_BLOCKS = 128;  // per camera; a multiple of 64 (tile_rowscan_kernel, tile_offsets_kernel)
constexpr int TB_THREADS = 1024;
constexpr int TB_BINS = 16384;    // LDS tile bins per pass (64 KiB)
constexpr int SORT_SMALL = 1024;  // tile length up to which the tile sort runs in its short (small-LDS) class
constexpr int TS_CAP = 4096;      // per-tile LDS sort capacity (32 KiB of u64 keys, sorted in place)
constexpr int TS_CAP_LONG = 9600; // long-tile launch: 75 KiB (+ 8 KiB radix state), two workgroups per CU
constexpr int TS_WIDE_MEAN = 1024; // mean tile length from which the sort uses 512-thread workgroups

// Geometry buffer (per-Gaussian state kept from forward to backward).
struct GeomLayout {
  size_t rec, cov3D, clamped, tiles, rect, total;
  __host__ __device__ GeomLayout(int64_t P) {
    size_t o = 0;
    rec = o;       o = align_up(o + sizeof(float) * REC * P, 256);
    cov3D = o;     o = align_up(o + sizeof(float) * 6 * P, 256);
    clamped = o;   o = align_up(o + P, 256);
    tiles = o;     o = align_up(o + sizeof(uint32_t) * P, 256);
    // binning record, 16 B: tile rect x0 | y0 << 16, x1 | y1 << 16, depth
    // bits, tiles_touched -- everything the plan and bucket passes read, in
    // one 16-B load (the depth alone used to cost a 64-B render-record line)
    rect = o;      o = align_up(o + sizeof(uint32_t) * 4 * P, 256);
    total = o;
  }
};

// Binning buffer (per tile/Gaussian instance): the (depth bits, id) keys in
// tile-bucket order and the per-tile sorted id list the blend kernels read.
struct BinLayout {
  size_t plist, keys, keys2, total;
  __host__ __device__ BinLayout(int64_t L) {
    size_t o = 0;
    plist = o; o = align_up(o + sizeof(uint32_t) * L, 256);  // first: located without L
    keys = o;  o = align_up(o + sizeof(uint64_t) * L, 256);
    keys2 = o; o = align_up(o + sizeof(uint64_t) * L, 256);  // radix twin of long tiles
    total = o;
  }
};

// Scratch of the standalone radix sort entry point (gs_sort_pairs).
struct SortLayout {
  size_t keys1, vals1, hist, rowtot, total;
  __host__ __device__ SortLayout(int64_t n) {
    const int64_t nblk = sort_blocks(n);
    size_t o = 0;
    keys1 = o; o = align_up(o + sizeof(uint64_t) * n, 256);
    vals1 = o; o = align_up(o + sizeof(uint32_t) * n, 256);
    hist = o;  o = align_up(o + sizeof(uint32_t) * 256 * (nblk > 0 ? nblk : 1), 256);
    rowtot = o; o = align_up(o + sizeof(uint32_t) * 256, 256);
    total = o;
  }
};

// Image buffer (per pixel / per tile), also the binning plan: per-block tile
// histograms (turned into per-block offsets), tile totals and the 8-word
// header (gs_meta.h).
struct ImgLayout {
  size_t ranges, n_contrib, thist, ttotal, bsum, meta, order, smax, fmax, total;
  int64_t tiles;
  __host__ __device__ ImgLayout(int W, int H) {
    tiles = (int64_t)((W + TILE - 1) / TILE) * ((H + TILE - 1) / TILE);
    const int64_t t = tiles > 0 ? tiles : 1;
    size_t o = 0;
    ranges = o;    o = align_up(o + sizeof(uint32_t) * 2 * t, 256);
    n_contrib = o; o = align_up(o + sizeof(uint32_t) * (int64_t)W * H, 256);
    thist = o;     o = align_up(o + sizeof(uint32_t) * TB_BLOCKS * t, 256);
    ttotal = o;    o = align_up(o + sizeof(uint32_t) * t, 256);
    bsum = o;      o = align_up(o + sizeof(uint32_t) * TB_BLOCKS, 256);  // per-block rect instances
    meta = o;      o = align_up(o + sizeof(uint32_t) * M_WORDS, 256);
    // dispatch records {tile, range.x, range.y, 0}, longest list first: one
    // 16-B load gives a blend workgroup its tile and list
    order = o;     o = align_up(o + sizeof(uint32_t) * 4 * t, 256);
    smax = o;      o = align_up(o + sizeof(uint32_t) * 4 * t, 256);  // per strip item: longest pixel walk (forward -> backward)
    // per feature channel (F <= 64): the largest |feature| as float bits, for
    // the forward's fp16 feature contraction (camera 0's buffer of a batch)
    fmax = o;      o = align_up(o + sizeof(uint32_t) * 64, 256);
    total = o;
  }
};

// ---------------------------------------------------------------- camera batches
// A multi-camera batch: C cameras of one image size over one Gaussian set
// (the per-timestep multi-camera step).  Every per-camera buffer is the
// single-camera layout repeated: geometry and image buffers at a fixed
// stride, binning buffers at host-computed offsets (their lengths differ),
// images and radii [C, ...].  Kernels take the camera from blockIdx.y (or
// the minor index of a flattened grid); the single-camera entry points are
// the C = 1 case.  Camera parameters ride in the kernel arguments.
constexpr int GS_MAX_CAMS = 64;
struct CamBatch {
  int C;
  int64_t geom_stride;   // bytes between the cameras' geometry buffers
  int64_t img_stride;    // bytes between the cameras' image buffers
  const float* view;     // C x 16 column-major 4x4 (device)
  const float* proj;     // C x 16
  const float* campos;   // C x 3
  float c_x[GS_MAX_CAMS], c_y[GS_MAX_CAMS], tanx[GS_MAX_CAMS], tany[GS_MAX_CAMS];
  int64_t bin_off[GS_MAX_CAMS];  // byte offset of camera c's binning buffer
  int64_t bin_L[GS_MAX_CAMS];    // camera c's tile-list length (instances)
  uint16_t win[GS_MAX_CAMS][4];  // camera c's tile window [x0, x1) x [y0, y1) (gs_camera tile_*)
};
__host__ __device__ inline bool in_window(const CamBatch& cb, int c, int tx, int ty) {
  return tx >= cb.win[c][0] && tx < cb.win[c][2] && ty >= cb.win[c][1] && ty < cb.win[c][3];
}
template <class T>
__host__ __device__ inline T* shift_bytes(T* p, int64_t bytes) {
  return p ? reinterpret_cast<T*>(reinterpret_cast<char*>(const_cast<typename std::remove_const<T>::type*>(p)) + bytes)
           : p;
}

// ---------------------------------------------------------------- device math

// Can a Gaussian (mean (mx, my), conic (a, b, c), threshold tq on the
// quadratic form, see preprocess alpha_extent) reach alpha >= 1/255 at any
// pixel centre of the rectangle [sx0, sx1] x [sy0, sy1]?  The minimum of the
// form over the rectangle (0 when the mean is inside, else the least of the
// four clamped edge minima) against tq, which carries a margin over fp32
// rounding: exact in effect -- a culled Gaussian is one every pixel of the
// rectangle would skip in the reference's loop.  Shared by the binning (tile
// rectangles) and the blend kernels (strips), so their decisions agree.
__device__ inline bool rect_culled(float mx, float my, float a, float b, float c, float tq, float sx0,
                                   float sx1, float sy0, float sy1) {
  const float xlo = mx - sx1, xhi = mx - sx0;  // offsets mean - pixel
  const float ylo = my - sy1, yhi = my - sy0;
  if (xlo <= 0.f && xhi >= 0.f && ylo <= 0.f && yhi >= 0.f) return !(tq >= 0.f);
  auto qf = [&](float x, float y) { return fmaf(a * x, x, fmaf(c * y, y, 2.f * b * x * y)); };
  const float ra = __builtin_amdgcn_rcpf(a), rc = __builtin_amdgcn_rcpf(c);
  const float ty0 = fminf(fmaxf(-b * xlo * rc, ylo), yhi), ty1 = fminf(fmaxf(-b * xhi * rc, ylo), yhi);
  const float tx0 = fminf(fmaxf(-b * ylo * ra, xlo), xhi), tx1 = fminf(fmaxf(-b * yhi * ra, xlo), xhi);
  const float m = fminf(fminf(qf(xlo, ty0), qf(xhi, ty1)), fminf(qf(tx0, ylo), qf(tx1, yhi)));
  return m > tq;  // NaN keeps the Gaussian
}

// Block -> strip-item map of the blend kernels (item = tile * 4 + strip).
//
// Workgroups are dealt round-robin to the 8 XCDs (blockIdx % 8).  The
// contiguous remap of cdna_hip_programming.md T1 (consecutive items on one
// XCD) was measured SLOWER here (bench camera, F = 32: fwd 199 vs 182 us,
// bwd 292 vs 274 us): it hands each XCD a horizontal band of the image, and
// the bands through the scene centre carry most of the blend work, so the
// XCDs owning them finish last.  Plain dispatch order interleaves tiles over
// the XCDs (tile % 8 with a tile per workgroup) and balances the load.  (The
// wave-per-workgroup backward keeps a tile's 4 strip workgroups on one XCD:
// strip_of_block, gs_render.hip.)
__device__ inline int strip_item(int bid, int wpb) { return bid * wpb; }

__device__ inline float bits_f(uint32_t u) { return __uint_as_float(u); }
__device__ inline uint32_t f_bits(float f) { return __float_as_uint(f); }

// DPP lane permutations on gfx950 (row = 16 lanes).
template <int CTRL>
__device__ inline float dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_ROW_ROR8 = 0x128;      // lane i <- lane (i+8)%16: xor 8
constexpr int DPP_ROW_HALF_MIRROR = 0x141;  // lane i <- 7-i in each 8: partner differs in bit 2
constexpr int DPP_QUAD_XOR2 = 0x4E;      // quad_perm [2,3,0,1]
constexpr int DPP_QUAD_XOR1 = 0xB1;      // quad_perm [1,0,3,2]

// One level of the transposed wave reduction on a pair (a, b) for lane-bit
// `bit`: lanes with the bit clear end up with a's pair-sum, lanes with it set
// with b's.  LEVEL 0/1 use the gfx950 permlane32/16 swaps, 2..5 use DPP.
template <int LEVEL>
__device__ inline float red_pair(float a, float b, int lane) {
  if constexpr (LEVEL == 0) {
    auto r = __builtin_amdgcn_permlane32_swap(f_bits(a), f_bits(b), false, false);
    return bits_f(r[0]) + bits_f(r[1]);
  } else if constexpr (LEVEL == 1) {
    auto r = __builtin_amdgcn_permlane16_swap(f_bits(a), f_bits(b), false, false);
    return bits_f(r[0]) + bits_f(r[1]);
  } else {
    constexpr int bit = 5 - LEVEL;  // 3, 2, 1, 0
    const bool hi = (lane >> bit) & 1;
    const float keep = hi ? b : a;
    const float send = hi ? a : b;
    if constexpr (LEVEL == 2) return keep + dpp<DPP_ROW_ROR8>(send);
    else if constexpr (LEVEL == 3) return keep + dpp<DPP_ROW_HALF_MIRROR>(send);
    else if constexpr (LEVEL == 4) return keep + dpp<DPP_QUAD_XOR2>(send);
    else return keep + dpp<DPP_QUAD_XOR1>(send);
  }
}
template <int LEVEL>
__device__ inline float red_self(float a) {
  if constexpr (LEVEL == 0) {
    auto r = __builtin_amdgcn_permlane32_swap(f_bits(a), f_bits(a), false, false);
    return bits_f(r[0]) + bits_f(r[1]);
  } else if constexpr (LEVEL == 1) {
    auto r = __builtin_amdgcn_permlane16_swap(f_bits(a), f_bits(a), false, false);
    return bits_f(r[0]) + bits_f(r[1]);
  } else if constexpr (LEVEL == 2) return a + dpp<DPP_ROW_ROR8>(a);
  else if constexpr (LEVEL == 3) return a + dpp<DPP_ROW_HALF_MIRROR>(a);
  else if constexpr (LEVEL == 4) return a + dpp<DPP_QUAD_XOR2>(a);
  else return a + dpp<DPP_QUAD_XOR1>(a);
}

template <int LEVEL, int N>
__device__ inline void red_level(float (&v)[64], int lane) {
#pragma unroll
  for (int i = 0; i < N / 2; ++i) v[i] = red_pair<LEVEL>(v[2 * i], v[2 * i + 1], lane);
  if constexpr (N % 2) v[N / 2] = red_self<LEVEL>(v[N - 1]);
}

// Transposed wave64 reduction of N <= 64 per-lane components: on return,
// lane l holds the 64-lane sum of component bitrev6(l) (lanes whose
// bitrev6(l) >= N hold duplicates and must be ignored).  Costs about
// 2N + N/2 + ... VALU ops instead of 6N for N independent butterfly trees,
// and lets ONE atomic wave-instruction commit all N sums.
__device__ inline int bitrev6(int l) {
  return ((l & 1) << 5) | ((l & 2) << 3) | ((l & 4) << 1) | ((l & 8) >> 1) | ((l & 16) >> 3) | ((l & 32) >> 5);
}
template <int N>
__device__ inline float wave_reduce_transposed(float (&v)[64], int lane) {
  static_assert(N >= 1 && N <= 64, "N in [1,64]");
  constexpr int N1 = (N + 1) / 2, N2 = (N1 + 1) / 2, N3 = (N2 + 1) / 2, N4 = (N3 + 1) / 2,
                N5 = (N4 + 1) / 2;
  red_level<0, N>(v, lane);
  red_level<1, N1>(v, lane);
  red_level<2, N2>(v, lane);
  red_level<3, N3>(v, lane);
  red_level<4, N4>(v, lane);
  red_level<5, N5>(v, lane);
  return v[0];
}

__device__ inline float wave_max_f(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
  return x;
}
__device__ inline uint32_t wave_max_u(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t y = __shfl_xor(x, o, 64);
    x = x > y ? x : y;
  }
  return x;
}

}  // namespace gs
