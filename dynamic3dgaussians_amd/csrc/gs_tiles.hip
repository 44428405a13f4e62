// gs_tiles.hip -- tile binning: every (tile, Gaussian) instance into its
// tile's list, each list in (depth, Gaussian id) order.
//
// Reference: DGR/cuda_rasterizer/rasterizer_impl.cu:70-138 and :283-314
// (duplicateWithKeys over an inclusive scan of tiles_touched, a global cub
// radix sort of (tile << 32 | depth bits) keys on 32 + getHigherMsb(tiles)
// bits, identifyTileRanges).  That sort is stable, so inside a tile the list
// is ordered by depth bits with ties in Gaussian index order.
//
// MI355X design -- no global sort at all:
//  1. plan   (tile_hist_kernel): TB_BLOCKS workgroups each histogram the
//     instances of a contiguous slice of the Gaussians over the tiles in LDS
//     and write one row of a [block][tile] count matrix (contiguous);
//     (tile_rowscan_kernel) turns every tile column into per-block offsets
//     inside the tile and a tile total; (tile_offsets_kernel, one workgroup)
//     scans the totals into ranges[tile] and writes the 8-word plan header
//     {L, longest tile, the reference's num_rendered, status, sort-class
//     prefixes P1, Q1, P2, -} -- the one device->host read of the forward
//     (the reference's num_rendered read, :287).
//  2. bucket (tile_bucket_kernel): the same walk, each instance taking a slot
//     from an LDS cursor in its workgroup's run of its tile (the plan's
//     per-block counts, scanned), its 64-bit (depth bits << 32 | id) key
//     staged in LDS; the runs are then copied to their tiles' segments in
//     order, so consecutive lanes store consecutive keys (a workgroup with
//     more keys than the LDS holds stores each key where its slot lands,
//     tile_hist_kernel<true>) -- the order inside a segment is arbitrary.
//  3. sort   (tile_sort_kernel): one workgroup per tile sorts its segment by
//     the full key.  Common case, an MSD bucket sort: the top bits of the
//     tile's depth-bit span pick one of 1,024 buckets (LDS atomics give each
//     key its slot), one scan, one scatter, then every key takes its place
//     in its bucket by counting the bucket's smaller keys -- the keys go from
//     global memory to registers to one LDS buffer (the scatter target, then
//     the sorted ids over its start).  Tiles whose
//     keys crowd into few buckets fall back to an LSD radix sort in global
//     memory (wave-owned quarters, ballot-matched stable scatter, skipped
//     constant-digit passes, equal depths ordered by id).  Keys are unique,
//     so either way the list is exactly the reference's stable order.
//     Length classes (short / up to TS_CAP / up to TS_CAP_LONG, two
//     workgroups per CU / beyond in global memory) run as separate launches
//     over their prefix of the longest-first dispatch order (P1, Q1, P2 in
//     the header).
// Integer work, HBM- and latency-bound; 5 launches instead of the
// reference's scan + 6-pass 64-bit radix sort + ranges.
#include <cstdlib>

#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

// The Gaussian at walk position w of the binning passes: the caller's walk
// order (gs_gaussians.walk_order, a permutation) or the ids themselves.  The
// plan and bucket passes walk the same order, so their per-block counts
// match; the tile lists do not depend on it (the sort orders every list by
// its unique (depth bits, id) keys).
__device__ inline int walk_id(const TileArgs& a, int w) { return a.walk ? a.walk[w] : w; }

// Instances of one rect handled by one lane; larger rects are spread over the
// wave (a full-screen Gaussian must not serialize its wave for 2,500 tiles).
constexpr int LANE_TILES = 16;

// A Gaussian's instances are the tiles of its binning rect (preprocess: the
// reference's getRect cut to the bounding box of the alpha >= 1/255
// ellipse, so the dropped instances are ones no pixel of their tile blends).
// The reference's tiles_touched (its num_rendered) is summed per block
// alongside.
template <bool WRITE>
__global__ __launch_bounds__(TB_THREADS) void tile_hist_kernel(TileArgs a0, CamBatch cb, int t0, int nt) {
  const TileArgs a = cam_tile_args(a0, cb, blockIdx.y);
  // a binning buffer laid out for fewer instances than the plan counted
  // (gs_forward_batch's capacity): store nothing, the caller renders again
  if (WRITE && a.meta[M_L] > (uint64_t)cb.bin_L[blockIdx.y]) return;
  extern __shared__ uint32_t s_bin[];  // nt counters (hist) or cursors (bucket)
  __shared__ uint32_t s_rect[TB_THREADS / 64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int per = (a.P + TB_BLOCKS - 1) / TB_BLOCKS;
  const int g0 = b * per, g1 = min(a.P, g0 + per);
  // the first slice's rects are requested before the cursor set-up, so their
  // latency overlaps it (the set-up ends in a barrier the compiler does not
  // hoist loads across); walk position -> Gaussian id through the walk order
  int inext = g0 + tid < g1 ? walk_id(a, g0 + tid) : 0;
  uint4 rnext = g0 + tid < g1 ? a.rect[inext] : make_uint4(0u, 0u, 0u, 0u);
  for (int i = tid; i < nt; i += TB_THREADS)
    s_bin[i] = WRITE ? a.ranges[t0 + i].x + a.thist[(size_t)b * a.num_tiles + t0 + i] : 0u;
  __syncthreads();
  const int gx = a.grid_x;
  uint32_t rect_n = 0;
  for (int base = g0; base < g1; base += TB_THREADS) {
    const int g = base + tid;
    int x0 = 0, y0 = 0, w = 0, n = 0;
    uint64_t key = 0;
    const uint4 r = rnext;  // {x0 | y0 << 16, x1 | y1 << 16, depth bits, tiles_touched}
    const int gi = inext;   // the Gaussian at walk position g
    if (base + TB_THREADS < g1 && g + TB_THREADS < g1) {
      inext = walk_id(a, g + TB_THREADS);
      rnext = a.rect[inext];
    }
    if (g < g1) {
      x0 = (int)(r.x & 0xFFFFu);
      y0 = (int)(r.x >> 16);
      w = (int)(r.y & 0xFFFFu) - x0;
      n = w * ((int)(r.y >> 16) - y0);
      if (WRITE && n > 0) key = ((uint64_t)r.z << 32) | (uint32_t)gi;
      if (!WRITE) rect_n += r.w;
    }
    auto emit = [&](int x, int y, uint64_t k) {
      const uint32_t u = (uint32_t)(y * gx + x - t0);
      if (u < (uint32_t)nt) {
        if (WRITE) a.keys[atomicAdd(&s_bin[u], 1u)] = k;
        else atomicAdd(&s_bin[u], 1u);
      }
    };
    if (n > 0 && n <= LANE_TILES) {
      const int h = n / w;
      for (int y = y0; y < y0 + h; ++y)
        for (int x = x0; x < x0 + w; ++x) emit(x, y, key);
    }
    uint64_t big = __ballot(n > LANE_TILES);
    while (big) {
      const int j = __builtin_ctzll(big);
      big &= big - 1;
      const int bx0 = __shfl(x0, j, 64), by0 = __shfl(y0, j, 64), bw = __shfl(w, j, 64);
      const int bn = __shfl(n, j, 64);
      const uint64_t bk = WRITE ? (uint64_t)__shfl((long long)key, j, 64) : 0ull;
      for (int i = lane; i < bn; i += 64) emit(bx0 + i % bw, by0 + i / bw, bk);
    }
  }
  if (!WRITE) {
    // the reference's num_rendered: bounding-rect instances of this block
    // (counted once, in the first tile pass)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) rect_n += __shfl_xor(rect_n, o, 64);
    if (lane == 0) s_rect[tid >> 6] = rect_n;
    __syncthreads();
    for (int i = tid; i < nt; i += TB_THREADS) a.thist[(size_t)b * a.num_tiles + t0 + i] = s_bin[i];
    if (tid == 0 && t0 == 0) {
      uint32_t sum = 0;
      for (int w2 = 0; w2 < TB_THREADS / 64; ++w2) sum += s_rect[w2];
      a.bsum[b] = sum;
    }
  }
}

// The count pass as a 2-D difference array: each Gaussian adds +1 / -1 at
// the four corners of its tile rect (4 LDS atomics instead of one per
// instance -- 5.5 per Gaussian at the bench scene, 14.6 at configs[4] --
// and, in a coherent walk order, far fewer same-address collisions), then a
// row scan and a column scan over the (gy + 1) x (gx + 1) grid turn the
// corners into every tile's count (integer sums: exactly tile_hist_kernel's
// counts).  One launch over the whole tile grid (grids up to TB_BINS tiles;
// launch_tile_plan falls back to the per-instance count beyond).
__global__ __launch_bounds__(TB_THREADS) void tile_count_kernel(TileArgs a0, CamBatch cb) {
  const TileArgs a = cam_tile_args(a0, cb, blockIdx.y);
  extern __shared__ uint32_t s_d[];  // (gy + 1) x (gx + 1) difference counters
  __shared__ uint32_t s_rect[TB_THREADS / 64];
  constexpr int NW = TB_THREADS / 64;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int gx = a.grid_x, gy = a.grid_y, DX = gx + 1, ND = DX * (gy + 1);
  const int per = (a.P + TB_BLOCKS - 1) / TB_BLOCKS;
  const int g0 = b * per, g1 = min(a.P, g0 + per);
  for (int i = tid; i < ND; i += TB_THREADS) s_d[i] = 0u;
  __syncthreads();
  uint32_t rect_n = 0;
  for (int g = g0 + tid; g < g1; g += TB_THREADS) {
    const uint4 r = a.rect[walk_id(a, g)];  // {x0 | y0 << 16, x1 | y1 << 16, depth bits, tiles_touched}
    rect_n += r.w;
    const int x0 = min((int)(r.x & 0xFFFFu), gx), y0 = min((int)(r.x >> 16), gy);
    const int x1 = min((int)(r.y & 0xFFFFu), gx), y1 = min((int)(r.y >> 16), gy);
    if (x1 > x0 && y1 > y0) {
      atomicAdd(&s_d[y0 * DX + x0], 1u);
      atomicAdd(&s_d[y0 * DX + x1], 0xFFFFFFFFu);
      atomicAdd(&s_d[y1 * DX + x0], 0xFFFFFFFFu);
      atomicAdd(&s_d[y1 * DX + x1], 1u);
    }
  }
  __syncthreads();
  // inclusive scan of `n` entries at stride `step` from `base`, one wave
  auto wave_scan = [&](int base, int n, int step) {
    uint32_t carry = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int i = c0 + lane;
      uint32_t v = i < n ? s_d[base + i * step] : 0u;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
      }
      if (i < n) s_d[base + i * step] = v + carry;
      carry += __shfl(v, 63, 64);
    }
  };
  for (int y = wv; y <= gy; y += NW) wave_scan(y * DX, DX, 1);  // along x
  __syncthreads();
  for (int x = wv; x <= gx; x += NW) wave_scan(x, gy + 1, DX);  // along y
  __syncthreads();
  const int T = a.num_tiles;
  for (int t = tid; t < T; t += TB_THREADS) {
    const int y = t / gx, x = t - y * gx;
    a.thist[(size_t)b * T + t] = s_d[y * DX + x];
  }
  // the reference's num_rendered: bounding-rect instances of this block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) rect_n += __shfl_xor(rect_n, o, 64);
  if (lane == 0) s_rect[wv] = rect_n;
  __syncthreads();
  if (tid == 0) {
    uint32_t sum = 0;
    for (int w2 = 0; w2 < NW; ++w2) sum += s_rect[w2];
    a.bsum[b] = sum;
  }
}

// Bucket pass with the block's keys staged in LDS (the direct pass, the
// tile_hist_kernel<true> walk above, every key stored where its slot lands).
// Consecutive lanes of that walk hold unrelated Gaussians, so each key store
// is its own 8-B request to a different line; storing every key twice cost
// +0.7 ms per 27-camera step (profiles/r03u_ab_bucket_store2.log), i.e. the
// stores, not the walk, bound the pass.  Here the block first lays out its
// own per-tile runs in LDS (the count pass's per-block counts, scanned), the
// walk drops each key into its run there, and the block then copies the runs
// out in order: consecutive lanes store consecutive keys of a run.  A block
// with more keys than the LDS holds (cap, 10 B per key) stores directly, as
// before.
__global__ __launch_bounds__(TB_THREADS) void tile_bucket_kernel(TileArgs a0, CamBatch cb, int t0, int nt, int cap) {
  const TileArgs a = cam_tile_args(a0, cb, blockIdx.y);
  if (a.meta[M_L] > (uint64_t)cb.bin_L[blockIdx.y]) return;  // over capacity (tile_hist_kernel<true>)
  extern __shared__ uint64_t s_dyn64[];
  uint64_t* s_key = s_dyn64;                                    // cap keys
  uint32_t* s_cur = reinterpret_cast<uint32_t*>(s_key + cap);   // nt run cursors (local, or global if direct)
  uint32_t* s_dlt = s_cur + nt;                                 // nt: global slot - local slot of the tile's run
  uint16_t* s_til = reinterpret_cast<uint16_t*>(s_dlt + nt);    // cap: the key's tile (nt <= 65536)
  __shared__ uint32_t s_wsum[TB_THREADS / 64];
  __shared__ uint32_t s_total;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int per = (a.P + TB_BLOCKS - 1) / TB_BLOCKS;
  const int g0 = b * per, g1 = min(a.P, g0 + per);
  const int T = a.num_tiles;
  int inext = g0 + tid < g1 ? walk_id(a, g0 + tid) : 0;
  uint4 rnext = g0 + tid < g1 ? a.rect[inext] : make_uint4(0u, 0u, 0u, 0u);
  // this block's run length in every tile: the column scan left each block's
  // offset inside the tile in thist (the next block's offset, or the tile
  // total, ends the run)
  constexpr int KT = 16;  // tiles per thread in the local scan (TB_THREADS * KT >= nt)
  const int i0 = tid * ((nt + TB_THREADS - 1) / TB_THREADS);
  const int i1 = min(nt, i0 + (nt + TB_THREADS - 1) / TB_THREADS);
  uint32_t cnt[KT];
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    const int i = i0 + k;
    cnt[k] = 0;
    if (i < i1) {
      const size_t t = (size_t)t0 + i;
      const uint32_t beg = a.thist[(size_t)b * T + t];
      const uint32_t end = b + 1 < TB_BLOCKS ? a.thist[(size_t)(b + 1) * T + t] : a.ttotal[t];
      cnt[k] = end - beg;
      run += cnt[k];
    }
  }
  // exclusive scan of the per-thread sums over the block
  uint32_t incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wsum[wv] = incl;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < TB_THREADS / 64; ++w) {
      const uint32_t v = s_wsum[w];
      s_wsum[w] = acc;
      acc += v;
    }
    s_total = acc;
  }
  __syncthreads();
  const uint32_t total = s_total;
  const bool staged = total <= (uint32_t)cap;
  {
    uint32_t lo = s_wsum[wv] + incl - run;  // local start of this thread's first tile
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int i = i0 + k;
      if (i < i1) {
        const size_t t = (size_t)t0 + i;
        const uint32_t gbeg = a.ranges[t].x + a.thist[(size_t)b * T + t];
        s_cur[i] = staged ? lo : gbeg;
        s_dlt[i] = gbeg - lo;
        lo += cnt[k];
      }
    }
  }
  __syncthreads();
  const int gx = a.grid_x;
  for (int base = g0; base < g1; base += TB_THREADS) {
    const int g = base + tid;
    int x0 = 0, y0 = 0, w = 0, n = 0;
    uint64_t key = 0;
    const uint4 r = rnext;  // {x0 | y0 << 16, x1 | y1 << 16, depth bits, tiles_touched}
    const int gi = inext;
    if (base + TB_THREADS < g1 && g + TB_THREADS < g1) {
      inext = walk_id(a, g + TB_THREADS);
      rnext = a.rect[inext];
    }
    if (g < g1) {
      x0 = (int)(r.x & 0xFFFFu);
      y0 = (int)(r.x >> 16);
      w = (int)(r.y & 0xFFFFu) - x0;
      n = w * ((int)(r.y >> 16) - y0);
      if (n > 0) key = ((uint64_t)r.z << 32) | (uint32_t)gi;
    }
    auto emit = [&](int x, int y, uint64_t k) {
      const uint32_t u = (uint32_t)(y * gx + x - t0);
      if (u < (uint32_t)nt) {
        const uint32_t sl = atomicAdd(&s_cur[u], 1u);
        if (staged) {
          s_key[sl] = k;
          s_til[sl] = (uint16_t)u;
        } else {
          a.keys[sl] = k;
        }
      }
    };
    if (n > 0 && n <= LANE_TILES) {
      const int h = n / w;
      for (int y = y0; y < y0 + h; ++y)
        for (int x = x0; x < x0 + w; ++x) emit(x, y, key);
    }
    uint64_t big = __ballot(n > LANE_TILES);
    while (big) {
      const int j = __builtin_ctzll(big);
      big &= big - 1;
      const int bx0 = __shfl(x0, j, 64), by0 = __shfl(y0, j, 64), bw = __shfl(w, j, 64);
      const int bn = __shfl(n, j, 64);
      const uint64_t bk = (uint64_t)__shfl((long long)key, j, 64);
      for (int i = lane; i < bn; i += 64) emit(bx0 + i % bw, by0 + i / bw, bk);
    }
  }
  if (staged) {
    __syncthreads();
    for (uint32_t i = tid; i < total; i += TB_THREADS) a.keys[s_dlt[s_til[i]] + i] = s_key[i];
  }
}

// Column scan of the [block][tile] count matrix (each plan/bucket workgroup
// reads and writes its own row contiguously): for every tile, the exclusive
// scan over the blocks (each block's offset inside the tile) and the tile
// total.  A workgroup takes RS_T tiles; thread (bg, tt) walks blocks
// 16 bg .. 16 bg + 15 of tile tt (16 tiles x 4 B = one 64-B piece per block
// row and load), the RS_BG block-group partial sums are scanned through LDS.
static_assert(TB_BLOCKS % 64 == 0 && TB_BLOCKS <= 256, "tile_rowscan_kernel: 4 to 16 block groups of 16 blocks");
// RS_THREADS threads: RS_T = RS_THREADS / RS_BG tiles per workgroup, so each
// load instruction of a wave reads 64 consecutive tiles of one block row
// (256 contiguous bytes at 1024 threads; 4 x 64 B pieces at 256)
constexpr int RS_THREADS = 1024;
constexpr int RS_BG = TB_BLOCKS / 16, RS_T = RS_THREADS / RS_BG;
__global__ __launch_bounds__(RS_THREADS) void tile_rowscan_kernel(uint32_t* __restrict__ thist0,
                                                           uint32_t* __restrict__ ttotal0, int T, CamBatch cb) {
  uint32_t* __restrict__ thist = shift_bytes(thist0, blockIdx.y * cb.img_stride);
  uint32_t* __restrict__ ttotal = shift_bytes(ttotal0, blockIdx.y * cb.img_stride);
  __shared__ uint32_t s_part[RS_BG][RS_T];
  const int tid = threadIdx.x, tt = tid % RS_T, bg = tid / RS_T;
  const int t = blockIdx.x * RS_T + tt;
  const bool ok = t < T;
  uint32_t v[16];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] = ok ? thist[(size_t)(16 * bg + i) * T + t] : 0u;
    sum += v[i];
  }
  s_part[bg][tt] = sum;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int g = 0; g < RS_BG; ++g) {
    const uint32_t x = s_part[g][tt];
    off += g < bg ? x : 0u;
    tot += x;
  }
  if (ok) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      thist[(size_t)(16 * bg + i) * T + t] = off;
      off += v[i];
    }
    if (bg == 0) ttotal[t] = tot;
  }
}

// One workgroup: exclusive scan of the tile totals into ranges, and the header.
constexpr int OFF_T = 1024;
__global__ __launch_bounds__(OFF_T) void tile_offsets_kernel(const uint32_t* __restrict__ ttotal0, int T,
                                                             const uint32_t* __restrict__ bsum0,
                                                             uint2* __restrict__ ranges0,
                                                             uint32_t* __restrict__ meta0, int prefiltered,
                                                             CamBatch cb, uint32_t* __restrict__ hdr_host) {
  const int64_t io = blockIdx.x * cb.img_stride;  // one workgroup per camera
  const uint32_t* __restrict__ ttotal = shift_bytes(ttotal0, io);
  const uint32_t* __restrict__ bsum = shift_bytes(bsum0, io);
  uint2* __restrict__ ranges = shift_bytes(ranges0, io);
  uint32_t* __restrict__ meta = shift_bytes(meta0, io);
  __shared__ unsigned long long s_sum[OFF_T / 64];
  __shared__ unsigned long long s_lref;
  __shared__ uint32_t s_max, s_cnt[3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) { s_max = 0; s_lref = 0; s_cnt[0] = s_cnt[1] = s_cnt[2] = 0; }
  const int per = (T + OFF_T - 1) / OFF_T;
  const int a0 = min(T, tid * per), a1 = min(T, a0 + per);
  unsigned long long sum = 0;
  uint32_t mx = 0;
  for (int t = a0; t < a1; ++t) {
    const uint32_t v = ttotal[t];
    sum += v;
    mx = max(mx, v);
  }
  // wave inclusive scan, then across the 16 waves
  unsigned long long inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_sum[wave] = inc;
  __syncthreads();
  atomicMax(&s_max, mx);
  // the reference's num_rendered: sum of the per-block tiles_touched sums
  if (tid < TB_BLOCKS) {
    unsigned long long v = bsum[tid];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) atomicAdd(&s_lref, v);
  }
  __syncthreads();  // s_max complete (read by the sort-class counts below)
  unsigned long long woff = 0, total = 0;
#pragma unroll
  for (int w = 0; w < OFF_T / 64; ++w) {
    const unsigned long long v = s_sum[w];
    if (w < wave) woff += v;
    total += v;
  }
  unsigned long long run = woff + inc - sum;
  for (int t = a0; t < a1; ++t) {
    const uint32_t v = ttotal[t];
    // empty tiles keep (0, 0), as identifyTileRanges leaves them (rasterizer_impl.cu:116-138)
    ranges[t] = v ? make_uint2((uint32_t)run, (uint32_t)(run + v)) : make_uint2(0u, 0u);
    run += v;
  }
  // Where the sort's length classes sit in tile_order_kernel's dispatch order
  // (descending by the bucket v >> sh, the same sh): the tiles longer than
  // SORT_SMALL all lie in the prefix of the P1 tiles whose bucket reaches
  // (SORT_SMALL + 1) >> sh, the Q1 tiles whose bucket exceeds
  // SORT_SMALL >> sh are all long, and the P2 prefix likewise holds every
  // tile longer than TS_CAP -- so each class launch covers only its part.
  {
    const uint32_t mxl = s_max;
    const int sh = mxl >= OFF_T ? (32 - __builtin_clz(mxl)) - 10 : 0;
    uint32_t p1 = 0, q1 = 0, p2 = 0;
    for (int t = a0; t < a1; ++t) {
      const uint32_t b = ttotal[t] >> sh;
      p1 += b >= ((uint32_t)(SORT_SMALL + 1) >> sh) ? 1u : 0u;
      q1 += b > ((uint32_t)SORT_SMALL >> sh) ? 1u : 0u;
      p2 += b >= ((uint32_t)(TS_CAP + 1) >> sh) ? 1u : 0u;
    }
    if (p1) atomicAdd(&s_cnt[0], p1);
    if (q1) atomicAdd(&s_cnt[1], q1);
    if (p2) atomicAdd(&s_cnt[2], p2);
  }
  __syncthreads();
  if (tid == 0) {
    const unsigned long long lref = s_lref;
    // ranges are 32-bit, as in the reference
    const uint32_t ovf = (total > 0xFFFFFFFFull || lref > 0xFFFFFFFFull) ? 2u : 0u;
    uint32_t h[M_WORDS] = {0u};
    h[M_L] = (uint32_t)total;
    h[M_MAXN] = s_max;
    h[M_LREF] = (uint32_t)lref;
    h[M_STATUS] = prefiltered ? (meta[M_STATUS] | ovf) : ovf;
    h[M_SORT_P1] = s_cnt[0];
    h[M_SORT_Q1] = s_cnt[1];
    h[M_SORT_P2] = s_cnt[2];
#pragma unroll
    for (int w = 0; w < M_WORDS; ++w) meta[w] = h[w];
    // The host's copy of the header: page-locked, device-mapped, coherent
    // host memory written here directly (vector stores at system scope), so
    // no copy command sits in the stream between the plan and the render
    // launches.  The host polls the last word (its sentinel, 0 once written):
    // the other words first, a system fence, then the sentinel, so a host that
    // sees the sentinel sees the header.  (An event on this dispatch instead
    // idled the GPU 15-27 us behind it per step: profiles/r06gaps3/.)
    if (hdr_host) {
      uint32_t* o = hdr_host + (size_t)blockIdx.x * M_WORDS;
#pragma unroll
      for (int w = 0; w < M_WORDS - 1; ++w)
        __hip_atomic_store(o + w, h[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
      __hip_atomic_store(o + M_WORDS - 1, h[M_WORDS - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Dispatch order of the blend (and sort) kernels: the tiles by descending
// list length (a counting sort on the top 10 bits of the length), so the
// longest tiles start first and the short ones fill the end of the launch --
// the longest-processing-time-first rule for a greedy workgroup dispatcher
// (bench camera: render_fwd 143 -> 135 us, render_bwd 263 -> 250 us).  The
// order inside a bucket is arbitrary: every tile's result is independent of
// when it runs.  One workgroup; launched with the render phase, off the
// plan -> header-read path the host waits for.
__global__ __launch_bounds__(OFF_T) void tile_order_kernel(const uint32_t* __restrict__ ttotal0, int T,
                                                           const uint32_t* __restrict__ meta0,
                                                           const uint2* __restrict__ ranges0,
                                                           uint4* __restrict__ order0, uint32_t* __restrict__ fmax,
                                                           CamBatch cb, SortCover cv) {
  const int64_t io = blockIdx.x * cb.img_stride;  // one workgroup per camera
  // the forward's feature-range table starts at zero (launch_feature_absmax
  // runs later on the stream; this saves it a fill launch)
  if (blockIdx.x == 0 && threadIdx.x < 64) fmax[threadIdx.x] = 0u;
  const uint32_t* __restrict__ ttotal = shift_bytes(ttotal0, io);
  const uint32_t* __restrict__ meta = shift_bytes(meta0, io);
  const uint2* __restrict__ ranges = shift_bytes(ranges0, io);
  uint4* __restrict__ order = shift_bytes(order0, io);
  __shared__ uint32_t s_obin[OFF_T];
  __shared__ uint32_t s_owsum[OFF_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per = (T + OFF_T - 1) / OFF_T;
  const int a0 = min(T, tid * per), a1 = min(T, a0 + per);
  s_obin[tid] = 0;
  __syncthreads();
  const uint32_t mxl = meta[M_MAXN];
  // a camera whose lists exceed its binning buffer (gs_forward_batch's
  // capacity) gets empty dispatch records: the sort and blend kernels then
  // read nothing from that buffer, and the caller renders again
  bool over = meta[M_L] > (uint64_t)cb.bin_L[blockIdx.x];
  if (cv.on) {  // a tile outside the sort launches (SortCover): render nothing either
    const bool covered = meta[M_SORT_Q1] >= (uint32_t)cv.q1 &&
                         (mxl <= (uint32_t)SORT_SMALL || (cv.mid && meta[M_SORT_P1] <= (uint32_t)cv.p1)) &&
                         (mxl <= (uint32_t)TS_CAP || (cv.lng && meta[M_SORT_P2] <= (uint32_t)cv.p2));
    over = over || !covered;
  }
  const int sh = mxl >= OFF_T ? (32 - __builtin_clz(mxl)) - 10 : 0;
  for (int t = a0; t < a1; ++t) atomicAdd(&s_obin[OFF_T - 1 - min(ttotal[t] >> sh, (uint32_t)(OFF_T - 1))], 1u);
  __syncthreads();
  const uint32_t c = s_obin[tid];
  uint32_t ci = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(ci, o, 64);
    if (lane >= o) ci += y;
  }
  if (lane == 63) s_owsum[wave] = ci;
  __syncthreads();
  uint32_t base = ci - c;
  for (int w = 0; w < wave; ++w) base += s_owsum[w];
  s_obin[tid] = base;
  __syncthreads();
  for (int t = a0; t < a1; ++t) {
    const uint2 r = ranges[t];
    order[atomicAdd(&s_obin[OFF_T - 1 - min(ttotal[t] >> sh, (uint32_t)(OFF_T - 1))], 1u)] =
        over ? make_uint4((uint32_t)t, 0u, 0u, 0u) : make_uint4((uint32_t)t, r.x, r.y, 0u);
  }
}

// One tile per workgroup: LSD radix sort of its (depth bits << 32 | id) keys
// on the depth bits relative to the tile's minimum, 8 bits a pass, only as
// many passes as the tile's depth-bit span needs (and passes whose digit is
// the same for every key are skipped).  Wave w owns the contiguous quarter
// [w*q, (w+1)*q) of the keys; per pass it counts digits per wave (ballot
// match, one leader per digit and round), a 256-thread scan turns the counts
// into per-(wave, digit) bases, and each wave scatters its keys in order --
// stable, with no barrier inside the scatter.  LSD passes keep equal depths
// in their incoming (arbitrary bucket) order, so a last step sorts any run of
// equal depth by id: the result is the reference's (depth, index) order.
// Keys live in LDS (two buffers) or, for tiles longer than the launch's LDS
// capacity, in global memory (the keys segment and its twin in keys2).
__device__ inline uint64_t match_digit8(uint32_t d, uint64_t valid) {
  // peers &= (bit set ? ballot : ~ballot), per 32-bit half: with s = 0 / -1
  // the sign-extended bit, keep = ~(ballot ^ s) -> peers & ~(ballot ^ s)
  uint32_t lo = (uint32_t)valid, hi = (uint32_t)(valid >> 32);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t m = __ballot((d >> b) & 1u);
    const uint32_t sx = ~(uint32_t)__builtin_amdgcn_sbfe(d, b, 1);  // bit set -> 0, clear -> ~0
    lo &= ~((uint32_t)m ^ ~sx);
    hi &= ~((uint32_t)(m >> 32) ^ ~sx);
  }
  return ((uint64_t)hi << 32) | lo;
}

// Bucket bits of the MSD sort: 2^10 buckets, 2^11 for the longer length
// classes of long-tile scenes (tile_sort_launches).
constexpr int BS_BITS = 10, BS_BITS_LONG = 11;
constexpr int BS_KPT = 8;       // keys per thread held in registers (up to 8 NT keys per tile)
constexpr int BS_KPT_LONG = 16;  // for launches whose tiles exceed 8 NT keys (20 / 24 measured slower)
constexpr int BS_BUCKET_MAX = 48;  // fullest bucket the bucket sort ranks (each key reads its bucket's keys)

template <int NT, int BINS>
struct RadixSmem {
  static constexpr int TS_WAVES = NT / 64;
  union {
    uint32_t wcnt[TS_WAVES][256];  // radix: per-wave digit counts, then per-wave bases
    uint32_t bcnt[BINS];           // bucket sort: bucket counts, then bucket starts
  };
  uint32_t wsum[TS_WAVES > 4 ? TS_WAVES : 4];  // scan partials
  int skip, unsorted;
  uint32_t dmin, dmax;  // depth-bit range of the tile
};

template <class KP, int TS_THREADS, int BINS>
__device__ __attribute__((always_inline)) KP tile_radix_sort(KP A, KP B, int n, RadixSmem<TS_THREADS, BINS>& sm) {
  // one thread per 8-bit digit in the count scans below
  static_assert(TS_THREADS >= 256, "tile_radix_sort needs >= 256 threads per workgroup");
  constexpr int TS_WAVES = TS_THREADS / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const int q = (n + TS_WAVES - 1) / TS_WAVES;
  const int w0 = min(n, wave * q), w1 = min(n, w0 + q);
  KP src = A, dst = B;
  // Sort on depth bits relative to the tile's minimum: positive float bits
  // order like the floats, and only the bits that vary need passes.
  if (tid == 0) { sm.dmin = 0xFFFFFFFFu; sm.dmax = 0u; }
  uint32_t lmin = 0xFFFFFFFFu, lmax = 0u;
  for (int i = tid; i < n; i += TS_THREADS) {
    const uint32_t h = (uint32_t)(src[i] >> 32);
    lmin = min(lmin, h);
    lmax = max(lmax, h);
  }
  __syncthreads();
  atomicMin(&sm.dmin, lmin);
  atomicMax(&sm.dmax, lmax);
  __syncthreads();
  const uint32_t dmin = sm.dmin, span = sm.dmax - dmin;
  const int nbits = span ? 32 - __builtin_clz(span) : 0;
  for (int shift = 0; shift < nbits; shift += 8) {
    for (int i = tid; i < TS_WAVES * 256; i += TS_THREADS) (&sm.wcnt[0][0])[i] = 0;
    if (tid == 0) sm.skip = 0;
    __syncthreads();
    for (int i0 = w0; i0 < w1; i0 += 64) {
      const int i = i0 + lane;
      const bool valid = i < w1;
      // counts need no order: one LDS atomic per key
      if (valid) atomicAdd(&sm.wcnt[wave][(((uint32_t)(src[i] >> 32) - dmin) >> shift) & 255u], 1u);
    }
    __syncthreads();
    // digit d = tid (first 256 threads): total over the waves, exclusive
    // scan over the digits, then per-(wave, digit) bases
    uint32_t c[TS_WAVES];
    uint32_t tot = 0, inc = 0;
    if (tid < 256) {
#pragma unroll
      for (int w = 0; w < TS_WAVES; ++w) {
        c[w] = sm.wcnt[w][tid];
        tot += c[w];
      }
      if (tot == (uint32_t)n) sm.skip = 1;
      inc = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      if (lane == 63) sm.wsum[wave] = inc;
    }
    __syncthreads();
    const bool skip = sm.skip != 0;
    if (tid < 256) {
      uint32_t ex = inc - tot;
#pragma unroll
      for (int w = 0; w < 4; ++w) ex += w < wave ? sm.wsum[w] : 0u;
#pragma unroll
      for (int w = 0; w < TS_WAVES; ++w) {
        sm.wcnt[w][tid] = ex;
        ex += c[w];
      }
    }
    __syncthreads();
    if (skip) continue;  // uniform: one digit holds every key
    for (int i0 = w0; i0 < w1; i0 += 64) {
      const int i = i0 + lane;
      const bool valid = i < w1;
      const uint64_t k = valid ? src[i] : 0ull;
      const uint32_t d = (((uint32_t)(k >> 32) - dmin) >> shift) & 255u;
      const uint64_t peers = match_digit8(d, __ballot(valid));
      const uint64_t below = peers & lt;
      const uint32_t base = sm.wcnt[wave][d];
      if (valid) dst[base + (uint32_t)__popcll(below)] = k;
      if (valid && below == 0) sm.wcnt[wave][d] = base + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    const KP t = src;
    src = dst;
    dst = t;
  }
  // equal depths: order by id (rare; runs are short)
  if (tid == 0) sm.unsorted = 0;
  __syncthreads();
  for (int i = tid; i + 1 < n; i += TS_THREADS)
    if ((src[i] >> 32) == (src[i + 1] >> 32) && src[i + 1] < src[i]) sm.unsorted = 1;
  __syncthreads();
  if (sm.unsorted) {
    for (int i = tid; i < n; i += TS_THREADS) {
      if (i > 0 && (src[i - 1] >> 32) == (src[i] >> 32)) continue;  // not a run start
      int e = i + 1;
      while (e < n && (src[e] >> 32) == (src[i] >> 32)) ++e;
      for (int a = i + 1; a < e; ++a) {  // insertion sort of [i, e)
        const uint64_t v = src[a];
        int b = a - 1;
        while (b >= i && src[b] > v) { src[b + 1] = src[b]; --b; }
        src[b + 1] = v;
      }
    }
    __syncthreads();
  }
  return src;
}

// MSD bucket sort of a tile held in LDS -- the common case.  The top
// BITS bits of the tile's depth-bit span pick one of BS_BINS buckets
// (counted with returning LDS atomics: the returned count is the key's slot
// in its bucket), one scan turns the counts into bucket starts, one scatter
// places the keys in their buckets, and every key then finds its place in
// its bucket by counting the bucket's keys below it (the full (depth bits
// << 32 | id) key: unique, so the places are distinct and the order is the
// reference's (depth, index) order).  The ids are left in LDS in sorted
// order, as 32-bit words over the start of the key buffer.  Returns false,
// with A untouched, when the tile has more keys than the registers hold or
// some bucket more than BS_BUCKET_MAX keys (depths crowded into few
// buckets): the caller then runs the radix sort.
// (Round 5: the ranking replaced a per-thread insertion sort of each
// thread's run of buckets -- chains of dependent LDS round trips, each wave
// waiting for its longest run.  Tile sort per step 0.42 -> 0.31 ms at the
// bench scene, 0.59 -> 0.39 ms at configs[4]; profiles/r05/rank_sort/.)

template <int NT, int BITS, int BS_KPT>
__device__ __attribute__((always_inline)) bool tile_bucket_sort(const uint64_t* A, uint64_t* B, int n,
                                                                RadixSmem<NT, (1 << BITS)>& sm) {
  constexpr int BS_BINS = 1 << BITS;
  uint32_t* cnt = sm.bcnt;
  uint32_t* wsum = sm.wsum;
  // BPT bins per owning thread (the first BS_BINS / BPT threads)
  constexpr int BPT = BS_BINS >= NT ? BS_BINS / NT : 1, NW = NT / 64;
  static_assert(BS_BINS % BPT == 0, "bins per thread");
  const bool owner = threadIdx.x < BS_BINS / BPT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (n > BS_KPT * NT) return false;
  if (tid == 0) { sm.dmin = 0xFFFFFFFFu; sm.dmax = 0u; sm.skip = 0; }
  uint32_t lmin = 0xFFFFFFFFu, lmax = 0u;
  uint64_t k[BS_KPT];
#pragma unroll
  for (int j = 0; j < BS_KPT; ++j) {
    const int i = tid + j * NT;
    k[j] = i < n ? A[i] : 0ull;
    if (i < n) {
      lmin = min(lmin, (uint32_t)(k[j] >> 32));
      lmax = max(lmax, (uint32_t)(k[j] >> 32));
    }
  }
  if (owner) {
#pragma unroll
    for (int b = 0; b < BPT; ++b) cnt[tid * BPT + b] = 0u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lmin = min(lmin, (uint32_t)__shfl_xor((int)lmin, o, 64));
    lmax = max(lmax, (uint32_t)__shfl_xor((int)lmax, o, 64));
  }
  __syncthreads();
  if (lane == 0) {
    atomicMin(&sm.dmin, lmin);
    atomicMax(&sm.dmax, lmax);
  }
  __syncthreads();
  const uint32_t dmin = sm.dmin, span = sm.dmax - dmin;
  const int nbits = span ? 32 - __builtin_clz(span) : 0;
  const int shift = nbits > BITS ? nbits - BITS : 0;
  uint32_t bk[BS_KPT], rk[BS_KPT];
#pragma unroll
  for (int j = 0; j < BS_KPT; ++j) {
    const int i = tid + j * NT;
    bk[j] = (((uint32_t)(k[j] >> 32)) - dmin) >> shift;
    rk[j] = i < n ? atomicAdd(&cnt[bk[j]], 1u) : 0u;
  }
  __syncthreads();
  // thread t owns bins [t BPT, (t + 1) BPT)
  uint32_t c[BPT], run = 0;
  bool crowded = false;
#pragma unroll
  for (int b = 0; b < BPT; ++b) {
    c[b] = owner ? cnt[tid * BPT + b] : 0u;
    run += c[b];
    crowded = crowded || c[b] > (uint32_t)BS_BUCKET_MAX;
  }
  uint32_t inc = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wave] = inc;
  if (crowded) sm.skip = 1;
  __syncthreads();
  if (sm.skip) return false;  // uniform: a crowded tile goes to the radix sort
  uint32_t base = inc - run;
#pragma unroll
  for (int w = 0; w < NW; ++w) base += w < wave ? wsum[w] : 0u;
  if (owner) {
    uint32_t e = base;
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
      cnt[tid * BPT + b] = e;  // own bins only: no barrier before the next reads
      e += c[b];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < BS_KPT; ++j)
    if (tid + j * NT < n) B[cnt[bk[j]] + rk[j]] = k[j];
  __syncthreads();
  // each key's place: its bucket's start plus the bucket's keys below it
  uint32_t dst[BS_KPT];
#pragma unroll
  for (int j = 0; j < BS_KPT; ++j) {
    dst[j] = 0u;
    if (tid + j * NT < n) {
      const uint32_t b0 = cnt[bk[j]];
      const uint32_t b1 = bk[j] + 1 < (uint32_t)BS_BINS ? cnt[bk[j] + 1] : (uint32_t)n;
      uint32_t r = 0;
      for (uint32_t i = b0; i < b1; ++i) r += B[i] < k[j] ? 1u : 0u;
      dst[j] = b0 + r;
    }
  }
  __syncthreads();  // every key read: the ids overwrite the buffer's start
  uint32_t* ids = reinterpret_cast<uint32_t*>(B);
#pragma unroll
  for (int j = 0; j < BS_KPT; ++j)
    if (tid + j * NT < n) ids[dst[j]] = (uint32_t)k[j];
  __syncthreads();
  return true;
}

#ifdef GS_STATS
// stats build only: [0] tiles sorted in LDS, [1] of them by the radix fallback
__device__ unsigned long long g_sort_stats[2];
extern "C" int gs_sort_stats_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_stats), sizeof(g_sort_stats), 0, hipMemcpyDeviceToHost);
}
#endif

// One tile per workgroup of NT threads (tiles of length lo < n <= hi; the
// others exit).  Keys bucket-sorted up to `cap` (the launch's dynamic LDS):
// loaded from global memory straight into registers and scattered into one
// LDS buffer of cap keys, where they are ranked (no staging copy and
// no second buffer: twice the workgroups per CU of the two-buffer sort); a
// tile the bucket sort hands back (crowded depths, or more than KPT keys per
// thread) and one longer than cap are radix-sorted in global memory.
template <int NT, int BITS, int KPT>
__global__ __launch_bounds__(NT) void tile_sort_kernel(TileArgs a0, CamBatch cb, int cap, int lo, int hi, int ofs) {
  extern __shared__ uint64_t s_key[];  // cap keys
  __shared__ RadixSmem<NT, (1 << BITS)> sm;
  const TileArgs ta = cam_tile_args(a0, cb, blockIdx.y);
  uint64_t* __restrict__ keys = ta.keys;
  uint64_t* __restrict__ keys2 = ta.keys2;
  uint32_t* __restrict__ plist = ta.plist;
  const uint4 o = ta.order[blockIdx.x + ofs];  // longest tiles first; the launch covers [ofs, ofs + grid)
  const uint2 r = make_uint2(o.y, o.z);
  const int n = (int)(r.y - r.x);
  if (n == 0 || n <= lo || n > hi) return;
  if (n == 1) {
    if (threadIdx.x == 0) plist[r.x] = (uint32_t)keys[r.x];
    return;
  }
  if (n <= cap) {
    // keys straight from global memory into the bucket sort's registers
    // (no LDS staging copy: sort 0.457-0.462 vs 0.470-0.471 ms per bench step)
    if (tile_bucket_sort<NT, BITS, KPT>(keys + r.x, s_key, n, sm)) {
      const uint32_t* ids = reinterpret_cast<const uint32_t*>(s_key);  // sorted ids over the keys' start
      for (int i = threadIdx.x; i < n; i += NT) plist[r.x + i] = ids[i];
    } else {
#ifdef GS_STATS
      if (threadIdx.x == 0) atomicAdd(&g_sort_stats[1], 1ull);
#endif
      // the keys in global memory are untouched (the bucket sort gives up
      // before its scatter); the radix passes run there with the twin buffer
      const uint64_t* out = tile_radix_sort<uint64_t*, NT, (1 << BITS)>(keys + r.x, keys2 + r.x, n, sm);
      for (int i = threadIdx.x; i < n; i += NT) plist[r.x + i] = (uint32_t)out[i];
    }
#ifdef GS_STATS
    if (threadIdx.x == 0) atomicAdd(&g_sort_stats[0], 1ull);
#endif
  } else {  // longer than the LDS capacity of this launch: sort in global memory
    const uint64_t* out = tile_radix_sort<uint64_t*, NT, (1 << BITS)>(keys + r.x, keys2 + r.x, n, sm);
    for (int i = threadIdx.x; i < n; i += NT) plist[r.x + i] = (uint32_t)out[i];
  }
}

// ------------------------------------------------------------------ launchers

// Which count pass: the difference array (tile_count_kernel) with a
// spatially coherent walk order (its adjacent lanes' instances are
// same-tile LDS atomics: configs[4] plan 0.29 -> 0.13 ms), the per-instance
// one (tile_hist_kernel<false>) in id order, where its ~5 atomics per
// Gaussian spread over the grid cost less than the array's scans (bench plan
// 0.120 vs 0.126-0.132 ms).  Env GS_COUNT_MODE=diff / instance forces one
// (A/B).
static int count_mode() {  // 0 auto, 1 diff, 2 per instance
  static const int v = [] {
    const char* e = getenv("GS_COUNT_MODE");
    if (!e) return 0;
    if (e[0] == 'd') return 1;
    if (e[0] == 'i') return 2;
    return 0;
  }();
  return v;
}

void launch_tile_plan(const TileArgs& a, const CamBatch& cb, int prefiltered, uint32_t* hdr_host, hipStream_t s) {
  const int T = a.num_tiles;
  const size_t nd = (size_t)(a.grid_x + 1) * (a.grid_y + 1);
  const int mode = count_mode();
  const bool diff = mode == 1 || (mode == 0 && a.walk != nullptr);
  if (T <= TB_BINS && nd <= (size_t)TB_BINS + 1024 && diff) {
    hipLaunchKernelGGL(tile_count_kernel, dim3(TB_BLOCKS, cb.C), dim3(TB_THREADS), sizeof(uint32_t) * nd, s, a, cb);
  } else {
    for (int t0 = 0; t0 < T; t0 += TB_BINS) {
      const int nt = min(TB_BINS, T - t0);
      hipLaunchKernelGGL(tile_hist_kernel<false>, dim3(TB_BLOCKS, cb.C), dim3(TB_THREADS), sizeof(uint32_t) * nt, s,
                         a, cb, t0, nt);
    }
  }
  hipLaunchKernelGGL(tile_rowscan_kernel, dim3((T + RS_T - 1) / RS_T, cb.C), dim3(RS_THREADS), 0, s, a.thist, a.ttotal, T,
                     cb);
  // the host polls the headers' sentinels (publish_wait, gs_api.hip): no
  // event, no marker packet between this kernel and the render launches
  hipLaunchKernelGGL(tile_offsets_kernel, dim3(cb.C), dim3(OFF_T), 0, s, a.ttotal, T, a.bsum, a.ranges, a.meta,
                     prefiltered, cb, hdr_host);
}

void launch_tile_order(const TileArgs& a, const CamBatch& cb, const SortCover& cv, hipStream_t s) {
  hipLaunchKernelGGL(tile_order_kernel, dim3(cb.C), dim3(OFF_T), 0, s, a.ttotal, a.num_tiles, a.meta, a.ranges, a.order,
                     a.fmax, cb, cv);
}

void launch_tile_bucket(const TileArgs& a, const CamBatch& cb, hipStream_t s) {
  const int T = a.num_tiles;
  for (int t0 = 0; t0 < T; t0 += TB_BINS) {
    const int nt = min(TB_BINS, T - t0);
    // staged: the whole LDS of a CU (one workgroup) for the cursors, the run
    // offsets and as many keys as fit (10 B each: the key and its tile)
    constexpr int kLds = 160 * 1024 - 1024;  // minus the static arrays
    const int cap = ((kLds - 8 * nt) / 10) & ~3;
    if (nt <= TB_THREADS * 16 && cap >= 2048) {
      hipLaunchKernelGGL(tile_bucket_kernel, dim3(TB_BLOCKS, cb.C), dim3(TB_THREADS),
                         (size_t)10 * cap + (size_t)8 * nt, s, a, cb, t0, nt, cap);
      continue;
    }
    // more keys per workgroup than the LDS holds: every key stored where its
    // slot lands
    hipLaunchKernelGGL(tile_hist_kernel<true>, dim3(TB_BLOCKS, cb.C), dim3(TB_THREADS), sizeof(uint32_t) * nt, s,
                       a, cb, t0, nt);
  }
}

// One class launch of NT-thread workgroups over the dispatch-order positions
// [ofs, ofs + n) (SortClasses), LDS for `cap` keys, BITS / BITS_LONG bucket
// bits (lo == 0: the short class).
template <int NT, bool LONG_BITS>
static void tile_sort_class(const TileArgs& a, const CamBatch& cb, int cap, int lo, int hi, int ofs, int n,
                            hipStream_t s) {
  if (n <= 0) return;
  const dim3 grid(n, cb.C), block(NT);
  const int c = cap > 0 ? cap : 1;
  const size_t lds = sizeof(uint64_t) * (size_t)c;
  const bool wide = c > BS_KPT * NT;  // keys per thread of the bucket sort
  constexpr int B = LONG_BITS ? BS_BITS_LONG : BS_BITS;
  if (lo == 0 || !LONG_BITS) {
    if (wide) hipLaunchKernelGGL((tile_sort_kernel<NT, BS_BITS, BS_KPT_LONG>), grid, block, lds, s, a, cb, c, lo, hi, ofs);
    else hipLaunchKernelGGL((tile_sort_kernel<NT, BS_BITS, BS_KPT>), grid, block, lds, s, a, cb, c, lo, hi, ofs);
  } else {
    if (wide) hipLaunchKernelGGL((tile_sort_kernel<NT, B, BS_KPT_LONG>), grid, block, lds, s, a, cb, c, lo, hi, ofs);
    else hipLaunchKernelGGL((tile_sort_kernel<NT, B, BS_KPT>), grid, block, lds, s, a, cb, c, lo, hi, ofs);
  }
}

// Tile-length classes of the sort launches.  The LDS of a launch is sized to
// its longest tile, and the occupancy with it: the short tiles (most of them:
// ~660 keys on the bench camera) get their own launch with small LDS and many
// workgroups per CU, the long ones follow with LDS for their length (and
// global memory beyond TS_CAP_LONG).  Bench batch (27 cameras): sort 0.94 ->
// 0.80 ms per step with the small class at 1024 keys; one LDS buffer instead
// of two (twice the long-class workgroups per CU): 0.52 -> 0.47 ms, configs[4]
// 0.82 -> 0.51 ms with the LDS class up to 4096 keys; the classes past the
// short one with 512-thread workgroups at every scene: 0.46 -> 0.44 ms.
// NT: the short class's workgroup size (launch_tile_sort).
template <int NT>
static void tile_sort_launches(const TileArgs& a, const CamBatch& cb, int64_t max_len, const SortClasses& sc,
                               hipStream_t s) {
  const int big = 0x7FFFFFFF;
  // the short class sorts with BS_BITS bucket bits, the longer (512-thread)
  // classes with BS_BITS_LONG.  Measured: 1080p / 1M Gaussians sort 1.02 ->
  // 0.85 ms per 4 cameras at 11 bits; the bench scene's longer tiles, once
  // they too ran 512-thread workgroups: 0.435-0.437 -> 0.416-0.420 ms per step
  // (with 256 threads they had been faster at 10 bits).
  constexpr bool long_bits = BS_BITS_LONG != BS_BITS;
  const int T = a.num_tiles;
  if (max_len < 0) {  // unknown lengths: the LDS classes and the global-memory class
    tile_sort_class<512, long_bits>(a, cb, TS_CAP, 0, TS_CAP, 0, T, s);
    tile_sort_class<512, long_bits>(a, cb, TS_CAP_LONG, TS_CAP, big, 0, T, s);
    return;
  }
  const int64_t small = SORT_SMALL;
  const bool known = sc.valid;
  const int q1 = known ? sc.q1 : 0;
  tile_sort_class<NT, long_bits>(a, cb, (int)(max_len < small ? max_len : small), 0, (int)small, q1, T - q1, s);
  if (max_len > small)
    tile_sort_class<512, long_bits>(a, cb, (int)(max_len < TS_CAP ? max_len : TS_CAP), (int)small, TS_CAP, 0,
                                    known ? sc.p1 : T, s);
  if (max_len > TS_CAP)
    tile_sort_class<512, long_bits>(a, cb, (int)(max_len < TS_CAP_LONG ? max_len : TS_CAP_LONG), TS_CAP, big, 0,
                                    known ? sc.p2 : T, s);
}

void launch_tile_sort(const TileArgs& a, const CamBatch& cb, int64_t max_len, int64_t L, const SortClasses& sc,
                      hipStream_t s) {
  // workgroup size by the mean tile length: 256 threads keep short tiles'
  // per-pass overhead low (bench camera: ~660 keys per tile), 512 split long
  // tiles' passes over twice the waves (1080p / 1M Gaussians: ~1800)
  const int64_t mean = a.num_tiles > 0 ? L / ((int64_t)a.num_tiles * cb.C) : 0;
  if (L >= 0 && mean >= TS_WIDE_MEAN) tile_sort_launches<512>(a, cb, max_len, sc, s);
  else tile_sort_launches<256>(a, cb, max_len, sc, s);
}

}  // namespace gs
