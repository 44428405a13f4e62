// gs_binning.hip -- tile binning: a stable depth sort of the Gaussians, an
// inclusive scan of their tile counts in depth order, duplicate-with-keys,
// a stable LSD radix sort of the (tile, id) instances and per-tile ranges.
// All HBM-bound integer work.
//
// Reference: DGR/cuda_rasterizer/rasterizer_impl.cu:70-138 (duplicateWithKeys,
// identifyTileRanges), :283 (cub::DeviceScan::InclusiveSum), :306-314
// (cub::DeviceRadixSort::SortPairs on bits [0, 32 + getHigherMsb(tiles))).
// The sort is our own: wave64 match-by-ballot ranking keeps every pass
// stable, so the permutation equals cub's stable LSD sort bit for bit.
#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

// ------------------------------------------------------------------ scan

constexpr int SCAN_T = 256, SCAN_I = 8;  // 2048 items per block (GeomLayout::SCAN_ITEMS)

__device__ inline uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// Block-wide exclusive scan of one value per thread (256 threads); returns the
// exclusive prefix and writes the block total to *total.
__device__ inline uint32_t block_excl_scan(uint32_t x, uint32_t* sh /*[4]*/, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(x, lane);
  if (lane == 63) sh[wave] = inc;
  __syncthreads();
  uint32_t woff = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t v = sh[w];
    if (w < wave) woff += v;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return woff + inc - x;
}

__device__ inline uint32_t scan_in(const uint32_t* __restrict__ in, const uint32_t* __restrict__ perm, int i) {
  return in[perm ? perm[i] : (uint32_t)i];
}

__global__ __launch_bounds__(SCAN_T) void scan_reduce_kernel(const uint32_t* __restrict__ in,
                                                            const uint32_t* __restrict__ perm, int P,
                                                            uint32_t* __restrict__ sums) {
  __shared__ uint32_t sh[4];
  const int base = blockIdx.x * (SCAN_T * SCAN_I) + threadIdx.x * SCAN_I;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_I; ++k) s += (base + k < P) ? scan_in(in, perm, base + k) : 0u;
  uint32_t tot;
  block_excl_scan(s, sh, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// Single block: exclusive scan of the block sums in place (any count).
__global__ __launch_bounds__(SCAN_T) void scan_sums_kernel(uint32_t* __restrict__ sums, int nb) {
  __shared__ uint32_t sh[4];
  uint32_t carry = 0;
  for (int start = 0; start < nb; start += SCAN_T) {
    const int i = start + threadIdx.x;
    const uint32_t v = i < nb ? sums[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(v, sh, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(SCAN_T) void scan_apply_kernel(const uint32_t* __restrict__ in,
                                                           const uint32_t* __restrict__ perm, int P,
                                                           const uint32_t* __restrict__ sums,
                                                           uint32_t* __restrict__ out) {
  __shared__ uint32_t sh[4];
  const int base = blockIdx.x * (SCAN_T * SCAN_I) + threadIdx.x * SCAN_I;
  uint32_t v[SCAN_I], s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_I; ++k) { v[k] = (base + k < P) ? scan_in(in, perm, base + k) : 0u; s += v[k]; }
  uint32_t tot;
  uint32_t run = block_excl_scan(s, sh, &tot) + sums[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_I; ++k) {
    run += v[k];
    if (base + k < P) out[base + k] = run;
  }
}

void launch_scan(const uint32_t* in, const uint32_t* perm, uint32_t* out, uint32_t* tmp, int P, hipStream_t s) {
  if (P <= 0) return;
  const int nb = (P + SCAN_T * SCAN_I - 1) / (SCAN_T * SCAN_I);
  hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(SCAN_T), 0, s, in, perm, P, tmp);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(SCAN_T), 0, s, tmp, nb);
  hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(SCAN_T), 0, s, in, perm, P, tmp, out);
}

// ------------------------------------------------------------------ radix sort

constexpr int RS_T = SORT_THREADS;

// Lanes of the wave holding the same 8-bit digit (valid lanes only).
__device__ inline uint64_t match_digit(uint32_t d, uint64_t valid) {
  uint64_t peers = valid;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool set = (d >> b) & 1u;
    const uint64_t m = __ballot(set);
    peers &= set ? m : ~m;
  }
  return peers;
}

template <class K>
__global__ __launch_bounds__(RS_T) void radix_hist_kernel(const K* __restrict__ keys, int64_t n,
                                                          int shift, uint32_t* __restrict__ hist,
                                                          int64_t nblk, int rounds) {
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t base = (int64_t)blockIdx.x * RS_T * rounds;
  for (int r = 0; r < rounds; ++r) {
    const int64_t i = base + r * RS_T + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = valid ? (uint32_t)(keys[i] >> shift) & 255u : 0u;
    const uint64_t peers = match_digit(d, __ballot(valid));
    const uint64_t below = peers & ((1ull << lane) - 1ull);
    if (valid && below == 0) atomicAdd(&cnt[d], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nblk + blockIdx.x] = cnt[threadIdx.x];
}

// One block per digit: exclusive scan of hist[d][0..nblk) in place, row total out.
__global__ __launch_bounds__(RS_T) void radix_rowscan_kernel(uint32_t* __restrict__ hist, int64_t nblk,
                                                             uint32_t* __restrict__ rowtot) {
  __shared__ uint32_t sh[4];
  uint32_t* row = hist + (int64_t)blockIdx.x * nblk;
  uint32_t carry = 0;
  for (int64_t start = 0; start < nblk; start += RS_T) {
    const int64_t i = start + threadIdx.x;
    const uint32_t v = i < nblk ? row[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(v, sh, &tot);
    if (i < nblk) row[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) rowtot[blockIdx.x] = carry;
}

// Stable scatter of one 8-bit digit: items are ranked in block order (rounds
// of 256, waves in order, lanes in order) with ballot-matched peer masks.
template <class K>
__global__ __launch_bounds__(RS_T) void radix_scatter_kernel(
    const K* __restrict__ kin, const uint32_t* __restrict__ vin, K* __restrict__ kout,
    uint32_t* __restrict__ vout, int64_t n, int shift, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ rowtot, int64_t nblk, int rounds) {
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t sh[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  {
    uint32_t tot;
    const uint32_t digit_off = block_excl_scan(rowtot[tid], sh, &tot);
    base[tid] = digit_off + hist[(int64_t)tid * nblk + blockIdx.x];
    wcnt[0][tid] = 0; wcnt[1][tid] = 0; wcnt[2][tid] = 0; wcnt[3][tid] = 0;
  }
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * RS_T * rounds;
  for (int r = 0; r < rounds; ++r) {
    const int64_t i = b0 + r * RS_T + tid;
    const bool valid = i < n;
    K k = 0;
    uint32_t v = 0, d = 0;
    if (valid) { k = kin[i]; v = vin[i]; d = (uint32_t)(k >> shift) & 255u; }
    const uint64_t peers = match_digit(d, __ballot(valid));
    const uint64_t below = peers & ((1ull << lane) - 1ull);
    const uint32_t rank = (uint32_t)__popcll(below);
    if (valid && below == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = base[d] + rank;
      for (int w = 0; w < wave; ++w) pos += wcnt[w][d];
      kout[pos] = k;
      vout[pos] = v;
    }
    __syncthreads();
    base[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
    wcnt[0][tid] = 0; wcnt[1][tid] = 0; wcnt[2][tid] = 0; wcnt[3][tid] = 0;
    __syncthreads();
  }
}

template <class K>
int radix_sort_impl(int64_t n, K* keys0, uint32_t* vals0, K* keys1, uint32_t* vals1, uint32_t* hist,
                    uint32_t* rowtot, int end_bit, hipStream_t s) {
  if (n <= 1) return 0;
  const int64_t nblk = sort_blocks(n);
  const int rounds = sort_rounds(n);
  int cur = 0;
  K* kb[2] = {keys0, keys1};
  uint32_t* vb[2] = {vals0, vals1};
  for (int shift = 0; shift < end_bit; shift += 8) {
    hipLaunchKernelGGL(radix_hist_kernel<K>, dim3((unsigned)nblk), dim3(RS_T), 0, s, kb[cur], n, shift, hist, nblk,
                       rounds);
    hipLaunchKernelGGL(radix_rowscan_kernel, dim3(256), dim3(RS_T), 0, s, hist, nblk, rowtot);
    hipLaunchKernelGGL(radix_scatter_kernel<K>, dim3((unsigned)nblk), dim3(RS_T), 0, s, kb[cur], vb[cur],
                       kb[cur ^ 1], vb[cur ^ 1], n, shift, hist, rowtot, nblk, rounds);
    cur ^= 1;
  }
  return cur;
}

int launch_radix_sort(int64_t n, uint64_t* keys0, uint32_t* vals0, uint64_t* keys1, uint32_t* vals1,
                      uint32_t* hist, uint32_t* rowtot, int end_bit, hipStream_t s) {
  return radix_sort_impl<uint64_t>(n, keys0, vals0, keys1, vals1, hist, rowtot, end_bit, s);
}

int launch_radix_sort32(int64_t n, uint32_t* keys0, uint32_t* vals0, uint32_t* keys1, uint32_t* vals1,
                        uint32_t* hist, uint32_t* rowtot, int end_bit, hipStream_t s) {
  return radix_sort_impl<uint32_t>(n, keys0, vals0, keys1, vals1, hist, rowtot, end_bit, s);
}

// ------------------------------------------------------------------ depth-first binning
//
// The reference sorts (tile << 32 | depth bits) pairs, stable in Gaussian
// index, over 32 + msb(tiles) bits (6 passes of the L instances at 800x800).
// Equivalent order with less work: sort the P Gaussians once by depth bits
// (stable, so ties keep index order), emit each Gaussian's instances in that
// order, then stably sort the instances by tile id alone (msb(tiles) bits: 2
// passes of 4-byte keys).  Within a tile the result is (depth bits, index)
// order -- identical to the reference's list.

__global__ __launch_bounds__(256) void depth_keys_kernel(int P, const float* __restrict__ rec,
                                                         const int* __restrict__ radii,
                                                         uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ vals) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= P) return;
  // positive depths order like their bit patterns; culled Gaussians have no
  // instances, park them at the end
  keys[g] = radii[g] > 0 ? __float_as_uint(rec[(size_t)REC * g + R_DEPTH]) : 0x7FFFFFFFu;
  vals[g] = (uint32_t)g;
}

void launch_depth_keys(int P, const float* rec, const int* radii, uint32_t* keys, uint32_t* vals,
                       hipStream_t s) {
  if (P <= 0) return;
  hipLaunchKernelGGL(depth_keys_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, rec, radii, keys, vals);
}

__global__ __launch_bounds__(256) void duplicate_sorted_kernel(int P, const uint32_t* __restrict__ order,
                                                               const float* __restrict__ rec,
                                                               const uint32_t* __restrict__ offsets,
                                                               const int* __restrict__ radii, int gx, int gy,
                                                               uint32_t* __restrict__ keys,
                                                               uint32_t* __restrict__ vals) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const uint32_t g = order[i];
  const int r = radii[g];
  if (!(r > 0)) return;
  uint32_t off = (i == 0) ? 0u : offsets[i - 1];
  const float px = rec[(size_t)REC * g + R_X], py = rec[(size_t)REC * g + R_Y];
  // getRect (auxiliary.h:46-56), same float expression order as preprocess
  int a, x0, y0, x1, y1;
  a = (int)((px - (float)r) / (float)TILE); a = a > 0 ? a : 0; x0 = a < gx ? a : gx;
  a = (int)((py - (float)r) / (float)TILE); a = a > 0 ? a : 0; y0 = a < gy ? a : gy;
  a = (int)((((px + (float)r) + (float)TILE) - 1.0f) / (float)TILE); a = a > 0 ? a : 0; x1 = a < gx ? a : gx;
  a = (int)((((py + (float)r) + (float)TILE) - 1.0f) / (float)TILE); a = a > 0 ? a : 0; y1 = a < gy ? a : gy;
  for (int y = y0; y < y1; ++y)
    for (int x = x0; x < x1; ++x) {
      keys[off] = (uint32_t)(y * gx + x);
      vals[off] = g;
      ++off;
    }
}

void launch_duplicate_sorted(int P, const uint32_t* order, const float* rec, const uint32_t* offsets,
                             const int* radii, int grid_x, int grid_y, uint32_t* keys, uint32_t* vals,
                             hipStream_t s) {
  if (P <= 0) return;
  hipLaunchKernelGGL(duplicate_sorted_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, order, rec, offsets,
                     radii, grid_x, grid_y, keys, vals);
}

// ------------------------------------------------------------------ ranges

__global__ __launch_bounds__(256) void tile_ranges_kernel(int64_t L, const uint32_t* __restrict__ keys,
                                                          uint2* __restrict__ ranges) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const uint32_t cur = keys[i];
  if (i == 0) ranges[cur].x = 0;
  else {
    const uint32_t prev = keys[i - 1];
    if (cur != prev) { ranges[prev].y = (uint32_t)i; ranges[cur].x = (uint32_t)i; }
  }
  if (i == L - 1) ranges[cur].y = (uint32_t)L;
}

void launch_tile_ranges(int64_t L, const uint32_t* keys, uint2* ranges, int num_tiles, hipStream_t s) {
  (void)hipMemsetAsync(ranges, 0, sizeof(uint2) * (size_t)num_tiles, s);
  if (L <= 0) return;
  hipLaunchKernelGGL(tile_ranges_kernel, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, L, keys, ranges);
}

}  // namespace gs
