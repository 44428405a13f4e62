// gs_binning.hip -- stable LSD radix sort of (u64 key, u32 value) pairs, the
// library's standalone sort (gs_sort_pairs).  The rasterizer's own binning no
// longer needs a global sort (gs_tiles.hip); this entry point stays as a
// tested, cub::DeviceRadixSort::SortPairs-compatible utility
// (DGR/cuda_rasterizer/rasterizer_impl.cu:306-314 semantics: stable, bits
// [0, end_bit)).  Wave64 match-by-ballot ranking keeps every pass stable.
#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

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

}  // namespace gs
