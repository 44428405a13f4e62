// gs_render.hip -- tile-ordered alpha blending, forward and backward.
//
// Reference: DGR/cuda_rasterizer/forward.cu:274-408 (renderCUDA) and
// backward.cu:432-652 (renderCUDA backward).
//
// MI355X design:
//  * A 16x16 binning tile is four 8x8 pixel strips (STRIP_W x STRIP_H,
//    gs_common.h); one wave64 owns a strip (lane = pixel) and walks the
//    tile's depth-sorted list on its own -- no block barriers, every wave
//    exits when its own pixels are done.  Both kernels run a wave per
//    workgroup, a tile's 4 strip workgroups on one XCD (strip_of_block).
//  * The list is consumed in chunks of 64: lane j gathers the 64-B render
//    record (gs_common.h R_*) of the chunk's j-th Gaussian (prefetched one
//    chunk ahead, ids two chunks ahead), tests it against the wave's strip
//    (the Gaussian's alpha >= 1/255 extent) and parks it in a wave-private
//    LDS slot.  A ballot leaves the Gaussians the strip can see; the inner
//    loop visits only those, reading each record back with broadcast LDS
//    reads.  Culled Gaussians are exactly the ones every pixel of the strip
//    skips in the reference loop.
//  * Colour, depth, transmittance and the blend decisions are fp32 on the
//    VALU.  The dense per-Gaussian contractions go to the bf16 matrix cores
//    with every fp32 operand split into 3 bf16 pieces (split_bf16: 6 piece
//    products per product, <= 2^-26 relative, fp32 accumulation -- as exact
//    as the reference's fp32 fma / atomicAdd, tests/test_gpu_envelope.py):
//      forward   out_feat^T[ch][pix] += f[g][ch] * w[g][pix] over 16-Gaussian
//                batches (v_mfma_f32_32x32x16_bf16), F = 32 k (+ a 4-channel
//                VALU tail at F = 36);
//      backward  per 16-Gaussian batch, contractions over the strip's 64
//                pixels (v_mfma_f32_16x16x32_bf16): w = alpha T against
//                dL/dC, dL/dD, dL/dF and u = G dL/dopacity against the pixel
//                monomials {1, X, Y, X^2, XY, Y^2} (dL/dmean2D, dL/dconic).
//  * Backward per-Gaussian sums are committed with float atomics per 64-B
//    accumulation record (10 components) and per feature channel.
//  * A batch launch deals its cameras to the XCDs in groups of 8 (cam_slot),
//    so a backward tile's 4 strip workgroups share one XCD's L2.
#include "gs_common.h"
#include "gs_kernels.h"

namespace gs {

constexpr float ALPHA_MIN = 1.0f / 255.0f;
constexpr int CHUNK = 64;
// Waves per workgroup in the blend kernels: one.  Each wave owns one strip
// and never synchronises with the others.  Round 1 measured the forward
// faster with a tile (4 strips) per workgroup on one camera (its 4 waves
// gathered the same records through one CU's L1: 0.202 vs 0.223 ms); on the
// camera batches a workgroup's wave slots then idle until its longest strip
// is done (tools/batch_steps.py --stamps: 3298 of 4096 slots busy on average
// at 4 cameras, 3642 with a strip per workgroup), and with the XCD rotation
// of strip_of_block a strip per workgroup wins (4-camera step 1.58-1.60 vs
// 1.62-1.63 ms with tile workgroups, 1.65-1.66 before the rotation;
// 27 cameras within noise; profiles/r04j/).  The backward was already
// faster that way (its 12 KiB of LDS are released the moment its strip is
// done: 0.330 vs 0.342 ms).
constexpr int WPB_FWD = 1;
constexpr int WPB_BWD = 1;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float float4_t __attribute__((ext_vector_type(4)));

__device__ inline bool wave_any(bool p) { return __ballot(p) != 0ull; }
__device__ inline uint64_t clamp_u32(uint64_t v) { return v < 0xFFFFFFFFull ? v : 0xFFFFFFFFull; }

// Workgroup -> (camera, slot) of a batch launch: groups of 8 cameras one
// after the other, camera-minor inside a group -- block b of a group is
// camera g0 + b % 8, tile slot b / 8.  Workgroups are dealt to the 8 XCDs
// round-robin (b % 8), so while a group runs each XCD renders ONE camera:
// the 4 strip workgroups of a backward tile (slots 4t .. 4t+3, blocks 8 apart)
// and the neighbouring tiles of the camera share that XCD's L2, and every
// camera's longest tiles still start first.  Measured at the 27-camera batch
// (profiles/r03n_*): render_bwd HBM reads 6.3 vs 20.1 GB per launch against
// all 27 cameras interleaved (each tile's strips then sat on 4 different XCDs
// and fetched the tile's records 4 times), 5.26-5.39 vs 5.30-5.45 ms.
// Camera-major order (all of camera 0's workgroups, then camera 1's, ...)
// measured 5.55 vs 5.23 ms: every strip in flight adds into
// the same camera's accumulation records and the contended float atomics
// cost more than the locality gains.  A final group of C % 8 cameras is
// interleaved the same way without the one-camera-per-XCD property.
constexpr int CAM_GROUP = 8;  // cameras interleaved at a time (8 = one per XCD)
__device__ inline void cam_slot(int bid, int C, int per_cam, int& cam, int& slot) {
  // groups of CAM_GROUP cameras one after the other, camera-minor inside
  const int G = CAM_GROUP < C ? CAM_GROUP : C;
  const int grp = bid / (G * per_cam), r = bid - grp * G * per_cam;
  const int g0 = grp * G, gn = C - g0 < G ? C - g0 : G;  // the last group may be smaller
  cam = g0 + r % gn;
  slot = r / gn;
}
// Workgroup -> (camera, strip item) of the wave-per-workgroup blend
// kernels.  A (camera, tile) unit is 4 strip workgroups, and those 4 sit on
// one XCD (one L2 fill of the tile's records and feature rows): units are
// dealt 8 at a time, one per XCD -- the k-th group of 8 units is blocks
// 32k .. 32k+31, block 32k + 8s + x holding strip s of unit 8k + (x + r) mod 8
// on XCD x (r = k at C < 8, else 0: see below).  Units are ordered by
// cam_slot (groups of 8 cameras, camera-minor, longest tiles first).  At
// C < 8 (an 8-rank split: 3-4 cameras per rank) the groups are rotated by k:
// without it XCD x rendered only camera x mod C, and the XCDs holding the
// heavier cameras finished last (per-XCD work at 4 cameras 698-809 us of
// the 850 us backward, tools/batch_steps.py --stamps; 4-camera backward
// 0.785-0.798 vs 0.825-0.832 ms rotated, profiles/r04j/).  At C >= 8 each XCD
// renders one camera of a group at a time, unrotated: the rotation measured
// the same there but read 3.6 GB more per 27-camera step (render_fwd 4.25
// vs 2.56 GB, render_bwd 7.13 vs 5.19; profiles/r04q/).  The last U % 8
// units keep plain order.
__device__ inline void strip_of_block(int bid, int C, int num_tiles, int& cam, int& item) {
  const int U = C * num_tiles, full = U & ~7;
  int u, s;
  if (bid < 4 * full) {
    const int x = bid & 7, q = bid >> 3, k = q >> 2;
    s = q & 3;
    u = k * 8 + ((x + (C < CAM_GROUP ? k : 0)) & 7);
  } else {
    const int r = bid - 4 * full;
    u = full + (r >> 2);
    s = r & 3;
  }
  int tslot;
  cam_slot(u, C, num_tiles, cam, tslot);
  item = tslot * 4 + s;
}
template <class A>
__device__ inline int num_tiles_of(const A& a) { return a.num_tiles; }

// Dispatch record of slot `i`: {tile, range.x, range.y, 0}.  The plan's
// order puts the longest tile lists first (tile_order_kernel), so the
// long-running workgroups start early and short ones fill the end of the
// launch instead of a few long ones trailing; the record carries the tile's
// list range too, so a workgroup starts with one 16-B load instead of two
// dependent ones.
__device__ inline uint4 tile_rec(const uint4* __restrict__ order, int i) { return order[i]; }

// Work counters for kernel tuning (tools/render_stats.py); compiled only into
// the "stats" build variant (-DGS_STATS), never into the product library.
#ifdef GS_STATS
__device__ unsigned long long g_stats[32];
#define STAT(i, n)                                                               \
  do {                                                                           \
    const unsigned long long n_ = (unsigned long long)(n);                       \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_stats[i], n_);                     \
  } while (0)
#define STAT_DECL(v) unsigned long long v = 0
#define STAT_INC(v) (++v)
#define STAT_WAVE(i_max, i_hist, v)                                              \
  do {                                                                           \
    if ((threadIdx.x & 63) == 0) {                                               \
      atomicMax(&g_stats[i_max], v);                                             \
      const int b_ = v < 256 ? 0 : v < 512 ? 1 : v < 1024 ? 2 : v < 2048 ? 3 : 4; \
      atomicAdd(&g_stats[i_hist + b_], 1ull);                                    \
    }                                                                            \
  } while (0)
#else
#define STAT(i, n) ((void)0)
#define STAT_DECL(v) ((void)0)
#define STAT_INC(v) ((void)0)
#define STAT_WAVE(i_max, i_hist, v) ((void)0)
#endif

// Wave-lifetime stamps (diagnostic "stamps" build only, -DGS_STAMPS): each
// wave stores its stamps (s_memtime ticks since its start: loop start, loop
// end, last output issued, outputs drained) into a host-provided buffer, one
// 4 x u64 record per wave (forward waves first, backward waves at
// g_stamp_bwd_off); plain per-wave stores, so the stamps add no contended
// atomics.  The stamps serialise around themselves: read the shares.
#ifdef GS_STAMPS
__device__ unsigned long long* g_stamp_buf;
__device__ long long g_stamp_bwd_off;
__device__ inline unsigned long long stamp() {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP(v) const unsigned long long v = stamp()
// the chip-wide real-time clock (100 MHz), comparable across CUs and XCDs:
// each wave's absolute start and end, for the launch's waves-in-flight curve
#define RT_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
__device__ inline void stamp_store(long long wave_id, unsigned long long a, unsigned long long b,
                                   unsigned long long c, unsigned long long d, unsigned long long e = 0,
                                   unsigned long long f = 0, unsigned long long g = 0, unsigned long long h = 0) {
  if ((threadIdx.x & 63) == 0 && g_stamp_buf) {
    unsigned long long* o = g_stamp_buf + 8 * wave_id;
    o[0] = a; o[1] = b; o[2] = c; o[3] = d; o[4] = e; o[5] = f; o[6] = g; o[7] = h;
  }
}
// prologue stages of the backward, each after a full wait (GS_STAMPS_FINE):
// the stage latencies in isolation (the waits serialise the prologue)
#ifdef GS_STAMPS_FINE
#define FINE_STAMP(v) __builtin_amdgcn_s_waitcnt(0); const unsigned long long v = stamp()
#else
#define FINE_STAMP(v) const unsigned long long v = 0
#endif
extern "C" int gs_stamps_set(void* buf, long long bwd_off) {
  int e = (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &buf, sizeof(buf), 0, hipMemcpyHostToDevice);
  if (e) return e;
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_bwd_off), &bwd_off, sizeof(bwd_off), 0, hipMemcpyHostToDevice);
}
#else
#define STAMP(v) ((void)0)
#define RT_STAMP(v) ((void)0)
#endif

// 1/x as one v_rcp_f32 (1 ulp).
__device__ inline float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// Swap the upper half of `a` with the lower half of `b`:
// lo = [a_lo, b_lo], hi = [a_hi, b_hi].
__device__ inline void swap32(float a, float b, float& lo, float& hi) {
  auto r = __builtin_amdgcn_permlane32_swap(f_bits(a), f_bits(b), false, false);
  lo = bits_f(r[0]);
  hi = bits_f(r[1]);
}

// Gather the fields of list entry i's record the blend kernels use.  The index is clamped
// to the last entry of the (non-empty) range, so the loads are unconditional:
// lanes past the end re-read a valid record and are masked out by the caller.
// (A conditional update of a register struct made the compiler keep it in
// scratch memory.)
struct RecRegs {
  float4 q0, q1;
  float2 q2;  // b, depth
  float tq;   // cull threshold
  uint32_t gid;
};
__device__ inline uint32_t load_gid(const uint32_t* __restrict__ point_list, uint32_t i, uint32_t last_valid) {
  return point_list[i < last_valid ? i : last_valid];
}
__device__ inline RecRegs load_rec_gid(const float* __restrict__ rec, uint32_t gid) {
  RecRegs r;
  r.gid = gid;
  const float4* p = reinterpret_cast<const float4*>(rec + (size_t)gid * REC);
  r.q0 = p[0];  // x, y, conic a, conic b
  r.q1 = p[1];  // conic c, opacity, r, g
  r.q2 = reinterpret_cast<const float2*>(p)[4];  // b, depth (R_EX, R_EY, R_RAD unused)
  r.tq = reinterpret_cast<const float*>(p)[R_TQ];
  return r;
}
__device__ inline RecRegs load_rec(const uint32_t* __restrict__ point_list, const float* __restrict__ rec,
                                   uint32_t i, uint32_t last_valid) {
  return load_rec_gid(rec, load_gid(point_list, i, last_valid));
}

// Gaussian exponent at pixel offset (dx, dy) from the conic scaled once per
// record: h = (-a/2, -b, -c/2).  power = -1/2 (a dx^2 + c dy^2) - b dx dy
// (CR/forward.cu:353-355) in a fixed fma order shared by the forward and the
// backward kernel, so both make bit-identical alpha decisions.
// The exponent is carried in base 2: the half conic is scaled by log2(e) once
// per record, so alpha = opacity * 2^power' costs one v_exp_f32 and no
// multiply per pixel.
constexpr float HC_SCALE = 1.4426950408889634f;
__device__ inline float gauss_exp(float p) { return __builtin_amdgcn_exp2f(p); }
__device__ inline float4 half_conic(const float4& q0, const float4& q1) {
  return make_float4((-0.5f * HC_SCALE) * q0.z, -HC_SCALE * q0.w, (-0.5f * HC_SCALE) * q1.x, 0.0f);
}
__device__ inline float gauss_power(float dx, float dy, const float4& h) {
  return fmaf(h.x * dx, dx, fmaf(h.z * dy, dy, (h.y * dx) * dy));
}

// Can the Gaussian reach alpha >= 1/255 at any pixel centre of the strip
// [sx0, sx1] x [sy0, sy1]?  rect_culled (gs_common.h) on the record's mean,
// conic and threshold tq: exact up to tq's margin, so it culls the Gaussians
// whose bounding box touches the strip but whose ellipse does not.
__device__ inline bool strip_culled(const RecRegs& q, float sx0, float sx1, float sy0, float sy1) {
  return rect_culled(q.q0.x, q.q0.y, q.q0.z, q.q0.w, q.q1.x, q.tq, sx0, sx1, sy0, sy1);
}

// ------------------------------------------------------------------ bf16 split products
// fp32 contractions on the bf16 matrix cores (16x the fp32 MFMA rate).  Every
// fp32 operand is split into NSP bf16 pieces, x = p0 + p1 + p2 + r, each piece
// the bf16 rounding of what the previous ones leave (x - p0 and x - p0 - p1
// are exact in fp32), so |r| <= 2^-27 |x| for three pieces: x is carried to
// fp32's 24 bits.  A product a*b is summed as the piece products p_i q_j with
// i + j < NSP (NSP = 3: 6 products; the dropped ones are <= 2^-26 |ab|, under
// fp32's own 2^-24 rounding of a product), smallest first, into the fp32
// accumulator.  Each bf16 x bf16 product is exact in fp32.
// (Round 2 used a two-piece split: 3 products, ~2^-17 per product; DESIGN.md
// section 4.)
constexpr int NSP = 3;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
struct bsplit {
  bf16x8 p[NSP];
};

__device__ inline float4_t mfma_bf16(const bf16x8& a, const bf16x8& b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ inline f32x16 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// Two operands at a time: one v_cvt_pk_bf16_f32 rounds both (RNE, as the
// scalar conversion), and each piece is read back to fp32 from the packed
// word by a shift (low half) or a mask (high half) -- 5.5 vector
// instructions per operand for 3 pieces instead of the 7.5 the compiler
// emits for the per-element form (a one-element conversion plus a shift per
// piece and operand).  Bit-identical pieces.  The remainders are single
// v_sub_f32 (inline asm, so the compiler does not pair them into
// v_pk_add_f32, which issues beside the matrix instructions at a higher
// price and cost registers: F = 32 forward 126 VGPRs and no scratch vs 128
// and 24 B).  27-camera step (profiles/r03q_ab_split.log): render_fwd
// 3.21-3.30 vs 3.44-3.48 ms per-element, render_bwd 5.02-5.06 vs 5.24-5.35;
// the v_pk_add_f32 pairing 3.37-3.40 / 5.04-5.11.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ inline uint32_t cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
__device__ inline float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ inline float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// the remainders with one v_sub_f32 each (no packed fp32 pairing)
__device__ inline float split_sub(float a, float h) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(h));
  return r;
}
__device__ inline void split_bf16(const float (&x)[8], bsplit& s) {
  u32x4 w[NSP];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float a = x[2 * j], b = x[2 * j + 1];
#pragma unroll
    for (int i = 0; i < NSP; ++i) {
      const uint32_t u = cvt_pk_bf16(a, b);
      w[i][j] = u;
      if (i + 1 < NSP) {
        a = split_sub(a, bf16_lo(u));
        b = split_sub(b, bf16_hi(u));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NSP; ++i) s.p[i] = __builtin_bit_cast(bf16x8, w[i]);
}
// c += a * b over the split pieces (i + j < NSP), the smallest products first
template <class Acc>
__device__ inline Acc mfma_split(const bsplit& a, const bsplit& b, Acc c) {
#pragma unroll
  for (int o = NSP - 1; o >= 0; --o)
#pragma unroll
    for (int i = 0; i <= o; ++i) c = mfma_bf16(a.p[i], b.p[o - i], c);
  return c;
}
// c += a * x with x split here, one piece at a time (fewer live registers
// than mfma_split: x's pieces never coexist); largest products first
template <class Acc>
__device__ inline Acc mfma_split_x(const bsplit& a, const float (&x)[8], Acc c) {
  float r[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = x[e];
#pragma unroll
  for (int j = 0; j < NSP; ++j) {
    u32x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t u = cvt_pk_bf16(r[2 * e], r[2 * e + 1]);
      w[e] = u;
      if (j + 1 < NSP) {
        r[2 * e] = split_sub(r[2 * e], bf16_lo(u));
        r[2 * e + 1] = split_sub(r[2 * e + 1], bf16_hi(u));
      }
    }
    const bf16x8 b = __builtin_bit_cast(bf16x8, w);
#pragma unroll
    for (int i = 0; i + j < NSP; ++i) c = mfma_bf16(a.p[i], b, c);
  }
  return c;
}
// c += a * b for an operand a that is exact in bf16 (b split)
template <class Acc>
__device__ inline Acc mfma_exact_split(const bf16x8& a, const bsplit& b, Acc c) {
#pragma unroll
  for (int i = NSP - 1; i >= 0; --i) c = mfma_bf16(a, b.p[i], c);
  return c;
}

// ------------------------------------------------------------------ fp16 split products
// The same contraction on the fp16 matrix cores (the bf16 rate) for operands
// whose range is known: fp16 keeps 11 significant bits, so TWO pieces carry
// an operand to 22-24 bits (x = h0 + h1 + r, h0 the fp16 rounding of x, h1
// of x - h0; |r| <= 2^-24 |x| while x - h0 is a normal fp16) and a product
// a*b is summed as h0 g0 + h0 g1 + h1 g0 (3 matrix instructions instead of
// the bf16 split's 6; the dropped h1 g1 and remainders are ~3 * 2^-24 |ab|,
// fp32's own rounding of a product), each piece product exact in fp32.
// Range: an operand is scaled by a power of two into [2^-3, 2^16) wherever
// its size allows (exact, undone on the fp32 sums), so h0 stays normal and
// h1 exact; fp16 subnormals pass the conversions and the matrix inputs
// unflushed (MODE.denorm, hipcc's default), so smaller values lose relative
// precision only below 2^-24 of the operand's scale in absolute terms.
// Per 8 values: 4 v_cvt_pk_f16_f32 + 8 v_fma_mix_f32 (the remainder x - h0
// read straight from the packed half, negated, in one instruction) + 4
// v_cvt_pk_f16_f32 = 2 vector instructions per value (the 3-piece bf16
// split: 5.5).
constexpr int NSH = 2;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
struct hsplit {
  f16x8 p[NSH];
};
__device__ inline float4_t mfma_f16(const f16x8& a, const f16x8& b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ inline uint32_t cvt_pk_f16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, f16x2));
}
// a - (the fp16 in the low / high half of u), exact, one v_fma_mix_f32
__device__ inline float f16_rem_lo(float a, uint32_t u) {
  float r;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(u), "v"(a));
  return r;
}
__device__ inline float f16_rem_hi(float a, uint32_t u) {
  float r;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(u), "v"(a));
  return r;
}
__device__ inline void split_f16(const float (&x)[8], hsplit& s) {
  u32x4 w0, w1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t u = cvt_pk_f16(x[2 * j], x[2 * j + 1]);
    w0[j] = u;
    w1[j] = cvt_pk_f16(f16_rem_lo(x[2 * j], u), f16_rem_hi(x[2 * j + 1], u));
  }
  s.p[0] = __builtin_bit_cast(f16x8, w0);
  s.p[1] = __builtin_bit_cast(f16x8, w1);
}
// c += a * b over the pieces (h1 g0 and h0 g1 first, then h0 g0)
__device__ inline float4_t mfma_hsplit(const hsplit& a, const hsplit& b, float4_t c) {
  c = mfma_f16(a.p[1], b.p[0], c);
  c = mfma_f16(a.p[0], b.p[1], c);
  return mfma_f16(a.p[0], b.p[0], c);
}
__device__ inline f32x16 mfma_f16(const f16x8& a, const f16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// c += a * x with x split here (its two pieces made one after the other):
// h1 g0 first, then h0 g1, h0 g0
__device__ inline f32x16 mfma_hsplit_x(const hsplit& a, const float (&x)[8], f32x16 c) {
  u32x4 w0, w1;
#pragma unroll
  for (int j = 0; j < 4; ++j) w0[j] = cvt_pk_f16(x[2 * j], x[2 * j + 1]);
  const f16x8 b0 = __builtin_bit_cast(f16x8, w0);
  c = mfma_f16(a.p[1], b0, c);
#pragma unroll
  for (int j = 0; j < 4; ++j) w1[j] = cvt_pk_f16(f16_rem_lo(x[2 * j], w0[j]), f16_rem_hi(x[2 * j + 1], w0[j]));
  c = mfma_f16(a.p[0], __builtin_bit_cast(f16x8, w1), c);
  return mfma_f16(a.p[0], b0, c);
}
// The power of two that scales a row whose largest magnitude is m into
// [2^14, 2^15) (0 for an all-zero row; bounded so that its inverse stays a
// normal fp32 together with the weights' scale).
__device__ inline int row_scale_exp(float m) {
  if (!(m > 0.f)) return 0;
  const int e = __builtin_amdgcn_frexp_expf(m);  // m = f 2^e, f in [0.5, 1)
  const int s = 15 - e;
  return s < -100 ? -100 : (s > 100 ? 100 : s);
}

// ------------------------------------------------------------------ forward

// Waves per SIMD the forward asks the register allocator for: 4 for the
// matrix-core feature widths (the two-survivor loop would otherwise settle
// at 130 registers = 3 waves), else the compiler's choice.
template <int F>
constexpr int fwd_waves_per_simd() {
  return F == 32 ? 4 : F == 36 ? 3 : 1;  // F = 36: 0.188 vs 0.205 ms per camera at 4 (spills)
}
// This workgroup's share of a region the forward zeroes for the backward
// (gs_gaussians.zero_fill): 16-B stores issued as the strip's last memory
// operations, so nothing the wave waits for queues behind them.
__device__ inline void zero_share(float4* __restrict__ z, int64_t n) {
  if (!z || n <= 0) return;
  const int64_t per = (n + (int64_t)gridDim.x - 1) / (int64_t)gridDim.x;
  const int64_t z0 = (int64_t)blockIdx.x * per, z1 = z0 + per < n ? z0 + per : n;
  for (int64_t i = z0 + (threadIdx.x & 63); i < z1; i += 64) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int F, int COMPAT>
__global__ __launch_bounds__(64 * WPB_FWD) __attribute__((amdgpu_waves_per_eu(fwd_waves_per_simd<F>(), 8))) void render_fwd_kernel(
    RenderArgs a0, CamBatch cb) {
  // camera and strip of this workgroup (strip_of_block)
  STAMP(ts0);
  RT_STAMP(rt0);
  static_assert(WPB_FWD == 1, "strip_of_block maps one strip per workgroup");
  int cam, item0;
  strip_of_block(blockIdx.x, cb.C, num_tiles_of(a0), cam, item0);
  const RenderArgs ca = cam_render_args(a0, cb, cam);
  const int W = ca.W, H = ca.H, grid_x = ca.grid_x;
  const uint4* __restrict__ order = ca.order;
  const uint32_t* __restrict__ point_list = ca.point_list;
  const float* __restrict__ rec = ca.rec;
  const float* __restrict__ feats = ca.feats;
  const float* __restrict__ bg = ca.bg;
  float* __restrict__ out_color = ca.out_color;
  float* __restrict__ out_feature = ca.out_feature;
  float* __restrict__ out_depth = ca.out_depth;
  float* __restrict__ out_alpha = ca.out_alpha;
  uint32_t* __restrict__ n_contrib = ca.n_contrib;
  // Features: 4 / 8 / 16 channels on the VALU (fma with the Gaussian's row
  // in SGPRs, requested at the top of the iteration); 32-channel blocks on
  // the matrix cores: a wave parks the weights w = alpha T of 16 blending
  // Gaussians in LDS and contracts the batch as out_feature^T[ch][pix] +=
  // sum_g feat[g][ch] w[g][pix] (v_mfma_f32_32x32x16_bf16, K = Gaussians,
  // 3-piece bf16 split operands: 6 matrix instructions per 16 Gaussians and
  // 32 channels, fp32-equivalent, instead of 8 fp32 v_mfma_f32_32x32x2_f32 at
  // 64 cycles each).  F = 36 (32 + a 4-channel tail, e.g. the fused colour +
  // seg pass's 3 seg channels next to 32 user channels) runs the tail on the
  // VALU next to the one matrix block instead of padding to 64.
  constexpr bool MF = (F >= 32);
  constexpr int FB = MF ? F / 32 : 1;        // 32-channel blocks
  constexpr int FT = MF ? F - 32 * FB : 0;   // VALU tail of a matrix-core width
  static_assert(FT == 0 || FT == 4, "matrix-core feature widths: 32 k or 32 k + 4");
  constexpr int NSF = (!MF && F > 0) ? F : (FT > 0 ? FT : 1);
  constexpr int WBF = 16;                    // Gaussians per matrix batch
  // per record: (x, y, -a/2, -b) (-c/2, opacity, r, g) (b, depth, -, -)
  __shared__ float4 s_rec[WPB_FWD][CHUNK][3];
  // batch weights [slot][pixel] (row pad 4: conflict-free writes and reads)
  __shared__ float s_fw[WPB_FWD][MF ? WBF + 1 : 1][68];  // +1: a pair may overfill by one
  __shared__ __attribute__((aligned(16))) uint32_t s_gid[WPB_FWD][MF ? WBF + 4 : 1];  // batch ids (+ the overfill)

  // strip item = tile slot * 4 + strip (the tile slot in dispatch order)
  // lw: LDS slot of the wave (a constant 0 at one wave per workgroup)
  const int lane = threadIdx.x & 63, lw = WPB_FWD == 1 ? 0 : (int)(threadIdx.x >> 6);
  const int item = item0 + lw;
  const uint4 trec = tile_rec(order, item >> 2);
  const int tile = (int)trec.x, wave = item & 3;
  const int tx = tile % grid_x, ty = tile / grid_x;
  const int qx0 = strip_x0(tx, wave), qy0 = strip_y0(ty, wave);  // lane = strip pixel (lane % STRIP_W, lane / STRIP_W)
  const int px = qx0 + lane % STRIP_W, py = qy0 + lane / STRIP_W;
  const bool inside = px < W && py < H;
  const float pfx = (float)px, pfy = (float)py;
  const float sx0 = (float)qx0, sx1 = sx0 + (float)(STRIP_W - 1);
  const float sy0 = (float)qy0, sy1 = sy0 + (float)(STRIP_H - 1);
  const uint2 range = make_uint2(trec.y, trec.z);
  if (!in_window(cb, cam, tx, ty)) {
    // outside the camera's tile window (image sharding, gs_camera tile_*):
    // zeros, and an empty walk for the backward
    if (lane == 0) ca.smax[item] = 0u;
    if (inside) {
      const size_t HW = (size_t)H * W, pix = (size_t)py * W + px;
      n_contrib[pix] = 0u;
      out_color[pix] = 0.f;
      out_color[HW + pix] = 0.f;
      out_color[2 * HW + pix] = 0.f;
      out_depth[pix] = 0.f;
      if (out_alpha) out_alpha[pix] = 0.f;
      for (int c = 0; c < F; ++c) out_feature[(size_t)c * HW + pix] = 0.f;
    }
    zero_share(a0.zero, a0.zero_n);
    return;
  }

  float T = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f, Dp = 0.f;
  float SF[NSF];
#pragma unroll
  for (int c = 0; c < NSF; ++c) SF[c] = 0.f;
  // acc[2 fb + blk]: out_feature^T block (channels 32 fb .., strip pixels 32 blk ..)
  f32x16 acc[2 * FB];
#pragma unroll
  for (int i = 0; i < 2 * FB; ++i) acc[i] = f32x16{0};
  uint32_t last = 0;
  // lane still blending (the reference's !done); an integer, not a bool, so
  // that it lives in a VGPR instead of exec-mask bookkeeping across the loops
  uint32_t live = inside ? 1u : 0u;
  int nb = 0;          // batch fill

  // Contract the batch's nb Gaussians.  A[ch][k] = feat[gid_k][32 fb + ch]
  // (lane l: channel l&31, k = 8(l>>5) + j), B[k][pix] = w[k][pix] (lane l:
  // pixel (l&31) + 32 blk); slots k >= nb are zeroed on both sides.
  // Park record j's Gaussian as batch slot k: the lane holding the chunk's
  // j-th id stores it to the batch's id row, which the flush reads back with
  // two broadcast 16-B reads per lane (instead of a readlane and a lane
  // select per park and 8 lane shuffles per flush).  (Copying the feature
  // rows to LDS by LDS-DMA at park time was measured slower: DESIGN.md
  // section 4.)
  if (MF && lane < WBF + 4) s_gid[lw][lane] = 0u;  // stale slots gather row 0
  auto park_row = [&](uint32_t chunk_gid, int j, int k) {
    if (lane == j) s_gid[lw][k] = chunk_gid;
  };
  // feature rows addressed by unsigned 32-bit byte offsets through a buffer
  // resource over the P x F table (the host refuses tables over 4 GiB): 64-bit
  // pointer arithmetic per row cost 3 more vector instructions per row and
  // spilled registers at the 128-VGPR cap
  const uint64_t fbytes = (uint64_t)ca.P * F * 4u;
  // fp16 feature contraction: the weights w = alpha T in [3.9e-7, 0.99]
  // (T >= 1e-4, alpha >= 1/255) enter scaled by 2^15, the features by their
  // channel's power of two (fmax); acc holds both scales until the stores
  constexpr int FW_EXP = 15;
  constexpr float FW_SCALE = (float)(1 << FW_EXP);
  const uint32_t* __restrict__ fmax = ca.fmax;
  const auto frsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(feats), (short)0,
                                                       (int)(uint32_t)clamp_u32(fbytes), 0x00020000);
  auto flush = [&](int n) {
    // an opaque copy of the lane index keeps the compiler from hoisting the
    // flush's address arithmetic into loop-long registers
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int h = (ln >> 5) & 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int fb = 0; fb < FB; ++fb) {
      hsplit A;
      {
        // the channel's scale (its largest |feature| into [2^14, 2^15))
        const float fs = ldexpf(1.f, row_scale_exp(__uint_as_float(fmax[fb * 32 + (ln & 31)])));
        float fa[8];
        // 32-bit row offsets through a buffer resource: one address
        // instruction per row instead of 64-bit pointer arithmetic
        const uint4 ga = *reinterpret_cast<const uint4*>(&s_gid[lw][8 * h]);
        const uint4 gb = *reinterpret_cast<const uint4*>(&s_gid[lw][8 * h + 4]);
        const uint32_t gk[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 8 * h + j;
          const uint32_t g = gk[j];
          const uint32_t off = (g * (uint32_t)F + (uint32_t)(fb * 32 + (ln & 31))) * 4u;
          const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(frsrc, (int)off, 0, 0));
          fa[j] = k < n ? v * fs : 0.f;
        }
        split_f16(fa, A);
      }
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 8 * h + j;
          x[j] = k < n ? s_fw[lw][k][(ln & 31) + 32 * blk] * FW_SCALE : 0.f;
        }
        acc[2 * fb + blk] = mfma_hsplit_x(A, x, acc[2 * fb + blk]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  const uint32_t lastv = range.y > range.x ? range.y - 1 : range.x;
  // Records are prefetched one chunk ahead and their list ids two chunks
  // ahead, so the id -> record dependent load never waits inside a chunk.
  RecRegs q;
  uint32_t gnext = 0;
  if (range.y > range.x) {
    q = load_rec(point_list, rec, range.x + lane, lastv);
    gnext = load_gid(point_list, range.x + CHUNK + lane, lastv);
  }
  STAT_DECL(st_it);
  STAT(6, 1);
  STAT(7, range.y - range.x);
#ifdef GS_STAMPS
  const unsigned long long ts1 = stamp();
#endif
  if (!wave_any(live != 0u)) goto blend_done;
  for (uint32_t c0 = range.x; c0 < range.y; c0 += CHUNK) {
    const bool keep = (c0 + lane < range.y) && !strip_culled(q, sx0, sx1, sy0, sy1);
    {
      const float4 h = half_conic(q.q0, q.q1);
      s_rec[lw][lane][0] = make_float4(q.q0.x, q.q0.y, h.x, h.y);
      s_rec[lw][lane][1] = make_float4(h.z, q.q1.y, q.q1.z, q.q1.w);
      s_rec[lw][lane][2] = make_float4(q.q2.x, q.q2.y, 0.f, 0.f);
    }
    const uint32_t chunk_gid = q.gid;  // lane j: id of the chunk's j-th record
    uint64_t mask = __ballot(keep);
    const uint32_t lbase = c0 - range.x + 1;
    STAT(0, 1);
    STAT(1, range.y - c0 < CHUNK ? range.y - c0 : CHUNK);
    STAT(2, __builtin_popcountll(mask));
    q = load_rec_gid(rec, gnext);                                 // next chunk (clamped)
    gnext = load_gid(point_list, c0 + 2 * CHUNK + lane, lastv);    // the one after
    if constexpr (F == 0 || MF) {
      // Two survivors per iteration: their exponents are evaluated side by
      // side (independent work for the issue slots), then blended in order.
      // A missing second survivor gets power = +1 (never blends).
      auto blend_step = [&](int j, const float4& r1, const float4& r2, float power, float alpha,
                            const float4& ft) {
        const float test_T = T * (1 - alpha);
        const bool cand = live != 0u && !(power > 0.0f) && !(alpha < ALPHA_MIN);
        const bool fin = cand && test_T < 0.0001f;  // saturated: not blended, lane done
        const bool blend = cand && !fin;
        live = fin ? 0u : live;
        const float w = blend ? alpha * T : 0.0f;
        C0 = fmaf(r1.z, w, C0);
        C1 = fmaf(r1.w, w, C1);
        C2 = fmaf(r2.x, w, C2);
        Dp = fmaf(r2.y, w, Dp);
        if constexpr (FT > 0) {
          SF[0] = fmaf(ft.x, w, SF[0]);
          SF[1] = fmaf(ft.y, w, SF[1]);
          SF[2] = fmaf(ft.z, w, SF[2]);
          SF[3] = fmaf(ft.w, w, SF[3]);
        }
        T = blend ? test_T : T;
        last = blend ? lbase + (uint32_t)j : last;
        if constexpr (MF) {
          if (wave_any(blend)) {  // park it; the batch is flushed after the pair
            s_fw[lw][nb][lane] = w;  // 0 on non-blending lanes
            park_row(chunk_gid, j, nb);
            ++nb;
          }
        }
      };
      while (mask) {
        const int ja = __builtin_ctzll(mask);
        mask &= mask - 1;
        const bool two = mask != 0;
        const int jb = two ? __builtin_ctzll(mask) : ja;
        if (two) mask &= mask - 1;
        STAT(3, two ? 2 : 1);
        // the survivors' tail feature rows (scalar loads), requested before
        // their alphas are computed
        float4 fta = make_float4(0.f, 0.f, 0.f, 0.f), ftb = fta;
        if constexpr (FT > 0) {
          const uint32_t ga = __builtin_amdgcn_readlane(chunk_gid, ja);
          const uint32_t gb = __builtin_amdgcn_readlane(chunk_gid, jb < CHUNK ? jb : ja);
          fta = *reinterpret_cast<const float4*>(feats + (size_t)ga * F + 32 * FB);
          ftb = *reinterpret_cast<const float4*>(feats + (size_t)gb * F + 32 * FB);
        }
        const float4 a0 = s_rec[lw][ja][0], a1 = s_rec[lw][ja][1], a2 = s_rec[lw][ja][2];
        const float4 b0 = s_rec[lw][jb][0], b1 = s_rec[lw][jb][1], b2 = s_rec[lw][jb][2];
        const float pa = gauss_power(a0.x - pfx, a0.y - pfy, make_float4(a0.z, a0.w, a1.x, 0.f));
        float pb = gauss_power(b0.x - pfx, b0.y - pfy, make_float4(b0.z, b0.w, b1.x, 0.f));
        pb = two ? pb : 1.0f;
        const float ala = fminf(0.99f, a1.y * gauss_exp(pa));
        const float alb = fminf(0.99f, b1.y * gauss_exp(pb));
        blend_step(ja, a1, a2, pa, ala, fta);
        blend_step(jb, b1, b2, pb, alb, ftb);
        if constexpr (MF) {
          if (nb >= WBF) {  // 16 or 17 parked: contract 16, carry the 17th to slot 0
            flush(WBF);
            if (nb > WBF) {
              s_fw[lw][0][lane] = s_fw[lw][WBF][lane];
              if (lane == 0) s_gid[lw][0] = s_gid[lw][WBF];
            }
            nb -= WBF;
          }
        }
        if (!wave_any(live != 0u)) goto blend_done;
      }
    } else {
    while (mask) {
      const int j = __builtin_ctzll(mask);
      mask &= ~(1ull << j);
      // the survivor's feature row, requested before its alpha is computed so
      // the scalar loads overlap that work
      float fcur[NSF];
      if constexpr ((!MF && F > 0) || FT > 0) {
        const uint32_t g = __builtin_amdgcn_readlane(chunk_gid, j);
#pragma unroll
        for (int c = 0; c < NSF; ++c) fcur[c] = feats[(size_t)g * F + 32 * FB * (MF ? 1 : 0) + c];
      }
      STAT(3, 1);
      STAT_INC(st_it);
      const float4 r0 = s_rec[lw][j][0];
      const float4 r1 = s_rec[lw][j][1];
      const float4 r2 = s_rec[lw][j][2];
      const float dx = r0.x - pfx, dy = r0.y - pfy;
      const float power = gauss_power(dx, dy, make_float4(r0.z, r0.w, r1.x, 0.f));
      const float alpha = fminf(0.99f, r1.y * gauss_exp(power));
      const float test_T = T * (1 - alpha);
      // Branch-free blend (CR/forward.cu:350-380): non-blending lanes add
      // zero-weighted terms, and T / last / live are selected, so the loop
      // body has no exec-mask juggling.
      const bool cand = live != 0u && !(power > 0.0f) && !(alpha < ALPHA_MIN);
      const bool fin = cand && test_T < 0.0001f;  // saturated: not blended, lane done
      const bool blend = cand && !fin;
      live = fin ? 0u : live;
      const float w = blend ? alpha * T : 0.0f;
      C0 = fmaf(r1.z, w, C0);
      C1 = fmaf(r1.w, w, C1);
      C2 = fmaf(r2.x, w, C2);
      Dp = fmaf(r2.y, w, Dp);
      T = blend ? test_T : T;
      last = blend ? lbase + (uint32_t)j : last;
      STAT(4, wave_any(blend));
      STAT(5, __builtin_popcountll(__ballot(blend)));
      STAT(18, wave_any(blend) && ((__ballot(blend) & 0xFFFFFFFFull) == 0 || (__ballot(blend) >> 32) == 0));
      if constexpr ((!MF && F > 0) || FT > 0) {
        // keep the row loads above the blend decision (issued early, used late)
#pragma unroll
        for (int c = 0; c < NSF; ++c) asm volatile("" ::"s"(fcur[c]));
      }
      if constexpr (FT > 0) {
#pragma unroll
        for (int c = 0; c < FT; ++c) SF[c] = fmaf(fcur[c], w, SF[c]);
      }
      if (F > 0 && wave_any(blend)) {
        if constexpr (MF) {
          s_fw[lw][nb][lane] = w;  // 0 on non-blending lanes
          park_row(chunk_gid, j, nb);
          if (++nb == WBF) {
            flush(WBF);
            nb = 0;
          }
        } else {
#pragma unroll
          for (int c = 0; c < NSF; ++c) SF[c] = fmaf(fcur[c], w, SF[c]);
        }
      }
      if (!wave_any(live != 0u)) goto blend_done;
    }
    }
  }
blend_done:
  STAT_WAVE(16, 20, st_it);
  STAMP(ts2);
  {
    // the strip's longest pixel walk: where the backward starts its walk
    const uint32_t wl = wave_max_u(inside ? last : 0u);
    if (lane == 0) ca.smax[item] = wl;
  }
  if constexpr (MF) {
    if (nb > 0) flush(nb);
  }
  const size_t HW = (size_t)H * W;
  if (inside) {
    const size_t pix = (size_t)py * W + px;
    n_contrib[pix] = last;
    out_color[pix] = C0 + T * bg[0];
    out_color[HW + pix] = C1 + T * bg[1];
    out_color[2 * HW + pix] = C2 + T * bg[2];
    out_depth[pix] = Dp;
    if constexpr (!MF && F > 0) {
#pragma unroll
      for (int c = 0; c < F; ++c) {
        // Q4: the reference adds bg[ch] (an out-of-bounds read for ch >= 3;
        // zero here); the fixed mode adds no background to features.
        const float b = (COMPAT == COMPAT_REFERENCE && c < 3) ? bg[c] : 0.0f;
        out_feature[c * HW + pix] = SF[c] + T * b;
      }
    }
    if constexpr (FT > 0) {
      // tail channels 32 FB .. (>= 3: no background in either mode)
#pragma unroll
      for (int c = 0; c < FT; ++c) out_feature[(size_t)(32 * FB + c) * HW + pix] = SF[c];
    }
    // Q1: the reference never writes out_alpha (torch::full -> 0 stays 0);
    // we store that 0 here instead of a separate fill launch.
    if (COMPAT != COMPAT_REFERENCE) out_alpha[pix] = 1.0f - T;
    else if (out_alpha) out_alpha[pix] = 0.0f;
  }
  if constexpr (MF) {
    // acc[2*fb + blk] holds out_feat^T: lane l, register r ->
    // channel fb*32 + (r&3) + 8(r>>2) + 4(l>>5), strip pixel (l&31) + 32 blk;
    // undo the channel's and the weights' scales (exact powers of two)
#pragma unroll
    for (int fb = 0; fb < FB; ++fb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ch = fb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float un = ldexpf(1.f, -row_scale_exp(__uint_as_float(fmax[ch])) - FW_EXP);
        acc[2 * fb][r] *= un;
        acc[2 * fb + 1][r] *= un;
      }
    float t_lo, t_hi;
    swap32(T, T, t_lo, t_hi);  // T of strip pixel (l&31) and (l&31)+32
    // Buffer stores: one per-lane byte offset (pixel + the lane's channel
    // quarter) and the register's channel in the scalar offset, so the 16 x FB
    // stores per pixel cost no address arithmetic on the vector ALUs.
    const bool small = (uint64_t)F * HW * 4u < 0x7FFFFFFFull;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out_feature, (short)0,
                                                        small ? (int)((uint64_t)F * HW * 4u) : 0, 0x00020000);
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      const int p = (lane & 31) + 32 * blk;
      const int qx = qx0 + p % STRIP_W, qy = qy0 + p / STRIP_W;
      if (qx < W && qy < H) {
        const size_t pix = (size_t)qy * W + qx;
        const float Tp = blk ? t_hi : t_lo;
        if (small) {
          const uint32_t voff = (uint32_t)(pix + (size_t)(4 * (lane >> 5)) * HW) * 4u;
#pragma unroll
          for (int fb = 0; fb < FB; ++fb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int chs = fb * 32 + (r & 3) + 8 * (r >> 2);  // channel minus the lane's quarter
              const int ch = chs + 4 * (lane >> 5);
              const float b = (COMPAT == COMPAT_REFERENCE && ch < 3) ? bg[ch < 3 ? ch : 0] : 0.0f;
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[2 * fb + blk][r] + Tp * b), rsrc, (int)voff,
                                                    (int)((uint32_t)chs * (uint32_t)HW * 4u), 0);
            }
          continue;
        }
        // images over 2 GiB of features: 64-bit addresses
#pragma unroll
        for (int fb = 0; fb < FB; ++fb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ch = fb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const float b = (COMPAT == COMPAT_REFERENCE && ch < 3) ? bg[ch < 3 ? ch : 0] : 0.0f;
            out_feature[ch * HW + pix] = acc[2 * fb + blk][r] + Tp * b;
          }
      }
    }
  }
  zero_share(a0.zero, a0.zero_n);
#ifdef GS_STAMPS
  STAMP(ts3);
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(ts4);
  RT_STAMP(rt1);
  stamp_store((long long)blockIdx.x * WPB_FWD + lw, ts1 - ts0, ts2 - ts0, ts3 - ts0, ts4 - ts0, 0, 0, rt0, rt1);
#endif
}

// ------------------------------------------------------------------ backward

// s_w / s_u element (row r, column c) of a 64-float row: the 16-B group index
// XOR-swizzled by the row
__device__ inline int sw_idx(int r, int c) { return r * 64 + ((((c >> 2) ^ r) & 15) << 2) + (c & 3); }
//
// Every per-Gaussian sum of the backward is a contraction over the wave's 64
// pixels of one of two per-(Gaussian, pixel) weights with per-pixel
// constants:
//   w = alpha T            (dL/dcolour, dL/ddepth, dL/dfeature):
//       sum_pix w * {dL/dC_r, dL/dC_g, dL/dC_b, dL/dD, dL/dF_ch}
//   u = G dL/dopacity_pix  (dL/dopacity, dL/dmean2D, dL/dconic):
//       sum_pix u * {1, dx, dy, dx^2, dx dy, dy^2}  with dx = mean_x - px;
//       dx = m' - X/2 for the strip-centred pixel coordinate X = 2(px - cx)
//       (an odd integer), so these follow from the per-pixel monomials
//       {1, X, Y, X^2, XY, Y^2} (exact in bf16) and the Gaussian's m'.
// A wave parks w and u of 16 contributing Gaussians in LDS and contracts the
// batch on the matrix cores (v_mfma_f32_16x16x32_bf16, K = pixels) instead of
// reducing each Gaussian's sums over the wave with cross-lane VALU work.
// Operands are split into three bf16 (split_bf16: 6 piece products; the
// monomials are exact in bf16, so their products take three).
// Waves per SIMD the backward asks the register allocator for: 3 (<= 168
// VGPRs) where that fits, measured 0.336 vs 0.388 ms at 2 waves on the bench
// camera (F = 32); with the 3-piece split that needs the colour operand in
// LDS and one k-step's split weights live at a time (flush), else 27-camera
// render_bwd 6.0 ms at 2 waves vs 5.45 at 3; the widest instantiations keep 2.
template <int F, int COMPAT>
constexpr int bwd_waves_per_simd() {
  return (F < 32 || (F == 32 && COMPAT == COMPAT_REFERENCE)) ? 3 : 2;
}
template <int F, int COMPAT>
__global__ __launch_bounds__(64 * WPB_BWD) __attribute__((amdgpu_waves_per_eu(bwd_waves_per_simd<F, COMPAT>(), 8))) void render_bwd_kernel(
    RenderBwdArgs a0, CamBatch cb) {
  // camera and strip of this workgroup (strip_of_block)
  STAMP(ts0);
  RT_STAMP(rt0);
  static_assert(WPB_BWD == 1, "strip_of_block maps one strip per workgroup");
  int cam, bslot;
  strip_of_block(blockIdx.x, cb.C, num_tiles_of(a0), cam, bslot);
  const RenderBwdArgs ca = cam_render_bwd_args(a0, cb, cam);
  const int W = ca.W, H = ca.H, grid_x = ca.grid_x;
  const uint4* __restrict__ order = ca.order;
  const uint32_t* __restrict__ point_list = ca.point_list;
  const float* __restrict__ rec = ca.rec;
  const float* __restrict__ feats = ca.feats;
  const float* __restrict__ bg = ca.bg;
  const float* __restrict__ alphas = ca.alphas;
  const uint32_t* __restrict__ n_contrib = ca.n_contrib;
  const float* __restrict__ dL_dpix = ca.dL_dpix;
  const float* __restrict__ dL_dfeat = ca.dL_dfeat;
  const float* __restrict__ dL_ddepth = ca.dL_ddepth;
  const float* __restrict__ dL_dalpha = ca.dL_dalpha;
  float* __restrict__ acc = ca.acc;
  float* __restrict__ dsem = ca.dsem;
  constexpr int WB = 16;                      // Gaussians per matrix batch
  constexpr int CB = F >= 16 ? F / 16 : 0;    // 16-channel feature blocks with their own accumulators
  constexpr int CB1 = CB > 0 ? CB : 1;
  // feature channels 16 CB .. F as rows 4.. of the colour block (F = 4, 8,
  // and the 4-channel tail of F = 36)
  constexpr int FW = F - 16 * CB;
  static_assert(FW <= 12, "the colour block holds at most 12 feature rows");
  constexpr int NCOMP = A_FEAT + FW;  // committed components per Gaussian and batch
  // row stride of the feature gradients the atomics add into: F, or a
  // 64-B multiple when the 16-channel blocks would straddle segments
  // (F = 36: the host hands a 48-wide scratch, feature_grad_rows copies out)
  constexpr int FS = feature_grad_stride(F);
  constexpr bool FIXED_FEAT = (COMPAT != COMPAT_REFERENCE) && F > 0;
  // per record: (x, y, -a/2, -b) (-c/2, opacity, r, g) (b, depth, -, -): one
  // 48-B row, so a survivor's three reads share one address register
  __shared__ float4 s_rec[WPB_BWD][CHUNK][3];
  // Colour block operand rows 0..3 (dL/dC_r,g,b, dL/dD) and the FW <= 4
  // feature rows after them, split, in the A layout: [k-step][piece][row]
  // [pixel group of 8].  Kept in LDS (1.5 / 3 KiB) rather than in 24 VGPRs:
  // every lane reads row (l&15) & (XR-1), so the rows past 4 + FW of the
  // colour sums hold copies nobody reads.
  constexpr bool XW_LDS = (FW <= 4);
  constexpr int XR = FW == 0 ? 4 : 8;  // operand rows kept
  __shared__ f16x8 s_xw[WPB_BWD][XW_LDS ? 2 : 1][NSH][XR][4];
  // per colour-block row: the factor that undoes its scale and the weights'
  __shared__ __attribute__((aligned(16))) float s_rsc[WPB_BWD][16];
  // The weights w = alpha T enter the fp16 contractions scaled by 2^W_EXP:
  // reference mode walks back from T_final = 1 (Q1), so T <= 1e4 (the
  // forward stops before T < 1e-4) and w in [1/255, 9.9e3] -> x4; fixed
  // mode T <= 1, w in [3.9e-7, 0.99] -> x2^15.  The scale rides on T itself
  // (T, w, dL/dopacity and u all carry it exactly; undone on the sums).
  constexpr int W_EXP = COMPAT == COMPAT_REFERENCE ? 2 : 15;
  constexpr float W_SCALE = (float)(1 << W_EXP);
  // batch weights w ([0]) and u ([1]) as [slot][pixel]: 64-float rows, 16-B
  // groups XOR-swizzled by the row (sw_idx) so that the flush's 16-row operand
  // reads and the per-lane writes are both conflict-free without padding; one
  // array, so the u row is the w row's address plus an immediate offset
  __shared__ float s_wu[WPB_BWD][2][WB * 64];
  __shared__ float4 s_slot[WPB_BWD][WB];  // (mean x, mean y, opacity, id bits)

  // strip item = tile slot * 4 + strip (the tile slot in dispatch order)
  // lw: LDS slot of the wave (a constant 0 at one wave per workgroup, so LDS
  // addresses are offsets from scalars rather than from a per-wave register)
  const int lane = threadIdx.x & 63, lw = WPB_BWD == 1 ? 0 : (int)(threadIdx.x >> 6);
  const int item = strip_item(bslot, WPB_BWD) + lw;
  const uint4 trec = tile_rec(order, item >> 2);
  const int tile = (int)trec.x, wave = item & 3;
  const int tx = tile % grid_x, ty = tile / grid_x;
  const int qx0 = strip_x0(tx, wave), qy0 = strip_y0(ty, wave);  // lane = strip pixel (lane % STRIP_W, lane / STRIP_W)
  const int px = qx0 + lane % STRIP_W, py = qy0 + lane / STRIP_W;
  const bool inside = px < W && py < H;
  const float pfx = (float)px, pfy = (float)py;
  const float sx0 = (float)qx0, sx1 = sx0 + (float)(STRIP_W - 1);
  const float sy0 = (float)qy0, sy1 = sy0 + (float)(STRIP_H - 1);
  const float cx = sx0 + 0.5f * (STRIP_W - 1), cy = sy0 + 0.5f * (STRIP_H - 1);  // strip centre
  const uint2 range = make_uint2(trec.y, trec.z);
  if (!in_window(cb, cam, tx, ty)) return;  // outside the camera's tile window: no contribution
  const size_t HW = (size_t)H * W, pix = inside ? (size_t)py * W + px : 0;

#ifdef GS_STAMPS
  FINE_STAMP(tA);
#endif
  const float T_final = inside ? 1 - alphas[pix] : 0.0f;
  float T = T_final * W_SCALE;  // scaled (W_EXP)
  const uint32_t last = inside ? n_contrib[pix] : 0u;
  float dLp[3];
  // absent upstream gradients (NULL) are zeros
  dLp[0] = inside && dL_dpix ? dL_dpix[pix] : 0.f;
  dLp[1] = inside && dL_dpix ? dL_dpix[HW + pix] : 0.f;
  dLp[2] = inside && dL_dpix ? dL_dpix[2 * HW + pix] : 0.f;
  const float dLd = inside && dL_ddepth ? dL_ddepth[pix] : 0.f;
  const float dLa = inside && dL_dalpha ? dL_dalpha[pix] : 0.f;
  const float bg_dot = bg[0] * dLp[0] + bg[1] * dLp[1] + bg[2] * dLp[2];
  const float tf_bg = (T_final * W_SCALE) * bg_dot;  // the background term's per-pixel factor, scaled like T
  float dLf_own[FIXED_FEAT ? F : 1];  // fixed mode: f . dL/dF feeds dL/dalpha
  if constexpr (FIXED_FEAT) {
#pragma unroll
    for (int c = 0; c < F; ++c) dLf_own[c] = inside && dL_dfeat ? dL_dfeat[(size_t)c * HW + pix] : 0.f;
  }

#ifdef GS_STAMPS
  asm volatile("" ::"v"(T_final), "v"(last), "v"(dLp[0]), "v"(dLp[1]), "v"(dLp[2]), "v"(dLd), "v"(dLa));
  FINE_STAMP(tB);
#endif
  // Constant matrix operands.  Lane l, k-step s (pixels 32s .. 32s+31) holds
  // strip pixels p = 32s + 8(l>>4) + j, j = 0..7 (8 consecutive pixels of one
  // strip row: column p % STRIP_W, row p / STRIP_W):
  //   Xw: row l&15 of the colour block: 0..2 dL/dC, 3 dL/dD, 4.. dL/dF (F < 16)
  //   Bf: dL/dF[p][16cb + (l&15)] (F >= 16; B operand of the feature blocks)
  // Both are fp16 two-piece splits (they meet the weights w in the fp16
  // contractions), each row scaled by its own power of two (row_scale_exp of
  // the row's largest magnitude over the strip's 64 pixels: the row's 16
  // values in each of the 4 lanes l, l^16, l^32, l^48); fmul / s_rsc undo
  // the row's scale and the weights' on the sums.
  hsplit Xw[XW_LDS ? 1 : 2];
  hsplit Bf[CB1][2];
  float fmul[CB1];
  const int kp0 = 8 * (lane >> 4);  // first strip pixel of the lane at k-step 0
  {
    const int row = lane & 15;
    const float* src = nullptr;
    if (row < 3) src = dL_dpix ? dL_dpix + (size_t)row * HW : nullptr;
    else if (row == 3) src = dL_ddepth;
    else if (row - 4 < FW) src = dL_dfeat ? dL_dfeat + (size_t)(16 * CB + row - 4) * HW : nullptr;
    float xv[2][8], fv[CB1][2][8];
    // A lane's 8 pixels are one run of a strip row.  Fast path (the strip
    // lies inside the image, rows and planes 16-B aligned -- decided once per
    // wave): every operand row with two 16-B loads, all issued back to back
    // (a per-row branch made the compiler wait for each row before issuing
    // the next).  Absent planes read the alpha image and are zeroed after.
    // Slow path: per-pixel loads with bounds.
    const float* fplane0 = dL_dfeat ? dL_dfeat + (size_t)row * HW : nullptr;
    const bool lane_ok = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(fplane0) |
                           reinterpret_cast<uintptr_t>(alphas)) & 15) == 0;
    const bool fast = (W & 3) == 0 && (HW & 3) == 0 && qx0 + STRIP_W <= W && qy0 + STRIP_H <= H &&
                      __ballot(!lane_ok) == 0ull;
    if (fast) {
      const float* sp = src ? src : alphas;
      float4 rw[2][2], rf[CB1][2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int p8 = 32 * s + kp0;
        const size_t o = (size_t)(qy0 + p8 / STRIP_W) * W + qx0 + p8 % STRIP_W;
        rw[s][0] = *reinterpret_cast<const float4*>(sp + o);
        rw[s][1] = *reinterpret_cast<const float4*>(sp + o + 4);
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          const float* fp = fplane0 ? fplane0 + (size_t)(16 * cb) * HW : alphas;
          rf[cb][s][0] = *reinterpret_cast<const float4*>(fp + o);
          rf[cb][s][1] = *reinterpret_cast<const float4*>(fp + o + 4);
        }
      }
      auto unpack = [](const float4 (&v)[2], bool on, float (&x)[8]) {
        x[0] = on ? v[0].x : 0.f; x[1] = on ? v[0].y : 0.f; x[2] = on ? v[0].z : 0.f; x[3] = on ? v[0].w : 0.f;
        x[4] = on ? v[1].x : 0.f; x[5] = on ? v[1].y : 0.f; x[6] = on ? v[1].z : 0.f; x[7] = on ? v[1].w : 0.f;
      };
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        unpack(rw[s], src != nullptr, xv[s]);
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) unpack(rf[cb][s], fplane0 != nullptr, fv[cb][s]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int p8 = 32 * s + kp0;
        const int qy = qy0 + p8 / STRIP_W, qx = qx0 + p8 % STRIP_W;
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[s][j] = (src && qx + j < W && qy < H) ? src[(size_t)qy * W + qx + j] : 0.f;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          const float* fsrc = fplane0 ? fplane0 + (size_t)(16 * cb) * HW : nullptr;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            fv[cb][s][j] = (fsrc && qx + j < W && qy < H) ? fsrc[(size_t)qy * W + qx + j] : 0.f;
        }
      }
    }
    // scale each row into [2^14, 2^15) by a power of two (exact), split
    auto scale_row = [&](float (&v)[2][8]) -> int {
      float m = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[s][j]));
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      const int e = row_scale_exp(m);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[s][j] = ldexpf(v[s][j], e);
      return e;
    };
    {
      const int e = scale_row(xv);
      if (lane < 16) s_rsc[lw][lane] = ldexpf(1.f, -e - W_EXP);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr (XW_LDS) {
          hsplit t;
          split_f16(xv[s], t);
          if ((lane & 15) < XR) {
#pragma unroll
            for (int i = 0; i < NSH; ++i) s_xw[lw][s][i][lane & 15][lane >> 4] = t.p[i];
          }
        } else {
          split_f16(xv[s], Xw[s]);
        }
      }
    }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const int e = scale_row(fv[cb]);
      fmul[cb] = ldexpf(1.f, -e - W_EXP);
#pragma unroll
      for (int s = 0; s < 2; ++s) split_f16(fv[cb][s], Bf[cb][s]);
    }
    if constexpr (CB == 0) fmul[0] = 0.f;
  }

#ifdef GS_STAMPS
  FINE_STAMP(tC);
#endif
  // Contract the batch's nb slots and commit their sums (one atomic per
  // (Gaussian, component); slots >= nb hold stale weights whose results are
  // dropped -- the matrix rows are independent).
  auto flush = [&](int nb) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int g = lane & 15;
    // every id the commits below need, read up front (independent LDS reads,
    // one wait) instead of one dependent read per atomic
    // (FW > 0: the component ids are read at the commit instead, fewer live
    // registers)
    constexpr int NAG = FW > 0 ? 1 : (WB * NCOMP + 63) / 64;
    uint32_t fgid[4], agid[NAG];
#pragma unroll
    for (int r = 0; r < 4; ++r) fgid[r] = f_bits(s_slot[lw][(lane >> 4) * 4 + r].w);
#pragma unroll
    for (int t = 0; t < NAG; ++t) {
      const int i = lane + 64 * t;
      agid[t] = (FW == 0 && i < WB * NCOMP) ? f_bits(s_slot[lw][i / NCOMP].w) : 0u;
    }
    // All sums of the batch first, one k-step (32 pixels) at a time, so that
    // only one k-step's split weights are live:
    //   cw: colour / depth (/ small features) C[row][slot] = sum_p Xw[row][p] w[slot][p]
    //   cu: geometry rows, the monomials of the lane's pixels against u
    //   cf: features C[slot][ch] = sum_p w[slot][p] dL/dF[p][ch]
    float4_t cw = float4_t{0.f, 0.f, 0.f, 0.f};
    float4_t cu = float4_t{0.f, 0.f, 0.f, 0.f};
    float4_t cf[CB1];
#pragma unroll
    for (int cb = 0; cb < CB1; ++cb) cf[cb] = float4_t{0.f, 0.f, 0.f, 0.f};
    constexpr int NKS = 2;  // k-steps of 32 pixels
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int p0 = 32 * s + 8 * (lane >> 4);
      {
        // the weights w (scaled by 2^W_EXP): colour block and features, fp16
        hsplit Ws;
        {
          float x[8];
          const float4 a0 = *reinterpret_cast<const float4*>(&s_wu[lw][0][sw_idx(g, p0)]);
          const float4 a1 = *reinterpret_cast<const float4*>(&s_wu[lw][0][sw_idx(g, p0 + 4)]);
          x[0] = a0.x; x[1] = a0.y; x[2] = a0.z; x[3] = a0.w; x[4] = a1.x; x[5] = a1.y; x[6] = a1.z; x[7] = a1.w;
          split_f16(x, Ws);
        }
        if constexpr (XW_LDS) {
          hsplit xw;
#pragma unroll
          for (int i = 0; i < NSH; ++i) xw.p[i] = s_xw[lw][s][i][lane & (XR - 1)][(lane >> 4) & 3];
          cw = mfma_hsplit(xw, Ws, cw);
        } else {
          cw = mfma_hsplit(Xw[s], Ws, cw);
        }
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) cf[cb] = mfma_hsplit(Ws, Bf[cb][s], cf[cb]);
      }
      // the weights u: geometry rows, the monomials 1, X, Y, X^2, XY, Y^2 of
      // the lane's pixels (X = 2 (px - cx) = 2 col - (STRIP_W - 1),
      // Y = 2 row - (STRIP_H - 1) for strip pixel p = 32s + 8(l>>4) + j)
      bsplit Us;
      {
        float y[8];
        const float4 b0 = *reinterpret_cast<const float4*>(&s_wu[lw][1][sw_idx(g, p0)]);
        const float4 b1 = *reinterpret_cast<const float4*>(&s_wu[lw][1][sw_idx(g, p0 + 4)]);
        y[0] = b0.x; y[1] = b0.y; y[2] = b0.z; y[3] = b0.w; y[4] = b1.x; y[5] = b1.y; y[6] = b1.z; y[7] = b1.w;
        split_bf16(y, Us);
      }
      bf16x8 xu;
      {
        // recomputed at every flush (an opaque copy of the lane index keeps
        // the compiler from hoisting them into 8 loop-long registers):
        // row value = a + X (b + c X) with (a, b, c) = (1,0,0), (0,1,0),
        // (Y,0,0), (0,0,1), (0,Y,0), (Y^2,0,0) for rows 0..5, else 0
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int row = ln & 15;
        const int p8 = 32 * s + 8 * ((ln >> 4) & 3);
        const float Y = (float)(2 * (p8 / STRIP_W) - (STRIP_H - 1));
        const float ca = row == 0 ? 1.f : row == 2 ? Y : row == 5 ? Y * Y : 0.f;
        const float cb = row == 1 ? 1.f : row == 4 ? Y : 0.f;
        const float cc = row == 3 ? 1.f : 0.f;
        const float X0 = (float)(2 * (p8 % STRIP_W) - (STRIP_W - 1));
        u32x4 xw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float Xa = X0 + (float)(4 * e), Xb = Xa + 2.f;
          xw[e] = cvt_pk_bf16(fmaf(Xa, fmaf(cc, Xa, cb), ca), fmaf(Xb, fmaf(cc, Xb, cb), ca));
        }
        xu = __builtin_bit_cast(bf16x8, xw);
      }
      cu = mfma_exact_split(xu, Us, cu);
    }
    // undo the scales: colour-block row (l>>4)*4 + r (its row's and the
    // weights'), feature channel l&15 (fmul), the weights' on u
    {
      const float4 rs = *reinterpret_cast<const float4*>(&s_rsc[lw][(lane >> 4) * 4]);
      cw[0] *= rs.x;
      cw[1] *= rs.y;
      cw[2] *= rs.z;
      cw[3] *= rs.w;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) cf[cb] *= fmul[cb];
      cu *= 1.0f / W_SCALE;
    }
    // lane l < 16 holds rows 0..3 of slot l; rows 4, 5 of cu come from lane l + 16
    const float s_xy = __shfl_down(cu[0], 16, 64);
    const float s_yy = __shfl_down(cu[1], 16, 64);
    // lanes 0..15 turn slot l's sums into its 10 accumulator components and
    // park them as [slot][component] in the batch's (consumed) u rows, so
    // that each atomic wave-instruction below adds whole 40-B component
    // records (~7 cache lines) instead of one component of 16 Gaussians; the
    // FW feature rows of the colour block (lanes 16.., row (l>>4)*4 + r) ride
    // along as components A_FEAT.. (their target is the feature gradient row,
    // FW contiguous floats: one request per Gaussian instead of one per
    // channel).
    float* s_out = &s_wu[lw][1][0];
    if (lane < 16) {
      const float4 sl = s_slot[lw][lane];
      const float mx = sl.x - cx, my = sl.y - cy, op = sl.z;
      const float S1 = cu[0], Sx = cu[1], Sy = cu[2], Sxx = cu[3];
      // sum u dx = m' S1 - Sx/2, sum u dx^2 = m'^2 S1 - m' Sx + Sxx/4, ...
      const float ux = fmaf(mx, S1, -0.5f * Sx), uy = fmaf(my, S1, -0.5f * Sy);
      const float uxx = fmaf(mx, fmaf(mx, S1, -Sx), 0.25f * Sxx);
      const float uyy = fmaf(my, fmaf(my, S1, -Sy), 0.25f * s_yy);
      const float uxy = fmaf(mx, fmaf(my, S1, -0.5f * Sy), fmaf(-0.5f * my, Sx, 0.25f * s_xy));
      float* o = s_out + NCOMP * lane;
      o[A_MX] = op * ux;
      o[A_MY] = op * uy;
      o[A_CA] = op * uxx;
      o[A_CB] = op * uxy;
      o[A_CC] = op * uyy;
      o[A_OP] = S1;
      o[A_R] = cw[0];
      o[A_G] = cw[1];
      o[A_B] = cw[2];
      o[A_DEPTH] = cw[3];
    }
    if constexpr (FW > 0) {
      if (lane >= 16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ch = (lane >> 4) * 4 + r - 4;
          if (ch < FW) s_out[NCOMP * g + A_FEAT + ch] = cw[r];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int t = 0; t < (WB * NCOMP + 63) / 64; ++t) {
      const int i = lane + 64 * t;
      if (i >= WB * NCOMP) break;
      const int slot = i / NCOMP, comp = i - NCOMP * slot;
      const uint32_t gi = FW > 0 ? f_bits(s_slot[lw][slot].w) : agid[t < NAG ? t : 0];
      float* dst = comp < A_FEAT ? acc + (size_t)ACC_STRIDE * gi + comp
                                 : dsem + (size_t)gi * FS + 16 * CB + (comp - A_FEAT);
      if (slot < nb) atomicAdd(dst, s_out[i]);
    }
    // features: C[slot][ch] = sum_p w[slot][p] dL/dF[p][ch]; lane l holds
    // channel 16cb + (l&15) of slots (l>>4)*4 + r
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int slot = (lane >> 4) * 4 + r;
        const uint32_t gi = fgid[r];
        if (slot < nb) atomicAdd(dsem + (size_t)gi * FS + 16 * cb + g, cf[cb][r]);
      }
    }
  };

  // The reference carries per-channel "accum_rec" recurrences
  // (CR/backward.cu:560-615): for every channel k with colour c_k and upstream
  // gradient g_k,  rec_k <- la*last_k + (1-la)*rec_k  and  dL/dalpha += (c_k -
  // rec_k)*g_k.  Since g_k is fixed per pixel, only the dot products matter:
  // with  cdot = sum_k c_k g_k  (colour, depth, alpha with c = 1, and in fixed
  // mode the features) and  Q = sum_k rec_k g_k  the recurrence is
  //   Q <- Q + la*(last_cdot - Q),   dL/dalpha = cdot - Q  -- the same value
  // with fewer operations (fp32 reassociation only).
  float Q = 0.f, lcd = 0.f, la = 0.f;
  int nb = 0;  // batch fill

  // the strip's longest pixel walk, from the forward (max n_contrib)
  const uint32_t wmax = __builtin_amdgcn_readfirstlane(ca.smax[item]);
  const uint32_t top = range.x + wmax;  // exclusive end of this wave's walk
  STAT(14, 1);
  STAT(15, wmax);
  STAT_DECL(st_it);
  // records one chunk ahead, list ids two chunks ahead (see the forward)
  RecRegs q;
  uint32_t gnext = 0;
  if (top > range.x) {
    const uint32_t c0 = top > range.x + CHUNK ? top - CHUNK : range.x;
    q = load_rec(point_list, rec, c0 + lane, top - 1);
    const uint32_t n0 = c0 > range.x + CHUNK ? c0 - CHUNK : range.x;
    gnext = load_gid(point_list, n0 + lane, top - 1);
  }
#ifdef GS_STAMPS
#ifdef GS_STAMPS_FINE
  if (top > range.x) asm volatile("" ::"v"(q.q0.x), "v"(gnext));
#endif
  FINE_STAMP(tD);
  const unsigned long long ts1 = stamp();
#endif
  for (uint32_t hi = top; hi > range.x;) {
    const uint32_t c0 = hi > range.x + CHUNK ? hi - CHUNK : range.x;
    const bool keep = (c0 + lane < hi) && !strip_culled(q, sx0, sx1, sy0, sy1);
    {
      const float4 h = half_conic(q.q0, q.q1);
      s_rec[lw][lane][0] = make_float4(q.q0.x, q.q0.y, h.x, h.y);
      s_rec[lw][lane][1] = make_float4(h.z, q.q1.y, q.q1.z, q.q1.w);
      s_rec[lw][lane][2] = make_float4(q.q2.x, q.q2.y, 0.f, 0.f);
    }
    const uint32_t chunk_gid = q.gid;  // lane j: id of the chunk's j-th record
    // chunk entry j is in front of this pixel's last contributor iff j < lrel
    int lrel = (int)last - (int)(c0 - range.x);
    asm volatile("" : "+v"(lrel));  // kept in a register, not recomputed per survivor
    uint64_t mask = __ballot(keep);
    STAT(8, 1);
    STAT(9, hi - c0);
    STAT(10, __builtin_popcountll(mask));
    {
      const uint32_t n0 = c0 > range.x + CHUNK ? c0 - CHUNK : range.x;
      const uint32_t nn0 = n0 > range.x + CHUNK ? n0 - CHUNK : range.x;
      q = load_rec_gid(rec, gnext);                        // the next (lower) chunk
      gnext = load_gid(point_list, nn0 + lane, top - 1);   // the one after
    }
    while (mask) {
      const int j = 63 - __builtin_clzll(mask);
      mask &= ~(1ull << j);
      // all three fields read up front from one row address (r2 is only used
      // by blending survivors, but a separate read would need its own address)
      const float4 r0 = s_rec[lw][j][0];
      const float4 r1 = s_rec[lw][j][1];
      const float2 r2 = *reinterpret_cast<const float2*>(&s_rec[lw][j][2]);
      const float dx = r0.x - pfx, dy = r0.y - pfy;
      const float op = r1.y;
      const float power = gauss_power(dx, dy, make_float4(r0.z, r0.w, r1.x, 0.f));
      const float G = gauss_exp(power);
      const float alpha = fminf(0.99f, op * G);
      const bool valid = (j < lrel) && !(power > 0.0f) && !(alpha < ALPHA_MIN);
      STAT(11, 1);
      STAT_INC(st_it);
      STAT(12, wave_any(valid));
      STAT(13, __builtin_popcountll(__ballot(valid)));
      // r2 read with r0 / r1 (not sunk into the branch below, where its own
      // address would cost a vector instruction)
      asm volatile("" ::"v"(r2.x), "v"(r2.y));
      if (!wave_any(valid)) continue;
      // Invalid lanes park w = u = 0, which zeroes their contributions.
      float w = 0.f, u = 0.f;
      if (valid) {
        const float rinv = fast_rcp(1.f - alpha);
        T = T * rinv;
        w = alpha * T;
        float cdot = fmaf(r2.y, dLd, fmaf(r2.x, dLp[2], fmaf(r1.w, dLp[1], r1.z * dLp[0]))) + dLa;
        if constexpr (FIXED_FEAT) {
          // fixed mode: the features feed dL/dalpha (Q5 fixed)
          const uint32_t gid = __builtin_amdgcn_readlane(chunk_gid, j);
          const float* f = feats + (size_t)gid * F;
          float fd = 0.f;
#pragma unroll
          for (int c = 0; c < F; ++c) fd = fmaf(f[c], dLf_own[c], fd);
          cdot += fd;
        }
        Q = fmaf(la, lcd - Q, Q);
        const float dL_dopa = fmaf(-tf_bg, rinv, (cdot - Q) * T);
        lcd = cdot;
        la = alpha;
        u = G * dL_dopa;
      }
      {
        // sw_idx(nb, lane) in bytes is ((4 lane) ^ (nb << 4)) + 256 nb (nb < 16):
        // one v_xad_u32 for both rows instead of four address instructions
        char* const wu = reinterpret_cast<char*>(&s_wu[lw][0][0]);
        const uint32_t off = (((uint32_t)lane << 2) ^ ((uint32_t)nb << 4)) + ((uint32_t)nb << 8);
        *reinterpret_cast<float*>(wu + off) = w;
        *reinterpret_cast<float*>(wu + off + WB * 64 * 4) = u;
      }
      // the slot record from lane j, which holds the record's id: no
      // readlane, and the centring on the strip is left to the flush
      if (lane == j) {
        // three stores straight from the registers the fields sit in (one
        // 16-B store would need them moved into four consecutive registers)
        float* const sl = reinterpret_cast<float*>(&s_slot[lw][nb]);
        *reinterpret_cast<float2*>(sl) = make_float2(r0.x, r0.y);
        asm volatile("" ::: "memory");
        sl[2] = op;
        asm volatile("" ::: "memory");
        sl[3] = bits_f(chunk_gid);
      }
      if (++nb == WB) {
        flush(WB);
        nb = 0;
      }
    }
    hi = c0;
  }
  STAT_WAVE(17, 25, st_it);
  STAMP(ts2);
  if (nb > 0) flush(nb);
#ifdef GS_STAMPS
  STAMP(ts3);
  __builtin_amdgcn_s_waitcnt(0);
  STAMP(ts4);
  RT_STAMP(rt1);
#ifdef GS_STAMPS_FINE
  stamp_store(g_stamp_bwd_off + (long long)blockIdx.x * WPB_BWD + lw, ts1 - ts0, ts2 - ts0, ts3 - ts0, ts4 - ts0,
              tA - ts0, tB - ts0, tC - ts0, tD - ts0);
#else
  stamp_store(g_stamp_bwd_off + (long long)blockIdx.x * WPB_BWD + lw, ts1 - ts0, ts2 - ts0, ts3 - ts0, ts4 - ts0,
              0, 0, rt0, rt1);
#endif
#endif
}

// ------------------------------------------------------------------ dispatch

// Feature gradients of a padded-stride scratch (F = 36: rows of 48) into the
// caller's P x F rows: out = (accumulate ? out : 0) + scratch, coalesced on
// the output.
__global__ __launch_bounds__(256) void feature_grad_rows_kernel(const float* __restrict__ pad, float* __restrict__ out,
                                                                int64_t n, int F, int FS, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t g = i / F, c = i - g * F;
  const float v = pad[g * FS + c];
  out[i] = accumulate ? out[i] + v : v;
}
// Per-channel largest |feature| (float bits; non-negative floats order as
// their bits, so atomicMax on the bits is a float max).  Each thread owns one
// 4-channel group of a row (F % 4 == 0 for every matrix-core width) and walks
// rows 16-B load by 16-B load, two in flight: a block step covers 256 / (F/4)
// whole rows, contiguous, so a wave's loads are one coalesced run.  At most
// 256 blocks: every block ends in F global float-max atomics on the one
// table, and those cost ~10 ns per block at the memory side whatever the
// addresses (tools/micro/absmax_bench.hip, 300k x 32: the read alone 9-10 us
// at any grid; with the atomics 13 us at 256 blocks, 30 us at 2,048, 52 at
// 4,096 -- replicas of the table did not change it).
__global__ __launch_bounds__(256) void feature_absmax_kernel(const float* __restrict__ f, int64_t P, int F,
                                                             uint32_t* __restrict__ out) {
  __shared__ uint32_t s_m[64];
  const int t = threadIdx.x, G = F >> 2, per = 256 / G;
  if (t < 64) s_m[t] = 0u;
  __syncthreads();
  if (t < per * G) {
    const int gq = t % G;
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* __restrict__ f4 = reinterpret_cast<const float4*>(f);
    const int64_t step = (int64_t)gridDim.x * per;
    int64_t r = (int64_t)blockIdx.x * per + t / G;
    for (; r + step < P; r += 2 * step) {
      const float4 v = f4[r * G + gq], u = f4[(r + step) * G + gq];
      m.x = fmaxf(m.x, fmaxf(fabsf(v.x), fabsf(u.x)));
      m.y = fmaxf(m.y, fmaxf(fabsf(v.y), fabsf(u.y)));
      m.z = fmaxf(m.z, fmaxf(fabsf(v.z), fabsf(u.z)));
      m.w = fmaxf(m.w, fmaxf(fabsf(v.w), fabsf(u.w)));
    }
    if (r < P) {
      const float4 v = f4[r * G + gq];
      m.x = fmaxf(m.x, fabsf(v.x));
      m.y = fmaxf(m.y, fabsf(v.y));
      m.z = fmaxf(m.z, fabsf(v.z));
      m.w = fmaxf(m.w, fabsf(v.w));
    }
    atomicMax(&s_m[4 * gq], __float_as_uint(m.x));
    atomicMax(&s_m[4 * gq + 1], __float_as_uint(m.y));
    atomicMax(&s_m[4 * gq + 2], __float_as_uint(m.z));
    atomicMax(&s_m[4 * gq + 3], __float_as_uint(m.w));
  }
  __syncthreads();
  if (t < F) atomicMax(&out[t], s_m[t]);
}
void launch_feature_absmax(const float* feats, int64_t P, int F, uint32_t* out, hipStream_t s) {
  // `out` is zero already (tile_order_kernel)
  if (P <= 0 || F <= 0 || F > 64 || (F & 3) || !feats) return;
  const int per = 256 / (F >> 2);
  const int64_t blocks = (P + 2 * per - 1) / (2 * per);
  hipLaunchKernelGGL(feature_absmax_kernel, dim3((unsigned)(blocks < 256 ? (blocks > 0 ? blocks : 1) : 256)),
                     dim3(256), 0, s, feats, P, F, out);
}
void launch_feature_grad_rows(const float* pad, float* out, int64_t P, int F, int accumulate, hipStream_t s) {
  const int64_t n = P * (int64_t)F;
  if (n <= 0) return;
  hipLaunchKernelGGL(feature_grad_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pad, out, n, F,
                     feature_grad_stride(F), accumulate);
}

template <int F>
static void fwd_f(const RenderArgs& a, const CamBatch& cb, hipStream_t s) {
  dim3 grid(a.num_tiles * (4 / WPB_FWD) * cb.C), block(64 * WPB_FWD);
  if (a.compat == COMPAT_REFERENCE)
    timed_launch(render_fwd_kernel<F, COMPAT_REFERENCE>, grid, block, 0, s, a, cb);
  else
    timed_launch(render_fwd_kernel<F, COMPAT_FIXED>, grid, block, 0, s, a, cb);
}

template <int F>
static void bwd_f(const RenderBwdArgs& a, const CamBatch& cb, hipStream_t s) {
  dim3 grid(a.num_tiles * (4 / WPB_BWD) * cb.C), block(64 * WPB_BWD);
  if (a.compat == COMPAT_REFERENCE)
    timed_launch(render_bwd_kernel<F, COMPAT_REFERENCE>, grid, block, 0, s, a, cb);
  else
    timed_launch(render_bwd_kernel<F, COMPAT_FIXED>, grid, block, 0, s, a, cb);
}

bool launch_render_fwd(const RenderArgs& a, const CamBatch& cb, hipStream_t s) {
  if (a.num_tiles <= 0) return true;
  switch (a.F) {
    case 0: fwd_f<0>(a, cb, s); return true;
    case 4: fwd_f<4>(a, cb, s); return true;
    case 8: fwd_f<8>(a, cb, s); return true;
    case 16: fwd_f<16>(a, cb, s); return true;
    case 32: fwd_f<32>(a, cb, s); return true;
    case 36: fwd_f<36>(a, cb, s); return true;
    case 64: fwd_f<64>(a, cb, s); return true;
    default: return false;
  }
}

bool launch_render_bwd(const RenderBwdArgs& a, const CamBatch& cb, hipStream_t s) {
  if (a.num_tiles <= 0) return true;
  switch (a.F) {
    case 0: bwd_f<0>(a, cb, s); return true;
    case 4: bwd_f<4>(a, cb, s); return true;
    case 8: bwd_f<8>(a, cb, s); return true;
    case 16: bwd_f<16>(a, cb, s); return true;
    case 32: bwd_f<32>(a, cb, s); return true;
    case 36: bwd_f<36>(a, cb, s); return true;
    case 64: bwd_f<64>(a, cb, s); return true;
    default: return false;
  }
}

#ifdef GS_STATS
extern "C" int gs_stats_read(unsigned long long* out, int n) {
  if (n > 32) n = 32;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stats), sizeof(unsigned long long) * n, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int gs_stats_reset(void) {
  static const unsigned long long z[32] = {0};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#endif

// ------------------------------------------------------------------ self-test

template <int N>
__global__ void test_wave_reduce_kernel(const float* __restrict__ in, float* __restrict__ out) {
  const int lane = threadIdx.x;
  float v[64];
#pragma unroll
  for (int c = 0; c < N; ++c) v[c] = in[c * 64 + lane];
  const float s = wave_reduce_transposed<N>(v, lane);
  const int comp = bitrev6(lane);
  if (comp < N) out[comp] = s;
}

void launch_test_wave_reduce(int n, const float* in, float* out, hipStream_t s) {
#define CASE(K) case K: hipLaunchKernelGGL(test_wave_reduce_kernel<K>, dim3(1), dim3(64), 0, s, in, out); break;
  switch (n) {
    CASE(1) CASE(2) CASE(3) CASE(10) CASE(13) CASE(18) CASE(26) CASE(42) CASE(64)
    default: break;
  }
#undef CASE
}

}  // namespace gs
