// Micro-benchmark: issue rate of packed vs scalar fp32 FMA on gfx950
// (v_pk_fma_f32 does two fp32 FMAs per lane: does it issue at the rate of
// one v_fma_f32?).  8 independent accumulator chains per lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int N = 4096;
__global__ __launch_bounds__(256) void scalar_k(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < N; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void packed_k(float* out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = (f2){(float)threadIdx.x + i, (float)i};
  const f2 av = {a, a}, bv = {b, b};
  for (int it = 0; it < N; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(av), "v"(bv));
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  float* d;
  const int blocks = 256 * 8;
  hipMalloc(&d, sizeof(float) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int kind = 0; kind < 2; ++kind) {
      hipEventRecord(e0);
      if (kind == 0) hipLaunchKernelGGL(scalar_k, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 0.001f);
      else hipLaunchKernelGGL(packed_k, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 0.001f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double fmas = (double)blocks * 256 * N * 8 * (kind ? 2 : 1);
      printf("%s: %.3f ms, %.1f TFLOP/s fp32\n", kind ? "v_pk_fma_f32" : "v_fma_f32", ms, 2 * fmas / ms / 1e9);
    }
  }
  return 0;
}
