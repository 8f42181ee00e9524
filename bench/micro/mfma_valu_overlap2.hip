// Throughput version: VALU waves issue independent v_max_f32 / v_and_b32 / v_add_u32
// (the epilogue mix of lenet_band.hip) from 16 independent registers, MFMA waves issue
// independent 32x32x16 bf16 MFMAs; both sized to ~equal solo time.  mode: 1 MFMA only,
// 2 VALU only, 3 both (same SIMDs: wave w and w+4 share SIMD w%4).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512) void k(float* out, int mode, int iters, int viters) {
  const int wave = threadIdx.x >> 6;
  float r = 0.f;
  if (wave < 4 && (mode & 1)) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(threadIdx.x * 0.001f + j); b[j] = (__bf16)(j * 0.5f); }
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    for (int j = 0; j < 16; ++j) r += c0[j] + c1[j] + c2[j] + c3[j];
  }
  if (wave >= 4 && (mode & 2)) {
    float v[8];
    unsigned u[8];
    for (int j = 0; j < 8; ++j) { v[j] = threadIdx.x + j; u[j] = threadIdx.x * 3 + j; }
    float m = 0.5f;
    for (int i = 0; i < viters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        asm volatile("v_max_f32 %0, %0, %1" : "+v"(v[j]) : "v"(m));
        asm volatile("v_and_b32 %0, 0xfffffffc, %0" : "+v"(u[j]));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[j]) : "v"(j));
    }
    for (int j = 0; j < 8; ++j) r += v[j] + u[j];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  float* out;
  const int blocks = 256, iters = 4000;
  const int viters = 4000 * 128 / (24 * 2);    // 24 VALU/iter at 2 cycles ~ MFMA time (128 cycles/iter)
  if (hipMalloc(&out, blocks * 512 * 4) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 1; mode <= 3; ++mode) {
      hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, out, mode, iters, viters);
      (void)hipEventRecord(e0);
      for (int t = 0; t < 5; ++t) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, out, mode, iters, viters);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("mode %d (%s): %.3f ms per launch  [MFMA %d x 32 cyc, VALU %d instrs/wave]\n", mode,
             mode == 1 ? "MFMA waves only" : mode == 2 ? "VALU waves only" : "both", ms / 5, iters * 4,
             viters * 24);
    }
  return 0;
}
