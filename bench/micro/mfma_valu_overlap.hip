// Can a VALU-only wave and an MFMA-only wave on the same SIMD run concurrently on gfx950?
// 256-thread block (one wave per SIMD) or 512 (two per SIMD): wave w < 4 runs MFMAs,
// waves >= 4 run dependent-free VALU; mode selects which roles are active.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512) void k(float* out, int mode, int iters) {
  const int wave = threadIdx.x >> 6;
  const bool mf = wave < 4;
  float r = 0.f;
  if (mf && (mode & 1)) {
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
  if (!mf && (mode & 2)) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < iters * 16; ++i) {   // 8 independent chains, 8 VALU per step
      x0 = fmaf(x0, 1.0001f, 0.5f); x1 = fmaf(x1, 1.0001f, 0.5f); x2 = fmaf(x2, 1.0001f, 0.5f); x3 = fmaf(x3, 1.0001f, 0.5f);
      x4 = fmaf(x4, 1.0001f, 0.5f); x5 = fmaf(x5, 1.0001f, 0.5f); x6 = fmaf(x6, 1.0001f, 0.5f); x7 = fmaf(x7, 1.0001f, 0.5f);
    }
    r = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  float* out;
  const int blocks = 256, iters = 2000;
  if (hipMalloc(&out, blocks * 512 * 4) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 1; mode <= 3; ++mode) {
      hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, out, mode, iters);
      hipEventRecord(e0);
      for (int t = 0; t < 5; ++t) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 0, 0, out, mode, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("mode %d (%s): %.3f ms per launch; MFMA-only cycles @2.1GHz ~ %.3f ms\n", mode,
             mode == 1 ? "MFMA waves only" : mode == 2 ? "VALU waves only" : "both", ms / 5,
             iters * 4 * 32 / 2.1e9 * 1e3);
    }
  return 0;
}
