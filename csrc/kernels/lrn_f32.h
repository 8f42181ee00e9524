// fp32 LRN (tf.nn.local_response_normalization across channels) building blocks shared by
// the fp32 LRN kernels (f32.hip) and the kernels that fold an LRN into their staging
// (conv1_f32.hip): 4 channels per lane, the G = C/4 lanes of a pixel adjacent inside one
// 16-lane DPP row; the window's neighbours (radius r <= 4) come from the adjacent lanes by
// DPP row shifts (zero at the pixel's first / last lane).
#pragma once
#include "common.h"

namespace mnistx {
namespace {

DEV float pow_neg(float n, float b) { return exp2f(-b * log2f(n)); }   // n^-b, n >= bias > 0
// n^-b (bitwise pow_neg) and n^-(b+1) from one log2: the backward's g x n^-b / n without the
// IEEE division (~10 VALU per channel; one more v_exp_f32 instead)
DEV void pow_neg2(float n, float b, float& p, float& p1) {
  const float lg = log2f(n);
  p = exp2f(-b * lg);
  p1 = exp2f(-(b + 1.f) * lg);
}

DEV float f32_from_left(float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, true)); }
DEV float f32_from_right(float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xf, 0xf, true)); }
DEV f32x4 win4(const f32x4& v, int c4, int G, int r) {
  float e[12];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float l = f32_from_left(v[j]), rr = f32_from_right(v[j]);
    e[j] = c4 == 0 ? 0.f : l;
    e[8 + j] = c4 == G - 1 ? 0.f : rr;
    e[4 + j] = v[j];
  }
  f32x4 s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float a = 0.f;
#pragma unroll
    for (int d = -4; d <= 4; ++d)
      if (d >= -r && d <= r) a = fmaf(1.f, e[4 + j + d], a);
    s[j] = a;
  }
  return s;
}

// dx = dL/d(LRN input) of one 4-channel vector: x = the LRN input, g = dL/d(LRN output);
// every lane of the wave must call it (DPP exchanges)
DEV f32x4 lrn_f32_bwd4(const f32x4& v, const f32x4& g, int c4, int G, int r, float bias, float alpha, float beta,
                       int relu_mask) {
  // no FMA contraction: every kernel that inlines this rounds alike (the fused norm1 fold in
  // conv1_f32.hip and lrn_f32_bwd_v4_k give bitwise-equal gradients, tests/test_f32_gpu.py)
#pragma clang fp contract(off)
  const f32x4 s = win4(v * v, c4, G, r);
  f32x4 nb, tt;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float p0, p1;
    pow_neg2(fmaf(alpha, s[j], bias), beta, p0, p1);
    nb[j] = p0;
    tt[j] = g[j] * v[j] * p1;
  }
  const f32x4 u = win4(tt, c4, G, r);
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float d = g[j] * nb[j] - 2.f * alpha * beta * v[j] * u[j];
    if (relu_mask && !(v[j] > 0.f)) d = 0.f;
    o[j] = d;
  }
  return o;
}

}  // namespace
}  // namespace mnistx
