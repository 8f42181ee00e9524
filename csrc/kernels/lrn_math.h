// LRN (tf.nn.local_response_normalization) building blocks shared by the LRN kernels
// (misc.hip) and the kernels that fold an LRN into their staging (convpool.hip).
// Channel-parallel: each lane owns 8 channels (one 16-byte bf16 vector) of a pixel,
// the C/8 lanes of a pixel sit side by side inside one 16-lane DPP row, and the R
// channels a window needs from the neighbouring vectors come over DPP row shifts
// (zeroed at the pixel's first / last vector).
#pragma once
#include "common.h"

namespace mnistx {
namespace {

DEV float dpp_from_left(float v) {   // lane i <- lane i-1 within its 16-lane row (0 at the row start)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, true));
}
DEV float dpp_from_right(float v) {  // lane i <- lane i+1 within its 16-lane row (0 at the row end)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xf, 0xf, true));
}

// running window sums of an 8-channel vector: e = R left neighbours, the 8 values, R right
// neighbours (zeros past the pixel's channels).  One full sum, then +entering -leaving (the
// inputs are non-negative squares or same-scale products, so the running form loses nothing
// at bf16 output).  Every LRN kernel sums through this, in this order.
template <int R, class T>
DEV void window_sums_e(const T (&e)[8 + 2 * R], T (&s)[8]) {
  // never fused with the multiplies that produced e (squares, products): every caller then
  // sums the same rounded values, whatever it inlines (bitwise equality across kernels)
#pragma clang fp contract(off)
  T a = T{};
#pragma unroll
  for (int d = 0; d <= 2 * R; ++d) a += e[d];
  s[0] = a;
#pragma unroll
  for (int j = 1; j < 8; ++j) {
    a += e[j + 2 * R] - e[j - 1];
    s[j] = a;
  }
}

// window sums over channels of the 8 values of this lane, with the R neighbours on
// either side taken from the adjacent lanes of the same pixel (G lanes per pixel)
template <int G, int R>
DEV void lane_window_sums(const float (&v)[8], int c8, float (&s)[8]) {
  static_assert(R <= 8 && 16 % G == 0, "neighbours must come from the adjacent lane of one DPP row");
  float e[8 + 2 * R];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[R + j] = v[j];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    float l = dpp_from_left(v[8 - R + k]), r = dpp_from_right(v[k]);
    if constexpr (G == 1) {
      l = 0.f;
      r = 0.f;
    }
    e[k] = c8 == 0 ? 0.f : l;
    e[R + 8 + k] = c8 == G - 1 ? 0.f : r;
  }
  window_sums_e<R>(e, s);
}

// x^p for x > 0 as exp2(p log2 x): two transcendental ops, no ln/log2e rescaling
DEV float powp(float x, float p) { return __builtin_amdgcn_exp2f(p * __builtin_amdgcn_logf(x)); }
// sc^-beta and sc^-(beta+1).  The reference's beta = 0.75 (mnist_input.py:151,167) takes two
// transcendentals, r = sc^-1/2 and q = r^1/2: sc^-0.75 = r q, sc^-1.75 = r^3 q (log + exp +
// rcp otherwise).  B075 is a template argument, chosen on the host from the kernel's beta: a
// runtime test on beta, uniform as it is, was compiled into one branch per value (32 per
// pixel vector in lrn_pool_bwd_k, each with its exec-mask juggling and s_nop padding).
template <bool B075>
DEV void pow_beta(float sc, float beta, float& pw, float& pw1) {
  if constexpr (B075) {
    const float r = __builtin_amdgcn_rsqf(sc), q = __builtin_amdgcn_sqrtf(r);
    pw = r * q;
    pw1 = pw * (r * r);
  } else {
    pw = powp(sc, -beta);
    pw1 = pw * __builtin_amdgcn_rcpf(sc);
  }
}

// The contractable spots of the LRN math are written as explicit fmaf: every kernel that
// inlines these helpers (lrn_*_k, lrn_pool_*_k, the staging folds) then rounds identically,
// whatever hipcc's fp-contract would fuse in each context (the fused-vs-two-step bitwise tests)
DEV float lrn_scale(float s, float bias, float alpha) { return fmaf(alpha, s, bias); }
DEV float lrn_out(float v, float s, float bias, float alpha, float beta) {
  return v * powp(lrn_scale(s, bias, alpha), -beta);
}

DEV void unpack8(const u32x4& u, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = u4_get(u, j);
}


// LRN forward of one 8-channel vector (G lanes per pixel): y = x s^-beta, s = bias +
// alpha * window sum of x^2, rounded to bf16 (bitwise lrn_fwd_k).
template <int G, int R>
DEV u32x4 lrn_fwd8(const u32x4& xv, int c8, float bias, float alpha, float beta) {
  float v[8], sq[8], s[8];
  unpack8(xv, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) sq[j] = v[j] * v[j];
  lane_window_sums<G, R>(sq, c8, s);
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = lrn_out(v[2 * j], s[2 * j], bias, alpha, beta);
    const float b = lrn_out(v[2 * j + 1], s[2 * j + 1], bias, alpha, beta);
    o[j] = pack2(a, b);
  }
  return o;
}

// LRN backward of one 8-channel vector (x = LRN input, g = dL/dy; G lanes per pixel):
// dx[c] = g[c] s[c]^-b - 2ab x[c] sum_{|c'-c|<=R} g[c'] x[c'] s[c']^(-b-1), s = bias +
// alpha * window sum of x^2; relu_mask zeroes dx where x <= 0.  Rounded to bf16.
template <int G, int R, bool B075 = false>
DEV u32x4 lrn_bwd8_vals(const float (&v)[8], const float (&g)[8], int c8, float bias, float alpha, float beta,
                        int relu_mask) {
  float w[8], s[8], u[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = v[j] * v[j];
  lane_window_sums<G, R>(w, c8, s);             // s = window sum of x^2
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float sc = lrn_scale(s[j], bias, alpha);
    float pw, pw1;                                  // sc^-beta, sc^-(beta+1)
    pow_beta<B075>(sc, beta, pw, pw1);
    s[j] = pw;
    w[j] = g[j] * v[j] * pw1;
  }
  lane_window_sums<G, R>(w, c8, u);
  const float k = 2.f * alpha * beta;
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float r2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 2 * j + h;
      float d = fmaf(g[c], s[c], -((k * v[c]) * u[c]));
      if (relu_mask && !(v[c] > 0.f)) d = 0.f;
      r2[h] = d;
    }
    o[j] = pack2(r2[0], r2[1]);
  }
  return o;
}
template <int G, int R, bool B075 = false>
DEV u32x4 lrn_bwd8(const u32x4& xv, const u32x4& gv, int c8, float bias, float alpha, float beta, int relu_mask) {
  float v[8], g[8];
  unpack8(xv, v);
  unpack8(gv, g);
  return lrn_bwd8_vals<G, R, B075>(v, g, c8, bias, alpha, beta, relu_mask);
}

// ---- packed forms: two independent vectors per lane (two pool windows, or two pixels of
// one), so the element-wise work issues as v_pk_{mul,add,fma}_f32.  Each half runs the
// scalar helpers' IEEE operations in the same order: bitwise the scalar forms above.
typedef float f2 __attribute__((ext_vector_type(2)));
DEV f2 f2s(float a) { return f2{a, a}; }
DEV f2 f2fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <int G, int R>
DEV void lane_window_sums2(const f2 (&v)[8], int c8, f2 (&s)[8]) {
  static_assert(R <= 8 && 16 % G == 0 && G > 1, "neighbours must come from the adjacent lane of one DPP row");
  f2 e[8 + 2 * R];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[R + j] = v[j];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const f2 l = f2{dpp_from_left(v[8 - R + k].x), dpp_from_left(v[8 - R + k].y)};
    const f2 r = f2{dpp_from_right(v[k].x), dpp_from_right(v[k].y)};
    e[k] = c8 == 0 ? f2{} : l;
    e[R + 8 + k] = c8 == G - 1 ? f2{} : r;
  }
  window_sums_e<R>(e, s);
}

// lrn_out on two values
DEV f2 lrn_out2(f2 v, f2 s, float bias, float alpha, float beta) {
  const f2 sc = f2fma(f2s(alpha), s, f2s(bias));
  const f2 p = f2s(-beta) * f2{__builtin_amdgcn_logf(sc.x), __builtin_amdgcn_logf(sc.y)};
  return v * f2{__builtin_amdgcn_exp2f(p.x), __builtin_amdgcn_exp2f(p.y)};
}

// lrn_bwd8_vals<G, R, true> (beta = 0.75) on two vectors
template <int G, int R>
DEV void lrn_bwd2_b075(const f2 (&v)[8], const f2 (&g)[8], int c8, float bias, float alpha, float beta, int relu_mask,
                       f2 (&o)[8]) {
  f2 w[8], s[8], u[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = v[j] * v[j];
  lane_window_sums2<G, R>(w, c8, s);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f2 sc = f2fma(f2s(alpha), s[j], f2s(bias));
    const f2 r = f2{__builtin_amdgcn_rsqf(sc.x), __builtin_amdgcn_rsqf(sc.y)};
    const f2 q = f2{__builtin_amdgcn_sqrtf(r.x), __builtin_amdgcn_sqrtf(r.y)};
    const f2 pw = r * q;
    const f2 pw1 = pw * (r * r);
    s[j] = pw;
    w[j] = g[j] * v[j] * pw1;
  }
  lane_window_sums2<G, R>(w, c8, u);
  const f2 k = f2s(2.f * alpha * beta);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f2 d = f2fma(g[j], s[j], -((k * v[j]) * u[j]));
    if (relu_mask) {
      d.x = v[j].x > 0.f ? d.x : 0.f;
      d.y = v[j].y > 0.f ? d.y : 0.f;
    }
    o[j] = d;
  }
}

// lrn_bwd8<G, R, true> of two independent 8-channel vectors (same lane layout) at once
template <int G, int R>
DEV void lrn_bwd8x2_b075(const u32x4& x0, const u32x4& g0, const u32x4& x1, const u32x4& g1, int c8, float bias,
                         float alpha, float beta, int relu_mask, u32x4& o0, u32x4& o1) {
  f2 v[8], g[8], o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = f2{u4_get(x0, j), u4_get(x1, j)};
    g[j] = f2{u4_get(g0, j), u4_get(g1, j)};
  }
  lrn_bwd2_b075<G, R>(v, g, c8, bias, alpha, beta, relu_mask, o);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o0[j] = pack2(o[2 * j].x, o[2 * j + 1].x);
    o1[j] = pack2(o[2 * j].y, o[2 * j + 1].y);
  }
}

}  // namespace
}  // namespace mnistx
