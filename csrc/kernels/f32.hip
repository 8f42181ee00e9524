// Reference-precision (fp32) kernels for gfx950: --precision fp32.
//
// The reference trains in fp32 (mnist_input.py:86,107 `dtype = tf.float32`).  The
// bf16 kernels stay the default; this file is the fp32 execution path of the
// same model specs:
//   * one MFMA GEMM engine on v_mfma_f32_16x16x4_f32 (fp32 operands, fp32
//     accumulate) with operand "loaders" for dense fwd / dgrad / wgrad and the
//     implicit-GEMM conv fwd / dgrad (flipped filter) / wgrad (im2col^T, split-K
//     into deterministic fp32 slabs reduced by misc.hip splitk_reduce);
//   * fp32 2x2/2 SAME max-pool fwd/bwd (argmax byte), LRN fwd/bwd across
//     channels, softmax-CE with fp32 logit gradients (ce_stats.h partials) and the
//     u8 -> fp32 batch gather/normalise.
//
// GEMM tiling: 64x64 output tile per 256-thread block, four waves in a 2x2 layout,
// each wave 2x2 16x16 fragments; K staged 16 at a time through LDS stored k-major
// ([k][m], 68-float rows: a fragment read is 16 consecutive floats per k row),
// register double-buffered (global -> VGPR for step t+1 while step t computes).
// v_mfma_f32_16x16x4_f32: A lane l = (row l%16, k l/16), B lane l = (k l/16, col
// l%16), D lane l = rows 4(l/16)..+3 of col l%16.
#include "common.h"
#include "ce_stats.h"
#include "launchers.h"
#include "lrn_f32.h"

#include <cstdlib>

namespace mnistx {
namespace {

constexpr int FBK = 16, FNT = 256;
// BM x BM output tile per 256-thread block (BM = 64, or 128 for large problems: half the
// L2 operand traffic per MAC); LDS row stride BM + 4 floats
template <int BM> constexpr int fvpt() { return BM * FBK / 4 / FNT; }   // 4-vectors per thread per operand tile
template <int BM> constexpr int fld() { return BM + 4; }

// ---------------------------------------------------------------- loaders
// load4(r, k): 4 operand elements along the operand's contiguous direction -- k..k+3
// of row r (KC: consecutive k are contiguous in memory) or rows r..r+3 at k (!KC) --
// zero outside; one 16-byte load when the 4 are contiguous and aligned.
DEV f32x4 ld4(const float* p) { return *(const f32x4*)p; }
DEV bool al16(const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <bool KC_>
struct StridedF {
  static constexpr bool KC = KC_;
  const float* p;
  int R, K, ld;
  int ones_r;  // virtual row of ones (bias-gradient row), -1 = none
  DEV float get(int r, int k) const {
    if (k >= K) return 0.f;
    if (r == ones_r) return 1.f;
    if (r >= R) return 0.f;
    return KC ? p[(int64_t)r * ld + k] : p[(int64_t)k * ld + r];
  }
  DEV f32x4 load4(int r, int k) const {
    if constexpr (KC) {
      if (r < R && r != ones_r && k + 3 < K && (ld & 3) == 0 && al16(p)) return ld4(p + (int64_t)r * ld + k);
      return f32x4{get(r, k), get(r, k + 1), get(r, k + 2), get(r, k + 3)};
    } else {
      if (k < K && r + 3 < R && (ones_r < r || ones_r > r + 3) && (ld & 3) == 0 && al16(p))
        return ld4(p + (int64_t)k * ld + r);
      return f32x4{get(r, k), get(r + 1, k), get(r + 2, k), get(r + 3, k)};
    }
  }
};

// conv fwd A: row m = output pixel (n, oh, ow), k = (kh, kw, ci)
struct Im2colF {
  static constexpr bool KC = true;
  const float* x;
  int H, W, C, OH, OW, KW, ph, pw, M, K;
  FastDiv fOHW, fOW, fC, fKW;
  DEV float get(int m, int k) const {
    if (m >= M || k >= K) return 0.f;
    const int n = fOHW.div(m), rem = fOHW.mod(m, n);
    const int oh = fOW.div(rem), ow = fOW.mod(rem, oh);
    const int tap = fC.div(k), ci = fC.mod(k, tap);
    const int kh = fKW.div(tap), kw = fKW.mod(tap, kh);
    const int ih = oh - ph + kh, iw = ow - pw + kw;
    if (ih < 0 || ih >= H || iw < 0 || iw >= W) return 0.f;
    return x[(((int64_t)n * H + ih) * W + iw) * C + ci];
  }
  DEV f32x4 load4(int m, int k) const {
    if ((C & 3) == 0 && al16(x) && m < M && k + 3 < K) {   // k..k+3: 4 channels of one tap
      const int n = fOHW.div(m), rem = fOHW.mod(m, n);
      const int oh = fOW.div(rem), ow = fOW.mod(rem, oh);
      const int tap = fC.div(k), ci = fC.mod(k, tap);
      const int kh = fKW.div(tap), kw = fKW.mod(tap, kh);
      const int ih = oh - ph + kh, iw = ow - pw + kw;
      if (ih < 0 || ih >= H || iw < 0 || iw >= W) return f32x4{0.f, 0.f, 0.f, 0.f};
      return ld4(x + (((int64_t)n * H + ih) * W + iw) * C + ci);
    }
    return f32x4{get(m, k), get(m, k + 1), get(m, k + 2), get(m, k + 3)};
  }
};

// conv wgrad A (im2col^T): row m = (kh, kw, ci) (+ ones row at Mreal), k = output pixel
struct Im2colTF {
  static constexpr bool KC = false;
  const float* x;
  int H, W, C, OH, OW, KW, ph, pw, P, Mreal;
  FastDiv fOHW, fOW, fC, fKW;
  DEV float get(int m, int k) const {
    if (k >= P) return 0.f;
    if (m == Mreal) return 1.f;
    if (m > Mreal) return 0.f;
    const int n = fOHW.div(k), rem = fOHW.mod(k, n);
    const int oh = fOW.div(rem), ow = fOW.mod(rem, oh);
    const int tap = fC.div(m), ci = fC.mod(m, tap);
    const int kh = fKW.div(tap), kw = fKW.mod(tap, kh);
    const int ih = oh - ph + kh, iw = ow - pw + kw;
    if (ih < 0 || ih >= H || iw < 0 || iw >= W) return 0.f;
    return x[(((int64_t)n * H + ih) * W + iw) * C + ci];
  }
  DEV f32x4 load4(int m, int k) const {
    if ((C & 3) == 0 && al16(x) && k < P && m + 3 < Mreal) {   // m..m+3: 4 channels of one tap
      const int n = fOHW.div(k), rem = fOHW.mod(k, n);
      const int oh = fOW.div(rem), ow = fOW.mod(rem, oh);
      const int tap = fC.div(m), ci = fC.mod(m, tap);
      const int kh = fKW.div(tap), kw = fKW.mod(tap, kh);
      const int ih = oh - ph + kh, iw = ow - pw + kw;
      if (ih < 0 || ih >= H || iw < 0 || iw >= W) return f32x4{0.f, 0.f, 0.f, 0.f};
      return ld4(x + (((int64_t)n * H + ih) * W + iw) * C + ci);
    }
    return f32x4{get(m, k), get(m + 1, k), get(m + 2, k), get(m + 3, k)};
  }
};

// conv dgrad A: row m = input pixel (n, ih, iw), k = (kh, kw, co): dy[n, ih+ph-kh, iw+pw-kw, co]
struct DyIm2colF {
  static constexpr bool KC = true;
  const float* dy;
  int H, W, OH, OW, Co, KW, ph, pw, M, K;
  FastDiv fHW, fW, fCo, fKW;
  DEV float get(int m, int k) const {
    if (m >= M || k >= K) return 0.f;
    const int n = fHW.div(m), rem = fHW.mod(m, n);
    const int ih = fW.div(rem), iw = fW.mod(rem, ih);
    const int tap = fCo.div(k), co = fCo.mod(k, tap);
    const int kh = fKW.div(tap), kw = fKW.mod(tap, kh);
    const int oh = ih + ph - kh, ow = iw + pw - kw;
    if (oh < 0 || oh >= OH || ow < 0 || ow >= OW) return 0.f;
    return dy[(((int64_t)n * OH + oh) * OW + ow) * Co + co];
  }
  DEV f32x4 load4(int m, int k) const {
    if ((Co & 3) == 0 && al16(dy) && m < M && k + 3 < K) {
      const int n = fHW.div(m), rem = fHW.mod(m, n);
      const int ih = fW.div(rem), iw = fW.mod(rem, ih);
      const int tap = fCo.div(k), co = fCo.mod(k, tap);
      const int kh = fKW.div(tap), kw = fKW.mod(tap, kh);
      const int oh = ih + ph - kh, ow = iw + pw - kw;
      if (oh < 0 || oh >= OH || ow < 0 || ow >= OW) return f32x4{0.f, 0.f, 0.f, 0.f};
      return ld4(dy + (((int64_t)n * OH + oh) * OW + ow) * Co + co);
    }
    return f32x4{get(m, k), get(m, k + 1), get(m, k + 2), get(m, k + 3)};
  }
};

// conv dgrad B: row = ci, k = (kh, kw, co): W[kh][kw][ci][co]
struct WFlipF {
  static constexpr bool KC = true;
  const float* w;
  int Ci, Co, K;
  FastDiv fCo;
  DEV float get(int ci, int k) const {
    if (ci >= Ci || k >= K) return 0.f;
    const int tap = fCo.div(k), co = fCo.mod(k, tap);
    return w[((int64_t)tap * Ci + ci) * Co + co];
  }
  DEV f32x4 load4(int ci, int k) const {
    if ((Co & 3) == 0 && al16(w) && ci < Ci && k + 3 < K) {
      const int tap = fCo.div(k), co = fCo.mod(k, tap);
      return ld4(w + ((int64_t)tap * Ci + ci) * Co + co);
    }
    return f32x4{get(ci, k), get(ci, k + 1), get(ci, k + 2), get(ci, k + 3)};
  }
};

struct EpiF {
  float* out;            // output (mode 0) or slab base (mode 1)
  int ldc;
  int mode;              // 0: store, 1: split-K slab [z][M][N]
  const float* bias;     // mode 0: + bias[n] (n < bias_n)
  int bias_n;
  int relu;
  const float* mask;     // mode 0: keep v where mask[m * ldm + n] > 0 (ReLU backward)
  int ldm;
  int64_t slab_stride;
};

// Tile staging: BM rows x FBK k = fvpt<BM>() four-element vectors per thread, taken along
// the operand's contiguous direction; LDS keeps the tile k-major ([k][row]).
template <int BM, class L>
DEV void stage_load(const L& ld, int r0, int k0, int tid, f32x4 (&v)[fvpt<BM>()]) {
#pragma unroll
  for (int i = 0; i < fvpt<BM>(); ++i) {
    const int idx = tid + i * FNT;
    if constexpr (L::KC) v[i] = ld.load4(r0 + idx / (FBK / 4), k0 + 4 * (idx % (FBK / 4)));
    else v[i] = ld.load4(r0 + 4 * (idx % (BM / 4)), k0 + idx / (BM / 4));
  }
}

template <int BM, class L>
DEV void stage_store(float* lds, int tid, const f32x4 (&v)[fvpt<BM>()]) {
  constexpr int LD = fld<BM>();
#pragma unroll
  for (int i = 0; i < fvpt<BM>(); ++i) {
    const int idx = tid + i * FNT;
    if constexpr (L::KC) {
      const int r = idx / (FBK / 4), k = 4 * (idx % (FBK / 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) lds[(k + j) * LD + r] = v[i][j];
    } else {
      *(f32x4*)(lds + (idx / (BM / 4)) * LD + 4 * (idx % (BM / 4))) = v[i];
    }
  }
}

// C[M,N] = sum_k A(m,k) B(k,n) over this split's K range [z*kc, min(K, (z+1)*kc))
// Four waves in a 2x2 layout, each (BM/2)^2 = FI x FI 16x16 fragments.
template <int BM, class AL, class BL>
__global__ __launch_bounds__(FNT) void gemm_f32_k(AL A, BL Bm, int M, int N, int K, int kc, EpiF ep) {
  constexpr int LD = fld<BM>(), FI = BM / 32, VP = fvpt<BM>();
  __shared__ float As[2][FBK * LD];
  __shared__ float Bs[2][FBK * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (N + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BM;
  const int z = blockIdx.y;
  const int kb = z * kc, ke = min(K, kb + kc);
  f32x4 acc[FI][FI];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 va[VP], vb[VP];
  if (kb < ke) {
    stage_load<BM>(A, m0, kb, tid, va);
    stage_load<BM>(Bm, n0, kb, tid, vb);
  }
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += FBK) {
    stage_store<BM, AL>(As[buf], tid, va);
    stage_store<BM, BL>(Bs[buf], tid, vb);
    __syncthreads();
    if (k0 + FBK < ke) {
      stage_load<BM>(A, m0, k0 + FBK, tid, va);
      stage_load<BM>(Bm, n0, k0 + FBK, tid, vb);
    }
    const float* as = As[buf];
    const float* bs = Bs[buf];
    const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int ks = 0; ks < FBK / 4; ++ks) {
      float a[FI], b[FI];
#pragma unroll
      for (int i = 0; i < FI; ++i) a[i] = as[(4 * ks + kr) * LD + wm * (BM / 2) + i * 16 + cl];
#pragma unroll
      for (int j = 0; j < FI; ++j) b[j] = bs[(4 * ks + kr) * LD + wn * (BM / 2) + j * 16 + cl];
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FI; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    buf ^= 1;   // the next step writes the other buffer: one barrier per K step
  }
  // epilogue: lane holds rows 4(l/16)+r of column l%16 of each fragment
  const int rg = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + 4 * rg + r;
        const int n = n0 + wn * (BM / 2) + j * 16 + cl;
        if (m >= M || n >= N) continue;
        float v = acc[i][j][r];
        if (ep.mode == 1) {
          ep.out[(int64_t)z * ep.slab_stride + (int64_t)m * N + n] = v;
        } else {
          if (ep.bias && n < ep.bias_n) v += ep.bias[n];
          if (ep.relu) v = fmaxf(v, 0.f);
          if (ep.mask && !(ep.mask[(int64_t)m * ep.ldm + n] > 0.f)) v = 0.f;
          ep.out[(int64_t)m * ep.ldc + n] = v;
        }
      }
}

// 128x128 tiles when both dims fill them and the problem has >= 4 per CU (incl. splits):
// half the L2 operand traffic per MAC of the 64x64 tile.  Measured (profiles/r3/fp32): the
// reference CNN's local3 forward 1.12 -> 0.95 ms, dgrad unchanged, and its split-K wgrad
// (600 tiles) SLOWER (1.29 -> 1.43 ms), hence the 4-per-CU threshold.  MNISTX_F32_TILE=64
// forces the small tile.
template <class AL, class BL>
hipError_t launch_f32(const AL& A, const BL& Bm, int M, int N, int K, int splits, const EpiF& ep, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  splits = splits < 1 ? 1 : splits;
  int kc = (K + splits - 1) / splits;
  kc = (kc + FBK - 1) / FBK * FBK;
  const int64_t big = (int64_t)((M + 127) / 128) * ((N + 127) / 128) * splits;
  if (big >= 1024 && N >= 128 && M >= 128) {
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
    hipLaunchKernelGGL((gemm_f32_k<128, AL, BL>), dim3(tiles, splits), dim3(FNT), 0, st, A, Bm, M, N, K, kc, ep);
  } else {
    const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
    hipLaunchKernelGGL((gemm_f32_k<64, AL, BL>), dim3(tiles, splits), dim3(FNT), 0, st, A, Bm, M, N, K, kc, ep);
  }
  return hipGetLastError();
}

EpiF store_epi(float* out, int ldc, const float* bias, int bias_n, int relu, const float* mask, int ldm) {
  return EpiF{out, ldc, 0, bias, bias_n, relu, mask, ldm, 0};
}
EpiF slab_epi(float* slab, int64_t stride) { return EpiF{slab, 0, 1, nullptr, 0, 0, nullptr, 0, stride}; }

// ---------------------------------------------------------------- max-pool 2x2/2 SAME
__global__ void maxpool_f32_fwd_k(const float* __restrict__ x, int Nb, int H, int W, int C, int OH, int OW,
                                  float* __restrict__ y, uint8_t* __restrict__ arg) {
  const int64_t total = (int64_t)Nb * OH * OW * C;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const int64_t pix = t / C;
    const int ow = (int)(pix % OW);
    const int oh = (int)((pix / OW) % OH);
    const int64_t n = pix / ((int64_t)OW * OH);
    float best = -INFINITY;
    int bi = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int ih = 2 * oh + (d >> 1), iw = 2 * ow + (d & 1);
      if (ih < H && iw < W) {
        const float v = x[((n * H + ih) * W + iw) * C + c];
        if (v > best) { best = v; bi = d; }   // first maximum wins (TF MaxPool)
      }
    }
    y[t] = best;
    arg[t] = (uint8_t)bi;
  }
}

// dx at the argmax position gets dy; relu_mask: the pooled input was a ReLU output, so
// its gradient also needs y > 0 (the max of a ReLU window is > 0 iff its winner is)
__global__ void maxpool_f32_bwd_k(const float* __restrict__ dy, const uint8_t* __restrict__ arg,
                                  const float* __restrict__ y, int relu_mask, int Nb, int H, int W, int C, int OH,
                                  int OW, float* __restrict__ dx) {
  const int64_t total = (int64_t)Nb * H * W * C;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const int64_t pix = t / C;
    const int iw = (int)(pix % W);
    const int ih = (int)((pix / W) % H);
    const int64_t n = pix / ((int64_t)W * H);
    const int oh = ih >> 1, ow = iw >> 1, d = ((ih & 1) << 1) | (iw & 1);
    const int64_t o = ((n * OH + oh) * OW + ow) * C + c;
    float g = 0.f;
    if (arg[o] == d && (!relu_mask || y[o] > 0.f)) g = dy[o];
    dx[t] = g;
  }
}

// ---------------------------------------------------------------- LRN across channels (C <= 64)
// y = x * (bias + alpha * sum_{|j-c| <= r} x_j^2)^-beta   (tf.nn.local_response_normalization)
// One thread per (pixel, channel); a block stages 256 / C whole pixels in LDS, so the
// window sums read neighbours from LDS and every global access is coalesced.
constexpr int LRN_MAXC = 64;

__global__ __launch_bounds__(256) void lrn_f32_fwd_k(const float* __restrict__ x, int64_t P, int C, int r,
                                                     float bias, float alpha, float beta, float* __restrict__ y) {
  __shared__ float xs[256];
  const int PB = 256 / C, t = threadIdx.x, pl = t / C, c = t - pl * C;
  for (int64_t p0 = (int64_t)blockIdx.x * PB; p0 < P; p0 += (int64_t)gridDim.x * PB) {
    const bool ok = pl < PB && p0 + pl < P;
    __syncthreads();
    xs[t] = ok ? x[p0 * C + t] : 0.f;
    __syncthreads();
    if (ok) {
      float s = 0.f;
      for (int j = max(0, c - r); j <= min(C - 1, c + r); ++j) s = fmaf(xs[pl * C + j], xs[pl * C + j], s);
      y[p0 * C + t] = xs[t] * pow_neg(fmaf(alpha, s, bias), beta);
    }
  }
}

// dx_i = dy_i N_i^-b - 2 a b x_i sum_{j: |i-j| <= r} dy_j x_j N_j^(-b-1),  N_j = bias + a sum x^2
// relu_mask: x is a ReLU output, dx_i = 0 where x_i <= 0
__global__ __launch_bounds__(256) void lrn_f32_bwd_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                     int64_t P, int C, int r, float bias, float alpha, float beta,
                                                     int relu_mask, float* __restrict__ dx) {
  __shared__ float xs[256], ts[256];
  const int PB = 256 / C, t = threadIdx.x, pl = t / C, c = t - pl * C;
  for (int64_t p0 = (int64_t)blockIdx.x * PB; p0 < P; p0 += (int64_t)gridDim.x * PB) {
    const bool ok = pl < PB && p0 + pl < P;
    __syncthreads();
    const float xv = ok ? x[p0 * C + t] : 0.f, g = ok ? dy[p0 * C + t] : 0.f;
    xs[t] = xv;
    __syncthreads();
    float s = 0.f;
    if (ok)
      for (int j = max(0, c - r); j <= min(C - 1, c + r); ++j) s = fmaf(xs[pl * C + j], xs[pl * C + j], s);
    const float n = fmaf(alpha, s, bias);
    float nb, nb1;
    pow_neg2(n, beta, nb, nb1);
    ts[t] = g * xv * nb1;
    __syncthreads();
    if (ok) {
      float u = 0.f;
      for (int j = max(0, c - r); j <= min(C - 1, c + r); ++j) u += ts[pl * C + j];
      float d = g * nb - 2.f * alpha * beta * xv * u;
      if (relu_mask && !(xv > 0.f)) d = 0.f;
      dx[p0 * C + t] = d;
    }
  }
}

// ---------------------------------------------------------------- softmax cross-entropy, fp32 gradient
__global__ __launch_bounds__(256) void softmax_ce_f32_k(const float* __restrict__ logits, int ldl,
                                                        const int32_t* __restrict__ labels, int B, int NC,
                                                        float scale, float* __restrict__ dl, int ldd,
                                                        float* __restrict__ stats, float* __restrict__ probs,
                                                        float* __restrict__ work) {
  float loss = 0.f, corr = 0.f, bad = 0.f;
  for (int row = blockIdx.x * 256 + threadIdx.x; row < B; row += gridDim.x * 256) {
    const float* l = logits + (int64_t)row * ldl;
    float mx = -INFINITY;
    for (int c = 0; c < NC; ++c) mx = fmaxf(mx, l[c]);
    float se = 0.f;
    for (int c = 0; c < NC; ++c) se += expf(l[c] - mx);
    const float inv = 1.f / se;
    const int lab = labels ? labels[row] : -1;
    if (labels) {
      const float ll = l[lab];
      const float lo = -(ll - mx - logf(se));
      loss += lo;
      corr += ll >= mx ? 1.f : 0.f;
      if (!isfinite(lo)) bad = 1.f;
    }
    if (dl)
      for (int c = 0; c < ldd; ++c)
        dl[(int64_t)row * ldd + c] = c < NC ? (expf(l[c] - mx) * inv - (c == lab ? 1.f : 0.f)) * scale : 0.f;
    if (probs)
      for (int c = 0; c < NC; ++c) probs[(int64_t)row * NC + c] = expf(l[c] - mx) * inv;
  }
  if (stats) ce_block_stats<4>(loss, corr, bad, stats, work);
}

// ---------------------------------------------------------------- u8 batch -> fp32 x/255 - 0.5
__global__ void prep_images_f32_k(const uint8_t* __restrict__ src, const int64_t* __restrict__ idx,
                                  const int32_t* __restrict__ lab_src, int B, int HW, int Csrc, int Cdst,
                                  float* __restrict__ out, int32_t* __restrict__ lab_out) {
  const int64_t total = (int64_t)B * HW * Cdst;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(t % Cdst);
    const int64_t pix = t / Cdst;
    const int b = (int)(pix / HW), q = (int)(pix % HW);
    const int cs = Csrc == Cdst ? c : 0;   // 1 -> Cdst channel replication
    out[t] = u8_norm(src[(idx[b] * HW + q) * Csrc + cs]);
    if (lab_out && t < B) lab_out[t] = lab_src[idx[t]];
  }
}

// ---------------------------------------------------------------- vectorised pool / LRN
// One lane per (pool window | pixel, 4 channels): 16-byte loads and stores, 32-bit
// FastDiv index math.  The per-element kernels above did three 64-bit divisions per
// element (1.17 ms for the 411 MB pool1 gradient at B = 16384, ~10x its HBM time);
// they remain the fallback for odd sizes / unaligned buffers.
__global__ __launch_bounds__(256) void maxpool_f32_fwd_v4_k(const float* __restrict__ x, int total, FastDiv fC4,
                                                            FastDiv fOW, FastDiv fOH, int C, float* __restrict__ y,
                                                            uint32_t* __restrict__ arg) {
  const int W = 2 * (int)fOW.d;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int win = fC4.div(t), cv = fC4.mod(t, win);
    const int r = fOW.div(win), ow = fOW.mod(win, r);
    const int n = fOH.div(r), oh = fOH.mod(r, n);
    const int64_t base = (((int64_t)n * 2 * fOH.d + 2 * oh) * W + 2 * ow) * C + 4 * cv;
    f32x4 v[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) v[d] = *(const f32x4*)(x + base + ((d >> 1) * W + (d & 1)) * C);
    f32x4 best = v[0];
    uint32_t code = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t bi = 0;
#pragma unroll
      for (int d = 1; d < 4; ++d)
        if (v[d][j] > best[j]) { best[j] = v[d][j]; bi = d; }   // first maximum wins (TF MaxPool)
      code |= bi << (8 * j);
    }
    *(f32x4*)(y + (int64_t)t * 4) = best;
    arg[t] = code;
  }
}

__global__ __launch_bounds__(256) void maxpool_f32_bwd_v4_k(const float* __restrict__ dy,
                                                            const uint32_t* __restrict__ arg,
                                                            const float* __restrict__ y, int relu_mask, int total,
                                                            FastDiv fC4, FastDiv fOW, FastDiv fOH, int C,
                                                            float* __restrict__ dx) {
  const int W = 2 * (int)fOW.d;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int win = fC4.div(t), cv = fC4.mod(t, win);
    const int r = fOW.div(win), ow = fOW.mod(win, r);
    const int n = fOH.div(r), oh = fOH.mod(r, n);
    const int64_t base = (((int64_t)n * 2 * fOH.d + 2 * oh) * W + 2 * ow) * C + 4 * cv;
    const f32x4 g = *(const f32x4*)(dy + (int64_t)t * 4);
    const uint32_t a = arg[t];
    f32x4 yy = {1.f, 1.f, 1.f, 1.f};
    if (relu_mask) yy = *(const f32x4*)(y + (int64_t)t * 4);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (((a >> (8 * j)) & 0xffu) == (uint32_t)d && yy[j] > 0.f) ? g[j] : 0.f;
      *(f32x4*)(dx + base + ((d >> 1) * W + (d & 1)) * C) = o;
    }
  }
}

// LRN with 4 channels per lane (lrn_f32.h: the C/4 lanes of a pixel adjacent inside one
// 16-lane DPP row, neighbours by DPP row shifts).
__global__ __launch_bounds__(256) void lrn_f32_fwd_v4_k(const float* __restrict__ x, int total, int G, int r,
                                                        float bias, float alpha, float beta, float* __restrict__ y) {
  // uniform trip count over whole waves: every lane takes part in the DPP exchanges
  for (int b0 = blockIdx.x * blockDim.x; b0 < total; b0 += gridDim.x * blockDim.x) {
    const int t = b0 + threadIdx.x;
    const bool ok = t < total;
    const int c4 = threadIdx.x % G;
    const f32x4 v = ok ? *(const f32x4*)(x + (int64_t)t * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 s = win4(v * v, c4, G, r);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[j] * pow_neg(fmaf(alpha, s[j], bias), beta);
    if (ok) *(f32x4*)(y + (int64_t)t * 4) = o;
  }
}

__global__ __launch_bounds__(256) void lrn_f32_bwd_v4_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                        int total, int G, int r, float bias, float alpha, float beta,
                                                        int relu_mask, float* __restrict__ dx) {
  for (int b0 = blockIdx.x * blockDim.x; b0 < total; b0 += gridDim.x * blockDim.x) {
    const int t = b0 + threadIdx.x;
    const bool ok = t < total;
    const int c4 = threadIdx.x % G;
    const f32x4 v = ok ? *(const f32x4*)(x + (int64_t)t * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 g = ok ? *(const f32x4*)(dy + (int64_t)t * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 o = lrn_f32_bwd4(v, g, c4, G, r, bias, alpha, beta, relu_mask);
    if (ok) *(f32x4*)(dx + (int64_t)t * 4) = o;
  }
}

// LRN then 2x2/2 max-pool in one pass (the reference's norm2 -> pool2, mnist_input.py:166-172):
// the LRN output (the 822 MB conv2-sized tensor at B = 16384) is never written.  Thread =
// (pooled pixel, 4 channels), the C/4 lanes of a pixel in one DPP row; each of the 4 window
// positions is normalised exactly as lrn_f32_fwd_v4_k does and the max taken in position
// order with the first maximum winning (maxpool_f32_fwd_v4_k), so outputs and codes are
// bitwise the unfused pair's.
__global__ __launch_bounds__(256) void lrn_pool_f32_fwd_k(const float* __restrict__ x, int total, FastDiv fC4,
                                                          FastDiv fOW, FastDiv fOH, int C, int r, float bias,
                                                          float alpha, float beta, float* __restrict__ y,
                                                          uint32_t* __restrict__ arg) {
  const int W = 2 * (int)fOW.d, G = (int)fC4.d;
  for (int b0 = blockIdx.x * blockDim.x; b0 < total; b0 += gridDim.x * blockDim.x) {
    const int t = b0 + threadIdx.x;
    const bool ok = t < total;
    const int tt = ok ? t : total - 1;
    const int win = fC4.div(tt), cv = fC4.mod(tt, win);
    const int rr = fOW.div(win), ow = fOW.mod(win, rr);
    const int n = fOH.div(rr), oh = fOH.mod(rr, n);
    const int64_t base = (((int64_t)n * 2 * fOH.d + 2 * oh) * W + 2 * ow) * C + 4 * cv;
    f32x4 best = {0.f, 0.f, 0.f, 0.f};
    uint32_t code = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const f32x4 v = ok ? *(const f32x4*)(x + base + ((d >> 1) * W + (d & 1)) * C) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 sq = v * v;
      const f32x4 sw = win4(sq, threadIdx.x % G, G, r);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float o = v[j] * pow_neg(fmaf(alpha, sw[j], bias), beta);
        if (d == 0 || o > best[j]) {
          best[j] = o;
          code = (code & ~(0xffu << (8 * j))) | ((uint32_t)d << (8 * j));
        }
      }
    }
    if (ok) {
      *(f32x4*)(y + (int64_t)t * 4) = best;
      arg[t] = code;
    }
  }
}

// the backward of that pair: un-pool dL/d pool into the LRN output gradient of each window
// position (the code's position only) and run the LRN backward there (lrn_f32_bwd_v4_k's
// arithmetic), writing dL/d(LRN input) once -- the unpooled gradient is never stored.
__global__ __launch_bounds__(256) void lrn_pool_f32_bwd_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                          const uint32_t* __restrict__ arg, int total, FastDiv fC4,
                                                          FastDiv fOW, FastDiv fOH, int C, int r, float bias,
                                                          float alpha, float beta, int relu_mask,
                                                          float* __restrict__ dx) {
  const int W = 2 * (int)fOW.d, G = (int)fC4.d;
  for (int b0 = blockIdx.x * blockDim.x; b0 < total; b0 += gridDim.x * blockDim.x) {
    const int t = b0 + threadIdx.x;
    const bool ok = t < total;
    const int tt = ok ? t : total - 1;
    const int win = fC4.div(tt), cv = fC4.mod(tt, win);
    const int rr = fOW.div(win), ow = fOW.mod(win, rr);
    const int n = fOH.div(rr), oh = fOH.mod(rr, n);
    const int64_t base = (((int64_t)n * 2 * fOH.d + 2 * oh) * W + 2 * ow) * C + 4 * cv;
    const f32x4 gp = ok ? *(const f32x4*)(dy + (int64_t)t * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    const uint32_t a = ok ? arg[t] : 0u;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int64_t off = base + ((d >> 1) * W + (d & 1)) * C;
      const f32x4 v = ok ? *(const f32x4*)(x + off) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 g;
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = ((a >> (8 * j)) & 0xffu) == (uint32_t)d ? gp[j] : 0.f;
      // the shared LRN backward (no FMA contraction): bitwise the unfused LRNF + PoolF pair
      const f32x4 o = lrn_f32_bwd4(v, g, threadIdx.x % G, G, r, bias, alpha, beta, relu_mask);
      if (ok) *(f32x4*)(dx + off) = o;
    }
  }
}

int ew_grid(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

}  // namespace

// ---------------------------------------------------------------- host launchers
// The local3-sized GEMMs (>= one round of 256 x 256 tiles) run on gemm256.hip's fp32 LDS-DMA
// kernel; everything smaller stays on gemm_f32_k.
static bool al16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

hipError_t f32_dense_fwd(const float* x, const float* w, int M, int N, int K, const float* bias, int bias_n, int relu,
                         float* y, int ldy, hipStream_t st) {
  if (gemm256f_ok(M, N, K) && (ldy & 3) == 0 && al16p(x) && al16p(w) && al16p(y))
    return gemm256f_fwd(x, w, M, N, K, bias, bias_n, relu, y, ldy, st);
  return launch_f32(StridedF<true>{x, M, K, K, -1}, StridedF<false>{w, N, K, N, -1}, M, N, K, 1,
                    store_epi(y, ldy, bias, bias_n, relu, nullptr, 0), st);
}

hipError_t f32_dense_dgrad(const float* dy, const float* w, int M, int Din, int Dout, const float* mask, float* dx,
                           hipStream_t st) {
  // dx[m][i] = sum_o dy[m][o] W[i][o]
  if (gemm256f_ok(M, Din, Dout) && al16p(dy) && al16p(w) && al16p(dx) && al16p(mask))
    return gemm256f_dgrad(dy, w, M, Din, Dout, mask, dx, st);
  return launch_f32(StridedF<true>{dy, M, Dout, Dout, -1}, StridedF<true>{w, Din, Dout, Dout, -1}, M, Din, Dout, 1,
                    store_epi(dx, Din, nullptr, 0, 0, mask, Din), st);
}

int f32_wgrad_splits_cap(int Din, int Dout, int B) {
  const int cus = gemm256_cus();
  return cus > 0 ? gemm256f_wgrad_splits(Din, Dout, B, cus) : 0;
}

hipError_t f32_dense_wgrad(const float* x, const float* dy, int B, int Din, int Dout, int splits, float* slab,
                           hipStream_t st, int* used) {
  // slab[z][Din + 1][Dout]: rows < Din = x^T dy, row Din = column sums of dy (bias)
  if (used) {
    *used = splits;
    const int s2 = f32_wgrad_splits_cap(Din, Dout, B);
    if (s2 > 0 && s2 <= splits && al16p(x) && al16p(dy) && al16p(slab)) {
      *used = s2;
      return gemm256f_wgrad(x, dy, B, Din, Dout, s2, slab, st);
    }
  }
  return launch_f32(StridedF<false>{x, Din, B, Din, Din}, StridedF<false>{dy, Dout, B, Dout, -1}, Din + 1, Dout, B,
                    splits, slab_epi(slab, (int64_t)(Din + 1) * Dout), st);
}

hipError_t f32_conv_fwd(const float* x, const float* w, int Nb, int H, int W, int C, int OH, int OW, int KH, int KW,
                        int ph, int pw, int Cout, const float* bias, int relu, float* y, hipStream_t st) {
  if (f32_conv1_ok(H, W, C, OH, OW, KH, KW, ph, pw, Cout) && (reinterpret_cast<uintptr_t>(y) & 15) == 0)
    return f32_conv1_fwd(x, w, Nb, bias, relu, y, st);
  if (f32_halo_fwd_ok(H, W, C, OH, OW, KH, KW, ph, pw, Cout) && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0)
    return f32_halo_fwd(x, w, Nb, C, Cout, bias, relu, y, st);
  const int M = Nb * OH * OW, K = KH * KW * C;
  const Im2colF A{x, H, W, C, OH, OW, KW, ph, pw, M, K, FastDiv(OH * OW), FastDiv(OW), FastDiv(C), FastDiv(KW)};
  return launch_f32(A, StridedF<false>{w, Cout, K, Cout, -1}, M, Cout, K,
                    1, store_epi(y, Cout, bias, Cout, relu, nullptr, 0), st);
}

hipError_t f32_conv_dgrad(const float* dy, const float* w, int Nb, int OH, int OW, int Cout, int H, int W, int KH,
                          int KW, int ph, int pw, int Cin, const float* mask, float* dx, hipStream_t st) {
  if (f32_halo_dgrad_ok(OH, OW, Cout, H, W, KH, KW, ph, pw, Cin) && (reinterpret_cast<uintptr_t>(dy) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(dx) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(mask) & 15) == 0)
    return f32_halo_dgrad(dy, w, Nb, Cout, Cin, mask, dx, st);
  const int M = Nb * H * W, K = KH * KW * Cout;
  const DyIm2colF A{dy, H, W, OH, OW, Cout, KW, ph, pw, M, K, FastDiv(H * W), FastDiv(W), FastDiv(Cout), FastDiv(KW)};
  return launch_f32(A, WFlipF{w, Cin, Cout, K, FastDiv(Cout)}, M, Cin, K, 1,
                    store_epi(dx, Cin, nullptr, 0, 0, mask, Cin), st);
}

hipError_t f32_conv_wgrad(const float* x, const float* dy, int Nb, int H, int W, int C, int OH, int OW, int KH,
                          int KW, int ph, int pw, int Cout, int splits, float* slab, hipStream_t st) {
  // slab[z][KH*KW*C + 1][Cout], row KH*KW*C = bias
  if (f32_conv1_ok(H, W, C, OH, OW, KH, KW, ph, pw, Cout))
    return f32_conv1_wgrad(x, dy, Nb, splits, slab, st);   // one partial per workgroup, `splits` workgroups
  if (f32_halo_wgrad_ok(H, W, C, OH, OW, KH, KW, ph, pw, Cout) && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(dy) & 15) == 0)
    return f32_halo_wgrad(x, dy, Nb, splits, slab, st);   // one partial per workgroup, `splits` workgroups
  const int P = Nb * OH * OW, Mr = KH * KW * C;
  const Im2colTF A{x, H, W, C, OH, OW, KW, ph, pw, P, Mr, FastDiv(OH * OW), FastDiv(OW), FastDiv(C), FastDiv(KW)};
  return launch_f32(A, StridedF<false>{dy, Cout, P, Cout, -1}, Mr + 1,
                    Cout, P, splits, slab_epi(slab, (int64_t)(Mr + 1) * Cout), st);
}

static bool al16h(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static bool pool_v4_ok(int64_t nwin, int H, int W, int C, int OH, int OW) {
  return H == 2 * OH && W == 2 * OW && C % 4 == 0 && nwin * (C / 4) < (int64_t)1 << 30;
}

hipError_t f32_maxpool_fwd(const float* x, int Nb, int H, int W, int C, int OH, int OW, float* y, uint8_t* arg,
                           hipStream_t st) {
  if (pool_v4_ok((int64_t)Nb * OH * OW, H, W, C, OH, OW) && al16h(x) && al16h(y) && al16h(arg)) {
    const int total = Nb * OH * OW * (C / 4);
    hipLaunchKernelGGL(maxpool_f32_fwd_v4_k, dim3(ew_grid(total)), dim3(256), 0, st, x, total, FastDiv(C / 4),
                       FastDiv(OW), FastDiv(OH), C, y, (uint32_t*)arg);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(maxpool_f32_fwd_k, dim3(ew_grid((int64_t)Nb * OH * OW * C)), dim3(256), 0, st, x, Nb, H, W, C,
                     OH, OW, y, arg);
  return hipGetLastError();
}

hipError_t f32_maxpool_bwd(const float* dy, const uint8_t* arg, const float* y, int relu_mask, int Nb, int H, int W,
                           int C, int OH, int OW, float* dx, hipStream_t st) {
  if (pool_v4_ok((int64_t)Nb * OH * OW, H, W, C, OH, OW) && al16h(dy) && al16h(arg) && al16h(y) && al16h(dx)) {
    const int total = Nb * OH * OW * (C / 4);
    hipLaunchKernelGGL(maxpool_f32_bwd_v4_k, dim3(ew_grid(total)), dim3(256), 0, st, dy, (const uint32_t*)arg, y,
                       relu_mask, total, FastDiv(C / 4), FastDiv(OW), FastDiv(OH), C, dx);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(maxpool_f32_bwd_k, dim3(ew_grid((int64_t)Nb * H * W * C)), dim3(256), 0, st, dy, arg, y,
                     relu_mask, Nb, H, W, C, OH, OW, dx);
  return hipGetLastError();
}

hipError_t f32_lrn_fwd(const float* x, int64_t P, int C, int r, float bias, float alpha, float beta, float* y,
                       hipStream_t st) {
  if (C > LRN_MAXC || C < 1) return hipErrorInvalidValue;
  if ((C == 32 || C == 64) && r <= 4 && P * (C / 4) < ((int64_t)1 << 30) && al16h(x) && al16h(y)) {
    const int total = (int)(P * (C / 4));
    hipLaunchKernelGGL(lrn_f32_fwd_v4_k, dim3(ew_grid(total)), dim3(256), 0, st, x, total, C / 4, r, bias, alpha,
                       beta, y);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(lrn_f32_fwd_k, dim3(ew_grid(P * C)), dim3(256), 0, st, x, P, C, r, bias, alpha, beta, y);
  return hipGetLastError();
}

hipError_t f32_lrn_bwd(const float* x, const float* dy, int64_t P, int C, int r, float bias, float alpha, float beta,
                       int relu_mask, float* dx, hipStream_t st) {
  if (C > LRN_MAXC || C < 1) return hipErrorInvalidValue;
  if ((C == 32 || C == 64) && r <= 4 && P * (C / 4) < ((int64_t)1 << 30) && al16h(x) && al16h(dy) && al16h(dx)) {
    const int total = (int)(P * (C / 4));
    hipLaunchKernelGGL(lrn_f32_bwd_v4_k, dim3(ew_grid(total)), dim3(256), 0, st, x, dy, total, C / 4, r, bias, alpha,
                       beta, relu_mask, dx);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(lrn_f32_bwd_k, dim3(ew_grid(P * C)), dim3(256), 0, st, x, dy, P, C, r, bias, alpha, beta,
                     relu_mask, dx);
  return hipGetLastError();
}

bool f32_lrn_pool_ok(int H, int W, int C, int r) {
  return (C == 32 || C == 64) && r <= 4 && H % 2 == 0 && W % 2 == 0;
}
hipError_t f32_lrn_pool_fwd(const float* x, int Nb, int H, int W, int C, int r, float bias, float alpha, float beta,
                            float* y, uint8_t* arg, hipStream_t st) {
  const int OH = H / 2, OW = W / 2;
  if (!f32_lrn_pool_ok(H, W, C, r) || !al16h(x) || !al16h(y) || !al16h(arg) ||
      (int64_t)Nb * OH * OW * (C / 4) >= ((int64_t)1 << 30))
    return hipErrorInvalidValue;
  if (Nb <= 0) return hipSuccess;
  const int total = Nb * OH * OW * (C / 4);
  hipLaunchKernelGGL(lrn_pool_f32_fwd_k, dim3(ew_grid(total)), dim3(256), 0, st, x, total, FastDiv(C / 4), FastDiv(OW),
                     FastDiv(OH), C, r, bias, alpha, beta, y, (uint32_t*)arg);
  return hipGetLastError();
}
hipError_t f32_lrn_pool_bwd(const float* x, const float* dy, const uint8_t* arg, int Nb, int H, int W, int C, int r,
                            float bias, float alpha, float beta, int relu_mask, float* dx, hipStream_t st) {
  const int OH = H / 2, OW = W / 2;
  if (!f32_lrn_pool_ok(H, W, C, r) || !al16h(x) || !al16h(dy) || !al16h(arg) || !al16h(dx) ||
      (int64_t)Nb * OH * OW * (C / 4) >= ((int64_t)1 << 30))
    return hipErrorInvalidValue;
  if (Nb <= 0) return hipSuccess;
  const int total = Nb * OH * OW * (C / 4);
  hipLaunchKernelGGL(lrn_pool_f32_bwd_k, dim3(ew_grid(total)), dim3(256), 0, st, x, dy, (const uint32_t*)arg, total,
                     FastDiv(C / 4), FastDiv(OW), FastDiv(OH), C, r, bias, alpha, beta, relu_mask, dx);
  return hipGetLastError();
}

hipError_t f32_softmax_ce(const float* logits, int ldl, const int32_t* labels, int B, int NC, float scale, float* dl,
                          int ldd, float* stats, float* probs, float* work, hipStream_t st) {
  int nb = (B + 255) / 256;
  nb = nb < 1 ? 1 : (nb > CE_MAXB ? CE_MAXB : nb);
  hipLaunchKernelGGL(softmax_ce_f32_k, dim3(nb), dim3(256), 0, st, logits, ldl, labels, B, NC, scale, dl, ldd, stats,
                     probs, work);
  return hipGetLastError();
}

hipError_t f32_prep_images(const uint8_t* src, const int64_t* idx, const int32_t* lab_src, int B, int HW, int Csrc,
                           int Cdst, float* out, int32_t* lab_out, hipStream_t st) {
  hipLaunchKernelGGL(prep_images_f32_k, dim3(ew_grid((int64_t)B * HW * Cdst)), dim3(256), 0, st, src, idx, lab_src,
                     B, HW, Csrc, Cdst, out, lab_out);
  return hipGetLastError();
}

}  // namespace mnistx
