// Bandwidth-bound kernels of the MNIST step on gfx950:
//   input prep (K10), max-pool fwd/bwd (K6), LRN fwd/bwd (K7), softmax-CE (K8),
//   split-K slab reduce (K3 tail), fused optimizer + EMA + LR schedule (K9),
//   step finalisation (loss EMAs, global_step, NaN flag).
// All 16-byte vectorised over 8 bf16 channels (NHWC with channels padded to 8).
// Reference ops replaced: SURVEY.md §2.3 N6-N14 (mnist_input.py:37-39,149-172,
// 224-231,252-267,288-290).
#include "common.h"
#include "ce_stats.h"
#include "lrn_math.h"
#include "launchers.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <tuple>
#include <vector>

namespace mnistx {
namespace {

constexpr int TPB = 256;

inline int nblocks(int64_t n, int per_block = TPB, int cap = 1 << 20) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

// ------------------------------------------------------------------ epoch shuffle
// Stateless per-epoch permutation: position p of the (endless) sample stream maps
// to dataset row F_e(p mod N), e = p / N, where F_e is a 4-round keyed Feistel
// bijection on [0, 4^h) >= N restricted to [0, N) by cycle walking.  Replaces a
// device randperm (a radix sort: 0.23 ms per 1.08M-entry permutation, 0.70 ms at
// 8 ranks' 8.4M) with ~2 us of integer math per step, and makes the data order a
// pure function of (seed, position): resume seeks instead of replaying.
// data/device_loader.py::perm_positions is the bit-identical torch version.
DEV uint32_t mix32(uint32_t x) {
  x = (x ^ (x >> 16)) * 0x7feb352du;
  x = (x ^ (x >> 15)) * 0x846ca68bu;
  return x ^ (x >> 16);
}
DEV uint64_t feistel4(uint64_t x, const uint32_t* key, int h) {
  const uint64_t mask = (1ull << h) - 1;
  uint64_t L = x >> h, R = x & mask;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint64_t nR = L ^ ((uint64_t)mix32((uint32_t)R ^ key[r]) & mask);
    L = R;
    R = nR;
  }
  return (L << h) | R;
}
// lab_src / lab_out (optional): the labels of the chosen rows gathered in the same
// launch (the resident-dataset input modes need only the index and the labels).
DEV void perm_one(int i, int64_t* __restrict__ out, int64_t start, int n, int64_t N, uint32_t seed, int h,
                  const int32_t* __restrict__ lab_src, int32_t* __restrict__ lab_out) {
  if (i >= n) return;
  const int64_t p = start + i;
  const int64_t e = p / N;
  uint64_t x = (uint64_t)(p - e * N);
  const uint32_t ek = mix32((uint32_t)e ^ 0x9e3779b9u) ^ seed;
  uint32_t key[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) key[r] = mix32(ek + 0x85ebca77u * (uint32_t)(r + 1));
  do { x = feistel4(x, key, h); } while (x >= (uint64_t)N);
  out[i] = (int64_t)x;
  if (lab_out) lab_out[i] = lab_src[x];
}
__global__ void perm_positions_k(int64_t* __restrict__ out, int64_t start, int n, int64_t N, uint32_t seed, int h,
                                 const int32_t* __restrict__ lab_src, int32_t* __restrict__ lab_out) {
  perm_one(blockIdx.x * blockDim.x + threadIdx.x, out, start, n, N, seed, h, lab_src, lab_out);
}

// ------------------------------------------------------------------ K10 input prep
// out[b, p, c] = src[idx[b], p, c_src] / 255 - 0.5   (mnist_input.py:39)
__global__ void prep_images_k(const uint8_t* __restrict__ src, const int64_t* __restrict__ idx,
                              const int32_t* __restrict__ lab_src, int B, int HW, int Csrc, int Cdst,
                              bf16_t* __restrict__ out, int32_t* __restrict__ lab_out) {
  const int64_t per_img = (int64_t)HW * Cdst;  // multiple of 8 (HW = 784)
  const int64_t nvec = (int64_t)B * per_img / 8;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 8;
    const int64_t b = e / per_img;
    const int64_t w = e - b * per_img;
    const uint8_t* img = src + idx[b] * (int64_t)HW * Csrc;
    u32x4 o;
    if (Csrc == Cdst) {
      const uint8_t* s = img + w;
      uint32_t lo = *(const uint32_t*)s, hi = *(const uint32_t*)(s + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = u8_norm((lo >> (8 * j)) & 0xff);
        float c = u8_norm((hi >> (8 * j)) & 0xff);
        u4_set(o, j, f2bf(a));
        u4_set(o, j + 4, f2bf(c));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t ww = w + j;
        const int64_t p = ww / Cdst;
        const int c = (int)(ww - p * Cdst);
        const int cs = c < Csrc ? c : 0;  // 1 -> 3 channel replication
        u4_set(o, j, f2bf(u8_norm(img[p * Csrc + cs])));
      }
    }
    *(u32x4*)(out + e) = o;
  }
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (lab_out && t < B) lab_out[t] = lab_src[idx[t]];
}

// Hot path of K10 (28x28x1 -> 28x28x1): 16 pixels per thread = one 16-byte gather
// load and two 16-byte bf16 stores, 49 vectors per image, 32-bit index math with a
// constant divisor (the generic kernel above does a 64-bit divide per 8 pixels).
// One thread per image also copies the label.
constexpr int PREP_V = 784 / 16;
__global__ __launch_bounds__(256) void prep_images_784_k(const uint8_t* __restrict__ src,
                                                          const int64_t* __restrict__ idx,
                                                          const int32_t* __restrict__ lab_src, int B,
                                                          bf16_t* __restrict__ out, int32_t* __restrict__ lab_out) {
  const int nvec = B * PREP_V;
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += gridDim.x * blockDim.x) {
    const int b = v / PREP_V, w = v - b * PREP_V;
    const int64_t row = idx[b];
    const u32x4 px = *(const u32x4*)(src + row * 784 + 16 * w);
    u32x4 o0, o1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      o0[2 * j] = pack2(u8_norm(px[j] & 0xff), u8_norm((px[j] >> 8) & 0xff));
      o0[2 * j + 1] = pack2(u8_norm((px[j] >> 16) & 0xff), u8_norm(px[j] >> 24));
      o1[2 * j] = pack2(u8_norm(px[2 + j] & 0xff), u8_norm((px[2 + j] >> 8) & 0xff));
      o1[2 * j + 1] = pack2(u8_norm((px[2 + j] >> 16) & 0xff), u8_norm(px[2 + j] >> 24));
    }
    bf16_t* dst = out + (int64_t)b * 784 + 16 * w;
    *(u32x4*)dst = o0;
    *(u32x4*)(dst + 8) = o1;
    if (lab_out && w == 0) lab_out[b] = lab_src[row];
  }
}

// K10 hot path with the epoch shuffle fused in: the dataset row of batch entry b is
// the Feistel image of stream position start + b (perm_positions_k), computed by
// each thread (a few dozen integer ops) instead of by a separate launch + index array.
__global__ __launch_bounds__(256) void prep_images_784_perm_k(const uint8_t* __restrict__ src,
                                                               const int32_t* __restrict__ lab_src, int B,
                                                               int64_t start, int64_t N, uint32_t seed, int h,
                                                               bf16_t* __restrict__ out,
                                                               int32_t* __restrict__ lab_out) {
  const int nvec = B * PREP_V;
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += gridDim.x * blockDim.x) {
    const int b = v / PREP_V, w = v - b * PREP_V;
    const int64_t p = start + b;
    const int64_t e = p / N;
    uint64_t x = (uint64_t)(p - e * N);
    const uint32_t ek = mix32((uint32_t)e ^ 0x9e3779b9u) ^ seed;
    uint32_t key[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) key[r] = mix32(ek + 0x85ebca77u * (uint32_t)(r + 1));
    do { x = feistel4(x, key, h); } while (x >= (uint64_t)N);
    const int64_t row = (int64_t)x;
    const u32x4 px = *(const u32x4*)(src + row * 784 + 16 * w);
    u32x4 o0, o1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      o0[2 * j] = pack2(u8_norm(px[j] & 0xff), u8_norm((px[j] >> 8) & 0xff));
      o0[2 * j + 1] = pack2(u8_norm((px[j] >> 16) & 0xff), u8_norm(px[j] >> 24));
      o1[2 * j] = pack2(u8_norm(px[2 + j] & 0xff), u8_norm((px[2 + j] >> 8) & 0xff));
      o1[2 * j + 1] = pack2(u8_norm((px[2 + j] >> 16) & 0xff), u8_norm(px[2 + j] >> 24));
    }
    bf16_t* dst = out + (int64_t)b * 784 + 16 * w;
    *(u32x4*)dst = o0;
    *(u32x4*)(dst + 8) = o1;
    if (w == 0) lab_out[b] = lab_src[row];
  }
}

// ------------------------------------------------------------------ K6 max-pool 2x2/2 SAME
__global__ void maxpool_fwd_k(const bf16_t* __restrict__ x, int Nb, int H, int W, int C, int OH, int OW,
                              bf16_t* __restrict__ y, uint8_t* __restrict__ arg) {
  const int CV = C / 8;
  const int64_t total = (int64_t)Nb * OH * OW * CV;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    int64_t r = t / CV;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int ih = 2 * oh + (d >> 1), iw = 2 * ow + (d & 1);
      if (ih < H && iw < W) {
        const u32x4 v = *(const u32x4*)(x + (((int64_t)n * H + ih) * W + iw) * C + cv * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = u4_get(v, j);
          if (f > best[j]) { best[j] = f; bi[j] = d; }
        }
      }
    }
    u32x4 o;
    uint32_t a0 = 0, a1 = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u4_set(o, j, f2bf(best[j]));
      if (j < 4) a0 |= bi[j] << (8 * j);
      else a1 |= bi[j] << (8 * (j - 4));
    }
    const int64_t off = (((int64_t)n * OH + oh) * OW + ow) * C + cv * 8;
    *(u32x4*)(y + off) = o;
    *(u32x2*)(arg + off) = u32x2{a0, a1};
  }
}

__global__ void maxpool_bwd_k(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                              const bf16_t* __restrict__ y, int relu_mask, int Nb, int H, int W, int C, int OH,
                              int OW, bf16_t* __restrict__ dx) {
  const int CV = C / 8;
  const int64_t total = (int64_t)Nb * OH * OW * CV;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    int64_t r = t / CV;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    const int64_t off = (((int64_t)n * OH + oh) * OW + ow) * C + cv * 8;
    u32x4 g = *(const u32x4*)(dy + off);
    const u32x2 a = *(const u32x2*)(arg + off);
    if (relu_mask) {
      const u32x4 yv = *(const u32x4*)(y + off);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (!(u4_get(yv, j) > 0.f)) u4_set(g, j, 0);
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int ih = 2 * oh + (d >> 1), iw = 2 * ow + (d & 1);
      if (ih < H && iw < W) {
        u32x4 o = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t aj = ((j < 4 ? a[0] : a[1]) >> (8 * (j & 3))) & 0xff;
          if (aj == (uint32_t)d) u4_set(o, j, (bf16_t)((g[j >> 1] >> (16 * (j & 1))) & 0xffff));
        }
        *(u32x4*)(dx + (((int64_t)n * H + ih) * W + iw) * C + cv * 8) = o;
      }
    }
  }
}

// ------------------------------------------------------------------ K7 LRN (TF semantics)
// y[c] = x[c] * (bias + alpha * sum_{|c'-c|<=R} x[c']^2)^-beta
// Channel-parallel: each lane owns 8 channels (one 16-byte vector) of a pixel, the
// C/8 lanes of a pixel sit side by side inside one 16-lane DPP row, and the R
// channels a window needs from the neighbouring vectors come over DPP row shifts
// (zeroed at the pixel's first / last vector).  Loads and stores are fully
// coalesced 16-byte vectors and a lane needs ~40 VGPRs (the one-pixel-per-lane form
// held all C channels three times over: 2 waves/SIMD, 2-3x the HBM floor).
template <int C, int R>
__global__ __launch_bounds__(TPB) void lrn_fwd_k(const bf16_t* __restrict__ x, int64_t P, float bias, float alpha,
                                                 float beta, bf16_t* __restrict__ y) {
  constexpr int G = C / 8;
  const int64_t total = P * G;   // one 8-channel vector per lane; whole pixels per wave
  const int c8 = threadIdx.x % G;
  // uniform trip count: every lane takes part in the DPP exchanges
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < total; base += (int64_t)gridDim.x * TPB) {
    const int64_t t = base + threadIdx.x;
    const bool ok = t < total;
    const u32x4 xv = *(const u32x4*)(x + (ok ? t : 0) * 8);   // unconditional (clamped) load
    const u32x4 o = lrn_fwd8<G, R>(xv, c8, bias, alpha, beta);
    if (ok) *(u32x4*)(y + t * 8) = o;
  }
}

// dx[c] = dy[c] s[c]^-b - 2ab x[c] sum_{|c'-c|<=R} dy[c'] x[c'] s[c']^(-b-1)
template <int C, int R, bool B075 = false>
__global__ __launch_bounds__(TPB) void lrn_bwd_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                 int64_t P, float bias, float alpha, float beta, int relu_mask,
                                                 bf16_t* __restrict__ dx) {
  constexpr int G = C / 8;
  const int64_t total = P * G;
  const int c8 = threadIdx.x % G;
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < total; base += (int64_t)gridDim.x * TPB) {
    const int64_t t = base + threadIdx.x;
    const bool ok = t < total;
    const u32x4 xv = *(const u32x4*)(x + (ok ? t : 0) * 8);    // unconditional (clamped) loads
    const u32x4 gv = *(const u32x4*)(dy + (ok ? t : 0) * 8);
    const u32x4 o = lrn_bwd8<G, R, B075>(xv, gv, c8, bias, alpha, beta, relu_mask);
    if (ok) *(u32x4*)(dx + t * 8) = o;
  }
}

// ------------------------------------------------------------------ K7+K6 fused: LRN -> 2x2/2 max-pool
// The reference CNN's norm2 -> pool2 (mnist_input.py:168-172) as one pass: lane
// group = one pool window, lane = 8 channels of it; the LRN of the window's 4 pixels
// is computed in registers and only the pooled maximum (+ argmax byte) is written,
// so the full-resolution LRN output never goes to HBM (and is never re-read by the
// pool).  Pooling compares the bf16-rounded LRN values in window order, exactly
// like lrn_fwd + maxpool_fwd.  Backward: unpool dP through the argmax into the 4
// pixels' dY in registers and apply the LRN gradient directly (no dY image).
// LRNP_U pool windows per lane per iteration, the loads of both issued first: 142 -> 132 us
// at B = 16384 (the same unrolling of lrn_fwd_k, 4 vectors per lane, measured no change)
constexpr int LRNP_U = 2;
template <int C, int R>
__global__ __launch_bounds__(TPB) void lrn_pool_fwd_k(const bf16_t* __restrict__ x, int Nb, int H, int W, float bias,
                                                      float alpha, float beta, bf16_t* __restrict__ y,
                                                      uint8_t* __restrict__ arg) {
  constexpr int G = C / 8;
  const int OH = H / 2, OW = W / 2;
  const int64_t total = (int64_t)Nb * OH * OW * G;
  const int c8 = threadIdx.x % G;
  const int64_t step = (int64_t)gridDim.x * TPB;
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < total; base += LRNP_U * step) {
    // the windows' 4 pixel vectors: unconditional loads (clamped index), all in flight
    // before any math -- a load under `ok ?` made each wait for its own latency
    u32x4 xq[LRNP_U][4];
#pragma unroll
    for (int k = 0; k < LRNP_U; ++k) {
      const int64_t t = base + k * step + threadIdx.x;
      const int64_t win = t < total ? t / G : 0;
      const int ow = (int)(win % OW);
      const int64_t r = win / OW;
      const int oh = (int)(r % OH);
      const int64_t n = r / OH;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int ih = 2 * oh + (d >> 1), iw = 2 * ow + (d & 1);
        xq[k][d] = *(const u32x4*)(x + ((n * H + ih) * W + iw) * C + c8 * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < LRNP_U; ++k) {
      const int64_t t = base + k * step + threadIdx.x;
      float best[8];
      uint32_t bi[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float v[8], sq[8], s[8];
        unpack8(xq[k][d], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) sq[j] = v[j] * v[j];
        lane_window_sums<G, R>(sq, c8, s);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(f2bf(lrn_out(v[j], s[j], bias, alpha, beta)));
          if (f > best[j]) { best[j] = f; bi[j] = d; }
        }
      }
      if (t < total) {
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack2(best[2 * j], best[2 * j + 1]);
        const int64_t off = (t / G) * C + c8 * 8;
        *(u32x4*)(y + off) = o;
        *(u32x2*)(arg + off) = u32x2{bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                                     bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24)};
      }
    }
  }
}

template <int C, int R, bool B075 = false>
__global__ __launch_bounds__(TPB) void lrn_pool_bwd_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dP,
                                                      const uint8_t* __restrict__ arg, int Nb, int H, int W,
                                                      float bias, float alpha, float beta, int relu_mask,
                                                      bf16_t* __restrict__ dx) {
  constexpr int G = C / 8;
  const int OH = H / 2, OW = W / 2;
  const int64_t total = (int64_t)Nb * OH * OW * G;
  const int c8 = threadIdx.x % G;
  for (int64_t base = (int64_t)blockIdx.x * TPB; base < total; base += (int64_t)gridDim.x * TPB) {
    const int64_t t = base + threadIdx.x;
    const bool ok = t < total;
    const int64_t win = ok ? t / G : 0;
    const int ow = (int)(win % OW);
    const int64_t r = win / OW;
    const int oh = (int)(r % OH);
    const int64_t n = r / OH;
    const int64_t poff = win * C + c8 * 8;
    // unconditional loads (clamped index: win = 0 past the end), all issued up front
    const u32x4 pv = *(const u32x4*)(dP + poff);
    const u32x2 av = *(const u32x2*)(arg + poff);
    u32x4 xq[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int ih = 2 * oh + (d >> 1), iw = 2 * ow + (d & 1);
      xq[d] = *(const u32x4*)(x + ((n * H + ih) * W + iw) * C + c8 * 8);
    }
    float pg[8];
    unpack8(pv, pg);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int ih = 2 * oh + (d >> 1), iw = 2 * ow + (d & 1);
      const int64_t xoff = ((n * H + ih) * W + iw) * C + c8 * 8;
      float v[8], g[8];
      unpack8(xq[d], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t aj = ((j < 4 ? av[0] : av[1]) >> (8 * (j & 3))) & 0xffu;
        g[j] = aj == (uint32_t)d ? pg[j] : 0.f;          // max-unpool
      }
      const u32x4 o = lrn_bwd8_vals<G, R, B075>(v, g, c8, bias, alpha, beta, relu_mask);
      if (ok) *(u32x4*)(dx + xoff) = o;
    }
  }
}

// The reference CNN's norm2 -> pool2 (64 channels, 14 x 14, radius 4, post-ReLU input) on
// packed fp32.  lrn_pool_fwd_k / lrn_pool_bwd_k spend most of their issue slots on VALU work
// (profiles/r6/lrnpk/): 32-bit index math with the geometry as constants (no 64-bit divides),
// the element-wise LRN math of two vectors per lane as v_pk ops, and -- forward, input >= 0 --
// the 4-way max + first-argmax as an integer max of keys (bf16 bits << 16 | 3 - d: larger value,
// then earlier pixel, wins), instead of a compare and two selects per pixel.  Bitwise
// lrn_pool_fwd_k / lrn_pool_bwd_k (tests/test_kernels_gpu.py test_lrn_pool_packed).
constexpr int LP14_C = 64, LP14_G = 8, LP14_HW = 14, LP14_OW = 7, LP14_NWIN = 49;
template <int R>
__global__ __launch_bounds__(TPB) void lrn_pool14_fwd_k(const bf16_t* __restrict__ x, int Nb, float bias, float alpha,
                                                        float beta, bf16_t* __restrict__ y, uint8_t* __restrict__ arg) {
  constexpr int C = LP14_C, G = LP14_G, HW = LP14_HW;
  const unsigned total = (unsigned)Nb * LP14_NWIN * G;
  const int c8 = threadIdx.x % G;
  const unsigned step = gridDim.x * TPB;
  for (unsigned base = blockIdx.x * TPB; base < total; base += 2 * step) {
    u32x4 xq[2][4];
    unsigned wk[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const unsigned t = base + k * step + threadIdx.x;
      const unsigned win = t < total ? t / G : 0u;
      wk[k] = win;
      const unsigned n = win / LP14_NWIN, rem = win - n * LP14_NWIN, oh = rem / LP14_OW, ow = rem - oh * LP14_OW;
      const bf16_t* p = x + ((int64_t)((n * HW + 2 * oh) * HW + 2 * ow)) * C + c8 * 8;
      xq[k][0] = *(const u32x4*)p;
      xq[k][1] = *(const u32x4*)(p + C);
      xq[k][2] = *(const u32x4*)(p + HW * C);
      xq[k][3] = *(const u32x4*)(p + HW * C + C);
    }
    int best[2][8];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      f2 v[8], sq[8], s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = f2{u4_get(xq[0][d], j), u4_get(xq[1][d], j)};
        sq[j] = v[j] * v[j];
      }
      lane_window_sums2<G, R>(sq, c8, s);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f2 yv = lrn_out2(v[j], s[j], bias, alpha, beta);
        const uint32_t pk = pack2(yv.x, yv.y);   // window 0's bf16 low, window 1's high
        const int k0 = (int)((pk << 16) | (uint32_t)(3 - d)), k1 = (int)((pk & 0xffff0000u) | (uint32_t)(3 - d));
        best[0][j] = d == 0 ? k0 : max(best[0][j], k0);
        best[1][j] = d == 0 ? k1 : max(best[1][j], k1);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const unsigned t = base + k * step + threadIdx.x;
      if (t < total) {
        u32x4 o;
        uint32_t cw[2] = {0u, 0u};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = ((uint32_t)best[k][2 * j] >> 16) | ((uint32_t)best[k][2 * j + 1] & 0xffff0000u);
#pragma unroll
        for (int j = 0; j < 8; ++j) cw[j >> 2] |= (((uint32_t)best[k][j] & 3u) ^ 3u) << (8 * (j & 3));
        const int64_t off = (int64_t)wk[k] * C + c8 * 8;
        *(u32x4*)(y + off) = o;
        *(u32x2*)(arg + off) = u32x2{cw[0], cw[1]};
      }
    }
  }
}

template <int R>
__global__ __launch_bounds__(TPB) void lrn_pool14_bwd_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dP,
                                                        const uint8_t* __restrict__ arg, int Nb, float bias, float alpha,
                                                        float beta, int relu_mask, bf16_t* __restrict__ dx) {
  constexpr int C = LP14_C, G = LP14_G, HW = LP14_HW;
  const unsigned total = (unsigned)Nb * LP14_NWIN * G;
  const int c8 = threadIdx.x % G;
  for (unsigned base = blockIdx.x * TPB; base < total; base += gridDim.x * TPB) {
    const unsigned t = base + threadIdx.x;
    const bool ok = t < total;
    const unsigned win = ok ? t / G : 0u;
    const unsigned n = win / LP14_NWIN, rem = win - n * LP14_NWIN, oh = rem / LP14_OW, ow = rem - oh * LP14_OW;
    const int64_t poff = (int64_t)win * C + c8 * 8;
    const u32x4 pv = *(const u32x4*)(dP + poff);
    const u32x2 av = *(const u32x2*)(arg + poff);
    const int64_t x0 = ((int64_t)((n * HW + 2 * oh) * HW + 2 * ow)) * C + c8 * 8;
    u32x4 xq[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) xq[d] = *(const u32x4*)(x + x0 + ((d >> 1) * HW + (d & 1)) * C);
    float pg[8];
    unpack8(pv, pg);
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // pixels 2h, 2h + 1 (one row of the window) as the two halves
      f2 v[8], g[8], o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t aj = ((j < 4 ? av[0] : av[1]) >> (8 * (j & 3))) & 0xffu;
        v[j] = f2{u4_get(xq[2 * h], j), u4_get(xq[2 * h + 1], j)};
        g[j] = f2{aj == (uint32_t)(2 * h) ? pg[j] : 0.f, aj == (uint32_t)(2 * h + 1) ? pg[j] : 0.f};
      }
      lrn_bwd2_b075<G, R>(v, g, c8, bias, alpha, beta, relu_mask, o);
      if (ok) {
        *(u32x4*)(dx + x0 + (h * HW) * C) =
            u32x4{pack2(o[0].x, o[1].x), pack2(o[2].x, o[3].x), pack2(o[4].x, o[5].x), pack2(o[6].x, o[7].x)};
        *(u32x4*)(dx + x0 + (h * HW + 1) * C) =
            u32x4{pack2(o[0].y, o[1].y), pack2(o[2].y, o[3].y), pack2(o[4].y, o[5].y), pack2(o[6].y, o[7].y)};
      }
    }
  }
}

// ------------------------------------------------------------------ K8 softmax cross-entropy
// stats[0] += sum(-log p[label]) ; stats[1] += #(logit[label] == max) ; stats[2] = 1 if non-finite.
__global__ void softmax_ce_k(const float* __restrict__ logits, int ldl, const int32_t* __restrict__ labels, int B,
                             int NC, float scale, bf16_t* __restrict__ dl, int ldd, float* __restrict__ stats,
                             float* __restrict__ probs) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f, corr = 0.f;
  int bad = 0;
  if (row < B) {
    const float* l = logits + (int64_t)row * ldl;
    float mx = -INFINITY;
    for (int c = 0; c < NC; ++c) mx = fmaxf(mx, l[c]);
    float se = 0.f;
    for (int c = 0; c < NC; ++c) se += __expf(l[c] - mx);
    const float inv = 1.f / se;
    const int lab = labels ? labels[row] : -1;
    if (labels) {
      const float ll = l[lab];
      loss = -(ll - mx - __logf(se));
      corr = (ll >= mx) ? 1.f : 0.f;
      if (!isfinite(loss)) bad = 1;
    }
    if (dl) {
      bf16_t* d = dl + (int64_t)row * ldd;
      for (int c = 0; c < ldd; ++c) {
        float g = 0.f;
        if (c < NC) g = (__expf(l[c] - mx) * inv - (c == lab ? 1.f : 0.f)) * scale;
        d[c] = f2bf(g);
      }
    }
    if (probs)
      for (int c = 0; c < NC; ++c) probs[(int64_t)row * NC + c] = __expf(l[c] - mx) * inv;
  }
  if (stats) {
    loss = warp_sum(loss);
    corr = warp_sum(corr);
    bad = warp_sum_i(bad);
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&stats[0], loss);
      atomicAdd(&stats[1], corr);
      if (bad) stats[2] = 1.f;
    }
  }
}

// Row-vectorized variant for padded logit rows of LD = 16 / 32 floats (the
// classifier output is padded to >= 16 columns): one thread per row, f32x4 loads,
// 16-byte bf16 stores.  Statistics: warp + block reduction, then either one
// atomic per block or -- with a workspace -- per-block partials combined by the
// last block to finish (ticket counter) in block order: bitwise deterministic.
template <int LD>
__global__ __launch_bounds__(256) void softmax_ce_rows_k(const float* __restrict__ logits,
                                                         const int32_t* __restrict__ labels, int B, int NC,
                                                         float scale, bf16_t* __restrict__ dl,
                                                         float* __restrict__ stats, float* __restrict__ probs,
                                                         float* __restrict__ work, int defer_stats,
                                                         float* __restrict__ dbias) {
  float loss = 0.f, corr = 0.f, bad = 0.f;
  float cs[LD];   // fp32 column sums of dlogits (dbias: the last layer's bias gradient partial)
#pragma unroll
  for (int c = 0; c < LD; ++c) cs[c] = 0.f;
  for (int row = blockIdx.x * 256 + threadIdx.x; row < B; row += gridDim.x * 256) {
    float l[LD];
#pragma unroll
    for (int v = 0; v < LD / 4; ++v) {
      const f32x4 t = *(const f32x4*)(logits + (int64_t)row * LD + 4 * v);
      l[4 * v] = t[0];
      l[4 * v + 1] = t[1];
      l[4 * v + 2] = t[2];
      l[4 * v + 3] = t[3];
    }
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < LD; ++c)
      if (c < NC) mx = fmaxf(mx, l[c]);
    float e[LD], se = 0.f;
#pragma unroll
    for (int c = 0; c < LD; ++c) {
      e[c] = c < NC ? __expf(l[c] - mx) : 0.f;
      se += e[c];
    }
    const float inv = 1.f / se;
    const int lab = labels ? labels[row] : -1;
    if (labels) {
      float ll = 0.f;
#pragma unroll
      for (int c = 0; c < LD; ++c) ll = (c == lab) ? l[c] : ll;
      const float lo = -(ll - mx - __logf(se));
      loss += lo;
      corr += (ll >= mx) ? 1.f : 0.f;
      if (!isfinite(lo)) bad = 1.f;
    }
    if (dl) {
#pragma unroll
      for (int v = 0; v < LD / 8; ++v) {
        u32x4 o;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int c0 = 8 * v + 2 * h;
          const float g0 = c0 < NC ? (e[c0] * inv - (c0 == lab ? 1.f : 0.f)) * scale : 0.f;
          const float g1 = c0 + 1 < NC ? (e[c0 + 1] * inv - (c0 + 1 == lab ? 1.f : 0.f)) * scale : 0.f;
          o[h] = pack2(g0, g1);
          cs[c0] += g0;
          cs[c0 + 1] += g1;
        }
        *(u32x4*)(dl + (int64_t)row * LD + 8 * v) = o;
      }
    }
    if (probs)
#pragma unroll
      for (int c = 0; c < LD; ++c)
        if (c < NC) probs[(int64_t)row * NC + c] = e[c] * inv;
  }
  if (dl && dbias) block_colsum<4, LD>(cs, dbias + (int64_t)blockIdx.x * LD);
  if (stats) ce_block_stats<4>(loss, corr, bad, stats, work, defer_stats != 0);
}

// ------------------------------------------------------------------ split-K reduce
// dst weights [G][I][J] <- sum_s slab[s][g*Ipad + i][j] ; bias[j] <- sum_s slab[s][bias_row][j]
// Fixed summation order (deterministic).  Few slabs: one thread per output;
// many slabs (per-block partials of the fused conv kernels): one wave per
// output, lanes stride the slabs, then a wave reduction.
DEV int64_t reduce_row(int64_t t, int64_t nw, int G, int Ipad, int I, int J, int bias_row, int& j) {
  if (t < nw) {
    j = (int)(t % J);
    const int64_t gi = t / J;
    const int i = (int)(gi % I);
    const int g = (int)(gi / I);
    return (int64_t)g * Ipad + i;
  }
  j = (int)(t - nw);
  return bias_row;
}

__global__ void splitk_reduce_k(const float* __restrict__ slab, int S, int M, int N, int G, int Ipad, int I, int J,
                                int bias_row, float* __restrict__ wdst, float* __restrict__ bdst, float scale) {
  const int64_t nw = (int64_t)G * I * J;
  const int64_t total = nw + (bdst ? J : 0);
  const int64_t ss = (int64_t)M * N;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int j;
    const int64_t row = reduce_row(t, nw, G, Ipad, I, J, bias_row, j);
    float s = 0.f;
    const float* p = slab + row * N + j;
    for (int z = 0; z < S; ++z) s += p[z * ss];
    if (t < nw) wdst[t] = s * scale;
    else bdst[j] = s * scale;
  }
}

// Coalesced variant (N % 4 == 0), multi-tensor: ONE launch reduces the split-K
// slabs of several layers (RedTable, block ranges per descriptor), so a backward
// pass pays one reduce launch per gradient bucket instead of two per layer.
// Each lane owns 4 consecutive slab columns of one row (one 16-byte load per
// split), the 4 waves of a block take every 4th split, and the 4 partial sums
// are combined in a fixed order (deterministic).  Splits z*zstride, z < S, are
// summed (zstride > 1 after the partial pass).
constexpr int RED_CHUNK = 64;
constexpr int MAXRED = 8;
struct RedDesc {
  float* slab;
  float* wdst;
  float* bdst;
  int64_t nq;        // M * N / 4 quads per split
  int S, M, N, G, Ipad, I, J, bias_row;
  int qb, sb;        // reduce blocks; partial-pass split blocks (0 = no partial pass)
  int tick0;         // first ticket of this descriptor's quad blocks (fused launch, partial pass)
  float scale;
};
struct RedTable {
  RedDesc d[MAXRED];
  int pblk0[MAXRED + 1];  // partial-pass block prefix
  int rblk0[MAXRED + 1];  // reduce-pass block prefix
  int n;
};

DEV int red_find(const int* blk0, int n, int b) {
  int k = 0;
  for (int i = 1; i < n; ++i) k = b >= blk0[i] ? i : k;
  return k;
}

// the reduced quad qd (4 consecutive slab columns of one row) -> weight / bias destination
DEV void red_emit(const RedDesc& D, int64_t qd, const f32x4 t) {
  const int NQ = D.N >> 2;
  const int row = (int)(qd / NQ), j0 = (int)(qd - (int64_t)row * NQ) * 4;
  if (row == D.bias_row) {
    if (D.bdst)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (j0 + jj < D.J) D.bdst[j0 + jj] = t[jj] * D.scale;
    return;
  }
  const int g = row / D.Ipad, i = row - g * D.Ipad;
  if (g >= D.G || i >= D.I) return;
  float* d = D.wdst + ((int64_t)g * D.I + i) * D.J;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj)
    if (j0 + jj < D.J) d[j0 + jj] = t[jj] * D.scale;
}

// block b of the reduce pass: 64 quads, the 4 waves take every 4th split
DEV void red_reduce_block(const RedTable& tab, int b, f32x4 (*part)[64]) {
  const int k = red_find(tab.rblk0, tab.n, b);
  const RedDesc& D = tab.d[k];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nq = D.nq;
  const int64_t qd = (int64_t)(b - tab.rblk0[k]) * 64 + lane;
  const int S = D.sb ? D.sb : D.S;
  const int64_t zs = (int64_t)(D.sb ? RED_CHUNK : 1) * nq;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (qd < nq) {
    const f32x4* p = (const f32x4*)D.slab + qd;
    int z = wave;
    for (; z + 12 < S; z += 16) {
      const f32x4 a = p[z * zs], b2 = p[(z + 4) * zs];
      const f32x4 c = p[(z + 8) * zs], d = p[(z + 12) * zs];
      acc += a;
      acc += b2;
      acc += c;
      acc += d;
    }
    for (; z < S; z += 4) acc += p[z * zs];
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave != 0 || qd >= nq) return;
  red_emit(D, qd, ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]);
}

__global__ __launch_bounds__(256) void splitk_reduce4_k(RedTable tab) {
  __shared__ f32x4 part[4][64];
  red_reduce_block(tab, blockIdx.x, part);
}

// agent-scope relaxed store / load: written through to / read from the coherence point (no
// L2-wide write-back or invalidate: the fences those need cost ~18 us in the LeNet-5 step and
// ~190 us in the reference CNN's when every block of a launch ran one)
DEV void st_coh(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV float ld_coh(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// The last-block ticket ("fence-free" hand-off; splitk_fused4_k, fused_opt_k):
//   every block: st_coh its partials -> take_ticket -> the block whose ticket is the last one
//   reads every block's partials with ld_coh and combines them.
// Memory-model argument.  In the HIP / C++ model the relaxed stores and the relaxed fetch_add
// carry no happens-before, so the language alone does not order them; the protocol rests on the
// gfx950 lowering of agent-scope relaxed atomics, which is the hand-off the microarchitecture
// guide (MI355X_MICROARCH.md, "Valid forms", first table row) measures as correct without an
// acquire: (1) st_coh is `global_store_* sc1` -- written through past the XCD's L2 to the
// coherence point; (2) `s_waitcnt vmcnt(0)` before the ticket: every such store of the issuing
// wave has completed (vmcnt counts stores) before the atomic is issued, and the storing wave is
// the ticket-taking wave (thread 0's wave after a __syncthreads in fused_opt_k; wave 0, which
// did all the stores, in splitk_fused4_k); (3) the winner's ld_coh is `global_load_* sc1`,
// served from the coherence point, never from a stale L1 / L2 line; (4) the winner's loads are
// control-dependent on the ticket's returned value.  The compiler must not move (1) below the
// ticket or (3) above it: the s_waitcnt builtin is not a compiler barrier, so both sides get a
// signal fence (compiler-only: no instruction).  tests/test_isa_ticket.py disassembles the
// built code object and fails if any of sc1 stores, sc1 loads or the vmcnt(0) before the ticket
// atomic goes missing (a compiler or flag change); release/acquire fences instead cost +20 us
// (LeNet-5) / +180 us (reference CNN) per step (profiles/r5/launch_fusion/README.md).
DEV int take_ticket(int* t) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);
  const int v = __hip_atomic_fetch_add(t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  return v;
}

// First pass for many splits over a small output: block (q, s) of a descriptor
// sums splits [64 s, 64 s + 64) of its 64 quads and stores the sum IN PLACE in
// split 64 s (only this block reads or writes that range), so the reduce pass
// has S/64 splits.  COH: the store goes to the coherence point (fused launch).
template <bool COH>
DEV const RedDesc& red_partial_block(const RedTable& tab, int b, f32x4 (*part)[64], int& qblk, int64_t& qd_out) {
  const int k = red_find(tab.pblk0, tab.n, b);
  const RedDesc& D = tab.d[k];
  const int local = b - tab.pblk0[k];
  qblk = local % D.qb;
  const int sblk = local / D.qb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nq = D.nq;
  const int64_t qd = (int64_t)qblk * 64 + lane;
  qd_out = qd;
  const int z0 = sblk * RED_CHUNK, z1 = min(D.S, z0 + RED_CHUNK);
  f32x4* p = (f32x4*)D.slab + qd;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (qd < nq) {
    // all 16 loads in flight at once (a dependent chain was latency-bound), summed in order
    constexpr int PER = RED_CHUNK / 4;
    f32x4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int z = z0 + wave + 4 * u;
      v[u] = z < z1 ? p[(int64_t)z * nq] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) acc += v[u];
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && qd < nq) {
    const f32x4 t = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    if constexpr (COH) {
      float* d = (float*)(p + (int64_t)z0 * nq);
#pragma unroll
      for (int j = 0; j < 4; ++j) st_coh(d + j, t[j]);
    } else {
      p[(int64_t)z0 * nq] = t;
    }
  }
  return D;
}

__global__ __launch_bounds__(256) void splitk_partial4_k(RedTable tab) {
  __shared__ f32x4 part[4][64];
  int qblk;
  int64_t qd;
  red_partial_block<false>(tab, blockIdx.x, part, qblk, qd);
}

// ONE launch for both passes (the partial pass's blocks first, then the reduce blocks of the
// descriptors without one): wave 0 of the block that stores the last of a quad block's sb
// partials (coherent stores, then a ticket) sums them in split order (coherent loads) and
// emits.  The winner resets its ticket to 0.
__global__ __launch_bounds__(256) void splitk_fused4_k(RedTable tab, int* __restrict__ tickets) {
  __shared__ f32x4 part[4][64];
  const int pb = tab.pblk0[MAXRED];
  if ((int)blockIdx.x >= pb) {
    red_reduce_block(tab, (int)blockIdx.x - pb, part);
    return;
  }
  int qblk;
  int64_t qd;
  const RedDesc& D = red_partial_block<true>(tab, blockIdx.x, part, qblk, qd);
  if (threadIdx.x >= 64) return;   // wave 0 stored the partials
  int* tk = tickets + D.tick0 + qblk;
  int last = 0;
  if (threadIdx.x == 0) last = take_ticket(tk) == D.sb - 1;
  last = __shfl(last, 0, 64);
  if (!last) return;
  if (threadIdx.x == 0) *tk = 0;
  if (qd >= D.nq) return;
  const float* p = (const float*)((const f32x4*)D.slab + qd);
  const int64_t zs = (int64_t)RED_CHUNK * D.nq * 4;
  f32x4 acc = {ld_coh(p), ld_coh(p + 1), ld_coh(p + 2), ld_coh(p + 3)};
  for (int z = 1; z < D.sb; ++z) {
    const float* q = p + z * zs;
    acc += f32x4{ld_coh(q), ld_coh(q + 1), ld_coh(q + 2), ld_coh(q + 3)};
  }
  red_emit(D, qd, acc);
}

// ------------------------------------------------------------------ K9 fused optimizer
// Each workgroup owns one contiguous chunk of ONE segment (block -> segment
// table built on the host), so there is no per-element segment search and the
// L2 norm needed for the weight-decay loss is reduced in the workgroup and added
// with a single atomic per workgroup.
constexpr int MAXSEG = 16;
constexpr int FIN_WAVES = 4, FIN_MAXW = 64;
template <bool COH>
DEV void finalize_body(const FinArgs& f, float* wsum);
constexpr int OPT_EPT = 2;                       // elements per thread: one consecutive pair (fused_opt_k)
constexpr int OPT_CHUNK = TPB * OPT_EPT;         // elements per workgroup
struct SegTable {
  OptSeg s[MAXSEG];
  FastDiv fij[MAXSEG], fj[MAXSEG];   // I*J and J of each segment (bf16-copy index math)
  int blk0[MAXSEG + 1];
  int n;
  int l2n;                           // l2[0..l2n): per-tensor sums; l2[l2n + block]: partials
};

__global__ __launch_bounds__(TPB) void fused_opt_k(float* __restrict__ params, const float* __restrict__ grads,
                                                   float* __restrict__ mom, float* __restrict__ ema,
                                                   bf16_t* __restrict__ bf, SegTable tab,
                                                   const int64_t* __restrict__ step_p, OptParams op,
                                                   float* __restrict__ l2, FinArgs fin, PermJob pj) {
  __shared__ float red[TPB / 64];
  __shared__ float wsum[FIN_MAXW];
  __shared__ int last;
  const int nopt = pj.n > 0 ? pj.blk0 : (int)gridDim.x;   // optimizer blocks; the rest: the perm job
  if ((int)blockIdx.x >= nopt) {
    perm_one(((int)blockIdx.x - nopt) * TPB + threadIdx.x, pj.out, pj.start, pj.n, pj.N, pj.seed, pj.h, pj.lab_src,
             pj.lab_out);
    return;
  }
  if (op.guard && *op.guard != op.guard_want) {   // a stale / torn PS push: never applied
    if (blockIdx.x == 0 && threadIdx.x == 0) *op.guard_err = op.guard_id;
    return;
  }
  int si = 0;
  while (si + 1 < tab.n && (int)blockIdx.x >= tab.blk0[si + 1]) ++si;
  const OptSeg sg = tab.s[si];
  const int64_t step = *step_p;
  float lr = op.lr0;
  if (op.decay_steps > 0) lr *= powf(op.decay_rate, (float)(step / op.decay_steps));  // staircase
  float ema_d = 0.f;
  if (op.ema_max >= 0.f) ema_d = fminf(op.ema_max, (1.f + (float)step) / (10.f + (float)step));
  const int64_t lo = (int64_t)(blockIdx.x - tab.blk0[si]) * OPT_CHUNK;
  const int64_t ij = (int64_t)sg.I * sg.J;
  float sq = 0.f;
  // each thread owns a PAIR of consecutive elements (8-byte loads / stores of params, grads,
  // momentum and EMA; one 4-byte bf16 store when the pair stays in one row of the padded
  // copy), all loads issued before any use; the pair falls back to two scalar accesses in a
  // segment at an odd offset.  Out-of-range elements load element 0 and are never stored.
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const int64_t li0 = lo + 2 * (int64_t)threadIdx.x;
  const bool vec = (sg.off & 1) == 0 && li0 + 1 < sg.n;
  float pv[OPT_EPT], gv[OPT_EPT], mv[OPT_EPT], ev[OPT_EPT];
  if (vec) {
    const int64_t e = sg.off + li0;
    const f32x2_t p2 = *(const f32x2_t*)(params + e), g2 = *(const f32x2_t*)(grads + e);
    const f32x2_t m2 = op.use_momentum ? *(const f32x2_t*)(mom + e) : f32x2_t{0.f, 0.f};
    const f32x2_t e2 = op.ema_max >= 0.f ? *(const f32x2_t*)(ema + e) : f32x2_t{0.f, 0.f};
#pragma unroll
    for (int u = 0; u < OPT_EPT; ++u) {
      pv[u] = p2[u];
      gv[u] = g2[u];
      mv[u] = m2[u];
      ev[u] = e2[u];
    }
  } else {
#pragma unroll
    for (int u = 0; u < OPT_EPT; ++u) {
      const int64_t li = li0 + u;
      const int64_t e = sg.off + (li < sg.n ? li : 0);
      pv[u] = params[e];
      gv[u] = grads[e];
      mv[u] = op.use_momentum ? mom[e] : 0.f;
      ev[u] = op.ema_max >= 0.f ? ema[e] : 0.f;
    }
  }
  float po[OPT_EPT], mo[OPT_EPT], eo[OPT_EPT];
#pragma unroll
  for (int u = 0; u < OPT_EPT; ++u) {
    float p = pv[u];
    if (li0 + u < sg.n) sq += p * p;
    const float g = gv[u] * op.grad_scale + sg.wd * p;
    float upd = g;
    mo[u] = 0.f;
    if (op.use_momentum) {
      const float v = mv[u] * op.momentum + g;
      mo[u] = v;
      upd = op.nesterov ? g + op.momentum * v : v;
    }
    p -= lr * upd;
    po[u] = p;
    eo[u] = op.ema_max >= 0.f ? ev[u] - (1.f - ema_d) * (ev[u] - p) : 0.f;
  }
  if (vec) {
    const int64_t e = sg.off + li0;
    *(f32x2_t*)(params + e) = f32x2_t{po[0], po[1]};
    if (op.use_momentum) *(f32x2_t*)(mom + e) = f32x2_t{mo[0], mo[1]};
    if (op.ema_max >= 0.f) *(f32x2_t*)(ema + e) = f32x2_t{eo[0], eo[1]};
  } else {
#pragma unroll
    for (int u = 0; u < OPT_EPT; ++u) {
      if (li0 + u >= sg.n) continue;
      const int64_t e = sg.off + li0 + u;
      params[e] = po[u];
      if (op.use_momentum) mom[e] = mo[u];
      if (op.ema_max >= 0.f) ema[e] = eo[u];
    }
  }
  if (sg.bf_off >= 0) {
    // 32-bit magic-number divisions (segments < 2^31 elements): the 64-bit divides here
    // were most of this kernel's time on the 3.2M-element local3 weights
    int64_t bi[OPT_EPT];
    int jj0 = 0, ii0 = 0;
#pragma unroll
    for (int u = 0; u < OPT_EPT; ++u) {
      const int l32 = (int)(li0 + u);
      const int gg = tab.fij[si].div(l32);
      const int rem = l32 - gg * (int)ij;
      const int ii = tab.fj[si].div(rem), jj = rem - ii * sg.J;
      bi[u] = sg.bf_off + ((int64_t)gg * sg.Ip + ii) * sg.Jp + jj;
      if (u == 0) {
        jj0 = jj;
        ii0 = ii;
      }
    }
    const bf16_t b0 = f2bf(po[0]), b1 = f2bf(po[1]);
    if (vec && bi[1] == bi[0] + 1 && (bi[0] & 1) == 0) {
      *(uint32_t*)(bf + bi[0]) = (uint32_t)b0 | ((uint32_t)b1 << 16);
    } else {
      if (li0 < sg.n) bf[bi[0]] = b0;
      if (li0 + 1 < sg.n) bf[bi[1]] = b1;
    }
    if (sg.bft_off >= 0) {   // W^T copy (fused dense head): scattered 2-byte stores
      if (li0 < sg.n) bf[sg.bft_off + (int64_t)jj0 * sg.It + ii0] = b0;
      if (li0 + 1 < sg.n) {
        const int l32 = (int)(li0 + 1);
        const int gg = tab.fij[si].div(l32);
        const int rem = l32 - gg * (int)ij;
        const int ii = tab.fj[si].div(rem), jj = rem - ii * sg.J;
        bf[sg.bft_off + (int64_t)jj * sg.It + ii] = b1;
      }
    }
  }
  if (l2 && sg.track_l2) {
    // per-block partial, summed in block order by finalize_k: one float atomic per
    // block on ONE address serialised ~6.8K blocks (96 us of the reference CNN's
    // update) and made the weight-decay loss order-dependent
    sq = warp_sum(sq);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < TPB / 64; ++w) t += red[w];
      if (fin.ticket) st_coh(l2 + tab.l2n + blockIdx.x, t);
      else l2[tab.l2n + blockIdx.x] = t;
    }
  }
  if (!fin.ticket) return;
  // the step's finalize in this launch: the last block to take a ticket (thread 0, after its
  // coherent partial store) runs it, reading the partials coherently; every block has read
  // *step_p by now
  if (threadIdx.x == 0) last = take_ticket(fin.ticket) == nopt - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) *fin.ticket = 0;
  finalize_body<true>(fin, wsum);
}

// stats: [0] ce_sum acc [1] correct acc [2] nan flag [3] -
//        [4] ce_mean [5] accuracy [6] total_loss [7] steps done (float)
// loss_ema: n_ema x {biased, local_step, avg}  (TF zero-debiased EMA, decay 0.9:
//           mnist_input.py:288-290); order = weight losses..., cross_entropy, total_loss
static_assert(64 * FIN_WAVES == TPB, "finalize_body also runs as the last block of fused_opt_k");
// the body of finalize_k, run by one TPB-thread block: by finalize_k, or by the last block of
// fused_opt_k (FinArgs::ticket set), which then replaces the separate launch
template <bool COH>   // COH: the optimizer's l2 partials of this launch, read coherently
DEV void finalize_body(const FinArgs& f, float* wsum) {
  int64_t* step = f.step;
  float* stats = f.stats;
  float* l2 = f.l2;
  const int* l2r = f.l2r;
  const int l2base = f.l2base, nw = f.nw, n_ema = f.n_ema, batch = f.batch, increment = f.increment;
  const float* wds = f.wds;
  float* loss_ema = f.loss_ema;
  const float* ce_work = f.ce_work;
  const int ce_nblk = f.ce_nblk;
  // wave 0 lane i owns loss entry i (weight losses..., cross_entropy, total_loss), so the
  // EMA read-modify-writes run in parallel instead of as one dependent chain.  The per-
  // weight sum(w^2) partials are summed by all FIN_WAVES waves (weight w by wave w %
  // FIN_WAVES, the same per-weight order as one wave): their load latencies overlap
  // instead of queueing behind each other (LeNet: 5 weights, ~11 -> ~5 us).
  const int t = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // wave 0: the CE partials and every per-lane input of the EMA update, loaded up front;
  // waves 1..FIN_WAVES-1: the per-weight sum(w^2) partials -- the two phases' memory
  // round trips overlap instead of following each other
  float ce_sum = 0.f, corr_sum = 0.f, l2t = 0.f, wdt = 0.f, e0 = 0.f, e1 = 0.f;
  if (wv == 0) {
    ce_sum = stats[0];
    corr_sum = stats[1];
    if (l2 && t < nw) l2t = l2[t];
    if (t < nw) wdt = wds[t];
    if (loss_ema && t < n_ema && t < nw + 2) {
      e0 = loss_ema[3 * t];
      e1 = loss_ema[3 * t + 1];
    }
    if (ce_nblk > 0) {
      // deferred CE partials (ce_block_stats defer): the same lane-strided, fixed-tree sum as
      // the ticket combine's last block, so the loss is bitwise what that path produced;
      // 8 partials per lane in flight per round, summed in the same per-lane order
      float a = 0.f, b = 0.f, c = 0.f;
      int i = t;
      for (; i + 7 * 64 < ce_nblk; i += 8 * 64) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(ce_work + 4 * (i + 64 * u));
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          a += v[u][0];
          b += v[u][1];
          c += v[u][2];
        }
      }
      for (; i < ce_nblk; i += 64) {
        a += ce_work[4 * i];
        b += ce_work[4 * i + 1];
        c += ce_work[4 * i + 2];
      }
      a = warp_sum(a);
      b = warp_sum(b);
      c = warp_sum(c);
      ce_sum += a;
      corr_sum += b;
      if (t == 0 && c > 0.f) stats[2] = 1.f;
    }
  } else if (l2 && l2r) {
    for (int w = wv - 1; w < nw && w < FIN_MAXW; w += FIN_WAVES - 1) {
      const int b0 = l2r[3 * w + 1], b1 = l2r[3 * w + 2];
      // 4 independent chains per lane, combined in a fixed order; 16 loads in flight per
      // round (the reference CNN's local3 has thousands of partials: 4 per round left this
      // wave's round trips most of finalize_k's ~11 us)
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
      int b = b0 + t;
      for (; b + 64 * 15 < b1; b += 64 * 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = COH ? ld_coh(l2 + l2base + b + 64 * u) : l2[l2base + b + 64 * u];
#pragma unroll
        for (int u = 0; u < 16; ++u) s4[u & 3] += v[u];
      }
      for (; b + 192 < b1; b += 256) {
#pragma unroll
        for (int u = 0; u < 4; ++u) s4[u] += COH ? ld_coh(l2 + l2base + b + 64 * u) : l2[l2base + b + 64 * u];
      }
      for (; b < b1; b += 64) s4[0] += COH ? ld_coh(l2 + l2base + b) : l2[l2base + b];
      float sum = (s4[0] + s4[1]) + (s4[2] + s4[3]);
      sum = warp_sum(sum);
      if (t == 0) wsum[w] = sum;
    }
  }
  __syncthreads();
  if (wv != 0) return;
  const float ce = ce_sum / (float)batch;
  const float acc = corr_sum / (float)batch;
  // sum(w^2) of weight t: the fused optimizer's per-block partials l2[l2base + b],
  // b in [l2r[3w+1], l2r[3w+2]), summed by the whole wave in a fixed order
  float l2v = l2t;
  if (l2 && l2r)
    for (int w = 0; w < nw && w < FIN_MAXW; ++w)
      if (t == l2r[3 * w]) l2v += wsum[w];
  const float wl = t < nw ? wdt * 0.5f * l2v : 0.f;
  float total = ce;
  for (int i = 0; i < nw; ++i) total += __shfl(wl, i, 64);   // fixed order (bitwise as before)
  if (loss_ema && t < n_ema && t < nw + 2) {
    const float v = t < nw ? wl : (t == nw ? ce : total);
    float* e = loss_ema + 3 * t;
    const float b = 0.9f * e0 + 0.1f * v, n = e1 + 1.f;
    e[0] = b;
    e[1] = n;
    e[2] = b / (1.f - powf(0.9f, n));
  }
  if (l2 && t < nw) l2[t] = 0.f;
  if (t != 0) return;
  stats[4] = ce;
  stats[5] = acc;
  stats[6] = total;
  stats[7] += 1.f;
  if (!isfinite(total)) stats[2] = 1.f;
  stats[0] = 0.f;
  stats[1] = 0.f;
  if (increment) *step += 1;
}

__global__ __launch_bounds__(64 * FIN_WAVES) void finalize_k(FinArgs f) {
  __shared__ float wsum[FIN_MAXW];
  finalize_body<false>(f, wsum);
}

__global__ void cast_pad_k(const float* __restrict__ src, bf16_t* __restrict__ dst, int G, int I, int J, int Ip,
                           int Jp) {
  const int64_t total = (int64_t)G * Ip * Jp;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int jj = (int)(t % Jp);
    const int64_t r = t / Jp;
    const int ii = (int)(r % Ip);
    const int gg = (int)(r / Ip);
    float v = 0.f;
    if (ii < I && jj < J) v = src[((int64_t)gg * I + ii) * J + jj];
    dst[t] = f2bf(v);
  }
}

}  // namespace

static int g_grid_cap = 0;
int grid_cap() { return g_grid_cap; }
void set_grid_cap(int n) { g_grid_cap = n > 0 ? n : 0; }
static int g_reserve_cus = 0;
int reserve_cus() { return g_reserve_cus; }
void set_reserve_cus(int n) { g_reserve_cus = n > 0 ? n : 0; }

hipError_t perm_positions(int64_t* out, int64_t start, int n, int64_t N, uint32_t seed, int h, hipStream_t st,
                          const int32_t* lab_src, int32_t* lab_out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(perm_positions_k, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, st, out, start, n, N, seed, h,
                     lab_src, lab_out);
  return hipGetLastError();
}

hipError_t prep_images_perm(const uint8_t* src, const int32_t* lab_src, int B, int64_t start, int64_t N,
                            uint32_t seed, int h, bf16_t* out, int32_t* lab_out, hipStream_t st) {
  if ((uintptr_t)src % 16 || (uintptr_t)out % 16 || (int64_t)B * PREP_V >= (1ll << 31)) return hipErrorInvalidValue;
  const int64_t nvec = (int64_t)B * PREP_V;
  hipLaunchKernelGGL(prep_images_784_perm_k, dim3(nblocks(nvec, 256, 8192)), dim3(256), 0, st, src, lab_src, B, start,
                     N, seed, h, out, lab_out);
  return hipGetLastError();
}

hipError_t prep_images(const uint8_t* src, const int64_t* idx, const int32_t* lab_src, int B, int HW, int Csrc,
                       int Cdst, bf16_t* out, int32_t* lab_out, hipStream_t st) {
  if (HW == 784 && Csrc == 1 && Cdst == 1 && (uintptr_t)src % 16 == 0 && (uintptr_t)out % 16 == 0 &&
      (int64_t)B * PREP_V < (1ll << 31)) {
    const int64_t nvec = (int64_t)B * PREP_V;
    hipLaunchKernelGGL(prep_images_784_k, dim3(nblocks(nvec, 256, 8192)), dim3(256), 0, st, src, idx, lab_src, B,
                       out, lab_out);
    return hipGetLastError();
  }
  const int64_t nvec = (int64_t)B * HW * Cdst / 8;
  int nb = nblocks(nvec, TPB, 8192);
  const int need = (B + TPB - 1) / TPB;
  if (nb < need) nb = need;
  hipLaunchKernelGGL(prep_images_k, dim3(nb), dim3(TPB), 0, st, src, idx, lab_src, B, HW, Csrc, Cdst, out, lab_out);
  return hipGetLastError();
}

hipError_t maxpool_fwd(const bf16_t* x, int Nb, int H, int W, int C, int OH, int OW, bf16_t* y, uint8_t* arg,
                       hipStream_t st) {
  const int64_t total = (int64_t)Nb * OH * OW * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_k, dim3(nblocks(total, TPB, 16384)), dim3(TPB), 0, st, x, Nb, H, W, C, OH, OW, y,
                     arg);
  return hipGetLastError();
}

hipError_t maxpool_bwd(const bf16_t* dy, const uint8_t* arg, const bf16_t* y, int relu_mask, int Nb, int H, int W,
                       int C, int OH, int OW, bf16_t* dx, hipStream_t st) {
  const int64_t total = (int64_t)Nb * OH * OW * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_k, dim3(nblocks(total, TPB, 16384)), dim3(TPB), 0, st, dy, arg, y, relu_mask, Nb,
                     H, W, C, OH, OW, dx);
  return hipGetLastError();
}

#define LRN_CASE(KER, CC, RR, ...) \
  if (C == CC && r == RR) { hipLaunchKernelGGL((KER<CC, RR>), grid, dim3(TPB), 0, st, __VA_ARGS__); return hipGetLastError(); }
#define LRN_ALL(KER, ...)                                                                                     \
  LRN_CASE(KER, 8, 4, __VA_ARGS__) LRN_CASE(KER, 16, 4, __VA_ARGS__) LRN_CASE(KER, 32, 4, __VA_ARGS__)         \
  LRN_CASE(KER, 64, 4, __VA_ARGS__) LRN_CASE(KER, 32, 2, __VA_ARGS__) LRN_CASE(KER, 64, 2, __VA_ARGS__)        \
  LRN_CASE(KER, 32, 5, __VA_ARGS__) LRN_CASE(KER, 64, 5, __VA_ARGS__)

hipError_t lrn_fwd(const bf16_t* x, int P, int C, int r, float bias, float alpha, float beta, bf16_t* y,
                   hipStream_t st) {
  dim3 grid(nblocks((int64_t)P * (C / 8), TPB, 16384));   // one lane per 8-channel vector
  LRN_ALL(lrn_fwd_k, x, (int64_t)P, bias, alpha, beta, y)
  return hipErrorInvalidValue;  // (C, depth_radius) combination not instantiated
}

bool lrn_pool_supported(int H, int W, int C, int r) {
  return H % 2 == 0 && W % 2 == 0 && (C == 32 || C == 64) && r == 4;
}
// the packed 14 x 14 x 64 kernels (MNISTX_LRN_PK=0: the generic ones)
static int g_lrn_pk = [] { const char* e = getenv("MNISTX_LRN_PK"); return (e && e[0] == '0') ? 0 : 1; }();
void lrn_set_packed(int on) { g_lrn_pk = on; }
static bool lrn_pk14(int H, int W, int C, int r, int Nb) {
  return g_lrn_pk && H == LP14_HW && W == LP14_HW && C == LP14_C && r == 4 && (int64_t)Nb * LP14_NWIN * LP14_G < (1ll << 31);
}

hipError_t lrn_pool_fwd(const bf16_t* x, int Nb, int H, int W, int C, int r, float bias, float alpha, float beta,
                        bf16_t* y, uint8_t* arg, hipStream_t st, int nonneg) {
  if (!lrn_pool_supported(H, W, C, r)) return hipErrorInvalidValue;
  if (nonneg && lrn_pk14(H, W, C, r, Nb)) {
    if (Nb <= 0) return hipSuccess;
    dim3 grid(nblocks(((int64_t)Nb * LP14_NWIN * LP14_G + 1) / 2, TPB, 16384));
    hipLaunchKernelGGL((lrn_pool14_fwd_k<4>), grid, dim3(TPB), 0, st, x, Nb, bias, alpha, beta, y, arg);
    return hipGetLastError();
  }
  dim3 grid(nblocks(((int64_t)Nb * (H / 2) * (W / 2) * (C / 8) + LRNP_U - 1) / LRNP_U, TPB, 16384));
  if (C == 64) hipLaunchKernelGGL((lrn_pool_fwd_k<64, 4>), grid, dim3(TPB), 0, st, x, Nb, H, W, bias, alpha, beta, y, arg);
  else hipLaunchKernelGGL((lrn_pool_fwd_k<32, 4>), grid, dim3(TPB), 0, st, x, Nb, H, W, bias, alpha, beta, y, arg);
  return hipGetLastError();
}
hipError_t lrn_pool_bwd(const bf16_t* x, const bf16_t* dP, const uint8_t* arg, int Nb, int H, int W, int C, int r,
                        float bias, float alpha, float beta, int relu_mask, bf16_t* dx, hipStream_t st) {
  if (!lrn_pool_supported(H, W, C, r)) return hipErrorInvalidValue;
  dim3 grid(nblocks((int64_t)Nb * (H / 2) * (W / 2) * (C / 8), TPB, 16384));
  if (beta == 0.75f && lrn_pk14(H, W, C, r, Nb)) {
    if (Nb <= 0) return hipSuccess;
    hipLaunchKernelGGL((lrn_pool14_bwd_k<4>), grid, dim3(TPB), 0, st, x, dP, arg, Nb, bias, alpha, beta, relu_mask, dx);
    return hipGetLastError();
  }
#define LRN_PB(CC, BB) \
  hipLaunchKernelGGL((lrn_pool_bwd_k<CC, 4, BB>), grid, dim3(TPB), 0, st, x, dP, arg, Nb, H, W, bias, alpha, beta, relu_mask, dx)
  const bool b075 = beta == 0.75f;   // the reference's beta (lrn_math.h pow_beta)
  if (C == 64) {
    if (b075) LRN_PB(64, true);
    else LRN_PB(64, false);
  } else {
    if (b075) LRN_PB(32, true);
    else LRN_PB(32, false);
  }
#undef LRN_PB
  return hipGetLastError();
}

hipError_t lrn_bwd(const bf16_t* x, const bf16_t* dy, int P, int C, int r, float bias, float alpha, float beta,
                   int relu_mask, bf16_t* dx, hipStream_t st) {
  dim3 grid(nblocks((int64_t)P * (C / 8), TPB, 16384));
  if (beta == 0.75f && r == 4 && (C == 32 || C == 64)) {   // the reference CNN's layers: pow_beta<true>
    if (C == 32) hipLaunchKernelGGL((lrn_bwd_k<32, 4, true>), grid, dim3(TPB), 0, st, x, dy, (int64_t)P, bias, alpha, beta, relu_mask, dx);
    else hipLaunchKernelGGL((lrn_bwd_k<64, 4, true>), grid, dim3(TPB), 0, st, x, dy, (int64_t)P, bias, alpha, beta, relu_mask, dx);
    return hipGetLastError();
  }
  LRN_ALL(lrn_bwd_k, x, dy, (int64_t)P, bias, alpha, beta, relu_mask, dx)
  return hipErrorInvalidValue;
}

int softmax_ce_dbias_blocks(int B, int ldl) {
  return (ldl == 16 || ldl == 32) && B > 0 ? (int)std::min<int64_t>(CE_MAXB, ((int64_t)B + 255) / 256) : 0;
}

hipError_t softmax_ce(const float* logits, int ldl, const int32_t* labels, int B, int NC, float scale,
                      bf16_t* dlogits, int ldd, float* stats, float* probs, float* work, hipStream_t st,
                      int* defer_blocks, float* dbias) {
  const int nb = (int)std::min<int64_t>(CE_MAXB, ((int64_t)B + 255) / 256);
  if (defer_blocks) *defer_blocks = 0;
  const bool rows_ok = (ldl == 16 || ldl == 32) && NC <= ldl && (!dlogits || ldd == ldl) &&
                       ((uintptr_t)logits % 16 == 0) && (!dlogits || (uintptr_t)dlogits % 16 == 0);
  if (rows_ok && B > 0) {
    const int defer = (defer_blocks && work && stats) ? 1 : 0;
    if (defer) *defer_blocks = nb;
    if (ldl == 16)
      hipLaunchKernelGGL(softmax_ce_rows_k<16>, dim3(nb), dim3(256), 0, st, logits, labels, B, NC, scale, dlogits,
                         stats, probs, work, defer, dbias);
    else
      hipLaunchKernelGGL(softmax_ce_rows_k<32>, dim3(nb), dim3(256), 0, st, logits, labels, B, NC, scale, dlogits,
                         stats, probs, work, defer, dbias);
    return hipGetLastError();
  }
  if (dbias) return hipErrorInvalidValue;   // the row kernel's block partials only
  hipLaunchKernelGGL(softmax_ce_k, dim3((B + TPB - 1) / TPB), dim3(TPB), 0, st, logits, ldl, labels, B, NC, scale,
                     dlogits, ldd, stats, probs);
  return hipGetLastError();
}

// Tickets of the fused reduce (one int per partial-pass quad block of a launch: at most
// MAXRED * 512) and of the optimizer's finalize (slot MAXRED * 512): one zeroed buffer per
// (device, stream), left zeroed by every launch, so launches on different streams (the
// executor's overlapped side-stream reduces) never share a ticket, and launches on one
// stream are ordered.  nullptr (the two-launch path) when disabled (MNISTX_REDUCE_FUSED=0)
// or while the stream is being captured (graphs keep the two launches).
static int g_reduce_fused = -1;
void set_reduce_fused(int on) { g_reduce_fused = on; }
int reduce_fused_enabled() {
  if (g_reduce_fused < 0) {
    const char* e = getenv("MNISTX_REDUCE_FUSED");
    g_reduce_fused = (e && *e) ? atoi(e) != 0 : 1;
  }
  return g_reduce_fused;
}
static int* red_tickets(hipStream_t st, bool any_use = false) {
  if (!any_use && !reduce_fused_enabled()) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  static std::mutex mu;
  static std::vector<std::tuple<int, hipStream_t, int*>> bufs;
  std::lock_guard<std::mutex> lk(mu);
  for (const auto& b : bufs)
    if (std::get<0>(b) == dev && std::get<1>(b) == st) return std::get<2>(b);
  int* p = nullptr;
  const size_t bytes = (MAXRED * 512 + 64) * sizeof(int);   // + the optimizer's finalize ticket
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return nullptr;
  bufs.emplace_back(dev, st, p);
  return p;
}

hipError_t splitk_reduce_multi(const RedSpec* specs, int n, hipStream_t st) {
  if (n < 1) return hipSuccess;
  // one-split slabs (small batches: K below pick_splits' min_k) take the same multi-tensor
  // launch -- its S = 1 sum is the slab itself -- instead of one generic launch per tensor
  // (LeNet-5 at B = 128: 5 launches, ~31 us of a ~100 us step)
  bool vec = true;
  for (int i = 0; i < n; ++i) vec = vec && specs[i].N % 4 == 0 && specs[i].splits >= 1;
  if (!vec) {  // generic path, one launch per tensor
    for (int i = 0; i < n; ++i) {
      const RedSpec& r = specs[i];
      const int64_t total = (int64_t)r.G * r.I * r.J + (r.bdst ? r.J : 0);
      hipLaunchKernelGGL(splitk_reduce_k, dim3(nblocks(total, TPB, 8192)), dim3(TPB), 0, st, r.slab, r.splits, r.M,
                         r.N, r.G, r.Ipad, r.I, r.J, r.bias_row, r.wdst, r.bdst, r.scale);
    }
    return hipGetLastError();
  }
  int* tickets = red_tickets(st);
  for (int i0 = 0; i0 < n; i0 += MAXRED) {
    RedTable tab;
    tab.n = std::min(MAXRED, n - i0);
    int pb = 0, rb = 0, tk = 0;
    const bool fused = tickets != nullptr;
    for (int i = 0; i < tab.n; ++i) {
      const RedSpec& r = specs[i0 + i];
      RedDesc& D = tab.d[i];
      D.slab = r.slab;
      D.wdst = r.wdst;
      D.bdst = r.bdst;
      D.nq = (int64_t)r.M * (r.N / 4);
      D.S = r.splits;
      D.M = r.M;
      D.N = r.N;
      D.G = r.G;
      D.Ipad = r.Ipad;
      D.I = r.I;
      D.J = r.J;
      D.bias_row = r.bias_row;
      D.scale = r.scale;
      D.qb = (int)((D.nq + 63) / 64);
      D.sb = (D.S > RED_CHUNK && D.qb < 512) ? (D.S + RED_CHUNK - 1) / RED_CHUNK : 0;
      D.tick0 = tk;
      tab.pblk0[i] = pb;
      tab.rblk0[i] = rb;
      pb += D.sb ? D.qb * D.sb : 0;
      tk += D.sb ? D.qb : 0;
      rb += (fused && D.sb) ? 0 : D.qb;   // fused: the partial pass finishes its own quads
    }
    for (int i = tab.n; i <= MAXRED; ++i) {
      tab.pblk0[i] = pb;
      tab.rblk0[i] = rb;
    }
    if (fused) {
      if (pb + rb > 0) hipLaunchKernelGGL(splitk_fused4_k, dim3(pb + rb), dim3(256), 0, st, tab, tickets);
      continue;
    }
    if (pb > 0) hipLaunchKernelGGL(splitk_partial4_k, dim3(pb), dim3(256), 0, st, tab);
    hipLaunchKernelGGL(splitk_reduce4_k, dim3(rb), dim3(256), 0, st, tab);
  }
  return hipGetLastError();
}

hipError_t splitk_reduce(float* slab, int splits, int M, int N, int G, int Ipad, int I, int J, int bias_row,
                         float* wdst, float* bdst, float scale, hipStream_t st) {
  const RedSpec r{slab, wdst, bdst, splits, M, N, G, Ipad, I, J, bias_row, scale};
  return splitk_reduce_multi(&r, 1, st);
}

int fused_optimizer_blocks(const OptSeg* segs, int nseg) {
  int nb = 0;
  for (int i = 0; i < nseg; ++i) nb += (int)((segs[i].n + OPT_CHUNK - 1) / OPT_CHUNK);
  return nb;
}

static int g_opt_fin_fused = -1;
void set_opt_fin_fused(int on) { g_opt_fin_fused = on; }
int opt_fin_fused_enabled() {
  if (g_opt_fin_fused < 0) {
    const char* e = getenv("MNISTX_OPT_FIN_FUSED");
    g_opt_fin_fused = (e && *e) ? atoi(e) != 0 : 1;
  }
  return g_opt_fin_fused;
}

hipError_t finalize_step(const FinArgs& f, hipStream_t st) {
  if (f.nw > FIN_MAXW) return hipErrorInvalidValue;
  FinArgs a = f;
  a.ticket = nullptr;
  hipLaunchKernelGGL(finalize_k, dim3(1), dim3(64 * FIN_WAVES), 0, st, a);
  return hipGetLastError();
}

hipError_t fused_optimizer(float* params, const float* grads, float* mom, float* ema, bf16_t* bf, const OptSeg* segs,
                           int nseg, int64_t total, const int64_t* step, OptParams op, float* l2, int l2n,
                           hipStream_t st, const FinArgs* fin, const PermJob* perm) {
  if (nseg > MAXSEG || nseg < 1) return hipErrorInvalidValue;
  if (fin && fin->nw > FIN_MAXW) return hipErrorInvalidValue;
  SegTable tab;
  int nb = 0;
  for (int i = 0; i < nseg; ++i) {
    if (segs[i].n >= (1ll << 31) || (int64_t)segs[i].I * segs[i].J >= (1ll << 31)) return hipErrorInvalidValue;
    tab.s[i] = segs[i];
    tab.fij[i] = FastDiv((uint32_t)(segs[i].I * segs[i].J));
    tab.fj[i] = FastDiv((uint32_t)segs[i].J);
    tab.blk0[i] = nb;
    nb += (int)((segs[i].n + OPT_CHUNK - 1) / OPT_CHUNK);
  }
  tab.blk0[nseg] = nb;
  tab.n = nseg;
  tab.l2n = l2n;
  (void)total;
  FinArgs fa{};
  int* tickets = nullptr;
  if (fin && !op.guard && nb <= 1024 && opt_fin_fused_enabled()) tickets = red_tickets(st, true);
  if (tickets) {
    fa = *fin;
    fa.ticket = tickets + MAXRED * 512;   // the optimizer's slot after the reduce's
  }
  PermJob pj{};
  int npb = 0;
  if (perm && perm->n > 0) {
    pj = *perm;
    pj.blk0 = nb;
    npb = (pj.n + TPB - 1) / TPB;
  }
  hipLaunchKernelGGL(fused_opt_k, dim3(nb + npb), dim3(TPB), 0, st, params, grads, mom, ema, bf, tab, step, op, l2, fa,
                     pj);
  if (fin && !tickets) return finalize_step(*fin, st);
  return hipGetLastError();
}

hipError_t cast_f32_bf16_padded(const float* src, bf16_t* dst, int G, int I, int J, int Ip, int Jp, hipStream_t st) {
  const int64_t total = (int64_t)G * Ip * Jp;
  hipLaunchKernelGGL(cast_pad_k, dim3(nblocks(total, TPB, 8192)), dim3(TPB), 0, st, src, dst, G, I, J, Ip, Jp);
  return hipGetLastError();
}

}  // namespace mnistx
