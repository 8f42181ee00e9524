// fp32 (--precision fp32) first convolution of the reference CNN / LeNet geometry:
// 28x28x1 NHWC input, 5x5 SAME, Cout 32, on v_mfma_f32_16x16x4_f32.
//
// The generic fp32 GEMM path (f32.hip Im2colF / Im2colTF) spends 1.17 ms (fwd) and
// 1.89 ms (wgrad) per step on this layer at B = 16384 (profiles/r3/fp32): its loaders
// recompute the im2col index of every element with four FastDivs, and the 64-wide N
// tile is half empty at Cout 32.  Both are small problems (25 MACs per output) bound
// by HBM at the roofline (the 1.64 GB conv output / its gradient), so these kernels
// only have to get the operand plumbing out of the way:
//   * forward: the image is staged in LDS once per image as a zero-haloed tile; K = the
//     25 taps in order (7 MFMAs per fragment, Taps7), A = the filter (held in registers for
//     the whole launch), B = 16 output pixels of one row, one float per lane; D lane (i, g)
//     = channels 4g..4g+3 of pixel i -> one 16-byte store with bias + ReLU;
//   * weight gradient: M = 32 rows = 25 taps + the bias row (A = 1) + zero rows, N =
//     32 channels, K = pixels, 4 consecutive pixels of a row per k-step; the patch
//     operand is a 4-byte LDS read of the staged tile, dY a coalesced 64-byte global
//     read per lane group (each dY value is read once); one fp32 partial per
//     workgroup goes to the split-K slab [S][26][32] reduced by splitk_reduce.
//
// Replaces (SURVEY.md §2.3 N1, fp32 path): Conv2D / its filter gradient of conv1 at
// mnist_input.py:142-145 under the reference's tf.float32.
#include "common.h"
#include "launchers.h"
#include "lrn_f32.h"

namespace mnistx {
namespace {

constexpr int IH = 28, IW = 28, IPIX = IH * IW, COUT = 32, KS = 5;
constexpr int TR = 34;                        // padded tile rows (2 + 28 + 2, + 2 slack)
constexpr int NT1 = 256;

// The weight-gradient kernels read the tile one float per lane (16 taps x 2 pixels per 32-lane
// half): with 32-float rows the 5 kernel rows of a tap column share a bank (4-way / 2-way
// ds_read_b32 conflicts); 40-float rows put them 8 banks apart (conflict-free).
constexpr int TCW = 40, TSZW = TR * TCW + 8;
DEV void stage_image_w(float* tile, const float* __restrict__ x, int img, int tid) {
  for (int e = tid; e < IPIX; e += NT1) {
    const int y = e / IW, xx = e - y * IW;
    tile[(y + 2) * TCW + xx + 2] = x[(int64_t)img * IPIX + e];
  }
}

// Forward: K = the 25 taps in order, 4 per v_mfma_f32_16x16x4_f32 (7 MFMAs per output row
// fragment and channel half, 3 zero slots), each lane reading one float of the tile (its tap of
// its pixel).  The former (kh 0..5) x (kw 0..7) K layout read 4-float runs but spent 12 MFMAs
// per fragment (48 slots for 25 taps).  Row stride 52 floats: a 32-lane half reads two taps of
// 16 consecutive pixels, one row apart at a kernel-row wrap (offset 52 - 4 = 48 = 16 mod 32
// banks), so the two 16-float runs always sit in disjoint banks.
constexpr int TCF = 52, TSZF = TR * TCF;
DEV void stage_image_f(float* tile, const float* __restrict__ x, int img, int tid) {
  for (int e = tid; e < IPIX; e += NT1) {
    const int y = e / IW, xx = e - y * IW;
    tile[(y + 2) * TCF + xx + 2] = x[(int64_t)img * IPIX + e];
  }
}
// filter slots of this lane (channel 16 nf + i, k-group g): tap t = 4 j + g
struct Taps7 {
  float a[7][2];
  int off[7];
  DEV void init(const float* __restrict__ w, int i, int g) {
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int t = 4 * j + g;
      off[j] = t < KS * KS ? (t / KS) * TCF + (t % KS) : 0;
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) a[j][nf] = t < KS * KS ? w[t * COUT + 16 * nf + i] : 0.f;
    }
  }
  // acc[nf] += conv of output row `row`, columns x0 + (0..15): D lane (i, g) = channels
  // 16 nf + 4 g .. + 3 of pixel x0 + i
  DEV void row(const float* tile, int row, int x0, int i, f32x4 (&acc)[2]) const {
    const float* b = tile + row * TCF + x0 + i;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const float v = b[off[j]];
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) acc[nf] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][nf], v, acc[nf], 0, 0, 0);
    }
  }
};

__global__ __launch_bounds__(NT1) void conv1_f32_fwd_k(const float* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ bias, int relu, int B,
                                                       float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float tile[TSZF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  for (int e = tid; e < TSZF; e += NT1) tile[e] = 0.f;
  Taps7 tp;   // A = filter, tap-major K
  tp.init(w, i, g);
  float bs[2][4];
#pragma unroll
  for (int nf = 0; nf < 2; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs[nf][r] = bias ? bias[16 * nf + 4 * g + r] : 0.f;
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    __syncthreads();
    stage_image_f(tile, x, img, tid);
    __syncthreads();
    // units (row, 16-column segment): 28 x 2, dealt over the 4 waves
    for (int u = wave; u < 2 * IH; u += NT1 / 64) {
      const int row = u >> 1, x0 = 16 * (u & 1);
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      tp.row(tile, row, x0, i, acc);
      const int xx = x0 + i;
      if (xx < IW) {
        const int64_t px = (int64_t)img * IPIX + row * IW + xx;
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          f32x4 o = acc[nf];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            o[r] += bs[nf][r];
            if (relu) o[r] = fmaxf(o[r], 0.f);
          }
          *(f32x4*)(y + px * COUT + 16 * nf + 4 * g) = o;
        }
      }
    }
  }
}

// slab[blockIdx][m][co], m = kh*5 + kw (25 taps) and the bias row 25
constexpr int WROWS = KS * KS + 1;
__global__ __launch_bounds__(NT1) void conv1_f32_wgrad_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                         int B, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float tile[TSZW];
  __shared__ float red[NT1 / 64][2][2][64][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  for (int e = tid; e < TSZW; e += NT1) tile[e] = 0.f;
  // A rows of this lane: tap m = 16 mf + i -> tile offset of its (kh, kw), or the bias / zero rows
  int toff[2];
  float aconst[2];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf) {
    const int m = 16 * mf + i;
    toff[mf] = m < KS * KS ? (m / KS) * TCW + (m % KS) : -1;
    aconst[mf] = m == KS * KS ? 1.f : 0.f;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    __syncthreads();
    stage_image_w(tile, x, img, tid);
    __syncthreads();
    const float* dyi = dy + (int64_t)img * IPIX * COUT;
    // k-step q = (row, 4-pixel column block): pixels (row, 4c + g); 196 per image over 4 waves
#pragma unroll 4
    for (int q = wave; q < IH * (IW / 4); q += NT1 / 64) {
      const int row = q / (IW / 4), c4 = q - row * (IW / 4);
      const int p = row * IW + 4 * c4 + g;
      const float b0 = dyi[p * COUT + i], b1 = dyi[p * COUT + 16 + i];
      const int base = row * TCW + 4 * c4 + g;     // tile offset of the pixel's tap (0, 0)
#pragma unroll
      for (int mf = 0; mf < 2; ++mf) {
        const float av = toff[mf] >= 0 ? tile[base + toff[mf]] : aconst[mf];
        acc[mf][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc[mf][0], 0, 0, 0);
        acc[mf][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc[mf][1], 0, 0, 0);
      }
    }
  }
  // fixed-order cross-wave sum (deterministic), then one partial per block
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][mf][nf][lane][r] = acc[mf][nf][r];
  __syncthreads();
  if (wave == 0) {
    float* out = slab + (int64_t)blockIdx.x * WROWS * COUT;
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = ((red[0][mf][nf][lane][r] + red[1][mf][nf][lane][r]) + red[2][mf][nf][lane][r]) +
                          red[3][mf][nf][lane][r];
          const int m = 16 * mf + 4 * g + r;
          if (m < WROWS) out[m * COUT + 16 * nf + i] = v;
        }
  }
}

// conv1 + bias + ReLU + 2x2/2 max-pool (the reference's conv1 -> pool1, mnist_input.py:142-150)
// in one pass: the 1.64 GB conv1 output at B = 16384 is never written.  Units are (output row
// pair, 16-column segment), each lane computes the same MFMAs as conv1_f32_fwd_k for its pixel
// on both rows; the vertical pool is in the lane, the horizontal one with the lane i ^ 1
// partner (DPP quad swap).  Pooled values and the first-maximum position order (0..3 =
// row-major window position) are maxpool_f32's; the code is 4 where the pooled ReLU output is
// 0 (no gradient: the unfused backward's y > 0 mask).  Even lanes store channels 0-15, odd
// lanes 16-31 of their pooled pixel.
DEV float quad_swap(float v) {   // lane i <- lane i ^ 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
}
constexpr int PH = IH / 2, PW = IW / 2;
__global__ __launch_bounds__(NT1) void conv1_f32_fwd_pool_k(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, int B,
                                                            float* __restrict__ y, uint32_t* __restrict__ arg) {
  __shared__ __attribute__((aligned(16))) float tile[TSZF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  for (int e = tid; e < TSZF; e += NT1) tile[e] = 0.f;
  Taps7 tp;   // A = filter, tap-major K
  tp.init(w, i, g);
  float bs[2][4];
#pragma unroll
  for (int nf = 0; nf < 2; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs[nf][r] = bias ? bias[16 * nf + 4 * g + r] : 0.f;
  const int cp = i & 1;    // this lane's column parity: window positions cp (row 0) and 2 + cp (row 1)
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    __syncthreads();
    stage_image_f(tile, x, img, tid);
    __syncthreads();
    // units (row pair, 16-column segment): 14 x 2, dealt over the 4 waves
    for (int u = wave; u < 2 * PH; u += NT1 / 64) {
      const int rp = u >> 1, x0 = 16 * (u & 1);
      f32x4 acc[2][2];   // [row][nf]
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acc[h][0] = acc[h][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        tp.row(tile, 2 * rp + h, x0, i, acc[h]);
      }
      // bias + ReLU, then the window max in position order 0 (r0 c0), 1 (r0 c1), 2 (r1 c0), 3 (r1 c1)
      f32x4 best[2];
      uint32_t code[2] = {0u, 0u};
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v[4];
          const float m0 = fmaxf(acc[0][nf][r] + bs[nf][r], 0.f), m1 = fmaxf(acc[1][nf][r] + bs[nf][r], 0.f);
          const float o0 = quad_swap(m0), o1 = quad_swap(m1);      // the partner column's rows 0 / 1
          v[0] = cp ? o0 : m0;
          v[1] = cp ? m0 : o0;
          v[2] = cp ? o1 : m1;
          v[3] = cp ? m1 : o1;
          float bv = v[0];
          uint32_t bd = 0;
#pragma unroll
          for (int d = 1; d < 4; ++d)
            if (v[d] > bv) { bv = v[d]; bd = d; }   // first maximum wins (TF MaxPool)
          best[nf][r] = bv;
          code[nf] |= (bv > 0.f ? bd : 4u) << (8 * r);
        }
      const int pc = (x0 + i) >> 1;
      if (pc < PW) {
        const int64_t pp = (int64_t)img * (PH * PW) + rp * PW + pc;
        const int nf = cp;                     // even lanes: channels 0-15, odd lanes 16-31
        *(f32x4*)(y + pp * COUT + 16 * nf + 4 * g) = nf ? best[1] : best[0];
        arg[(pp * COUT + 16 * nf + 4 * g) >> 2] = nf ? code[1] : code[0];
      }
    }
  }
}

// conv1 weight gradient from dL/d pool1 and the pool codes (the unfused pool backward's
// dL/d conv1 -- 1.64 GB at B = 16384 -- is never written): a pixel's gradient is its pooled
// pixel's where the code names its window position, else 0 (code 4: ReLU output 0).
// Otherwise conv1_f32_wgrad_k.
__global__ __launch_bounds__(NT1) void conv1_f32_wgrad_unpool_k(const float* __restrict__ x,
                                                                const float* __restrict__ dp,
                                                                const uint8_t* __restrict__ codes, int B,
                                                                float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float tile[TSZW];
  __shared__ float red[NT1 / 64][2][2][64][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  for (int e = tid; e < TSZW; e += NT1) tile[e] = 0.f;
  int toff[2];
  float aconst[2];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf) {
    const int m = 16 * mf + i;
    toff[mf] = m < KS * KS ? (m / KS) * TCW + (m % KS) : -1;
    aconst[mf] = m == KS * KS ? 1.f : 0.f;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    __syncthreads();
    stage_image_w(tile, x, img, tid);
    __syncthreads();
    const float* dpi = dp + (int64_t)img * (PH * PW) * COUT;
    const uint8_t* cdi = codes + (int64_t)img * (PH * PW) * COUT;
#pragma unroll 4
    for (int q = wave; q < IH * (IW / 4); q += NT1 / 64) {
      const int row = q / (IW / 4), c4 = q - row * (IW / 4);
      const int col = 4 * c4 + g;
      const int pp = (row >> 1) * PW + (col >> 1);
      const uint32_t pos = (uint32_t)(2 * (row & 1) + (col & 1));
      const float d0 = dpi[pp * COUT + i], d1 = dpi[pp * COUT + 16 + i];
      const uint32_t k0 = cdi[pp * COUT + i], k1 = cdi[pp * COUT + 16 + i];
      const float b0 = k0 == pos ? d0 : 0.f, b1 = k1 == pos ? d1 : 0.f;
      const int base = row * TCW + col;
#pragma unroll
      for (int mf = 0; mf < 2; ++mf) {
        const float av = toff[mf] >= 0 ? tile[base + toff[mf]] : aconst[mf];
        acc[mf][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc[mf][0], 0, 0, 0);
        acc[mf][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc[mf][1], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][mf][nf][lane][r] = acc[mf][nf][r];
  __syncthreads();
  if (wave == 0) {
    float* out = slab + (int64_t)blockIdx.x * WROWS * COUT;
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = ((red[0][mf][nf][lane][r] + red[1][mf][nf][lane][r]) + red[2][mf][nf][lane][r]) +
                          red[3][mf][nf][lane][r];
          const int m = 16 * mf + 4 * g + r;
          if (m < WROWS) out[m * COUT + 16 * nf + i] = v;
        }
  }
}

// The same weight gradient with norm1's backward folded in (reference CNN, pool1 -> norm1 ->
// conv2, mnist_input.py:149-156): reads dL/d norm1, pool1 (the LRN input) and the codes, and
// runs lrn_f32_bwd4 -- the unfused lrn_f32_bwd_v4_k's arithmetic -- while staging, so dL/d
// pool1 (411 MB at B = 16384, written and read back by the unfused pair) never reaches HBM.
// Per image the staged dL/d pool1 and codes live in LDS; the next image's operands are loaded
// into registers during this image's MFMAs (the unfused kernel's per-k-step global loads were
// latency bound: 570 us against a ~170 us MFMA floor).  Summation order = conv1_f32_wgrad_unpool_k
// for the same grid.
constexpr int NPP = PH * PW;                   // 196 pooled pixels
constexpr int LT = NPP * (COUT / 4);           // LRN tasks per image: (pooled pixel, 4 channels)
constexpr int LR = (LT + NT1 - 1) / NT1;       // 7 staging rounds (the last: 32 tasks)
constexpr int XR = (IPIX + NT1 - 1) / NT1;     // 4 input rounds
__global__ __launch_bounds__(NT1) void conv1_f32_wgrad_lrn_k(const float* __restrict__ x,
                                                             const float* __restrict__ dn,
                                                             const float* __restrict__ p1,
                                                             const uint8_t* __restrict__ codes, int B, float lbias,
                                                             float lalpha, float lbeta, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) float tile[TSZW];
  __shared__ __attribute__((aligned(16))) float dps[NPP * COUT];     // dL/d pool1 of the image
  __shared__ __attribute__((aligned(16))) uint32_t cds[LT];          // its codes, 4 per word
  static_assert(sizeof(float) * NPP * COUT >= sizeof(float) * (NT1 / 64) * 2 * 2 * 64 * 4, "red aliases dps");
  float(*red)[2][2][64][4] = (float(*)[2][2][64][4])dps;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  for (int e = tid; e < TSZW; e += NT1) tile[e] = 0.f;
  int toff[2];
  float aconst[2];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf) {
    const int m = 16 * mf + i;
    toff[mf] = m < KS * KS ? (m / KS) * TCW + (m % KS) : -1;
    aconst[mf] = m == KS * KS ? 1.f : 0.f;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};

  // next image's operands in registers: branch-free buffer loads, zeros past the batch
  f32x4 pv[LR], gv[LR];
  uint32_t cv[LR];
  float xv[XR];
  auto load = [&](int img) {
    const bool ok = img < B;
    const int64_t b = ok ? img : 0;
    const auto rx = buf_rsrc(x + b * IPIX, ok ? IPIX * 4u : 0u);
    const auto rp = buf_rsrc(p1 + b * LT * 4, ok ? LT * 16u : 0u);
    const auto rg = buf_rsrc(dn + b * LT * 4, ok ? LT * 16u : 0u);
    const auto rc = buf_rsrc(codes + b * LT * 4, ok ? LT * 4u : 0u);
#pragma unroll
    for (int u = 0; u < XR; ++u) {
      const int e = tid + u * NT1;
      xv[u] = __uint_as_float(buf_b32(rx, e < IPIX ? 4u * e : BUF_OOB));
    }
#pragma unroll
    for (int u = 0; u < LR; ++u) {
      const int t = tid + u * NT1;
      const uint32_t o = t < LT ? 0u : BUF_OOB;
      pv[u] = __builtin_bit_cast(f32x4, buf_b128(rp, 16u * t + o));
      gv[u] = __builtin_bit_cast(f32x4, buf_b128(rg, 16u * t + o));
      cv[u] = buf_b32(rc, 4u * t + o);
    }
  };
  load(blockIdx.x);
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    __syncthreads();   // the previous image's k-steps no longer read tile / dps / cds
#pragma unroll
    for (int u = 0; u < XR; ++u) {
      const int e = tid + u * NT1;
      if (e < IPIX) {
        const int y = e / IW, xx = e - y * IW;
        tile[(y + 2) * TCW + xx + 2] = xv[u];
      }
    }
#pragma unroll
    for (int u = 0; u < LR; ++u) {   // every lane runs the DPP exchanges; stores are masked
      const int t = tid + u * NT1;
      const f32x4 d = lrn_f32_bwd4(pv[u], gv[u], tid % (COUT / 4), COUT / 4, 4, lbias, lalpha, lbeta, 0);
      if (t < LT) {
        *(f32x4*)(dps + 4 * t) = d;
        cds[t] = cv[u];
      }
    }
    load(img + gridDim.x);
    __syncthreads();
    const uint8_t* cdb = (const uint8_t*)cds;
#pragma unroll 4
    for (int q = wave; q < IH * (IW / 4); q += NT1 / 64) {
      const int row = q / (IW / 4), c4 = q - row * (IW / 4);
      const int col = 4 * c4 + g;
      const int pp = (row >> 1) * PW + (col >> 1);
      const uint32_t pos = (uint32_t)(2 * (row & 1) + (col & 1));
      const float d0 = dps[pp * COUT + i], d1 = dps[pp * COUT + 16 + i];
      const uint32_t k0 = cdb[pp * COUT + i], k1 = cdb[pp * COUT + 16 + i];
      const float b0 = k0 == pos ? d0 : 0.f, b1 = k1 == pos ? d1 : 0.f;
      const int base = row * TCW + col;
#pragma unroll
      for (int mf = 0; mf < 2; ++mf) {
        const float av = toff[mf] >= 0 ? tile[base + toff[mf]] : aconst[mf];
        acc[mf][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc[mf][0], 0, 0, 0);
        acc[mf][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc[mf][1], 0, 0, 0);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][mf][nf][lane][r] = acc[mf][nf][r];
  __syncthreads();
  if (wave == 0) {
    float* out = slab + (int64_t)blockIdx.x * WROWS * COUT;
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = ((red[0][mf][nf][lane][r] + red[1][mf][nf][lane][r]) + red[2][mf][nf][lane][r]) +
                          red[3][mf][nf][lane][r];
          const int m = 16 * mf + 4 * g + r;
          if (m < WROWS) out[m * COUT + 16 * nf + i] = v;
        }
  }
}

int resident(const void* k) {
  int dev = 0, cus = 0, pc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k, NT1, 0) == hipSuccess && hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && pc > 0)
    return pc * cus;
  return 1024;
}

}  // namespace

bool f32_conv1_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout) {
  static const bool on = [] { const char* e = getenv("MNISTX_F32_HALO"); return !(e && e[0] == '0'); }();
  return on && H == IH && W == IW && C == 1 && OH == IH && OW == IW && KH == KS && KW == KS && ph == 2 && pw == 2 &&
         Cout == COUT;
}
int f32_conv1_wgrad_grid() {
  static const int n = resident((const void*)conv1_f32_wgrad_k);
  return n;
}
hipError_t f32_conv1_fwd(const float* x, const float* w, int Nb, const float* bias, int relu, float* y,
                         hipStream_t st) {
  if (Nb <= 0) return hipSuccess;
  static const int n = resident((const void*)conv1_f32_fwd_k);
  hipLaunchKernelGGL(conv1_f32_fwd_k, dim3(cap_grid(Nb < n ? Nb : n)), dim3(NT1), 0, st, x, w, bias, relu, Nb, y);
  return hipGetLastError();
}
hipError_t f32_conv1_fwd_pool(const float* x, const float* w, int Nb, const float* bias, float* y, uint8_t* arg,
                              hipStream_t st) {
  if (Nb <= 0) return hipSuccess;
  static const int n = resident((const void*)conv1_f32_fwd_pool_k);
  hipLaunchKernelGGL(conv1_f32_fwd_pool_k, dim3(cap_grid(Nb < n ? Nb : n)), dim3(NT1), 0, st, x, w, bias, Nb, y,
                     (uint32_t*)arg);
  return hipGetLastError();
}
int f32_conv1_wgrad_unpool_grid() {
  static const int n = resident((const void*)conv1_f32_wgrad_unpool_k);
  return n;
}
hipError_t f32_conv1_wgrad_unpool(const float* x, const float* dp, const uint8_t* codes, int Nb, int splits,
                                  float* slab, hipStream_t st) {
  if (Nb <= 0 || splits <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv1_f32_wgrad_unpool_k, dim3(splits), dim3(NT1), 0, st, x, dp, codes, Nb, slab);
  return hipGetLastError();
}
int f32_conv1_wgrad_lrn_grid() {
  static const int n = resident((const void*)conv1_f32_wgrad_lrn_k);
  return n;
}
hipError_t f32_conv1_wgrad_lrn(const float* x, const float* dn, const float* p1, const uint8_t* codes, int Nb,
                               int splits, float bias, float alpha, float beta, float* slab, hipStream_t st) {
  if (Nb <= 0 || splits <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv1_f32_wgrad_lrn_k, dim3(splits), dim3(NT1), 0, st, x, dn, p1, codes, Nb, bias, alpha, beta,
                     slab);
  return hipGetLastError();
}
hipError_t f32_conv1_wgrad(const float* x, const float* dy, int Nb, int splits, float* slab, hipStream_t st) {
  if (Nb <= 0 || splits <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv1_f32_wgrad_k, dim3(splits), dim3(NT1), 0, st, x, dy, Nb, slab);
  return hipGetLastError();
}

}  // namespace mnistx
