// LDS-halo implicit-GEMM 5x5 convolution for the reference CNN's conv2 geometry
// (14x14 NHWC images, stride 1, SAME padding, Cin % 32 == 0): forward
// (conv + bias + ReLU) and data gradient (the same convolution of dY with the
// 180-degree-flipped, in/out-swapped filter, optional ReLU mask).
//
// The generic GEMM path (gemm.hip Im2colK) gathers every im2col element from
// L2: each input value is fetched 25 times (once per tap), and at Cin = 32..64
// the 16-byte gathers -- not the MFMAs -- bound it (conv2 dgrad 1.2 ms for
// 164 GFLOP at B = 16384).  Here a workgroup keeps
//   * its slice of the filter resident in LDS for the whole (persistent) launch,
//     as [tap][out channel][in channel] rows (B fragments = one ds_read_b128), and
//   * one zero-haloed 18x18xCin image at a time (A fragments = one ds_read_b128
//     of 8 channels of one (pixel, tap)),
// so HBM/L2 see each input image once per output-channel slice.  16-byte chunks
// are XOR-swizzled by row so a fragment's 16 rows hit 16 distinct bank groups.
// A wave computes four 16-pixel M-fragments per pass (B fragments shared), with
// v_mfma_f32_16x16x32_bf16 and K ordered (tap, channel block).  The next image is
// prefetched into VGPRs while the current one computes.
//
// Replaces: Conv2D / Conv2DBackpropInput of conv2,
// mnist_input.py:161 (reference CNN); the gemm.hip launchers route to it.
#include "common.h"
#include "launchers.h"
#include "lrn_math.h"

#include <cstdlib>

namespace mnistx {
namespace {

constexpr int HW = 14, KS = 5, HP = HW + 4, NPIX = HW * HW, NTAP = KS * KS;
// Forward / dgrad tile: 18 rows x WR = 20 pixels (interior at rows/cols 2..15).  An
// M-fragment is ONE output row of 16 pixels (columns 14/15 are padding whose results
// are dropped; they read the zero columns 16..19), so a fragment's 16 lanes read 16
// CONSECUTIVE tile pixels -- the property the swizzle below needs.
constexpr int WR = 20;
constexpr int MFR = HW;                      // 14 row fragments per image

// 16-byte chunk swizzle of tile/filter row r (CH chunks per row), for ds_read_b128
// by 16 consecutive rows x one chunk per lane group: with 64-B rows (CH 4, four rows
// per 256-B bank line) chunk ^= bit2(r)*2, with 128-B rows (CH 8) chunk ^= r & 6 --
// each of the instruction's four 16-lane bank groups ({0-3,12-15,20-27}, ...) then
// hits 16 distinct 16-byte bank slots for ANY start row (exhaustive check:
// bench/lds_sim.py halo).  (The previous c ^ (r & 3) over 13 wrapped 16-pixel runs
// measured 45-51 % LDS bank-conflict cycles.)
template <int CH>
DEV int swz(int r, int c) {
  if constexpr (CH == 4) return c ^ ((r >> 1) & 2);
  else return c ^ (r & 6);
}

// Lane i <- lane i + N of its 16-lane row, zero past the row's end (DPP row_shl; the
// zero is exactly the tile's right halo: see ROWS below)
template <int N>
DEV uint32_t row_shl(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + N, 0xf, 0xf, true);
}
DEV u32x4 row_shl4(const u32x4& v, int n) {
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    o[j] = n == 1 ? row_shl<1>(v[j]) : n == 2 ? row_shl<2>(v[j]) : n == 3 ? row_shl<3>(v[j]) : row_shl<4>(v[j]);
  return o;
}

// MODE 0 = forward: out[p][n] = relu(sum_{tap,ci} x[p+tap][ci] W[tap][ci][n] + b[n])
// MODE 1 = data gradient: out[p][n] = mask * sum_{tap,ci} dy[p+tap][ci] W[24-tap][n][ci]
//   (W is the conv's [kh][kw][cin][cout] filter; here ci runs over the conv's
//    output channels and n over its input channels)
// LRNX: x is the input of an LRN (radius 4) whose output is the convolution's input;
// the LRN is applied to each staged 16-byte vector (the CH lanes of a pixel are
// adjacent), bitwise lrn_fwd_k, so the LRN output never exists in HBM.
// ROWS: a wave's FR output rows (one image, FR | 14) read each of the FR + 4 tile rows
// they touch ONCE per channel block (one ds_read_b128 at columns 0..15) instead of once
// per (row, tap): tap column kw is the fragment shifted by kw lanes (DPP row_shl), and
// the lanes it shifts in past column 15 are the zero halo columns 16..19 the tile holds
// there anyway (only output columns i < 14 are kept, i + kw <= 17).  Tile-row reuse
// across kh comes from fragment h + kh.  The A-side LDS reads drop from 25 FR to FR + 4
// per channel block: the B (filter) reads, one per (tap, nf) shared by the FR rows, are
// then most of the LDS traffic.
template <int CIN, int CW, int NW, int MODE, int FR, int IMGS, bool LRNX = false, bool ROWS = false>
__global__ __launch_bounds__(64 * NW) void conv5_halo_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                        int wcin, int wcout, const float* __restrict__ bias, int bias_n,
                                                        int relu, const bf16_t* __restrict__ mask, int ldm, int B,
                                                        bf16_t* __restrict__ out, int ldo, const LrnParams lrn) {
  constexpr int NT = 64 * NW;
  constexpr int CH = CIN / 8;                 // 16-byte chunks per pixel / filter row
  constexpr int NF = CW / 16;
  constexpr int KC = CIN / 32;                // 32-wide k-steps per tap
  constexpr int XE = HP * WR * CIN;           // image tile elements (one image)
  constexpr int WE = NTAP * CW * CIN;         // filter slice elements
  constexpr int NV = NPIX * CH;               // 16-byte vectors per input image
  constexpr int PER = (IMGS * NV + NT - 1) / NT;
  constexpr int NGRP = (IMGS * MFR + FR - 1) / FR;   // fragment groups per image group (FR share the B reads)
  static_assert(CIN % 32 == 0 && CW % 16 == 0 && (CH == 4 || CH == 8), "conv5_halo geometry");
  __shared__ __attribute__((aligned(16))) bf16_t xs[IMGS * XE];
  __shared__ __attribute__((aligned(16))) bf16_t ws[WE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.y * CW;

  for (int e = tid; e < IMGS * XE / 8; e += NT) *(u32x4*)(xs + 8 * e) = u32x4{0u, 0u, 0u, 0u};   // halo stays zero
  // filter slice -> ws[(tap*CW + n)][ci] (swizzled chunks), once per block
  if constexpr (MODE == 0) {
    // W[tap][ci][n0 + n .. +7] is contiguous: one vector load, 8 scattered 2-byte LDS stores
    for (int e = tid; e < NTAP * CIN * (CW / 8); e += NT) {
      const int nv = e % (CW / 8), rest = e / (CW / 8), ci = rest % CIN, t = rest / CIN;
      const u32x4 v = *(const u32x4*)(w + ((int64_t)t * wcin + ci) * wcout + n0 + 8 * nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = t * CW + 8 * nv + j;
        ws[r * CIN + (swz<CH>(r, ci >> 3) << 3) + (ci & 7)] = (bf16_t)((v[j >> 1] >> (16 * (j & 1))) & 0xffffu);
      }
    }
  } else {
    // flipped tap, row n = conv input channel n0 + n, columns = conv output channels (contiguous)
    for (int e = tid; e < NTAP * CW * CH; e += NT) {
      const int c = e % CH, r = e / CH, n = r % CW, t = r / CW;
      const u32x4 v = *(const u32x4*)(w + ((int64_t)(NTAP - 1 - t) * wcin + n0 + n) * wcout + 8 * c);
      *(u32x4*)(ws + r * CIN + (swz<CH>(r, c) << 3)) = v;
    }
  }

  // this lane's bias values (output channels n0 + nf*16 + 4g + r), loaded once: a
  // conditional load inside the epilogue stalled every fragment on its latency
  float bsv[NF][4];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int nb = n0 + nf * 16 + 4 * g + r;
      bsv[nf][r] = (MODE == 0 && bias != nullptr && nb < bias_n) ? bias[nb] : 0.f;
    }

  u32x4 pre[PER];
  auto gload = [&](int img0) {               // images img0 .. img0+IMGS-1 are contiguous in HBM
    // branch-free buffer loads (common.h): images past the batch read zeros
    const auto r = buf_rsrc(x + (int64_t)img0 * NPIX * CIN, (uint32_t)(max(0, min(IMGS, B - img0)) * NPIX * CIN * 2));
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int v = tid + u * NT;
      pre[u] = buf_b128(r, v < IMGS * NV ? (uint32_t)(16 * v) : BUF_OOB);
    }
  };
  const int gstride = gridDim.x * IMGS;
  gload(blockIdx.x * IMGS);
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += gstride) {
    __syncthreads();                            // previous group's fragments consumed
    if constexpr (LRNX) {                       // every lane: the DPP exchanges read neighbours
      static_assert(CH == 4 && NT % CH == 0, "LRN fold: 32 channels = 4 lanes per pixel");
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        pre[u] = lrn_fwd8<CH, 4>(pre[u], tid % CH, lrn.bias, lrn.alpha, lrn.beta);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int v = tid + u * NT;
      if (v < IMGS * NV) {
        const int im = v / NV, vv = v - im * NV;
        const int p = vv / CH, c = vv - p * CH;
        const int P = (p / HW + 2) * WR + (p % HW) + 2;
        const int PI = im * (XE / CIN) + P;      // pixel index across the group's tiles
        *(u32x4*)(xs + PI * CIN + (swz<CH>(PI, c) << 3)) = pre[u];
      }
    }
    __syncthreads();
    gload(img0 + gstride);                      // next group in flight during the MFMAs
    for (int gr = wave; gr < NGRP; gr += NW) {
      // fragments FR*gr .. FR*gr+FR-1 = (image, output row); lane i = output column
      int P0[FR];                               // tile pixel under tap (0,0) of this lane's output pixel
#pragma unroll
      for (int h = 0; h < FR; ++h) {
        const int f = min(FR * gr + h, IMGS * MFR - 1), im = f / MFR;
        P0[h] = im * (XE / CIN) + (f - im * MFR) * WR + i;
      }
      // dgrad ReLU mask of this group's outputs, loaded before the MFMAs so its latency hides
      // behind them (loaded in the epilogue, every wave of the block stalled on it at once)
      u32x2 mkv[FR][NF];
      if (MODE == 1 && mask != nullptr) {
#pragma unroll
        for (int h = 0; h < FR; ++h) {
          const int f = FR * gr + h, im = f / MFR;
          const int q = (f - im * MFR) * HW + i;
          const bool ok = f < IMGS * MFR && i < HW && img0 + im < B;
          const int64_t row = (int64_t)(img0 + im) * NPIX + q;
#pragma unroll
          for (int nf = 0; nf < NF; ++nf)
            mkv[h][nf] = ok ? *(const u32x2*)(mask + row * ldm + n0 + nf * 16 + 4 * g) : u32x2{0u, 0u};
        }
      }
      f32x4 acc[FR][NF];
#pragma unroll
      for (int h = 0; h < FR; ++h)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) acc[h][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (ROWS) {
        static_assert(MFR % FR == 0, "ROWS: row groups inside one image");
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const int c = 4 * kc + g;
          u32x4 R[FR + 4];
#pragma unroll
          for (int t = 0; t < FR + 4; ++t) {
            const int P = P0[0] + t * WR;
            R[t] = *(const u32x4*)(xs + P * CIN + (swz<CH>(P, c) << 3));
          }
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            u32x4 Sh[FR + 4];
#pragma unroll
            for (int t = 0; t < FR + 4; ++t) Sh[t] = kw == 0 ? R[t] : row_shl4(R[t], kw);
#pragma unroll
            for (int kh = 0; kh < KS; ++kh) {
              const int t = kh * KS + kw;
              bf16x8 b[NF];
#pragma unroll
              for (int nf = 0; nf < NF; ++nf) {
                const int r = t * CW + nf * 16 + i;
                b[nf] = __builtin_bit_cast(bf16x8, *(const u32x4*)(ws + r * CIN + (swz<CH>(r, c) << 3)));
              }
#pragma unroll
              for (int h = 0; h < FR; ++h)
#pragma unroll
                for (int nf = 0; nf < NF; ++nf)
                  acc[h][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nf], __builtin_bit_cast(bf16x8, Sh[h + kh]),
                                                                       acc[h][nf], 0, 0, 0);
            }
          }
        }
      } else
      for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const int t = kh * KS + kw;
          const int dP = kh * WR + kw;
#pragma unroll
          for (int kc = 0; kc < KC; ++kc) {
            const int c = 4 * kc + g;
            bf16x8 a[FR], b[NF];
#pragma unroll
            for (int h = 0; h < FR; ++h) {
              const int P = P0[h] + dP;
              a[h] = __builtin_bit_cast(bf16x8, *(const u32x4*)(xs + P * CIN + (swz<CH>(P, c) << 3)));
            }
#pragma unroll
            for (int nf = 0; nf < NF; ++nf) {
              const int r = t * CW + nf * 16 + i;
              b[nf] = __builtin_bit_cast(bf16x8, *(const u32x4*)(ws + r * CIN + (swz<CH>(r, c) << 3)));
            }
#pragma unroll
            for (int h = 0; h < FR; ++h)
#pragma unroll
              for (int nf = 0; nf < NF; ++nf)
                // filter rows as the A operand: D = (W x)^T, so a lane holds 4 CONSECUTIVE
                // output channels of one pixel (one 8-byte store) instead of one channel of
                // 4 pixels (four 2-byte stores)
                acc[h][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nf], a[h], acc[h][nf], 0, 0, 0);
          }
        }
      }
      // D row 4g + r = output channel n0 + nf*16 + 4g + r, column i = output column ow
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
        const int nb = n0 + nf * 16 + 4 * g;
        const float* bn = bsv[nf];
#pragma unroll
        for (int h = 0; h < FR; ++h) {
          const int f = FR * gr + h, im = f / MFR;
          const int q = (f - im * MFR) * HW + i;
          if (f < IMGS * MFR && i < HW && img0 + im < B) {
            const int64_t row = (int64_t)(img0 + im) * NPIX + q;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] = acc[h][nf][r] + bn[r];
              if (relu) v[r] = fmaxf(v[r], 0.f);
            }
            if (MODE == 1 && mask != nullptr) {
              const u32x2 mk = mkv[h][nf];
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (!(bf2f((bf16_t)((mk[r >> 1] >> (16 * (r & 1))) & 0xffffu)) > 0.f)) v[r] = 0.f;
            }
            *(u32x2*)(out + row * ldo + nb) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
// dW[tap][ci][co] = sum_p x[p + tap][ci] dY[p][co]  (+ bias row: sum_p dY[p][co]).
// M = (tap, ci) rows (25*CIN + the bias row), N = COUT, K = pixels.  A persistent
// block keeps the whole M x N partial in registers (8 waves, row tiles dealt
// round-robin, all NFW column tiles each) and streams images: per image the x
// tile (zero halo) and dY (14 x 16 pixel rows, columns 14/15 zero) are staged in
// LDS once and every (tap, ci-block) row tile reads its A fragments straight from
// the x tile with ds_read_b64_tr_b16 (k = 16 consecutive pixels of an image row,
// +16 = the next row).  The pixel padding (columns 14/15) multiplies zero dY.
// One fp32 partial per block goes to the split-K slab ([S][25*CIN+1][COUT] rows
// (tap*CIN + ci), bias row 25*CIN), reduced by splitk_reduce like the GEMM path.
template <int CIN, int COUT, int NW, bool LRNX = false>
__global__ __launch_bounds__(64 * NW) void conv5_halo_wgrad_k(const bf16_t* __restrict__ x,
                                                              const bf16_t* __restrict__ dy, int B,
                                                              float* __restrict__ slab, const LrnParams lrn) {
  constexpr int NT = 64 * NW;
  constexpr int SX = CIN + 16, SD = COUT + 16;          // tr-read row strides (gemm.hip ImgStride rule)
  constexpr int XP = HP * HP + 8;                       // tile pixels + zero over-read slack
  constexpr int DPIX = HW * 16;                         // dY rows: 14 image rows x 16 columns
  constexpr int MREAL = NTAP * CIN, MTOT = MREAL + 1;
  constexpr int RT = NTAP * (CIN / 16) + 1;             // row tiles incl. the bias tile
  constexpr int NFW = COUT / 16;
  constexpr int RPW = (RT + NW - 1) / NW;               // row tiles per wave (max)
  constexpr int KSTEPS = HW / 2;                        // 32 pixels (two image rows) per k-step
  constexpr int XV = NPIX * CIN / 8, DV = NPIX * COUT / 8;
  constexpr int PX = (XV + NT - 1) / NT, PD = (DV + NT - 1) / NT;
  static_assert(CIN % 16 == 0 && COUT % 16 == 0 && HW % 2 == 0, "");
  __shared__ __attribute__((aligned(16))) bf16_t xs[XP * SX];
  __shared__ __attribute__((aligned(16))) bf16_t ds[DPIX * SD];
  __shared__ __attribute__((aligned(16))) bf16_t ones[32 * 16];   // bias A tile: column 0 = 1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  for (int e = tid; e < XP * SX / 8; e += NT) *(u32x4*)(xs + 8 * e) = u32x4{0u, 0u, 0u, 0u};
  for (int e = tid; e < DPIX * SD / 8; e += NT) *(u32x4*)(ds + 8 * e) = u32x4{0u, 0u, 0u, 0u};
  for (int e = tid; e < 32 * 16; e += NT) ones[e] = (e & 15) == 0 ? (bf16_t)0x3f80 : (bf16_t)0;

  f32x4 acc[RPW][NFW];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int n = 0; n < NFW; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 px[PX], pd[PD];
  auto gload = [&](int img) {                 // branch-free buffer loads; past the batch: zeros
    const bool in = img < B;
    const auto rx = buf_rsrc(x + (int64_t)(in ? img : 0) * NPIX * CIN, in ? (uint32_t)(NPIX * CIN * 2) : 0u);
    const auto rd = buf_rsrc(dy + (int64_t)(in ? img : 0) * NPIX * COUT, in ? (uint32_t)(NPIX * COUT * 2) : 0u);
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int v = tid + u * NT;
      px[u] = buf_b128(rx, v < XV ? (uint32_t)(16 * v) : BUF_OOB);
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int v = tid + u * NT;
      pd[u] = buf_b128(rd, v < DV ? (uint32_t)(16 * v) : BUF_OOB);
    }
  };
  gload(blockIdx.x);
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    __syncthreads();
    if constexpr (LRNX) {   // x is the LRN input: normalise while staging (bitwise lrn_fwd_k)
      static_assert(CIN == 32 && NT % 4 == 0, "LRN fold: 4 lanes per pixel");
#pragma unroll
      for (int u = 0; u < PX; ++u) {
        px[u] = lrn_fwd8<CIN / 8, 4>(px[u], tid % (CIN / 8), lrn.bias, lrn.alpha, lrn.beta);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int v = tid + u * NT;
      if (v < XV) {
        const int pix = v / (CIN / 8), c = v - pix * (CIN / 8);
        const int P = (pix / HW + 2) * HP + (pix % HW) + 2;
        *(u32x4*)(xs + P * SX + 8 * c) = px[u];
      }
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int v = tid + u * NT;
      if (v < DV) {
        const int pix = v / (COUT / 8), c = v - pix * (COUT / 8);
        const int Q = (pix / HW) * 16 + (pix % HW);
        *(u32x4*)(ds + Q * SD + 8 * c) = pd[u];
      }
    }
    __syncthreads();
    gload(img + gridDim.x);
    for (int ks = 0; ks < KSTEPS; ++ks) {
      // B fragments: dY rows (2ks, 2ks+1) x 16 columns, all column tiles
      bf16x8 b[NFW];
      const bf16_t* db = ds + (2 * ks * 16 + 4 * g + q) * SD + 4 * p4;
#pragma unroll
      for (int n = 0; n < NFW; ++n)
        b[n] = join(lds_tr4(db + 16 * n), lds_tr4(db + 16 * SD + 16 * n));
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const int rt = wave + r * NW;
        if (rt < RT) {                            // wave-uniform
          bf16x8 a;
          if (rt < RT - 1) {
            const int t = rt / (CIN / 16), cb = rt - t * (CIN / 16);
            const int P = (2 * ks + t / KS) * HP + (t % KS) + 4 * g + q;   // pixel k = 4g+q of row 2ks, tap t
            const bf16_t* ab = xs + P * SX + 16 * cb + 4 * p4;
            a = join(lds_tr4(ab), lds_tr4(ab + HP * SX));                  // +16 k = next image row
          } else {
            const bf16_t* ob = ones + (4 * g + q) * 16 + 4 * p4;
            a = join(lds_tr4(ob), lds_tr4(ob + 16 * 16));
          }
#pragma unroll
          for (int n = 0; n < NFW; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[n], acc[r][n], 0, 0, 0);
        }
      }
    }
  }
  // partial -> slab[blockIdx][m][n]: D rows 4g + r2 of the tile, column (lane & 15)
  float* out = slab + (int64_t)blockIdx.x * MTOT * COUT;
  const int li = lane & 15;
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int rt = wave + r * NW;
    if (rt < RT) {
#pragma unroll
      for (int n = 0; n < NFW; ++n)
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2) {
          const int m = rt * 16 + 4 * g + r2;
          if (m < MTOT) out[(int64_t)m * COUT + 16 * n + li] = acc[r][n][r2];
        }
    }
  }
}

template <int CIN, int COUT, int NW>
int halo_wgrad_resident(int* per_cu = nullptr) {
  static int per = -1, pc = 1;
  if (per < 0) {
    int dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, conv5_halo_wgrad_k<CIN, COUT, NW>, 64 * NW, 0) ==
            hipSuccess &&
        hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && pc > 0)
      per = pc * cus;
    else
      per = 256, pc = 1;
  }
  if (per_cu) *per_cu = pc;
  return per;
}

template <int CIN, int CW, int NW, int MODE, int FR, int IMGS, bool LRNX = false, bool ROWS = false>
int halo_grid(int B) {
  static int per = -1, pc = 1;
  if (per < 0) {
    int dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, conv5_halo_k<CIN, CW, NW, MODE, FR, IMGS, LRNX, ROWS>, 64 * NW, 0) ==
            hipSuccess &&
        hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && pc > 0)
      per = pc * cus;
    else
      per = 256, pc = 1;
  }
  const int groups = (B + IMGS - 1) / IMGS, res = reserve_cut(per, pc);
  return cap_grid(groups < res ? groups : res);
}

template <int CIN, int CW, int NW, int MODE, int FR, int IMGS = 1, bool LRNX = false, bool ROWS = false>
hipError_t run_halo(const bf16_t* x, const bf16_t* w, int wcin, int wcout, const float* bias, int bias_n, int relu,
                    const bf16_t* mask, int ldm, int B, bf16_t* out, int ncols, int ldo, hipStream_t st,
                    LrnParams lrn = LrnParams{0.f, 0.f, 0.f, 0}) {
  if (B <= 0) return hipSuccess;
  dim3 grid(halo_grid<CIN, CW, NW, MODE, FR, IMGS, LRNX, ROWS>(B), ncols / CW);
  hipLaunchKernelGGL((conv5_halo_k<CIN, CW, NW, MODE, FR, IMGS, LRNX, ROWS>), grid, dim3(64 * NW), 0, st, x, w, wcin, wcout, bias,
                     bias_n, relu, mask, ldm, B, out, ldo, lrn);
  return hipGetLastError();
}

}  // namespace

// Geometry the halo kernels cover: 14x14, 5x5, pad 2, stride 1; fwd Cin 32 -> Cout % 32,
// dgrad dY 64 channels -> dX 32.
bool conv5_halo_fwd_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout) {
  return H == 14 && W == 14 && OH == 14 && OW == 14 && KH == 5 && KW == 5 && ph == 2 && pw == 2 && C == 32 &&
         Cout % 32 == 0;
}
bool conv5_halo_dgrad_ok(int OH, int OW, int Cout, int H, int W, int KH, int KW, int ph, int pw, int Cin) {
  return H == 14 && W == 14 && OH == 14 && OW == 14 && KH == 5 && KW == 5 && ph == 2 && pw == 2 && Cout == 64 &&
         Cin % 32 == 0;
}

// Launch variant (index; measured in profiles/r2/halo): the defaults below, or
// set_halo_variants() (the tests run every variant in one process).
static int g_halo_override[2] = {-1, -1};
static int halo_variant(const char* name, int dflt) {
  const int which = name[12] == 'F' ? 0 : 1;   // "MNISTX_HALO_FWD" / "MNISTX_HALO_DGRAD"
  return g_halo_override[which] >= 0 ? g_halo_override[which] : dflt;
}

// Launch shapes (profiles/r2/halo: per-kernel us at B = 16384).  More resident waves
// beat bigger per-wave tiles: 8 waves x 2 row fragments 350 us fwd / 326 us dgrad vs
// 4 x 4 fragments 435 / 520 us.
hipError_t conv5_halo_fwd(const bf16_t* x, const bf16_t* w, int Nb, int C, int Cout, const float* bias, int bias_n,
                          int relu, bf16_t* out, hipStream_t st, LrnParams lrn) {
  if (lrn.on)   // norm1 folded into the staging: the default launch shape only
    return run_halo<32, 32, 8, 0, 7, 4, true, true>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout,
                                                     st, lrn);
  const int v = halo_variant("MNISTX_HALO_FWD", 0);
  switch (v) {
    case 1:   // whole Cout per block (NF = 4): 125 KB LDS, 1 block / CU
      if (Cout == 64) return run_halo<32, 64, 4, 0, 4>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
      break;
    case 2:   // 4 waves x 4 row fragments
      return run_halo<32, 32, 4, 0, 4>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
    case 3:   // 16 waves x 1 row fragment
      return run_halo<32, 32, 16, 0, 1>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
    case 4:   // two images per block, 8 waves x 2 row fragments (7 of 8 groups busy twice)
      return run_halo<32, 32, 8, 0, 2, 2>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
    case 5:   // whole Cout, 8 waves x 2 row fragments
      if (Cout == 64) return run_halo<32, 64, 8, 0, 2>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
      break;
    case 6:   // ROWS: 7 waves x 2 row fragments (every wave busy)
      return run_halo<32, 32, 7, 0, 2, 1, false, true>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
    case 7:   // ROWS: four images, 8 waves x 7 row fragments
      return run_halo<32, 32, 8, 0, 7, 4, false, true>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
    case 9:   // ROWS: two images, 14 waves x 2 row fragments (one workgroup per CU)
      return run_halo<32, 32, 14, 0, 2, 2, false, true>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
    case 8:   // the pre-ROWS default: 8 waves x 2 row fragments, 25 A reads per row and channel block
      return run_halo<32, 32, 8, 0, 2>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
    default: break;
  }
  return run_halo<32, 32, 8, 0, 7, 4, false, true>(x, w, C, Cout, bias, bias_n, relu, nullptr, 0, Nb, out, Cout, Cout, st);
}

hipError_t conv5_halo_dgrad(const bf16_t* dy, const bf16_t* w, int Nb, int Cout, int Cin, const bf16_t* mask,
                            bf16_t* dx, hipStream_t st) {
  const int v = halo_variant("MNISTX_HALO_DGRAD", 0);
  switch (v) {
    case 1:   // 4 waves x 4 row fragments
      return run_halo<64, 32, 4, 1, 4>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 2:   // half the input channels of the conv per block (NF = 1)
      return run_halo<64, 16, 4, 1, 4>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 3:   // 16 waves x 1 row fragment
      return run_halo<64, 32, 16, 1, 1>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 4:   // half the channels, 8 waves x 2 row fragments (97 KB LDS)
      return run_halo<64, 16, 8, 1, 2>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 5:   // 2 waves x 7 row fragments
      return run_halo<64, 32, 2, 1, 7>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 6:   // ROWS: 7 waves x 2 row fragments
      return run_halo<64, 32, 7, 1, 2, 1, false, true>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 7:   // ROWS: half the channels, two images, 4 waves x 7 row fragments (143 KB LDS)
      return run_halo<64, 16, 4, 1, 7, 2, false, true>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 9:   // ROWS: half the channels, two images, 14 waves x 2 row fragments (143 KB LDS)
      return run_halo<64, 16, 14, 1, 2, 2, false, true>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    case 8:   // the pre-ROWS default
      return run_halo<64, 32, 8, 1, 2>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
    default: break;
  }
  return run_halo<64, 32, 7, 1, 2, 1, false, true>(dy, w, Cin, Cout, nullptr, 0, 0, mask, Cin, Nb, dx, Cin, Cin, st);
}

void set_halo_variants(int fwd, int dgrad) {
  g_halo_override[0] = fwd;
  g_halo_override[1] = dgrad;
}

bool conv5_halo_wgrad_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout,
                         int with_bias) {
  return with_bias && H == 14 && W == 14 && OH == 14 && OW == 14 && KH == 5 && KW == 5 && ph == 2 && pw == 2 &&
         C == 32 && Cout == 64;
}
int conv5_halo_wgrad_grid(int Nb) {
  int pc = 1;
  const int r = reserve_cut(halo_wgrad_resident<32, 64, 8>(&pc), pc);
  return Nb < r ? (Nb < 1 ? 1 : Nb) : r;
}
hipError_t conv5_halo_wgrad(const bf16_t* x, const bf16_t* dy, int Nb, int grid, float* slab, hipStream_t st,
                            LrnParams lrn) {
  if (Nb <= 0) return hipSuccess;
  if (lrn.on)
    hipLaunchKernelGGL((conv5_halo_wgrad_k<32, 64, 8, true>), dim3(grid), dim3(512), 0, st, x, dy, Nb, slab, lrn);
  else
    hipLaunchKernelGGL((conv5_halo_wgrad_k<32, 64, 8>), dim3(grid), dim3(512), 0, st, x, dy, Nb, slab, lrn);
  return hipGetLastError();
}

}  // namespace mnistx
