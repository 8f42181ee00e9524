// Fused small-channel conv blocks for gfx950: conv(5x5, stride 1) + bias + ReLU + 2x2/2 max-pool.
//
// The first conv layers of MNIST nets have tiny channel counts (Cin 1/3/8, Cout
// 8/16/32), so a generic implicit GEMM wastes its tiles and spends its time in
// index arithmetic.  These kernels are specialised at compile time on the
// layer geometry and keep one padded input image per LDS tile:
//
// * Pool-window-major GEMM rows: output pixel row r = 4*window + d with
//   d = (dy, dx) inside the 2x2 pooling window.  A v_mfma_f32_16x16x32_bf16
//   accumulator gives each lane rows 4g..4g+3 of one column, i.e. exactly one
//   pooling window of one channel — so bias + ReLU + max-pool + argmax happen
//   in registers and the full-resolution conv output never touches HBM.
// * im2col fragments are gathered straight from the LDS tile with per-lane
//   offsets precomputed once per kernel (no division in the inner loop);
//   weight fragments stay in VGPRs for the whole persistent grid-stride loop.
// * Backward (wgrad): the max-unpool + ReLU mask is applied while building the
//   dY operand from the pooled gradient (argmax byte + pooled value > 0), the
//   bias gradient is a virtual ones-row of the im2col operand, per-block fp32
//   partials go to a slab reduced deterministically by splitk_reduce.
// * Backward (dgrad, LeNet conv2): the unpooled dY image is staged in LDS with
//   a KS-1-PAD halo; the flipped-filter implicit GEMM reads its K-contiguous
//   operand with ds_read_b64.
//
// Replaces: Conv2D + BiasAdd + Relu + MaxPool and
// their gradients at mnist_input.py:142-150 (conv1 -> pool1) and the LeNet-5
// conv blocks.
#include "common.h"
#include "launchers.h"

namespace mnistx {
namespace {

// smallest column count >= c whose byte width (c * cin * 2) is a multiple of 16
constexpr int align_cols(int c, int cin) {
  while ((c * cin * 2) % 16 != 0) ++c;
  return c;
}

template <int CIN_, int COUT_, int KS_, int PAD_, int H_, int W_>
struct Geo {
  static constexpr int CIN = CIN_, COUT = COUT_, KS = KS_, PAD = PAD_, H = H_, W = W_;
  static constexpr int HP = H + 2 * PAD, WP = W + 2 * PAD;
  static constexpr int OH = HP - KS + 1, OW = WP - KS + 1;
  // LDS tile rows: the interior starts at column X0 >= PAD and every row is a
  // multiple of 16 bytes, so the interior rows are filled with 8-byte vectors.
  static constexpr int X0 = align_cols(PAD, CIN);
  static constexpr int WS = align_cols(X0 + W + PAD, CIN);
  static constexpr int XOFF = X0 - PAD;
  static constexpr int ROWV = W * CIN / 4;            // 8-byte vectors per interior row
  static_assert((W * CIN) % 4 == 0, "interior rows must be whole 8-byte vectors");
  static constexpr int PH = OH / 2, PW = OW / 2;
  static constexpr int NWIN = PH * PW;
  static constexpr int NPIX = OH * OW;
  static constexpr int MF = (NPIX + 15) / 16;
  static constexpr int KC = KS * KS * CIN;
  static constexpr int KSTEPS = (KC + 31) / 32;
  static constexpr int NF = (COUT + 15) / 16;
  static constexpr int NCOL = NF * 16;
  static constexpr int TILE = HP * WS * CIN;
  static constexpr int INTERIOR = H * W * CIN;
  static constexpr int KM = ((KC + 1) + 15) / 16 * 16;  // wgrad rows incl. the bias (ones) row
  static constexpr int MFW = KM / 16;
  static constexpr int RSTEPS = (NPIX + 31) / 32;
  static_assert(OH % 2 == 0 && OW % 2 == 0, "pool-window-major order needs an even conv output");
  static_assert(NPIX == 4 * NWIN, "");

  // LDS offset of im2col column k = (kh, kw, ci) relative to the pixel base
  static DEV int kdelta(int k) {
    const int tap = k / CIN, ci = k - (k / CIN) * CIN;
    const int kh = tap / KS, kw = tap - (tap / KS) * KS;
    return (kh * WS + kw) * CIN + ci;
  }
  // LDS offset of the top-left input pixel feeding pool window w
  static DEV int wbase(int w) {
    const int ph = w / PW, pw = w - (w / PW) * PW;
    return ((2 * ph) * WS + 2 * pw + XOFF) * CIN;
  }
  static DEV int doff(int d) { return ((d >> 1) * WS + (d & 1)) * CIN; }
};

DEV __bf16 as_bf(bf16_t v) { return __builtin_bit_cast(__bf16, v); }

constexpr int NTH = 256;

// Copy IMGS input images (NHWC, interior only) into their LDS tiles with
// 8-byte vectors; the zero border written once at kernel start is untouched.
template <class G, int IMGS>
DEV void fill_tiles(bf16_t* tile, const bf16_t* __restrict__ x, int img0, int B, int tid) {
  constexpr int NV = IMGS * G::H * G::ROWV;
  for (int e = tid; e < NV; e += NTH) {
    const int im = e / (G::H * G::ROWV), rem = e - im * (G::H * G::ROWV);
    const int hh = rem / G::ROWV, vv = rem - hh * G::ROWV;
    u32x2 v = {0u, 0u};
    if (img0 + im < B) v = *(const u32x2*)(x + (int64_t)(img0 + im) * G::INTERIOR + hh * G::W * G::CIN + 4 * vv);
    *(u32x2*)(tile + im * G::TILE + ((hh + G::PAD) * G::WS + G::X0) * G::CIN + 4 * vv) = v;
  }
}

// ------------------------------------------------------------------ forward
template <class G, int IMGS>
__global__ __launch_bounds__(NTH) void convpool_fwd_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const float* __restrict__ bias, int bias_n, int B,
                                                      bf16_t* __restrict__ pooled, uint8_t* __restrict__ arg) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[IMGS * G::TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  for (int e = tid; e < IMGS * G::TILE; e += NTH) tile[e] = 0;

  int dl[G::KSTEPS][8];
  bf16x8 bfr[G::KSTEPS][G::NF];
#pragma unroll
  for (int s = 0; s < G::KSTEPS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 4 * g + (j & 3) + 16 * (j >> 2);
      dl[s][j] = k < G::KC ? G::kdelta(k) : 0;
#pragma unroll
      for (int nf = 0; nf < G::NF; ++nf) {
        const int n = nf * 16 + li;
        bfr[s][nf][j] = as_bf((k < G::KC && n < G::COUT) ? w[k * G::COUT + n] : (bf16_t)0);
      }
    }
  float bs[G::NF];
#pragma unroll
  for (int nf = 0; nf < G::NF; ++nf) {
    const int n = nf * 16 + li;
    bs[nf] = n < bias_n ? bias[n] : 0.f;
  }

  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += gridDim.x * IMGS) {
    __syncthreads();
    fill_tiles<G, IMGS>(tile, x, img0, B, tid);
    __syncthreads();
    for (int f = wave; f < IMGS * G::MF; f += NTH / 64) {
      const int im = f / G::MF, fm = f - im * G::MF;
      const int r = min(fm * 16 + li, G::NPIX - 1);
      const bf16_t* tb = tile + im * G::TILE + G::wbase(r >> 2) + G::doff(r & 3);
      f32x4 acc[G::NF];
#pragma unroll
      for (int nf = 0; nf < G::NF; ++nf) acc[nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) {
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = as_bf(tb[dl[s][j]]);
#pragma unroll
        for (int nf = 0; nf < G::NF; ++nf) acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[s][nf], acc[nf], 0, 0, 0);
      }
      const int win = fm * 4 + g;
      if (win < G::NWIN && img0 + im < B) {
#pragma unroll
        for (int nf = 0; nf < G::NF; ++nf) {
          const int n = nf * 16 + li;
          if (n < G::COUT) {
            float best = -INFINITY;
            int bi = 0;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              const float v = fmaxf(acc[nf][d] + bs[nf], 0.f);
              if (v > best) { best = v; bi = d; }
            }
            const int64_t off = ((int64_t)(img0 + im) * G::NWIN + win) * G::COUT + n;
            pooled[off] = f2bf(best);
            arg[off] = (uint8_t)bi;
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
template <class G, int IMGS>
__global__ __launch_bounds__(NTH) void convpool_wgrad_k(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dP,
                                                        const uint8_t* __restrict__ arg,
                                                        const bf16_t* __restrict__ P, int B,
                                                        float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[IMGS * G::TILE];
  __shared__ __attribute__((aligned(16))) bf16_t dys[IMGS * G::NWIN * G::COUT];
  __shared__ __attribute__((aligned(16))) uint8_t args[IMGS * G::NWIN * G::COUT];
  __shared__ float red[G::KM * G::NCOL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  for (int e = tid; e < IMGS * G::TILE; e += NTH) tile[e] = 0;

  int dk[G::MFW];
  int kind[G::MFW];  // 0: im2col column, 1: bias ones-row, 2: zero pad
#pragma unroll
  for (int mf = 0; mf < G::MFW; ++mf) {
    const int k = mf * 16 + li;
    dk[mf] = k < G::KC ? G::kdelta(k) : 0;
    kind[mf] = k < G::KC ? 0 : (k == G::KC ? 1 : 2);
  }
  f32x4 acc[G::MFW][G::NF];
#pragma unroll
  for (int mf = 0; mf < G::MFW; ++mf)
#pragma unroll
    for (int nf = 0; nf < G::NF; ++nf) acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int DEL = IMGS * G::NWIN * G::COUT;
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += gridDim.x * IMGS) {
    __syncthreads();
    fill_tiles<G, IMGS>(tile, x, img0, B, tid);
    static_assert(DEL % 8 == 0, "");
    for (int e8 = tid; e8 < DEL / 8; e8 += NTH) {
      const int e = 8 * e8;
      const int im = e / (G::NWIN * G::COUT);
      u32x4 v = {0u, 0u, 0u, 0u};
      u32x2 a = {0xffffffffu, 0xffffffffu};
      if (img0 + im < B) {
        const int64_t o = (int64_t)img0 * G::NWIN * G::COUT + e;
        const u32x4 pv = *(const u32x4*)(P + o);
        v = *(const u32x4*)(dP + o);
        a = *(const u32x2*)(arg + o);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!(u4_get(pv, j) > 0.f)) u4_set(v, j, 0);   // ReLU mask: pooled value > 0
      }
      *(u32x4*)(dys + e) = v;
      *(u32x2*)(args + e) = a;
    }
    __syncthreads();
    for (int it = wave; it < IMGS * G::RSTEPS; it += NTH / 64) {
      const int im = it / G::RSTEPS, s = it - im * G::RSTEPS;
      // this lane's two pool windows for the 8 reduction slots
      const int w0 = 8 * s + g, w1 = w0 + 4;
      const bool v0 = w0 < G::NWIN, v1 = w1 < G::NWIN;
      const bf16_t* tb = tile + im * G::TILE;
      const int b0 = v0 ? G::wbase(w0) : 0, b1 = v1 ? G::wbase(w1) : 0;
      bf16x8 bfr[G::NF];
#pragma unroll
      for (int nf = 0; nf < G::NF; ++nf) {
        const int n = nf * 16 + li;
        const bool nv = n < G::COUT;
        const int i0 = (im * G::NWIN + w0) * G::COUT + n, i1 = (im * G::NWIN + w1) * G::COUT + n;
        const bf16_t y0 = (nv && v0) ? dys[i0] : (bf16_t)0, y1 = (nv && v1) ? dys[i1] : (bf16_t)0;
        const int a0 = (nv && v0) ? args[i0] : 0xff, a1 = (nv && v1) ? args[i1] : 0xff;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bfr[nf][d] = as_bf(a0 == d ? y0 : (bf16_t)0);
          bfr[nf][4 + d] = as_bf(a1 == d ? y1 : (bf16_t)0);
        }
      }
#pragma unroll
      for (int mf = 0; mf < G::MFW; ++mf) {
        bf16x8 a;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bf16_t e0 = 0, e1 = 0;
          if (kind[mf] == 0) {
            e0 = v0 ? tb[b0 + G::doff(d) + dk[mf]] : (bf16_t)0;
            e1 = v1 ? tb[b1 + G::doff(d) + dk[mf]] : (bf16_t)0;
          } else if (kind[mf] == 1) {
            e0 = v0 ? (bf16_t)0x3f80 : (bf16_t)0;
            e1 = v1 ? (bf16_t)0x3f80 : (bf16_t)0;
          }
          a[d] = as_bf(e0);
          a[4 + d] = as_bf(e1);
        }
#pragma unroll
        for (int nf = 0; nf < G::NF; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[nf], acc[mf][nf], 0, 0, 0);
      }
    }
  }
  // cross-wave reduction in LDS in a FIXED wave order (bitwise reproducible:
  // no float atomics), then one fp32 slab per block
  for (int wv = 0; wv < NTH / 64; ++wv) {
    __syncthreads();
    if (wave == wv) {
#pragma unroll
      for (int mf = 0; mf < G::MFW; ++mf)
#pragma unroll
        for (int nf = 0; nf < G::NF; ++nf)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float& dst = red[(mf * 16 + 4 * g + r) * G::NCOL + nf * 16 + li];
            dst = (wv == 0) ? acc[mf][nf][r] : dst + acc[mf][nf][r];
          }
    }
  }
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * G::KM * G::COUT;
  for (int e = tid; e < G::KM * G::COUT; e += NTH) {
    const int m = e / G::COUT, n = e - m * G::COUT;
    out[e] = red[m * G::NCOL + n];
  }
}

// ------------------------------------------------------------------ data gradient (pooled dY -> dX)
template <class G, int IMGS>
__global__ __launch_bounds__(NTH) void convpool_dgrad_k(const bf16_t* __restrict__ dP, const uint8_t* __restrict__ arg,
                                                        const bf16_t* __restrict__ P, const bf16_t* __restrict__ w,
                                                        int B, bf16_t* __restrict__ dx) {
  constexpr int Q = G::KS - 1 - G::PAD;
  constexpr int OHQ = G::OH + 2 * Q, OWQ = G::OW + 2 * Q;
  constexpr int DT = OHQ * OWQ * G::COUT;
  constexpr int KD = G::KS * G::KS * G::COUT;
  constexpr int KSD = (KD + 31) / 32;
  constexpr int NPX = G::H * G::W;
  constexpr int MFD = (NPX + 15) / 16;
  constexpr int NFD = (G::CIN + 15) / 16;
  static_assert(G::COUT % 16 == 0, "dgrad operand reads need Cout % 16 == 0");
  __shared__ __attribute__((aligned(16))) bf16_t dyt[IMGS * DT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  for (int e = tid; e < IMGS * DT; e += NTH) dyt[e] = 0;

  int dd[KSD][2];
  bf16x8 bw[KSD][NFD];
#pragma unroll
  for (int s = 0; s < KSD; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * s + 4 * g + 16 * h;  // 4 consecutive co at one flipped tap
      const int tp = k / G::COUT, co = k - tp * G::COUT;
      const int kh = tp / G::KS, kw = tp - kh * G::KS;
      dd[s][h] = k < KD ? (kh * OWQ + kw) * G::COUT + co : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 4 * g + (j & 3) + 16 * (j >> 2);
      const int tp = k / G::COUT, co = k - tp * G::COUT;
      const int tap = G::KS * G::KS - 1 - tp;
#pragma unroll
      for (int nf = 0; nf < NFD; ++nf) {
        const int ci = nf * 16 + li;
        bw[s][nf][j] = as_bf((k < KD && ci < G::CIN) ? w[(tap * G::CIN + ci) * G::COUT + co] : (bf16_t)0);
      }
    }
  }
  constexpr int NWC = G::NWIN * G::COUT;
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += gridDim.x * IMGS) {
    __syncthreads();
    for (int e8 = tid; e8 < IMGS * NWC / 8; e8 += NTH) {
      const int e = 8 * e8;
      const int im = e / NWC, rem = e - im * NWC;
      const int win = rem / G::COUT, co = rem - win * G::COUT;
      u32x4 v = {0u, 0u, 0u, 0u};
      u32x2 a = {0xffffffffu, 0xffffffffu};
      if (img0 + im < B) {
        const int64_t o = (int64_t)img0 * NWC + e;
        const u32x4 pv = *(const u32x4*)(P + o);
        v = *(const u32x4*)(dP + o);
        a = *(const u32x2*)(arg + o);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!(u4_get(pv, j) > 0.f)) u4_set(v, j, 0);
      }
      const int ph = win / G::PW, pw = win - ph * G::PW;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int oh = 2 * ph + (d >> 1) + Q, ow = 2 * pw + (d & 1) + Q;
        u32x4 o = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t aj = ((j < 4 ? a[0] : a[1]) >> (8 * (j & 3))) & 0xff;
          if (aj == (uint32_t)d) u4_set(o, j, (bf16_t)((v[j >> 1] >> (16 * (j & 1))) & 0xffff));
        }
        *(u32x4*)(dyt + im * DT + (oh * OWQ + ow) * G::COUT + co) = o;
      }
    }
    __syncthreads();
    for (int f = wave; f < IMGS * MFD; f += NTH / 64) {
      const int im = f / MFD, mf = f - im * MFD;
      const int m = min(mf * 16 + li, NPX - 1);
      const int ih = m / G::W, iw = m - ih * G::W;
      const bf16_t* tb = dyt + im * DT + (ih * OWQ + iw) * G::COUT;
      f32x4 acc[NFD];
#pragma unroll
      for (int nf = 0; nf < NFD; ++nf) acc[nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSD; ++s) {
        const s16x4 lo = *(const s16x4*)(tb + dd[s][0]);
        const s16x4 hi = *(const s16x4*)(tb + dd[s][1]);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const bf16x8 a = __builtin_bit_cast(bf16x8, (s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int nf = 0; nf < NFD; ++nf) acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[s][nf], acc[nf], 0, 0, 0);
      }
      if (img0 + im < B) {
#pragma unroll
        for (int nf = 0; nf < NFD; ++nf) {
          const int ci = nf * 16 + li;
          if (ci < G::CIN) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int mm = mf * 16 + 4 * g + r;
              if (mm < NPX) dx[((int64_t)(img0 + im) * NPX + mm) * G::CIN + ci] = f2bf(acc[nf][r]);
            }
          }
        }
      }
    }
  }
}

int grid_for(int B, int imgs, int cap) {
  int n = (B + imgs - 1) / imgs;
  return n < cap ? (n < 1 ? 1 : n) : cap;
}

template <class G, int IMGS>
hipError_t run_fwd(const bf16_t* x, const bf16_t* w, const float* bias, int bias_n, int B, bf16_t* pooled, uint8_t* arg,
                   hipStream_t st) {
  hipLaunchKernelGGL((convpool_fwd_k<G, IMGS>), dim3(grid_for(B, IMGS, 2048)), dim3(NTH), 0, st, x, w, bias, bias_n, B,
                     pooled, arg);
  return hipGetLastError();
}

template <class G, int IMGS>
hipError_t run_wgrad(const bf16_t* x, const bf16_t* dP, const uint8_t* arg, const bf16_t* P, int B, float* slab,
                     int grid, hipStream_t st) {
  hipLaunchKernelGGL((convpool_wgrad_k<G, IMGS>), dim3(grid), dim3(NTH), 0, st, x, dP, arg, P, B, slab);
  return hipGetLastError();
}

template <class G, int IMGS>
hipError_t run_dgrad(const bf16_t* dP, const uint8_t* arg, const bf16_t* P, const bf16_t* w, int B, bf16_t* dx,
                     hipStream_t st) {
  hipLaunchKernelGGL((convpool_dgrad_k<G, IMGS>), dim3(grid_for(B, IMGS, 2048)), dim3(NTH), 0, st, dP, arg, P, w, B,
                     dx);
  return hipGetLastError();
}

using LeNetC1 = Geo<1, 8, 5, 2, 28, 28>;
using LeNetC2 = Geo<8, 16, 5, 0, 14, 14>;
using RefC1g = Geo<1, 32, 5, 2, 28, 28>;
using RefC1c = Geo<3, 32, 5, 2, 28, 28>;

}  // namespace

int convpool_config(int cin, int cout, int ks, int pad, int h, int w) {
  if (ks != 5) return -1;
  if (cin == 1 && cout == 8 && pad == 2 && h == 28 && w == 28) return 0;
  if (cin == 8 && cout == 16 && pad == 0 && h == 14 && w == 14) return 1;
  if (cin == 1 && cout == 32 && pad == 2 && h == 28 && w == 28) return 2;
  if (cin == 3 && cout == 32 && pad == 2 && h == 28 && w == 28) return 3;
  return -1;
}

int convpool_wgrad_rows(int cfg) {
  switch (cfg) {
    case 0: return LeNetC1::KM;
    case 1: return LeNetC2::KM;
    case 2: return RefC1g::KM;
    case 3: return RefC1c::KM;
  }
  return -1;
}

hipError_t convpool_fwd(int cfg, const bf16_t* x, const bf16_t* w, const float* bias, int bias_n, int B,
                        bf16_t* pooled, uint8_t* arg, hipStream_t st) {
  switch (cfg) {
    case 0: return run_fwd<LeNetC1, 4>(x, w, bias, bias_n, B, pooled, arg, st);
    case 1: return run_fwd<LeNetC2, 4>(x, w, bias, bias_n, B, pooled, arg, st);
    case 2: return run_fwd<RefC1g, 4>(x, w, bias, bias_n, B, pooled, arg, st);
    case 3: return run_fwd<RefC1c, 4>(x, w, bias, bias_n, B, pooled, arg, st);
  }
  return hipErrorInvalidValue;
}

hipError_t convpool_wgrad(int cfg, const bf16_t* x, const bf16_t* dP, const uint8_t* arg, const bf16_t* P, int B,
                          float* slab, int grid, hipStream_t st) {
  switch (cfg) {
    case 0: return run_wgrad<LeNetC1, 4>(x, dP, arg, P, B, slab, grid, st);
    case 1: return run_wgrad<LeNetC2, 4>(x, dP, arg, P, B, slab, grid, st);
    case 2: return run_wgrad<RefC1g, 2>(x, dP, arg, P, B, slab, grid, st);
    case 3: return run_wgrad<RefC1c, 2>(x, dP, arg, P, B, slab, grid, st);
  }
  return hipErrorInvalidValue;
}

hipError_t convpool_dgrad(int cfg, const bf16_t* dP, const uint8_t* arg, const bf16_t* P, const bf16_t* w, int B,
                          bf16_t* dx, hipStream_t st) {
  switch (cfg) {
    case 1: return run_dgrad<LeNetC2, 4>(dP, arg, P, w, B, dx, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace mnistx
