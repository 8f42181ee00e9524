// fp32 (--precision fp32) LDS-halo 5x5 convolution for the reference CNN's conv2
// geometry (14x14 NHWC, stride 1, SAME): forward (conv + bias + ReLU) and data
// gradient (the same convolution of dY with the 180-degree-flipped, in/out-swapped
// filter, optional ReLU mask) on v_mfma_f32_16x16x4_f32.
//
// The generic fp32 path (f32.hip Im2colF / DyIm2colF) gathers every im2col element
// through index math from L2: 5.8 / 6.7 ms per step for conv fwd / conv2 dgrad at
// B = 16384 (profiles/r2/fp32).  Here, as in the bf16 conv_halo.hip design, a
// persistent workgroup keeps its filter slice resident in LDS for the whole launch
// and stages one zero-haloed 18x20 image tile (32 channels) at a time, so each input
// value is fetched from HBM once per output-channel slice and every MFMA operand
// is a 16-byte LDS read:
//   * A = filter rows (output channel n, 16 per fragment), B = image pixels (one
//     output row of 16 columns, 14 real); D lane (i, g) holds output channels
//     4g..4g+3 of pixel column i, so the epilogue is one 16-byte store per fragment;
//   * the K order inside a 16-channel block is permuted so that lane group g's four
//     k-steps s = 0..3 read channels 4(4cb+g)+s -- ONE ds_read_b128 per operand
//     feeds four MFMAs (for the filter, rows are [tap][n][ci] with ci contiguous);
//   * 16-byte chunks are XOR-swizzled per row (c ^ (r & 6), 128-byte rows) so a
//     read of 16 consecutive rows x one chunk per lane group is conflict-free
//     (bench/lds_sim.py halo, the bf16 kernel's proven swizzle);
//   * dgrad reduces over 64 channels in two 32-channel passes over the same tile
//     buffer (its two filter halves stay resident), accumulators carried across.
// Occupancy: 46 KB tile + 102 KB filter = one 8-wave workgroup per CU.
//
// Replaces (SURVEY.md §2.3 N1/N2, fp32 path): Conv2D / Conv2DBackpropInput of conv2
// at mnist_input.py:161 under the reference's tf.float32.
#include "common.h"
#include <type_traits>
#include "launchers.h"

namespace mnistx {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int HW = 14, KS = 5, HP = HW + 4, WR = 20, NPIX = HW * HW, NTAP = KS * KS, MFR = HW;
constexpr int CP = 32;                 // channels staged per pass (one 128-byte pixel row)
constexpr int CHK = CP / 4;            // 16-byte chunks per pixel row

DEV int swz(int r, int c) { return c ^ (r & 6); }

// MODE 0 = forward: out[p][n] = relu(sum_{tap,ci} x[p+tap][ci] W[tap][ci][n] + b[n])
// MODE 1 = data gradient: out[p][n] = mask * sum_{tap,c} dy[p+tap][c] W[24-tap][n][c]
// (W = [kh][kw][cin][cout]; for MODE 1, c runs over the conv's output channels, n over
// its input channels).  CR = reduction channels (32 fwd, 64 dgrad), CW = output
// channels per workgroup (grid.y = ncols / CW), FR = row fragments per wave.
// UPW > 0 (FR = 1): the block's 14 x NF (output row, 16-channel fragment) units are dealt
// round-robin to the waves, UPW per wave at most -- with 8 waves and NF = 2 that is 4 + 3
// units on every SIMD (waves w and w + 4 share one), where 7 two-row groups on 8 waves leave
// one SIMD's second wave idle and the step waits for the SIMDs that ran two groups.
template <int CR, int CW, int NW, int MODE, int FR, int UPW = 0>
__global__ __launch_bounds__(64 * NW) void conv5_halo_f32_k(const float* __restrict__ x, const float* __restrict__ w,
                                                            int wcin, int wcout, const float* __restrict__ bias,
                                                            int relu, const float* __restrict__ mask, int ldm, int B,
                                                            float* __restrict__ out, int ldo) {
  constexpr int NT = 64 * NW;
  constexpr int NPASS = CR / CP;
  constexpr int NF = CW / 16;
  constexpr int XE = HP * WR * CP;               // tile floats
  constexpr int WE = NTAP * CW * CP;             // filter floats per pass
  constexpr int NV = NPIX * CHK;                 // 16-byte vectors per image pass
  constexpr int PER = (NV + NT - 1) / NT;
  constexpr int NGRP = (MFR + FR - 1) / FR;
  static_assert(CR % CP == 0 && CW % 16 == 0 && (UPW > 0 || NGRP <= NW), "conv5_halo_f32 geometry: one row group per wave");
  static_assert(UPW == 0 || (FR == 1 && UPW * NW >= MFR * NF && (UPW - 1) * NW < MFR * NF), "unit mode geometry");
  __shared__ __attribute__((aligned(16))) float xs[XE];
  __shared__ __attribute__((aligned(16))) float ws[NPASS * WE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.y * CW;

  for (int e = tid; e < XE / 4; e += NT) *(f32x4*)(xs + 4 * e) = f32x4{0.f, 0.f, 0.f, 0.f};   // halo stays zero
  // filter -> ws[pass][(tap*CW + n)][ci] (ci contiguous, swizzled 16-byte chunks)
  if constexpr (MODE == 0) {
    // W[tap][ci][n0 .. n0+CW) is contiguous: 4 output channels per load, 4 scattered stores
    for (int e = tid; e < NTAP * CP * (CW / 4); e += NT) {
      const int nv = e % (CW / 4), rest = e / (CW / 4), ci = rest % CP, t = rest / CP;
      const f32x4 v = *(const f32x4*)(w + ((int64_t)t * wcin + ci) * wcout + n0 + 4 * nv);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = t * CW + 4 * nv + j;
        ws[r * CP + swz(r, ci >> 2) * 4 + (ci & 3)] = v[j];
      }
    }
  } else {
    // flipped tap; row n = conv input channel n0 + n, columns = conv output channels
    for (int e = tid; e < NPASS * NTAP * CW * CHK; e += NT) {
      const int c = e % CHK, r0 = e / CHK, r = r0 % (NTAP * CW), pass = r0 / (NTAP * CW);
      const int n = r % CW, t = r / CW;
      const f32x4 v = *(const f32x4*)(w + ((int64_t)(NTAP - 1 - t) * wcin + n0 + n) * wcout + CP * pass + 4 * c);
      *(f32x4*)(ws + pass * WE + r * CP + swz(r, c) * 4) = v;
    }
  }
  float bsv[NF][4];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) bsv[nf][r] = (MODE == 0 && bias != nullptr) ? bias[n0 + nf * 16 + 4 * g + r] : 0.f;

  // this wave's row group: output rows FR*wave .. +FR-1 (clamped; the clamped duplicate's
  // results are dropped)
  const bool busy = wave < NGRP;
  int P0[FR];
#pragma unroll
  for (int h = 0; h < FR; ++h) P0[h] = min(FR * wave + h, MFR - 1) * WR + i;

  f32x4 pre[PER];
  auto gload = [&](int img, int pass) {   // channels [CP*pass, +CP) of image img (zeros past the batch)
    const bool in = img < B;
    const auto r = buf_rsrc(x + (int64_t)(in ? img : 0) * NPIX * CR, in ? (uint32_t)(NPIX * CR * 4) : 0u);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int v = tid + u * NT;
      const int p = v / CHK, c = v - p * CHK;
      pre[u] = __builtin_bit_cast(f32x4, buf_b128(r, v < NV ? (uint32_t)((p * CR + CP * pass + 4 * c) * 4) : BUF_OOB));
    }
  };
  gload(blockIdx.x, 0);
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    f32x4 uacc[UPW > 0 ? UPW : 1];
#pragma unroll
    for (int j = 0; j < (UPW > 0 ? UPW : 1); ++j) uacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 acc[FR][NF];
#pragma unroll
    for (int h = 0; h < FR; ++h)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[h][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
      __syncthreads();                          // previous pass / image consumed
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int v = tid + u * NT;
        if (v < NV) {
          const int p = v / CHK, c = v - p * CHK;
          const int P = (p / HW + 2) * WR + (p % HW) + 2;
          *(f32x4*)(xs + P * CP + swz(P, c) * 4) = pre[u];
        }
      }
      __syncthreads();
      if (pass + 1 < NPASS) gload(img, pass + 1);   // next pass / image in flight during the MFMAs
      else gload(img + gridDim.x, 0);
      if constexpr (UPW > 0) {
        // units u = wave + NW j: output row u % 14, fragment u / 14; this wave owns nmine
        const int nmine = (MFR * NF - wave + NW - 1) / NW;
        const float* wp = ws + pass * WE;
        auto units = [&](auto NUc) {
          constexpr int NU = decltype(NUc)::value;
          for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
            for (int kw = 0; kw < KS; ++kw) {
              const int t = kh * KS + kw, dP = kh * WR + kw;
#pragma unroll
              for (int cb = 0; cb < CP / 16; ++cb) {
                const int c = 4 * cb + g;
                f32x4 a[NU], b[NU];
#pragma unroll
                for (int j = 0; j < NU; ++j) {
                  const int u = wave + NW * j, r = t * CW + (u / MFR) * 16 + i, P = (u % MFR) * WR + i + dP;
                  a[j] = *(const f32x4*)(wp + r * CP + swz(r, c) * 4);
                  b[j] = *(const f32x4*)(xs + P * CP + swz(P, c) * 4);
                }
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                  for (int j = 0; j < NU; ++j)
                    uacc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][s], b[j][s], uacc[j], 0, 0, 0);
              }
            }
          }
        };
        if (nmine == UPW) units(std::integral_constant<int, UPW>{});
        else units(std::integral_constant<int, (UPW > 1 ? UPW - 1 : 1)>{});
      } else if (busy) {
        const float* wp = ws + pass * WE;
        for (int kh = 0; kh < KS; ++kh) {
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            const int t = kh * KS + kw, dP = kh * WR + kw;
#pragma unroll
            for (int cb = 0; cb < CP / 16; ++cb) {
              const int c = 4 * cb + g;
              f32x4 a[NF], b[FR];
#pragma unroll
              for (int nf = 0; nf < NF; ++nf) {
                const int r = t * CW + nf * 16 + i;
                a[nf] = *(const f32x4*)(wp + r * CP + swz(r, c) * 4);
              }
#pragma unroll
              for (int h = 0; h < FR; ++h) {
                const int P = P0[h] + dP;
                b[h] = *(const f32x4*)(xs + P * CP + swz(P, c) * 4);
              }
#pragma unroll
              for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int h = 0; h < FR; ++h)
#pragma unroll
                  for (int nf = 0; nf < NF; ++nf)
                    acc[h][nf] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[nf][s], b[h][s], acc[h][nf], 0, 0, 0);
            }
          }
        }
      }
    }
    // D row 4g + r = output channel n0 + nf*16 + 4g + r, column i = output column
    if constexpr (UPW > 0) {
      if (i < HW) {
#pragma unroll
        for (int j = 0; j < UPW; ++j) {
          const int u = wave + NW * j;
          if (u < MFR * NF) {
            const int row = u % MFR, nf = u / MFR;
            const int64_t px = (int64_t)img * NPIX + row * HW + i;
            const int nb = n0 + nf * 16 + 4 * g;
            f32x4 v = uacc[j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] += bsv[nf][r];
              if (relu) v[r] = fmaxf(v[r], 0.f);
            }
            if (mask != nullptr) {
              const f32x4 mk = *(const f32x4*)(mask + px * ldm + nb);
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (!(mk[r] > 0.f)) v[r] = 0.f;
            }
            *(f32x4*)(out + px * ldo + nb) = v;
          }
        }
      }
    } else if (busy && i < HW) {
#pragma unroll
      for (int h = 0; h < FR; ++h) {
        const int row = FR * wave + h;
        if (row < MFR) {
          const int64_t px = (int64_t)img * NPIX + row * HW + i;
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) {
            const int nb = n0 + nf * 16 + 4 * g;
            f32x4 v = acc[h][nf];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] += bsv[nf][r];
              if (relu) v[r] = fmaxf(v[r], 0.f);
            }
            if (mask != nullptr) {
              const f32x4 mk = *(const f32x4*)(mask + px * ldm + nb);
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (!(mk[r] > 0.f)) v[r] = 0.f;
            }
            *(f32x4*)(out + px * ldo + nb) = v;
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
// dW[tap][ci][co] = sum_p x[p + tap][ci] dY[p][co] (+ bias row: sum_p dY[p][co]).
// M = (tap, ci) in 16-row tiles T = 2 tap + ci/16 (50) + the bias tile, N = 64, K =
// pixels.  A persistent block keeps the whole 801 x 64 fp32 partial in registers:
// tile T belongs to wave T % 8 (accumulator slot T / 8), and the tap loop is unrolled
// so each tile's kw -- hence the alignment of its 4-pixel A reads -- is a compile-time
// constant (kw 0/4: one ds_read_b128, 2: two b64, odd: four b32).  Per image x and dY
// are staged TRANSPOSED ([channel][pixel], 16-byte vectors scattered to 4 channel
// rows) so a lane's four k-steps are 4 consecutive pixels of one channel row; a dY
// pixel row (16 columns, 14 real) is one k-block whose B fragments stay in registers
// for all 51 tiles.  Channel-row strides are 8 mod 64 dwords: the 128-bit reads of 16
// channels x 2 lane groups hit 16 distinct bank quads.  One fp32 partial per block
// goes to the split-K slab [S][801][64], reduced by splitk_reduce like the GEMM path.
template <int NW>
__global__ __launch_bounds__(64 * NW) void conv5_halo_f32_wgrad_k(const float* __restrict__ x,
                                                                  const float* __restrict__ dy, int B,
                                                                  float* __restrict__ slab) {
  constexpr int CIN = 32, COUT = 64, NT = 64 * NW;
  constexpr int NTL = NTAP * (CIN / 16);          // 50 tap x channel tiles
  constexpr int SLOTS = (NTL + 1 + NW - 1) / NW;  // accumulator slots per wave (bias tile included)
  constexpr int NFW = COUT / 16;
  constexpr int XRS = 392, DRS = 264;             // channel-row strides (floats), both 8 mod 64
  constexpr int MROWS = NTAP * CIN + 1;
  constexpr int XV = NPIX * CIN / 4, DV = NPIX * COUT / 4;
  constexpr int PX = (XV + NT - 1) / NT, PD = (DV + NT - 1) / NT;
  static_assert(NW == 8 && XRS >= HP * WR && DRS >= HW * 16, "");
  __shared__ __attribute__((aligned(16))) float xt[CIN * XRS];
  __shared__ __attribute__((aligned(16))) float dt[COUT * DRS];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, g = lane >> 4;
  for (int e = tid; e < CIN * XRS / 4; e += NT) *(f32x4*)(xt + 4 * e) = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = tid; e < COUT * DRS / 4; e += NT) *(f32x4*)(dt + 4 * e) = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 acc[SLOTS][NFW];
#pragma unroll
  for (int sl = 0; sl < SLOTS; ++sl)
#pragma unroll
    for (int n = 0; n < NFW; ++n) acc[sl][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 px[PX], pd[PD];
  auto gload = [&](int img) {                 // past the batch: zeros
    const bool in = img < B;
    const auto rx = buf_rsrc(x + (int64_t)(in ? img : 0) * NPIX * CIN, in ? (uint32_t)(NPIX * CIN * 4) : 0u);
    const auto rd = buf_rsrc(dy + (int64_t)(in ? img : 0) * NPIX * COUT, in ? (uint32_t)(NPIX * COUT * 4) : 0u);
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int v = tid + u * NT;
      px[u] = __builtin_bit_cast(f32x4, buf_b128(rx, v < XV ? (uint32_t)(16 * v) : BUF_OOB));
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int v = tid + u * NT;
      pd[u] = __builtin_bit_cast(f32x4, buf_b128(rd, v < DV ? (uint32_t)(16 * v) : BUF_OOB));
    }
  };
  gload(blockIdx.x);
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      const int v = tid + u * NT;
      if (v < XV) {
        const int p = v / (CIN / 4), c4 = v - p * (CIN / 4);
        const int P = (p / HW + 2) * WR + (p % HW) + 2;
#pragma unroll
        for (int j = 0; j < 4; ++j) xt[(4 * c4 + j) * XRS + P] = px[u][j];
      }
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int v = tid + u * NT;
      if (v < DV) {
        const int p = v / (COUT / 4), c4 = v - p * (COUT / 4);
        const int Q = (p / HW) * 16 + (p % HW);
#pragma unroll
        for (int j = 0; j < 4; ++j) dt[(4 * c4 + j) * DRS + Q] = pd[u][j];
      }
    }
    __syncthreads();
    gload(img + gridDim.x);
    for (int y = 0; y < HW; ++y) {
      // B fragments of this pixel row: lane (co = 16 n + i, pixels 4g..4g+3)
      f32x4 b[NFW];
#pragma unroll
      for (int n = 0; n < NFW; ++n) b[n] = *(const f32x4*)(dt + (16 * n + i) * DRS + 16 * y + 4 * g);
#pragma unroll
      for (int T = 0; T <= NTL; ++T) {
        if (T % NW != wave) continue;          // wave-uniform
        f32x4 a;
        if (T == NTL) {                        // bias tile: row 0 of A = ones
          const float one = i == 0 ? 1.f : 0.f;
          a = f32x4{one, one, one, one};
        } else {
          const int tap = T / 2, kh = tap / KS, kw = tap % KS, ci = (T % 2) * 16 + i;
          const float* ap = xt + ci * XRS + (y + kh) * WR + 4 * g + kw;
          if constexpr (true) {
            if (kw % 4 == 0) a = *(const f32x4*)ap;
            else if (kw % 2 == 0) {
              const f32x2 lo = *(const f32x2*)ap, hi = *(const f32x2*)(ap + 2);
              a = f32x4{lo[0], lo[1], hi[0], hi[1]};
            } else {
              a = f32x4{ap[0], ap[1], ap[2], ap[3]};
            }
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int n = 0; n < NFW; ++n)
            acc[T / NW][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[n][s], acc[T / NW][n], 0, 0, 0);
      }
    }
  }
  // partial -> slab[blockIdx][m][co]: D rows 4g + r of tile T, column i
  float* out = slab + (int64_t)blockIdx.x * MROWS * COUT;
#pragma unroll
  for (int T = 0; T <= NTL; ++T) {
    if (T % NW != wave) continue;
#pragma unroll
    for (int n = 0; n < NFW; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * T + 4 * g + r;
        if (m < MROWS) out[(int64_t)m * COUT + 16 * n + i] = acc[T / NW][n][r];
      }
  }
}

template <int CR, int CW, int NW, int MODE, int FR, int UPW = 0>
int halo_f32_grid(int B) {
  static int per = -1;
  if (per < 0) {
    int dev = 0, cus = 0, pc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, conv5_halo_f32_k<CR, CW, NW, MODE, FR, UPW>, 64 * NW, 0) ==
            hipSuccess &&
        hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && pc > 0)
      per = pc * cus;
    else
      per = 256;
  }
  return cap_grid(B < per ? B : per);
}

template <int CR, int CW, int NW, int MODE, int FR, int UPW = 0>
hipError_t run_halo_f32(const float* x, const float* w, int wcin, int wcout, const float* bias, int relu,
                        const float* mask, int ldm, int B, float* out, int ncols, int ldo, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (ncols % CW != 0) return hipErrorInvalidValue;
  dim3 grid(halo_f32_grid<CR, CW, NW, MODE, FR, UPW>(B), ncols / CW);
  hipLaunchKernelGGL((conv5_halo_f32_k<CR, CW, NW, MODE, FR, UPW>), grid, dim3(64 * NW), 0, st, x, w, wcin, wcout, bias,
                     relu, mask, ldm, B, out, ldo);
  return hipGetLastError();
}

}  // namespace

// Geometry: 14x14, 5x5, pad 2, stride 1; fwd Cin 32 -> Cout % 32 == 0; dgrad dY 64
// channels -> dX Cin % 16 == 0.  MNISTX_F32_HALO=0 keeps the generic im2col GEMM.
static bool f32_halo_on() {
  static const bool on = [] { const char* e = getenv("MNISTX_F32_HALO"); return !(e && e[0] == '0'); }();
  return on;
}
bool f32_halo_fwd_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout) {
  return f32_halo_on() && H == 14 && W == 14 && OH == 14 && OW == 14 && KH == 5 && KW == 5 && ph == 2 && pw == 2 &&
         C == 32 && Cout % 32 == 0;
}
bool f32_halo_dgrad_ok(int OH, int OW, int Cout, int H, int W, int KH, int KW, int ph, int pw, int Cin) {
  return f32_halo_on() && H == 14 && W == 14 && OH == 14 && OW == 14 && KH == 5 && KW == 5 && ph == 2 && pw == 2 &&
         Cout == 64 && Cin % 16 == 0;
}
static int g_f32_halo_fwd_variant = 0;
void set_f32_halo_fwd_variant(int v) { g_f32_halo_fwd_variant = v; }
static int f32_halo_fwd_variant() { return g_f32_halo_fwd_variant; }
hipError_t f32_halo_fwd(const float* x, const float* w, int Nb, int C, int Cout, const float* bias, int relu, float* y,
                        hipStream_t st) {
  // A/B hook (tests, bench/micro_halo_f32.py): 1 = the 7-group launch this replaced
  if (f32_halo_fwd_variant() == 1)
    return run_halo_f32<32, 32, 8, 0, 2>(x, w, C, Cout, bias, relu, nullptr, 0, Nb, y, Cout, Cout, st);
  return run_halo_f32<32, 32, 8, 0, 1, 4>(x, w, C, Cout, bias, relu, nullptr, 0, Nb, y, Cout, Cout, st);
}
hipError_t f32_halo_dgrad(const float* dy, const float* w, int Nb, int Cout, int Cin, const float* mask, float* dx,
                          hipStream_t st) {
  return run_halo_f32<64, 16, 8, 1, 2>(dy, w, Cin, Cout, nullptr, 0, mask, Cin, Nb, dx, Cin, Cin, st);
}

bool f32_halo_wgrad_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout) {
  return f32_halo_on() && H == 14 && W == 14 && OH == 14 && OW == 14 && KH == 5 && KW == 5 && ph == 2 && pw == 2 &&
         C == 32 && Cout == 64;
}
// one resident wave of wgrad workgroups (the caller sizes its split-K slab with it)
int f32_halo_wgrad_grid() {
  static int per = -1;
  if (per < 0) {
    int dev = 0, cus = 0, pc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, conv5_halo_f32_wgrad_k<8>, 512, 0) == hipSuccess &&
        hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && pc > 0)
      per = pc * cus;
    else
      per = 256;
  }
  return per;
}
// slab: [splits][801][64]; every one of the `splits` workgroups writes its partial
hipError_t f32_halo_wgrad(const float* x, const float* dy, int Nb, int splits, float* slab, hipStream_t st) {
  if (Nb <= 0 || splits <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv5_halo_f32_wgrad_k<8>, dim3(splits), dim3(512), 0, st, x, dy, Nb, slab);
  return hipGetLastError();
}

}  // namespace mnistx
