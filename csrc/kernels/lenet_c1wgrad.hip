// LeNet-5 conv1 weight gradient in pooled-K form, gfx950.
//
// dW1[dy][dx][c] = sum over conv1 outputs (y, x) of xpad[y + dy - 2][x + dx - 2] * G[y][x][c],
// G = the max-unpooled pool1 gradient: at most one position g = 2 py + px of each 2x2 window
// (its argmax code) carries dP1, the other three are 0.  Splitting the sum by g,
//
//   C[q][(g, c)] = sum over pooled pixels k of P[k][q] * B_g[k][c]
//   P[k][q]      = xpad[2 yp + qy - 2][2 xp + qx - 2]      q = (qy, qx) in the 6x6 window patch
//   B_g[k][c]    = code_c(k) == g ? dP1_c(k) : 0
//   dW1[dy][dx][c] = sum_g C[(dy + py_g) * 6 + dx + px_g][(g, c)],   db1[c] = sum_g C[36][(g, c)]
//
// is ONE GEMM with K = the 196 pooled pixels (not the 784 conv outputs), M = 36 patch
// positions + a ones row (bias) and N = 4 positions x 8 channels = 32: every MFMA column is
// a real (g, c) pair, and neither operand needs an unpooled image or an im2col gather:
//  * P comes from 6 shifted, column-deinterleaved copies of the image row (copy qx holds
//    x[r][2 (i + qx/2 - 1) + qx % 2] at i), so the 8 pooled pixels of a lane's k-slots are
//    8 CONSECUTIVE elements: one aligned ds_read_b128 per A fragment, no per-step VALU;
//  * B_g lives in LDS as [pooled pixel][(g, c)] rows; staging scatters each channel's dP1
//    into its code's column (2 VALU + one ds_write_b16 per channel; the previous image's
//    scatter positions are zeroed the same way, code 4 = ReLU-inactive lands in row padding)
//    and the MFMA reads it transposed (ds_read_b64_tr_b16), K-contiguous per lane.
// v_mfma_f32_16x16x32_bf16; a 4-wave workgroup per image, wave w = column tile w & 1 (g = 2(w & 1),
// 2(w & 1) + 1) x k-steps 4 (w >> 1) .. (7 k-steps of 32 pooled pixels: 2 pooled rows, xp padded
// to 16) x 3 row tiles; threads 0..195 stage one pooled pixel each, 196..251 the x copies.
// The workgroup folds its C into the [KM = 48][8] weight-gradient slab of
// convpool_wgrad_pair_k (rows kh * 8 + kw, bias row 40), so the split-K reduce and the
// rest of the step are unchanged.
//
// Replaces the unpool-to-LDS implicit GEMM (convpool_wgrad_pair_k<LeNetC1>) for the
// BASELINE config's conv1 (reference topology mnist_input.py:136-155, the same op).
#include "common.h"
#include "launchers.h"

#include <cstdlib>

namespace mnistx {
namespace {

constexpr int NT = 256;                  // 4 waves: (column tile, k-step half)
constexpr int XCS = 528;                 // copy stride (elements): [qx 6][row 32][16], bank-spread (see header)
constexpr int XC_E = 6 * XCS;
constexpr int ONES_E = 6 * 64 + 8;       // A rows q >= 36 read a ones strip (bias row), stepped like the copies
constexpr int BRS = 104;                 // B row stride (bytes): tr reads and b16 scatters <= 2-way, code-4 dump fits
constexpr int BROWS = 224;               // pooled pixel rows: yp 14 x xp 16 (xp 14, 15 stay zero)
constexpr int LDS_B = (XC_E + ONES_E) * 2 + BROWS * BRS;
static_assert(((XC_E + ONES_E) * 2) % 16 == 0, "B image 16-byte aligned");
static_assert(64 + 2 * 6 <= BRS, "code-4 scatter stays inside the row padding");
constexpr int KM = 48;                   // slab rows (convpool_wgrad_pair_k<LeNetC1> layout)

typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;
DEV s16x4 tr4(const uint8_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)p); }
DEV uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

struct C1wArgs {
  XSrc x;
  const bf16_t* dP;    // [B][14][14][8] pool1 gradient
  const uint8_t* arg;  // [B][196][4] packed codes: byte k = code(c = k) | code(c = k + 4) << 4
  int B;
  float* slab;         // [grid][KM][8]
};

// image row R (28 pixels) as 14 bf16 pairs, bf16 dataset / batch or uint8 dataset
struct XRow {
  uint32_t w[14];
  DEV void load(const C1wArgs& a, int img, int R, bool ok) {
    int64_t row = img;
    if (a.x.idx) {
      row = a.x.idx[img];
      row = row < 0 ? 0 : (row >= a.x.n ? a.x.n - 1 : row);
    }
    // buffer resources are wave-uniform (buf_rsrc reads the first lane): the image base
    // goes in the resource, the lane's row in the offset
    if (a.x.u8) {
      const auto r = buf_rsrc(a.x.u8 + row * 784, ok ? 784u : 0u);
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const uint32_t b = buf_b32(r, (uint32_t)R * 28u + 4u * i);
        w[2 * i] = pack2(u8_norm(b & 0xff), u8_norm((b >> 8) & 0xff));
        w[2 * i + 1] = pack2(u8_norm((b >> 16) & 0xff), u8_norm(b >> 24));
      }
    } else {
      const auto r = buf_rsrc(a.x.x + row * 784, ok ? 1568u : 0u);
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const u32x2 v = buf_b64(r, (uint32_t)R * 56u + 8u * i);
        w[2 * i] = v[0];
        w[2 * i + 1] = v[1];
      }
    }
  }
};

// SPLIT 0: wave w = (column tile w & 1, k-steps 4 (w >> 1) ..); SPLIT 1: wave w = k-steps 2w, 2w + 1
// for BOTH column tiles (each A fragment read once per image instead of twice)
template <int SPLIT>
__global__ __launch_bounds__(NT) void lenet_c1w_pk_k(const C1wArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_B];
  bf16_t* xc = (bf16_t*)lds;
  uint8_t* bt = lds + (XC_E + ONES_E) * 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int e = tid; e < LDS_B / 16; e += NT) ((u32x4*)lds)[e] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  for (int e = tid; e < ONES_E; e += NT) xc[XC_E + e] = (bf16_t)0x3f80;

  // A fragment of row tile mt: lane row m = lane % 16 (q = 16 mt + m), k-group kg = lane / 16
  // (pooled row 2s + kg / 2, pooled columns 8 (kg % 2) .. + 7)
  const int kg = lane >> 4;
  int aoff[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    const int q = 16 * mt + (lane & 15);
    if (q < 36) {
      const int qy = q / 6, qx = q - 6 * qy;
      aoff[mt] = qx * XCS + (2 * (kg >> 1) + qy) * 16 + 8 * (kg & 1);
    } else {
      aoff[mt] = XC_E;   // ones (q = 36: bias row; q > 36: unused rows)
    }
  }
  // B fragment (transposed reads): lane 4q' + p of its 16-lane group supplies row
  // 8 kg + 4h + q', columns 4p .. 4p + 3 of column tile nt
  const int nt = SPLIT ? 0 : (wave & 1), khalf = wave >> 1;
  const int boff = (8 * kg + ((lane & 15) >> 2)) * BRS + nt * 32 + 8 * (lane & 3);
  constexpr int NTW = SPLIT ? 2 : 1;   // column tiles per wave
  f32x4 acc[NTW][3];
#pragma unroll
  for (int n = 0; n < NTW; ++n)
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) acc[n][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging roles: thread p < 196 scatters pooled pixel p into B; threads 196..251 build the
  // x copies of row R = (tid - 196) / 2, parity tid & 1
  const bool prole = tid < 196, xrole = tid >= 196 && tid < 252;
  const int R = (tid - 196) >> 1, par = tid & 1;
  uint32_t oldc = 0x44444444u;   // previous image's codes (4 = nothing to clear)
  // global data of an image: this thread's pooled pixel (dP1 + codes) or x row.  Loaded
  // PF = 3 images ahead: one image's staging + MFMA phase is far shorter than an HBM round
  // trip, so a one-ahead prefetch left every workgroup waiting on memory once per image.
  struct Pre {
    u32x4 dv;
    uint32_t cv;
    XRow xr;
  };
  auto prefetch = [&](Pre& pf, int img) {
    const bool ok = img < a.B;
    const int im = ok ? img : 0;
    // wave-uniform resources; a pixel past 196 reads out of range (zeros)
    const auto rd = buf_rsrc(a.dP + ((int64_t)im * 196) * 8, ok ? 196u * 16u : 0u);
    const auto rc = buf_rsrc(a.arg + (int64_t)im * 784, ok ? 784u : 0u);
    pf.dv = buf_b128(rd, 16u * (uint32_t)tid);
    pf.cv = buf_b32(rc, 4u * (uint32_t)tid);
    if (xrole) pf.xr.load(a, im, R, ok);
  };
  auto body = [&](const Pre& pf) {
    __syncthreads();   // the previous image's MFMA reads are done
    // ---- B: zero the previous scatter positions, scatter this image's dP1 by code
    if (prole) {
      const int yp = tid / 14, xp = tid - 14 * yp;
      uint8_t* row = bt + (yp * 16 + xp) * BRS;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const int sh = c < 4 ? 8 * c : 8 * (c - 4) + 4;
        const uint32_t co = (oldc >> sh) & 15u;
        *(uint16_t*)(row + co * 16 + 2 * c) = 0;
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const int sh = c < 4 ? 8 * c : 8 * (c - 4) + 4;
        const uint32_t cn = (pf.cv >> sh) & 15u;
        const uint32_t d = pf.dv[c >> 1];
        *(uint16_t*)(row + cn * 16 + 2 * c) = (uint16_t)((c & 1) ? (d >> 16) : d);
      }
      oldc = pf.cv;
    }
    // ---- A: the three shifted copies of this thread's (row, parity)
    if (xrole) {
      uint32_t e[7];   // D[2j], D[2j+1] with D[i] = x[R][2i + par]
#pragma unroll
      for (int j = 0; j < 7; ++j) e[j] = perm(pf.xr.w[2 * j + 1], pf.xr.w[2 * j], par ? 0x07060302u : 0x05040100u);
      bf16_t* r0 = xc + (R + 2) * 16;
      // qx = par (shift -1): (0, D0), (D1, D2), ..., (D13, 0)
      u32x4 lo, hi;
      lo = u32x4{e[0] << 16, perm(e[1], e[0], 0x05040302u), perm(e[2], e[1], 0x05040302u), perm(e[3], e[2], 0x05040302u)};
      hi = u32x4{perm(e[4], e[3], 0x05040302u), perm(e[5], e[4], 0x05040302u), perm(e[6], e[5], 0x05040302u), e[6] >> 16};
      *(u32x4*)(r0 + par * XCS) = lo;
      *(u32x4*)(r0 + par * XCS + 8) = hi;
      // qx = 2 + par (no shift): (D0, D1), ..., (D12, D13), (0, 0)
      *(u32x4*)(r0 + (2 + par) * XCS) = u32x4{e[0], e[1], e[2], e[3]};
      *(u32x4*)(r0 + (2 + par) * XCS + 8) = u32x4{e[4], e[5], e[6], 0u};
      // qx = 4 + par (shift +1): (D1, D2), ..., (D13, 0), (0, 0)
      lo = u32x4{perm(e[1], e[0], 0x05040302u), perm(e[2], e[1], 0x05040302u), perm(e[3], e[2], 0x05040302u),
                 perm(e[4], e[3], 0x05040302u)};
      hi = u32x4{perm(e[5], e[4], 0x05040302u), perm(e[6], e[5], 0x05040302u), e[6] >> 16, 0u};
      *(u32x4*)(r0 + (4 + par) * XCS) = lo;
      *(u32x4*)(r0 + (4 + par) * XCS + 8) = hi;
    }
    __syncthreads();
  };
  auto mfma_phase = [&]() {
    // ---- MFMA: this wave's k-steps (0..3 or 4..6) of 32 pooled pixels x 3 row tiles
    __builtin_amdgcn_s_setprio(1);
    constexpr int NS = SPLIT ? 2 : 4;
#pragma unroll
    for (int s4 = 0; s4 < NS; ++s4) {
      const int s = (SPLIT ? 2 * wave : 4 * khalf) + s4;
      if (s >= 7) break;
      const uint8_t* bp = bt + boff + s * 32 * BRS;
      bf16x8 b[NTW];
#pragma unroll
      for (int n = 0; n < NTW; ++n) b[n] = join(tr4(bp + 32 * n), tr4(bp + 32 * n + 4 * BRS));
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
        const bf16x8 av = *(const bf16x8*)(xc + aoff[mt] + 64 * s);
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          acc[n][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b[n], acc[n][mt], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  const int G = gridDim.x;
  Pre p0, p1, p2;
  prefetch(p0, blockIdx.x);
  prefetch(p1, blockIdx.x + G);
  prefetch(p2, blockIdx.x + 2 * G);
  for (int img = blockIdx.x; img < a.B; img += 3 * G) {
    body(p0);
    prefetch(p0, img + 3 * G);
    mfma_phase();
    if (img + G >= a.B) break;
    body(p1);
    prefetch(p1, img + 4 * G);
    mfma_phase();
    if (img + 2 * G >= a.B) break;
    body(p2);
    prefetch(p2, img + 5 * G);
    mfma_phase();
  }
  // ---- fold C[q][(g, c)] into the slab: dW[kh][kw][c] = sum_g C[(kh + py) * 6 + kw + px][(g, c)]
  __syncthreads();
  float* red = (float*)bt;   // [k half 2][48][32] (SPLIT 1: half 0 only, the waves added in order)
  if constexpr (SPLIT) {
    for (int wv = 0; wv < 4; ++wv) {
      if (wave == wv)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int mt = 0; mt < 3; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              float& d = red[(16 * mt + 4 * kg + i) * 32 + 16 * n + (lane & 15)];
              d = wv ? d + acc[n][mt][i] : acc[n][mt][i];
            }
      __syncthreads();
    }
    for (int e = tid; e < 1536; e += NT) red[1536 + e] = 0.f;
  } else {
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[khalf * 1536 + (16 * mt + 4 * kg + i) * 32 + 16 * nt + (lane & 15)] = acc[0][mt][i];
  }
  __syncthreads();
  float* out = a.slab + (int64_t)blockIdx.x * KM * 8;
  for (int e = tid; e < KM * 8; e += NT) {
    const int m = e >> 3, c = e & 7;
    float v = 0.f;
    if (m < 40) {
      const int kh = m >> 3, kw = m & 7;
      if (kw < 5)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int o = ((kh + (g >> 1)) * 6 + kw + (g & 1)) * 32 + g * 8 + c;
          v += red[o] + red[1536 + o];
        }
    } else if (m == 40) {
#pragma unroll
      for (int g = 0; g < 4; ++g) v += red[36 * 32 + g * 8 + c] + red[1536 + 36 * 32 + g * 8 + c];
    }
    out[e] = v;
  }
}

}  // namespace

// Opt-in (MNISTX_C1W_POOLK=1) until it measures faster than the unpool kernel on the step
bool lenet_c1w_pk_enabled() {
  static const int on = [] { const char* e = getenv("MNISTX_C1W_POOLK"); return (e && e[0] == '1') ? 1 : 0; }();
  return on != 0;
}

static int c1w_split() {
  static const int v = [] { const char* e = getenv("MNISTX_C1W_SPLIT"); return (e && e[0] == '1') ? 1 : 0; }();
  return v;
}

int lenet_c1w_pk_grid() {
  static int g = -1;
  if (g < 0) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -1;
    const hipError_t e = c1w_split() ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lenet_c1w_pk_k<1>, NT, 0)
                                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lenet_c1w_pk_k<0>, NT, 0);
    if (e != hipSuccess) return -1;
    g = per_cu * cus;
  }
  return g;
}

hipError_t lenet_c1w_pk(const XSrc& x, const bf16_t* dP, const uint8_t* arg, int B, float* slab, int grid,
                        hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (grid <= 0 || (!x.x && !x.u8)) return hipErrorInvalidValue;
  const C1wArgs a{x, dP, arg, B, slab};
  if (c1w_split()) hipLaunchKernelGGL(lenet_c1w_pk_k<1>, dim3(grid), dim3(NT), 0, st, a);
  else hipLaunchKernelGGL(lenet_c1w_pk_k<0>, dim3(grid), dim3(NT), 0, st, a);
  return hipGetLastError();
}

}  // namespace mnistx
