// LeNet-5 conv stack on banded (Toeplitz) MFMA tiles, gfx950.
//
// conv1 (5x5 SAME, 1 -> 6) + bias + ReLU + 2x2 max-pool and conv2 (5x5 VALID,
// 6 -> 16) + bias + ReLU + 2x2 max-pool as ONE persistent kernel per batch.
//
// Formulation (why it maps to CDNA4): a convolution over an image row is a GEMM
// with a banded ("Toeplitz") weight matrix: out[(x, c)] = sum_(x', ci) in[(x', ci)]
// * T[(x', ci)][(x, c)] with T = W[x' - x + pad] inside the band.  Written with the
// weights as the MFMA A operand and the activations as B, the B fragment of a lane
// is 8 CONSECUTIVE elements of one input row (one 16-byte load) -- there is no
// im2col gather at all, which is what bounds small-channel implicit-GEMM kernels
// (VALU + LDS address work per MFMA).  The band wastes part of each MFMA; at
// 2.5 PF of dense bf16 MFMA that is far cheaper than the gather it replaces.
//
// v_mfma_f32_32x32x16_bf16, columns = 32 = 16 images x 2 output-row parities
// (ypar = column & 1), rows = output features:
//  * conv1: rows = (window position g = 2 ypar + xpar, channel 3+1 per
//    lane half), columns = (pooled row half, image, pooled column parity xq); K = 16 =
//    (input row parity h, 8 input columns from 4u + 2xq - 2): 3 k-steps cover the 6
//    input rows of a pooled row.  Each lane then holds the 4 positions of its windows
//    in 4 registers: the pool is 3 v_max in the lane, no cross-lane exchange, and the
//    padded channels are never pooled (47 VALU per 3 MFMAs against 85 for a lane-pair
//    pooling layout; band kernel 201 -> 161 us, profiles/r3/lenet/inlane/).
//  * conv2 rows = (xpar 2, c2 16) of ONE pooled column x2p; K = 16 = 2 input
//    pixels x 8 channels; 3 k-steps x 5 kernel rows.  15 A fragments in total.
//  * bias added after pooling (4 values per lane instead of 16 accumulators).
//  * 2x2 pool: the x parity is a register pair of the same lane (rows m, m+4 /
//    m+8); the y parity is the neighbouring lane (one DPP quad-perm swap); the
//    argmax position rides in the 2 low mantissa bits of the fp32 sums (the same
//    encoding as convpool.hip, <= 3 ulp, far below bf16 resolution).
//  * the input tile and pool1 live in LDS (16 images, bank-conflict-free strides;
//    the next tile's input is loaded into registers while this tile computes);
//    conv2 reads pool1 as 16-byte B fragments.  pool1 is copied to HBM only when
//    the backward kernels still need it.
//
// Replaces: Conv2D + BiasAdd + Relu + MaxPool of the
// LeNet-5 conv blocks (BASELINE config; reference topology mnist_input.py:136-172
// uses the same ops).
#include "common.h"
#include "launchers.h"
#include "lrn_math.h"

#include <cstdlib>

namespace mnistx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NTH = 512;        // 8 waves: 0-3 conv1 (producers), 4-7 conv2 (consumers)
constexpr int BT = 8;           // images per tile (MFMA columns = 8 images x 2 row parities x 2 units)
constexpr int XROW = 28;        // input row (bf16 elements), 28x28x1 images
constexpr int XIMG = 784;
// LDS tiles (bf16 elements), rows split by parity into two planes so that the two
// output-row parities of an image (lanes 2i, 2i+1) read different bank halves;
// both rings are double-buffered (conv1 of tile k overlaps conv2 of tile k-1).
//  input : image [plane 2][14 rows][32 cols = x' -2..29], zero pad columns
constexpr int XRW = 32, XPL = 448, XIS = 900;
//  pool1 : image [plane 2][7 rows][14 px][8 ch]
constexpr int PRW = 112, PPL = 792, PIS = 1584;
constexpr int XBUF = BT * XIS, PBUF = BT * PIS;
constexpr int XZERO = 2 * XBUF;                 // one zero row: out-of-image input rows
constexpr int LDS_X = 2 * XBUF + XRW, LDS_P = 2 * PBUF;
static_assert((LDS_X + LDS_P) * 2 <= 81920, "two workgroups per CU");
constexpr int P1E = 14 * 14 * 8;    // pool1 elements per image in HBM ([14][14][8])
constexpr int P2E = 5 * 5 * 16;     // pool2 elements per image ([5][5][16])
constexpr uint32_t ARG_OFF = 4;     // argmax code of a window whose ReLU output is 0
constexpr int U1 = 49;              // conv1 units per tile: (pooled row pair yp0 / yp0 + 7, window u)
constexpr int U2 = 13;              // conv2 units per tile: (pooled pixel f0 / f0 + 13)

DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }
DEV float embed(float v, uint32_t d) { return __uint_as_float((__float_as_uint(v) & ~3u) | d); }
DEV float vmax(float a, float b) {  // bare v_max_f32 (fmaxf adds NaN-canonicalising moves)
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
DEV float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (round to nearest even)
DEV uint32_t pk2(float lo, float hi) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2)); }
DEV bf16x8 as_frag(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }
// Two LDS reads at a constant distance are fused by the compiler into ds_read2_b64,
// which runs at half the rate of two ds_read_b64 on gfx950; hiding the offset keeps
// them separate.
DEV int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

struct BandFwd {
  const bf16_t* x;        // images [n][784] bf16, normalised (or null with u8)
  const uint8_t* u8;      // images [n][784] uint8, normalised x/255 - 0.5 while staging (or null)
  const int64_t* idx;     // per-sample row of x [B]; null: sample b is row b
  int n;                  // rows in x
  const bf16_t* w1;       // [5][5][1][8]
  const float* b1;        // [b1n]
  int b1n;
  const bf16_t* w2;       // [5][5][8][16]
  const float* b2;        // [16]
  int B;
  bf16_t* p1;             // [B][14][14][8] pool1 (null: not written)
  uint8_t* arg1;          // [B][196][4] packed codes (with p1; null: p1 holds the combined records)
  bf16_t* p2;             // [B][5][5][16]
  uint8_t* arg2;          // [B][25][16]
  unsigned long long* prof;   // optional (experiments): per-role busy / barrier-wait clock sums
  int prio;                   // 1 = conv1 waves at s_setprio 1 (default), 2 = conv2 waves, 0 = none
};

// input tile fill by the conv1 waves: thread t (0..255) -> image t >> 5, 8-byte chunks
// (4 pixels) r = (t & 31) + 32 i of the image's 196
constexpr int FCH = (196 + 31) / 32;
struct XFill {
  u32x2 v[FCH];            // bf16 input: 4 pixels per chunk; uint8 input: v[i][0] = 4 pixels
  DEV void load(__amdgpu_buffer_rsrc_t rx, const BandFwd& a, int t0, int t) {
    const int gi = t0 + (t >> 5);
    const uint32_t esz = a.u8 ? 1u : 2u;
    uint32_t base = BUF_OOB;
    if (gi < a.B && t0 >= 0) {
      int64_t row = a.idx ? a.idx[gi] : (int64_t)gi;
      row = row < 0 ? 0 : (row >= a.n ? a.n - 1 : row);
      base = (uint32_t)row * (XIMG * esz);
    }
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int r = (t & 31) + 32 * i;
      if (a.u8) v[i] = u32x2{buf_b32(rx, r < 196 ? base + 4u * r : BUF_OOB), 0u};
      else v[i] = buf_b64(rx, r < 196 ? base + 8u * r : BUF_OOB);
    }
  }
  // LDS element offsets of this thread's chunks inside an input slot (tile-invariant:
  // computed once, so a tile's store is 7 ds_write2_b32 with no index arithmetic)
  int off[FCH];
  DEV void init(int t) {
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int r = (t & 31) + 32 * i, y = r / 7, k = r - 7 * y;
      off[i] = (t >> 5) * XIS + 2 + (y & 1) * XPL + (y >> 1) * XRW + 4 * k;
    }
  }
  DEV void store_pre(bf16_t* xb, int t, bool u8) const {
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int r = (t & 31) + 32 * i;
      if (r < 196) {
        uint32_t* d = (uint32_t*)(xb + off[i]);
        uint32_t lo = v[i][0], hi = v[i][1];
        if (u8) {
          const uint32_t b = v[i][0];
          lo = pack2(u8_norm(b & 0xff), u8_norm((b >> 8) & 0xff));
          hi = pack2(u8_norm((b >> 16) & 0xff), u8_norm(b >> 24));
        }
        d[0] = lo;
        d[1] = hi;
      }
    }
  }
};

// Warp-specialised pipeline over the block's tiles k = 0..nk-1 (tile blockIdx + k * grid):
// iteration k: conv1 waves turn input[k%2] into pool1[k%2] (and load tile k+1's input),
// conv2 waves turn pool1[(k-1)%2] into pool2 -- one barrier per iteration, nk+1 iterations.
// P1OUT: 0 = pool1 stays in LDS (eval / inference); 1 = pool1 [B][196][8] (channels 6-7 zero)
// + codes [B][196][4], the convpool layouts; 2 = one 16-byte record per pool1 window,
// channels 0-5 + the window's code word in the channel 6-7 slot -- the LDS record itself,
// copied out with one store, and what lenet_bwd_k reads (20 -> 16 bytes per window: 51 MB
// less written and read per step at B = 65536)
template <int P1OUT>
__global__ __launch_bounds__(NTH, 4) void lenet_band_fwd_k(const BandFwd a) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_X + LDS_P];
  bf16_t* xs = lds;
  bf16_t* p1s = lds + LDS_X;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 31, h = lane >> 5, ypar = col & 1, img = (col >> 1) & 7, half = col >> 4;
  const int ntiles = (a.B + BT - 1) / BT;
  const int nk = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  auto tile0 = [&](int k) { return ((int)blockIdx.x + k * (int)gridDim.x) * BT; };

  // weights -> LDS (pool1 ring, free until the first conv1 epilogue), zero the input ring
  constexpr int W1E = 5 * 5 * 8, W2E = 5 * 5 * 8 * 16;
  bf16_t* w1s = p1s;
  bf16_t* w2s = p1s + W1E + 8;   // zero slot at W1E: out-of-band taps read 0
  for (int e = tid; e < W2E / 8; e += NTH) *(u32x4*)(w2s + 8 * e) = *(const u32x4*)(a.w2 + 8 * e);
  for (int e = tid; e < W1E / 8; e += NTH) *(u32x4*)(w1s + 8 * e) = *(const u32x4*)(a.w1 + 8 * e);
  if (tid == 0) *(u32x4*)(w1s + W1E) = u32x4{0u, 0u, 0u, 0u};
  for (int e = tid; e < LDS_X / 8; e += NTH) *(u32x4*)(xs + 8 * e) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();

  if (wave < 4) {
    // ================================================================ conv1 + pool1 role, in-lane pooling
    // rows m = 8 g + 4 hh + i4: window position g = 2 ypar + xpar (= the argmax code), channel
    // c = ch(hh, i4) (3 per lane half, i4 = 3 is padding), so C register 4 g + i4 of a lane
    // holds all four positions of ONE 2x2 window: the pool is 3 v_max in the lane (no DPP,
    // no keep/send selects) and the padded channels 6-7 are never computed on.
    // columns = (half, img, xq): pooled pixel (yp0 + 7 half, 2u + xq) of image img.
    // B of column xq starts at input column 4u + 2xq - 2: 4-byte aligned for xq = 1, so a
    // fragment is two ds_read2_b32 (an 8-byte read off its alignment would replay).
    const int t = tid;
    if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
    // channel of C row (hh, i4): h = 0 holds 0,1,2; h = 1 holds 4,5,3 (so each lane's first
    // pair packs to its own 8-byte store and channel 3 moves to the h = 0 lane); -1: pad
    auto chan = [](int hh, int i4) { return i4 == 3 ? -1 : (hh == 0 ? i4 : (i4 == 2 ? 3 : 4 + i4)); };
    bf16x8 a1[3];
    {
      const int g = col >> 3, ypr = g >> 1, xpr = g & 1, c = chan((col >> 2) & 1, col & 3);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int dy = 2 * p + h - ypr, dx = j - xpr;
          const bool ok = c >= 0 && dy >= 0 && dy <= 4 && dx >= 0 && dx <= 4;
          a1[p][j] = __builtin_bit_cast(__bf16, w1s[ok ? (dy * 5 + dx) * 8 + c : W1E]);
        }
      }
    }
    float bias1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int c = chan(h, i);
      bias1[i] = c < a.b1n ? a.b1[c] : 0.f;
    }
    const int xq = col & 1;
    const auto rx = a.u8 ? buf_rsrc(a.u8, (uint32_t)a.n * XIMG) : buf_rsrc(a.x, (uint32_t)a.n * (XIMG * 2));
    // B rows: input row 2 yp - 2 + 2p + h = plane h, row yp0 + 7 half - 1 + p; column 4u + 2xq
    // (x' = 4u + 2xq - 2 with the 2-column left pad)
    const int xlane = img * XIS + h * XPL + (7 * half - 1) * XRW + 2 * xq;
    const bool top = half == 0, bot = half == 1;   // lanes whose p = 0 / p = 2 row can be padding
    // pool1 store: lane part + the (yp0 parity, half) part of pooled row yp = yp0 + 7 half
    const int store_lane = img * PIS + 8 * xq + 4 * h;
    const int row_even = half ? PPL + 3 * PRW : 0;   // yp0 even
    const int row_odd = half ? 4 * PRW : PPL;        // yp0 odd
    // code word: byte k = code(c = k) | code(c = k + 4) << 4; channels 6-7 are padding (code 4)
    const uint32_t sh0 = h ? 4u : 0u, sh1 = h ? 12u : 8u, sh2 = h ? 24u : 16u, kc = h ? 0x40400000u : 0u;
    XFill xf;
    xf.init(t);
    xf.load(rx, a, nk > 0 ? tile0(0) : -1, t);
    xf.store_pre(xs, t, a.u8 != nullptr);

    uint64_t busy = 0, wait = 0, tw = __builtin_amdgcn_s_memtime();
    for (int k = 0; k <= nk; ++k) {
      __syncthreads();
      const uint64_t tb = __builtin_amdgcn_s_memtime();
      wait += tb - tw;
      if (k < nk) {
        const bf16_t* xb = xs + (k & 1) * XBUF + xlane;
        bf16_t* pb = p1s + (k & 1) * PBUF + store_lane;
        xf.load(rx, a, k + 1 < nk ? tile0(k + 1) : -1, t);
        struct Frags { bf16x8 b[3]; };
        auto fetch = [&](int j) {
          const int f = min(wave + 4 * j, U1 - 1), yp0 = f / 7, u = f - 7 * yp0;
          const bf16_t* base = xb + yp0 * XRW + 4 * u;
          Frags fr;
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const bf16_t* rp = base + p * XRW;
            if (p == 0 && yp0 == 0) rp = top ? xs + XZERO : rp;   // input rows -2, -1
            if (p == 2 && yp0 == 6) rp = bot ? xs + XZERO : rp;   // input rows 28, 29
            const uint32_t* q = (const uint32_t*)rp;
            fr.b[p] = as_frag(u32x4{q[0], q[1], q[2], q[3]});
          }
          return fr;
        };
        auto window = [&](const Frags& fr) {
          f32x16 acc = {};
#pragma unroll
          for (int p = 0; p < 3; ++p) acc = mfma32(a1[p], fr.b[p], acc);
          return acc;
        };
        auto epilogue = [&](const f32x16& acc, int j) {
          const int f = wave + 4 * j, yp0 = f / 7, u = f - 7 * yp0;
          float o[3];
          uint32_t cw = kc;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            if constexpr (P1OUT != 0) {
              const float v = vmax(vmax3(__uint_as_float(__float_as_uint(acc[i]) & ~3u), embed(acc[4 + i], 1u),
                                         embed(acc[8 + i], 2u)), embed(acc[12 + i], 3u));
              o[i] = vmax(__uint_as_float(__float_as_uint(v) & ~3u) + bias1[i], 0.f);
              const uint32_t cd = o[i] > 0.f ? (__float_as_uint(v) & 3u) : ARG_OFF;
              cw |= cd << (i == 0 ? sh0 : i == 1 ? sh1 : sh2);
            } else {
              o[i] = vmax(vmax(vmax3(acc[i], acc[4 + i], acc[8 + i]), acc[12 + i]) + bias1[i], 0.f);
            }
          }
          const uint32_t w0 = pk2(o[0], o[1]);
          uint32_t w1;
          if constexpr (P1OUT != 0) {
            const uint32_t X = h ? __float_as_uint(o[2]) : cw;
            const auto sw = __builtin_amdgcn_permlane32_swap(X, X, false, false);
            w1 = h ? (cw | sw[0]) : pk2(o[2], __uint_as_float(sw[1]));
          } else {   // channels 6-7 stay 0 (zero weights in conv2)
            const uint32_t X = __float_as_uint(o[2]);
            const auto sw = __builtin_amdgcn_permlane32_swap(X, X, false, false);
            w1 = h ? 0u : pk2(o[2], __uint_as_float(sw[1]));
          }
          if (f < U1) {
            const int off = (yp0 & 1 ? row_odd : row_even) + (yp0 >> 1) * PRW + 16 * u;
            *(u32x2*)(pb + off) = u32x2{w0, w1};
          }
        };
        // 13 slots per wave (units wave + 4j, j = 0..12: 52 slots for the 49 units) -- the
        // 2-deep pipeline of the lane-pair layout ran 15 windows for 14 slots
        Frags fa = fetch(0), fb = fetch(1);
        f32x16 acca = window(fa), accb;
#pragma unroll 1
        for (int j = 0; j < 12; j += 2) {
          fa = fetch(j + 2);
          accb = window(fb);
          epilogue(acca, j);
          if (j + 3 < 13) fb = fetch(j + 3);
          acca = window(fa);
          epilogue(accb, j + 1);
        }
        epilogue(acca, 12);
        xf.store_pre(xs + ((k + 1) & 1) * XBUF, t, a.u8 != nullptr);
      }
      tw = __builtin_amdgcn_s_memtime();
      busy += tw - tb;
    }
    if (a.prof && lane == 0) {
      atomicAdd(a.prof + 0, (unsigned long long)busy);
      atomicAdd(a.prof + 2, (unsigned long long)wait);
    }
  } else {
    // ================================================================ conv2 + pool2 role
    const int t = tid - 256;
    if (a.prio == 2) __builtin_amdgcn_s_setprio(1);
    bf16x8 a2[15];   // (dy, q): rows (xpar, c2), k = (pixel h, channel j)
    {
      const int xpar = col >> 4, c2 = col & 15;
#pragma unroll
      for (int dy = 0; dy < 5; ++dy)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int dx = 2 * q + h - xpar;
          const bool ok = dx >= 0 && dx <= 4;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            a2[dy * 3 + q][j] = __builtin_bit_cast(__bf16, w1s[ok ? W1E + 8 + ((dy * 5 + dx) * 8 + j) * 16 + c2 : W1E]);
        }
    }
    const int w2v = wave - 4;
    const int cp_r = (t + 192) & 255;   // copy-out pixel of this thread (>= 196: none)
    const int cp_lds = ((cp_r / 14) & 1) * PPL + ((cp_r / 14) >> 1) * PRW + (cp_r % 14) * 8;
    uint64_t busy = 0, wait = 0, tw = __builtin_amdgcn_s_memtime();
    for (int k = 0; k <= nk; ++k) {
      __syncthreads();   // pool1[(k-1)%2] complete
      const uint64_t tb = __builtin_amdgcn_s_memtime();
      wait += tb - tw;
      tw = tb;
      if (k == 0) continue;
      const int t0 = tile0(k - 1), gi = t0 + img;
      const bool iv = gi < a.B;
      const bf16_t* pb = p1s + ((k - 1) & 1) * PBUF;
      if constexpr (P1OUT == 2) {     // combined pool1 / code records for lenet_bwd_k
        // all 196 records by wave 7 (4 rounds of 64 lanes): it runs one of the 7 conv2 units
        // where waves 4-6 run two, so the copy no longer lands on two of the busiest waves
        if (w2v == 3) {
          const int nimg = min(BT, a.B - t0);
          const auto rp1 = buf_rsrc(a.p1 + (int64_t)t0 * P1E, (uint32_t)nimg * (P1E * 2));
#pragma unroll 1
          for (int rr = 0; rr < 4; ++rr) {
            const int r = lane + 64 * rr;
            if (r < 196) {
              const bf16_t* src = pb + ((r / 14) & 1) * PPL + ((r / 14) >> 1) * PRW + (r % 14) * 8;
#pragma unroll
              for (int i0 = 0; i0 < BT; i0 += 4) {
                u32x4 cv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) cv[i] = *(const u32x4*)(src + (i0 + i) * PIS);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                  __builtin_amdgcn_raw_buffer_store_b128(cv[i], rp1, (uint32_t)r * 16u, (i0 + i) * (P1E * 2), 0);
              }
            }
          }
        }
      } else if constexpr (P1OUT == 1) {   // pool1 + argmax codes to HBM (convpool layouts)
        // copy thread ct owns pooled pixel ct (< 196) of every image of the tile: one LDS
        // offset per thread, image strides as instruction / scalar offsets (no per-element
        // index arithmetic).  ct is rotated so the wave with 4 conv2 units copies least.
        if (cp_r < 196) {
          const int nimg = min(BT, a.B - t0);
          const auto rp1 = buf_rsrc(a.p1 + (int64_t)t0 * P1E, (uint32_t)nimg * (P1E * 2));
          const auto ra1 = buf_rsrc(a.arg1 + (int64_t)t0 * 784, (uint32_t)nimg * 784);
          const bf16_t* src = pb + cp_lds;
#pragma unroll
          for (int i0 = 0; i0 < BT; i0 += 4) {
            u32x4 cv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) cv[i] = *(const u32x4*)(src + (i0 + i) * PIS);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{cv[i][0], cv[i][1], cv[i][2], 0u}, rp1, (uint32_t)cp_r * 16u,
                                                     (i0 + i) * (P1E * 2), 0);
              __builtin_amdgcn_raw_buffer_store_b32(cv[i][3], ra1, (uint32_t)cp_r * 4u, (i0 + i) * 784, 0);
            }
          }
        }
      }
      {
        // in-lane pooling: columns = (pooled-pixel slot, image), ONE accumulator per output-row
        // parity of the window, so a lane holds all 4 positions of 8 channels: the pool is
        // 3 v_max in the lane (no DPP, no keep/send selects, no chain sum).  Unit u = pooled
        // pixels 4u .. 4u+3 of the 8 images (7 units, the last 3 slots recomputed, no store);
        // the 6 pool1 rows 2 y2p .. 2 y2p + 5 are streamed once, each feeding both parities.
        // column -> (slot, image) bit order chosen for the pool1 B reads' bank groups:
        // 1.9-way average ds_read_b128 conflicts instead of 3.6-way for (col >> 3, col & 7)
        const int slot = (col >> 2) & 3, im2 = (col >> 4) | ((col & 3) << 1), gi2 = t0 + im2;
#pragma unroll 1
        for (int j = 0; j < 2; ++j) {
          const int u = w2v + 4 * j;
          if (u >= 7) break;
          const int f = 4 * u + slot, fc = min(f, 24);
          const int y2p = fc / 5, x2p = fc - 5 * y2p;
          const bf16_t* rb = pb + im2 * PIS + y2p * PRW + (2 * x2p + h) * 8;
          auto rowp = [&](int r) { return rb + (r & 1) * PPL + (r >> 1) * PRW; };
          bf16x8 bq[2][3];
#pragma unroll
          for (int q = 0; q < 3; ++q) bq[0][q] = *(const bf16x8*)(rowp(0) + 16 * q);
          f32x16 y0 = {}, y1 = {};
#pragma unroll
          for (int r = 0; r < 6; ++r) {
            if (r < 5) {
#pragma unroll
              for (int q = 0; q < 3; ++q) bq[(r + 1) & 1][q] = *(const bf16x8*)(rowp(r + 1) + 16 * q);
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) {
              if (r < 5) y0 = mfma32(a2[r * 3 + q], bq[r & 1][q], y0);
              if (r > 0) y1 = mfma32(a2[(r - 1) * 3 + q], bq[r & 1][q], y1);
            }
          }
          // channel ch of this lane: c2 = 8 (ch >> 2) + 4h + (ch & 3); xpar 0 / 1 at i0 / i0 + 8
          const f32x4 bl = *(const f32x4*)(a.b2 + 4 * h), bh = *(const f32x4*)(a.b2 + 8 + 4 * h);
          float o[8];
          uint32_t cd[8];
#pragma unroll
          for (int ch = 0; ch < 8; ++ch) {
            const int i0 = 4 * (ch >> 2) + (ch & 3);
            const float v = vmax(vmax3(__uint_as_float(__float_as_uint(y0[i0]) & ~3u), embed(y0[i0 + 8], 1u),
                                       embed(y1[i0], 2u)), embed(y1[i0 + 8], 3u));
            o[ch] = vmax(__uint_as_float(__float_as_uint(v) & ~3u) + (ch < 4 ? bl[ch] : bh[ch - 4]), 0.f);
            cd[ch] = o[ch] > 0.f ? (__float_as_uint(v) & 3u) : ARG_OFF;
          }
          if (gi2 < a.B && f < 25) {
            const int64_t e = (int64_t)gi2 * P2E + f * 16 + 4 * h;
            *(u32x2*)(a.p2 + e) = u32x2{pk2(o[0], o[1]), pk2(o[2], o[3])};
            *(u32x2*)(a.p2 + e + 8) = u32x2{pk2(o[4], o[5]), pk2(o[6], o[7])};
            *(uint32_t*)(a.arg2 + e) = cd[0] | (cd[1] << 8) | (cd[2] << 16) | (cd[3] << 24);
            *(uint32_t*)(a.arg2 + e + 8) = cd[4] | (cd[5] << 8) | (cd[6] << 16) | (cd[7] << 24);
          }
        }
      }
      tw = __builtin_amdgcn_s_memtime();
      busy += tw - tb;
    }
    if (a.prof && lane == 0) {
      atomicAdd(a.prof + 1, (unsigned long long)busy);
      atomicAdd(a.prof + 3, (unsigned long long)wait);
    }
  }
}

template <int P1OUT>
int fwd_grid(int ntiles) {
  static int per_cu = -1, cus = 0;
  if (per_cu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
    cus = prop.multiProcessorCount;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, lenet_band_fwd_k<P1OUT>, NTH, 0) != hipSuccess) return -1;
    per_cu = nb > 0 ? nb : 1;
  }
  const int res = reserve_cut(per_cu * cus, per_cu);
  return cap_grid(ntiles < res ? ntiles : res);
}


// ============================================================================ reference CNN conv1
// conv1 of the reference CNN (5x5 SAME, 1 -> 32 channels) + bias + ReLU + 2x2 max-pool on the
// same banded formulation and in-lane pooling as the LeNet conv1 role above (SURVEY §2.3 N1/N4/N6;
// /root/reference/mnist_input.py:146-155 conv1 -> pool1): rows = (window position g, 8 channels),
// so 32 channels are 4 column-sharing row groups; wave pair wp = wave >> 1 owns groups 2wp, 2wp + 1
// (6 A fragments), the two waves of a pair split the 49 (pooled row pair, window) units of a
// tile.  The pooled output and its argmax codes (one byte per channel, 4 = ReLU inactive: the
// convpool layout the LRN / backward kernels read) are stored straight from the lanes.
constexpr int RNTH = 256;
constexpr int RW_E = 5 * 5 * 32;               // weights [5][5][1][32]
constexpr int R_LDS = LDS_X + RW_E + 8;
static_assert(R_LDS * 2 <= 40960, "four workgroups per CU");

__global__ __launch_bounds__(RNTH) void refc1_band_fwd_k(const BandFwd a) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[R_LDS];
  bf16_t* xs = lds;
  bf16_t* ws = lds + LDS_X;                    // weights, then one zero slot of 8
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 31, h = lane >> 5, img = (col >> 1) & 7, half = col >> 4, xq = col & 1;
  const int ntiles = (a.B + BT - 1) / BT;
  const int nk = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  auto tile0 = [&](int k) { return ((int)blockIdx.x + k * (int)gridDim.x) * BT; };
  for (int e = tid; e < RW_E / 8; e += RNTH) *(u32x4*)(ws + 8 * e) = *(const u32x4*)(a.w1 + 8 * e);
  if (tid == 0) *(u32x4*)(ws + RW_E) = u32x4{0u, 0u, 0u, 0u};
  for (int e = tid; e < LDS_X / 8; e += RNTH) *(u32x4*)(xs + 8 * e) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  const int wp = wave >> 1, wi = wave & 1;     // channel-group pair, unit parity
  bf16x8 af[2][3];
  {
    const int g = col >> 3, ypr = g >> 1, xpr = g & 1, c8 = col & 7;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int dy = 2 * p + h - ypr, dx = j - xpr, c = 8 * (2 * wp + q) + c8;
          const bool ok = dy >= 0 && dy <= 4 && dx >= 0 && dx <= 4;
          af[q][p][j] = __builtin_bit_cast(__bf16, ws[ok ? (dy * 5 + dx) * 32 + c : RW_E]);
        }
  }
  float bias[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 8 * (2 * wp + q) + 4 * h + i;
      bias[q][i] = c < a.b1n ? a.b1[c] : 0.f;
    }
  const auto rx = a.u8 ? buf_rsrc(a.u8, (uint32_t)a.n * XIMG) : buf_rsrc(a.x, (uint32_t)a.n * (XIMG * 2));
  const int xlane = img * XIS + h * XPL + (7 * half - 1) * XRW + 2 * xq;
  const bool top = half == 0, bot = half == 1;
  XFill xf;
  xf.init(tid);
  xf.load(rx, a, nk > 0 ? tile0(0) : -1, tid);
  xf.store_pre(xs, tid, a.u8 != nullptr);
  constexpr int NU = (U1 + 1) / 2;             // 25 slots per wave (units wi + 2j)
  for (int k = 0; k < nk; ++k) {
    __syncthreads();                           // input[k % 2] landed; input[(k + 1) % 2] free
    const bf16_t* xb = xs + (k & 1) * XBUF + xlane;
    const int t0 = tile0(k), gi = t0 + img;
    xf.load(rx, a, k + 1 < nk ? tile0(k + 1) : -1, tid);
    struct Frags { bf16x8 b[3]; };
    auto fetch = [&](int j) {
      const int f = min(wi + 2 * j, U1 - 1), yp0 = f / 7, u = f - 7 * yp0;
      const bf16_t* base = xb + yp0 * XRW + 4 * u;
      Frags fr;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const bf16_t* rp = base + p * XRW;
        if (p == 0 && yp0 == 0) rp = top ? xs + XZERO : rp;
        if (p == 2 && yp0 == 6) rp = bot ? xs + XZERO : rp;
        const uint32_t* qq = (const uint32_t*)rp;
        fr.b[p] = as_frag(u32x4{qq[0], qq[1], qq[2], qq[3]});
      }
      return fr;
    };
    auto window = [&](const Frags& fr, int q) {
      f32x16 acc = {};
#pragma unroll
      for (int p = 0; p < 3; ++p) acc = mfma32(af[q][p], fr.b[p], acc);
      return acc;
    };
    auto epilogue = [&](const f32x16& acc, int j, int q) {
      const int f = wi + 2 * j, yp0 = f / 7, u = f - 7 * yp0;
      float o[4];
      uint32_t cw = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = vmax(vmax3(__uint_as_float(__float_as_uint(acc[i]) & ~3u), embed(acc[4 + i], 1u),
                                   embed(acc[8 + i], 2u)), embed(acc[12 + i], 3u));
        o[i] = vmax(__uint_as_float(__float_as_uint(v) & ~3u) + bias[q][i], 0.f);
        cw |= (o[i] > 0.f ? (__float_as_uint(v) & 3u) : ARG_OFF) << (8 * i);
      }
      if (f < U1 && gi < a.B) {
        const int yp = yp0 + 7 * half, px = 2 * u + xq;
        const int64_t e = ((int64_t)gi * 196 + yp * 14 + px) * 32 + 8 * (2 * wp + q) + 4 * h;
        *(u32x2*)(a.p1 + e) = u32x2{pk2(o[0], o[1]), pk2(o[2], o[3])};
        *(uint32_t*)(a.arg1 + e) = cw;
      }
    };
    Frags fa = fetch(0);
#pragma unroll 1
    for (int j = 0; j < NU; ++j) {
      const Frags fb = fetch(j + 1 < NU ? j + 1 : j);
      const f32x16 c0 = window(fa, 0);
      const f32x16 c1 = window(fa, 1);
      epilogue(c0, j, 0);
      epilogue(c1, j, 1);
      fa = fb;
    }
    if (k + 1 < nk) xf.store_pre(xs + ((k + 1) & 1) * XBUF, tid, a.u8 != nullptr);
  }
}

// ---------------------------------------------------------------------------- + norm1 in the epilogue
// The same conv1 + pool1 with ALL 32 channels of a unit in one wave (4 channel groups x 3
// k-steps = 12 MFMAs per unit, units w + 4 j), so the pooled pixel's 32 channels sit in the lane
// pair (l, l + 32): lane half h holds channels 8 q + 4 h + i of groups q = 0..3.  Two
// v_permlane32_swap per 4-channel block pair -- swap(P[k], P[k + 2]) -- turn that into
// channels 16 h .. 16 h + 15 per lane (the swap IS the transpose: no selects), so a lane
// stores 32 contiguous bytes of pool1, 16 of codes and 32 of norm1, and the norm1 LRN
// (mnist_input.py:152-153, radius 4) of its two 8-channel vectors needs no other data: the
// 4-channel neighbours are blocks the lane already holds.  The LRN arithmetic replays
// lrn_fwd8 (same squares of the bf16 pool1 values, same running window sum, same
// lrn_out), so norm1 is bitwise lrn_fwd_k's; pool1 and the codes are bitwise
// refc1_band_fwd_k's (same pooling expressions).  Replaces refc1_band_fwd_k + lrn_fwd_k:
// norm1 is computed from registers instead of a second 205 MB pool1 pass at B = 16384.
struct RefC1Lrn {
  bf16_t* norm;           // [B][196][32] norm1 (null: not written)
  float bias, alpha, beta;
};

// pool / bias / ReLU / code of channel group q (the accumulator of one unit): refc1_band_fwd_k's
// expressions, so pool1 and the codes are bitwise that kernel's
DEV void refc1_pool_q(const f32x16& acc, const float (&bias)[4], uint32_t (&P)[2], uint32_t& CW) {
  float o[4];
  uint32_t cw = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float v = vmax(vmax3(__uint_as_float(__float_as_uint(acc[i]) & ~3u), embed(acc[4 + i], 1u),
                               embed(acc[8 + i], 2u)), embed(acc[12 + i], 3u));
    o[i] = vmax(__uint_as_float(__float_as_uint(v) & ~3u) + bias[i], 0.f);
    cw |= (o[i] > 0.f ? (__float_as_uint(v) & 3u) : ARG_OFF) << (8 * i);
  }
  P[0] = pk2(o[0], o[1]);
  P[1] = pk2(o[2], o[3]);
  CW = cw;
}

// A unit's pooled pixel: lane half h holds channels 8 q + 4 h + i (P[q], CW[q]).  Transposes to
// channels 16 h .. 16 h + 15 per lane, stores pool1 / codes at element e (if st) and, with LRN,
// norm1 from the lane's own blocks (see refc1n_fwd_k).  PK: the two LRN vectors as packed
// (v_pk) halves -- refc1n_fwd_k; refc1n3_fwd_k keeps the scalar form (at 198 VGPRs with its
// A ring, the packed one spilled: 164 -> 207 us, profiles/r6/refc1pk/)
template <bool LRN, bool PK = true>
DEV void refc1_unit_out(const uint32_t (&P)[4][2], const uint32_t (&CW)[4], int h, int64_t e, bool st,
                        const BandFwd& a, const RefC1Lrn& l) {
  // lane half h: 4-channel blocks Bk = channels 16 h + 4 k .. + 3 (swap(P[k], P[k + 2]): lanes
  // of h = 0 keep P[k] in the first result and receive the partner's P[k] in the second;
  // lanes of h = 1 receive the partner's P[k + 2] in the first and keep P[k + 2] in the second)
  uint32_t Bk[4][2], Ck[4];
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2) {
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const auto sw = __builtin_amdgcn_permlane32_swap(P[k2][w], P[k2 + 2][w], false, false);
      Bk[2 * k2][w] = sw[0];
      Bk[2 * k2 + 1][w] = sw[1];
    }
    const auto sc = __builtin_amdgcn_permlane32_swap(CW[k2], CW[k2 + 2], false, false);
    Ck[2 * k2] = sc[0];
    Ck[2 * k2 + 1] = sc[1];
  }
  if (st) {
    *(u32x4*)(a.p1 + e) = u32x4{Bk[0][0], Bk[0][1], Bk[1][0], Bk[1][1]};
    *(u32x4*)(a.p1 + e + 8) = u32x4{Bk[2][0], Bk[2][1], Bk[3][0], Bk[3][1]};
    *(u32x4*)(a.arg1 + e) = u32x4{Ck[0], Ck[1], Ck[2], Ck[3]};
  }
  if constexpr (LRN) {
    // vector 0 = B0 B1 (left: channels 16 h - 4.. = own P[1] of h = 1, zeros for h = 0;
    // right: B2); vector 1 = B2 B3 (left B1; right: own P[2] of h = 0, zeros for h = 1)
    uint32_t lw[2], rw[2];
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      lw[w] = h ? P[1][w] : 0u;
      rw[w] = h ? 0u : P[2][w];
    }
    auto val = [](const uint32_t (&b)[2], int i) {
      const uint32_t w = b[i >> 1];
      return (i & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
    };
    uint32_t nv[2][4];
    if constexpr (PK) {
      // the two vectors as the halves of packed (v_pk) values: bitwise the scalar lrn_out path
      f2 v[8], e16[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = f2{val(Bk[0], i), val(Bk[2], i)};
        v[4 + i] = f2{val(Bk[1], i), val(Bk[3], i)};
        const f2 lv = f2{val(lw, i), val(Bk[1], i)}, rv = f2{val(Bk[2], i), val(rw, i)};
        e16[i] = lv * lv;
        e16[12 + i] = rv * rv;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) e16[4 + i] = v[i] * v[i];
      f2 s[8];
      window_sums_e<4>(e16, s);   // (never contracted with the squares: lrn_math.h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f2 y0 = lrn_out2(v[2 * i], s[2 * i], l.bias, l.alpha, l.beta);
        const f2 y1 = lrn_out2(v[2 * i + 1], s[2 * i + 1], l.bias, l.alpha, l.beta);
        nv[0][i] = pack2(y0.x, y1.x);
        nv[1][i] = pack2(y0.y, y1.y);
      }
    } else {
#pragma unroll
      for (int vec = 0; vec < 2; ++vec) {
        const uint32_t(&L)[2] = vec ? Bk[1] : lw;
        const uint32_t(&M0)[2] = vec ? Bk[2] : Bk[0];
        const uint32_t(&M1)[2] = vec ? Bk[3] : Bk[1];
        const uint32_t(&R)[2] = vec ? rw : Bk[2];
        float v[8], e16[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = val(M0, i);
          v[4 + i] = val(M1, i);
          const float lv = val(L, i), rv = val(R, i);
          e16[i] = lv * lv;
          e16[12 + i] = rv * rv;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) e16[4 + i] = v[i] * v[i];
        // materialised squares (the round-6 form: this scheduling keeps refc1n3 at 198 VGPRs)
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(e16[i]));
        float s[8];
        window_sums_e<4>(e16, s);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          nv[vec][i] = pack2(lrn_out(v[2 * i], s[2 * i], l.bias, l.alpha, l.beta),
                             lrn_out(v[2 * i + 1], s[2 * i + 1], l.bias, l.alpha, l.beta));
      }
    }
    if (st) {
      *(u32x4*)(l.norm + e) = u32x4{nv[0][0], nv[0][1], nv[0][2], nv[0][3]};
      *(u32x4*)(l.norm + e + 8) = u32x4{nv[1][0], nv[1][1], nv[1][2], nv[1][3]};
    }
  }
}

template <bool LRN>
__global__ __launch_bounds__(RNTH, 2) void refc1n_fwd_k(const BandFwd a, const RefC1Lrn l) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[R_LDS];
  bf16_t* xs = lds;
  bf16_t* ws = lds + LDS_X;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 31, h = lane >> 5, img = (col >> 1) & 7, half = col >> 4, xq = col & 1;
  const int ntiles = (a.B + BT - 1) / BT;
  const int nk = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  auto tile0 = [&](int k) { return ((int)blockIdx.x + k * (int)gridDim.x) * BT; };
  for (int e = tid; e < RW_E / 8; e += RNTH) *(u32x4*)(ws + 8 * e) = *(const u32x4*)(a.w1 + 8 * e);
  if (tid == 0) *(u32x4*)(ws + RW_E) = u32x4{0u, 0u, 0u, 0u};
  for (int e = tid; e < LDS_X / 8; e += RNTH) *(u32x4*)(xs + 8 * e) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  bf16x8 af[4][3];
  {
    const int g = col >> 3, ypr = g >> 1, xpr = g & 1, c8 = col & 7;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int dy = 2 * p + h - ypr, dx = j - xpr, c = 8 * q + c8;
          const bool ok = dy >= 0 && dy <= 4 && dx >= 0 && dx <= 4;
          af[q][p][j] = __builtin_bit_cast(__bf16, ws[ok ? (dy * 5 + dx) * 32 + c : RW_E]);
        }
  }
  float bias[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 8 * q + 4 * h + i;
      bias[q][i] = c < a.b1n ? a.b1[c] : 0.f;
    }
  const auto rx = a.u8 ? buf_rsrc(a.u8, (uint32_t)a.n * XIMG) : buf_rsrc(a.x, (uint32_t)a.n * (XIMG * 2));
  const int xlane = img * XIS + h * XPL + (7 * half - 1) * XRW + 2 * xq;
  const bool top = half == 0, bot = half == 1;
  XFill xf;
  xf.init(tid);
  xf.load(rx, a, nk > 0 ? tile0(0) : -1, tid);
  xf.store_pre(xs, tid, a.u8 != nullptr);
  const int nu = (U1 - wave + 3) / 4;          // units wave + 4 j: 13, 12, 12, 12
  for (int k = 0; k < nk; ++k) {
    __syncthreads();                           // input[k % 2] landed; input[(k + 1) % 2] free
    const bf16_t* xb = xs + (k & 1) * XBUF + xlane;
    const int t0 = tile0(k), gi = t0 + img;
    xf.load(rx, a, k + 1 < nk ? tile0(k + 1) : -1, tid);
    struct Frags { bf16x8 b[3]; };
    auto fetch = [&](int j) {
      const int f = min(wave + 4 * j, U1 - 1), yp0 = f / 7, u = f - 7 * yp0;
      const bf16_t* base = xb + yp0 * XRW + 4 * u;
      Frags fr;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const bf16_t* rp = base + p * XRW;
        if (p == 0 && yp0 == 0) rp = top ? xs + XZERO : rp;
        if (p == 2 && yp0 == 6) rp = bot ? xs + XZERO : rp;
        const uint32_t* qq = (const uint32_t*)rp;
        fr.b[p] = as_frag(u32x4{qq[0], qq[1], qq[2], qq[3]});
      }
      return fr;
    };
    Frags fa = fetch(0);
#pragma unroll 1
    for (int j = 0; j < nu; ++j) {
      const Frags fb = fetch(j + 1 < nu ? j + 1 : j);
      uint32_t P[4][2], CW[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x16 acc = {};
#pragma unroll
        for (int p = 0; p < 3; ++p) acc = mfma32(af[q][p], fa.b[p], acc);
        refc1_pool_q(acc, bias[q], P[q], CW[q]);
      }
      fa = fb;
      const int f = wave + 4 * j, yp0 = f / 7, u = f - 7 * yp0;
      const bool st = gi < a.B;
      const int64_t e = ((int64_t)(st ? gi : 0) * 196 + (yp0 + 7 * half) * 14 + 2 * u + xq) * 32 + 16 * h;
      refc1_unit_out<LRN>(P, CW, h, e, st, a, l);
    }
    if (k + 1 < nk) xf.store_pre(xs + ((k + 1) & 1) * XBUF, tid, a.u8 != nullptr);
  }
}

// ---------------------------------------------------------------------------- 3 input channels
// The reference's own records are 28x28x3 (mnist_input.py:13-15,134): the same banded GEMM per
// input plane, accumulated -- a unit is 4 groups x 3 k-steps x 3 planes = 36 MFMAs.  The 36 A
// fragments (144 VGPRs) live in an LDS table read lane-linearly (one conflict-free ds_read_b128
// each, 1 per MFMA: under the LDS array's 2-per-gap rate), the input is staged de-interleaved
// (one 12-byte load = 2 pixels x 3 channels -> one dword per plane), and the epilogue is
// refc1n_fwd_k's (pool1, codes, norm1).  512 threads, units w + 8 j; the double-buffered 3-plane
// input ring (86 KB) + table (36 KB) make it one block per CU.  bf16 input only (the batch, or
// the bf16 dataset through the batch index, as refc1_wgrad reads it).
constexpr int R3TH = 512, R3NW = 8;
constexpr int PLN = XIS;                        // one input plane of an image ([2][14][32] + pad)
constexpr int XIS3 = 3 * PLN, XBUF3 = BT * XIS3;
constexpr int XZERO3 = 2 * XBUF3;               // zero row (out-of-image input rows)
constexpr int AT_OFF = XZERO3 + XRW;            // A-fragment table [36][64 lanes] x 8 bf16
constexpr int R3_LDS = AT_OFF + 36 * 64 * 8;
static_assert(R3_LDS * 2 <= 163840, "one workgroup per CU");
static_assert(XBUF3 >= 5 * 5 * 3 * 32 + 8, "the weights are staged in input buffer 1");
constexpr int FC3 = 7;                          // 12-byte chunks per thread: 64 threads x 7 >= 392 per image

template <bool LRN>
__global__ __launch_bounds__(R3TH, 1) void refc1n3_fwd_k(const BandFwd a, const RefC1Lrn l) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds3[];
  bf16_t* xs = lds3;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 31, h = lane >> 5, img = (col >> 1) & 7, half = col >> 4, xq = col & 1;
  const int ntiles = (a.B + BT - 1) / BT;
  const int nk = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  auto tile0 = [&](int k) { return ((int)blockIdx.x + k * (int)gridDim.x) * BT; };
  constexpr int W3E = 5 * 5 * 3 * 32;
  {
    bf16_t* ws = xs + XBUF3;                     // weights [5][5][3][32] + one zero slot, in buffer 1
    for (int e = tid; e < W3E / 8; e += R3TH) *(u32x4*)(ws + 8 * e) = *(const u32x4*)(a.w1 + 8 * e);
    if (tid == 0) *(u32x4*)(ws + W3E) = u32x4{0u, 0u, 0u, 0u};
    for (int e = tid; e < (XBUF3 + 0) / 8; e += R3TH) *(u32x4*)(xs + 8 * e) = u32x4{0u, 0u, 0u, 0u};
    if (tid < XRW / 8) *(u32x4*)(xs + XZERO3 + 8 * tid) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    // A table: fragment fi = (q * 3 + p) * 3 + c, lane ln: W[dy][dx][c][8 q + c8] as in refc1n_fwd_k
    for (int e = tid; e < 36 * 64; e += R3TH) {
      const int fi = e >> 6, ln = e & 63, q = fi / 9, p = (fi / 3) % 3, c = fi % 3;
      const int cl = ln & 31, hh = ln >> 5, g = cl >> 3, ypr = g >> 1, xpr = g & 1, c8 = cl & 7;
      uint32_t wv[4];
#pragma unroll
      for (int j2 = 0; j2 < 4; ++j2) {
        uint32_t pr = 0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int j = 2 * j2 + t, dy = 2 * p + hh - ypr, dx = j - xpr;
          const bool ok = dy >= 0 && dy <= 4 && dx >= 0 && dx <= 4;
          pr |= (uint32_t)ws[ok ? ((dy * 5 + dx) * 3 + c) * 32 + 8 * q + c8 : W3E] << (16 * t);
        }
        wv[j2] = pr;
      }
      *(u32x4*)(xs + AT_OFF + 8 * e) = u32x4{wv[0], wv[1], wv[2], wv[3]};
    }
    __syncthreads();
    for (int e = tid; e < XBUF3 / 8; e += R3TH) *(u32x4*)(xs + XBUF3 + 8 * e) = u32x4{0u, 0u, 0u, 0u};
  }
  float bias[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 8 * q + 4 * h + i;
      bias[q][i] = c < a.b1n ? a.b1[c] : 0.f;
    }
  // input staging: thread t -> image t >> 6, pixel pairs r = (t & 63) + 64 i (< 392) of its row
  constexpr uint32_t IMGB = 784 * 3 * 2;
  const auto rx = buf_rsrc(a.x, (uint32_t)a.n * IMGB);
  int soff[FC3];
#pragma unroll
  for (int i = 0; i < FC3; ++i) {
    const int r = (tid & 63) + 64 * i, y = r / 14, x2 = 2 * (r - 14 * y);
    soff[i] = (tid >> 6) * XIS3 + 2 + (y & 1) * XPL + (y >> 1) * XRW + x2;
  }
  u32x4 xv[FC3];
  auto xload = [&](int t0) {
    const int gi2 = t0 + (tid >> 6);
    uint32_t base = BUF_OOB;
    if (t0 >= 0 && gi2 < a.B) {
      int64_t row = a.idx ? a.idx[gi2] : (int64_t)gi2;
      row = row < 0 ? 0 : (row >= a.n ? a.n - 1 : row);
      base = (uint32_t)row * IMGB;
    }
#pragma unroll
    for (int i = 0; i < FC3; ++i) {
      const int r = (tid & 63) + 64 * i;
      const auto v3 = __builtin_amdgcn_raw_buffer_load_b96(rx, r < 392 ? base + 12u * r : BUF_OOB, 0, 0);
      xv[i] = u32x4{v3[0], v3[1], v3[2], 0u};
    }
  };
  auto xstore = [&](bf16_t* xb) {
#pragma unroll
    for (int i = 0; i < FC3; ++i) {
      if ((tid & 63) + 64 * i < 392) {
        // (p0c0 p0c1) (p0c2 p1c0) (p1c1 p1c2) -> plane c = (p0c, p1c)
        const uint32_t d0 = xv[i][0], d1 = xv[i][1], d2 = xv[i][2];
        uint32_t* o = (uint32_t*)(xb + soff[i]);
        o[0] = (d0 & 0xffffu) | (d1 & 0xffff0000u);
        o[PLN / 2] = (d0 >> 16) | (d2 << 16);
        o[PLN] = (d1 & 0xffffu) | (d2 & 0xffff0000u);
      }
    }
  };
  xload(nk > 0 ? tile0(0) : -1);
  xstore(xs);
  const int xlane = img * XIS3 + h * XPL + (7 * half - 1) * XRW + 2 * xq;
  const bool top = half == 0, bot = half == 1;
  const bf16_t* at = xs + AT_OFF + 8 * lane;
  const int nu = (U1 - wave + R3NW - 1) / R3NW;   // units wave + 8 j: 7, 6, ..., 6
  for (int k = 0; k < nk; ++k) {
    __syncthreads();                              // input[k % 2] landed; input[(k + 1) % 2] free
    const bf16_t* xb = xs + (k & 1) * XBUF3 + xlane;
    const int t0 = tile0(k), gi = t0 + img;
    xload(k + 1 < nk ? tile0(k + 1) : -1);
    struct Frags { bf16x8 b[3][3]; };
    auto fetch = [&](int j) {
      const int f = min(wave + R3NW * j, U1 - 1), yp0 = f / 7, u = f - 7 * yp0;
      const bf16_t* base = xb + yp0 * XRW + 4 * u;
      Frags fr;
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const bf16_t* rp = base + p * XRW + c * PLN;
          if (p == 0 && yp0 == 0) rp = top ? xs + XZERO3 : rp;
          if (p == 2 && yp0 == 6) rp = bot ? xs + XZERO3 : rp;
          const uint32_t* qq = (const uint32_t*)rp;
          fr.b[p][c] = as_frag(u32x4{qq[0], qq[1], qq[2], qq[3]});
        }
      return fr;
    };
    Frags fa = fetch(0);
#pragma unroll 1
    for (int j = 0; j < nu; ++j) {
      const Frags fb = fetch(j + 1 < nu ? j + 1 : j);
      // A fragments of group q + 1 are read while group q's 9 MFMAs run (read one by one in
      // front of each dependent MFMA, every MFMA waited a full LDS latency)
      uint32_t P[4][2], CW[4];
      bf16x8 Ar[2][9];
#pragma unroll
      for (int i = 0; i < 9; ++i) Ar[0][i] = *(const bf16x8*)(at + i * 512);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q + 1 < 4) {
#pragma unroll
          for (int i = 0; i < 9; ++i) Ar[(q + 1) & 1][i] = *(const bf16x8*)(at + ((q + 1) * 9 + i) * 512);
        }
        f32x16 acc = {};
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int c = 0; c < 3; ++c) acc = mfma32(Ar[q & 1][p * 3 + c], fa.b[p][c], acc);
        refc1_pool_q(acc, bias[q], P[q], CW[q]);
      }
      fa = fb;
      const int f = wave + R3NW * j, yp0 = f / 7, u = f - 7 * yp0;
      const bool st = gi < a.B;
      const int64_t e = ((int64_t)(st ? gi : 0) * 196 + (yp0 + 7 * half) * 14 + 2 * u + xq) * 32 + 16 * h;
      refc1_unit_out<LRN, false>(P, CW, h, e, st, a, l);
    }
    if (k + 1 < nk) xstore(xs + ((k + 1) & 1) * XBUF3);
  }
}

int refc1_band_grid(int ntiles) {
  static int per_cu = -1, cus = 0;
  if (per_cu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
    cus = prop.multiProcessorCount;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, refc1_band_fwd_k, RNTH, 0) != hipSuccess) return -1;
    per_cu = nb > 0 ? nb : 1;
  }
  const int res = reserve_cut(per_cu * cus, per_cu);
  return cap_grid(ntiles < res ? ntiles : res);
}

}  // namespace

// MNISTX_REFC1_BAND=0 keeps the convpool kernel for the reference CNN's conv1 forward
bool refc1_band_enabled() {
  static const int on = [] { const char* e = getenv("MNISTX_REFC1_BAND"); return (e && e[0] == '0') ? 0 : 1; }();
  return on != 0;
}

// MNISTX_REFC1_FWD: 2 (default) = refc1n_fwd_k (all 32 channels per wave; norm1 in the epilogue
// when asked for), 1 = the round-5 refc1_band_fwd_k (two waves per unit; no norm1)
static int g_refc1_fwd = [] { const char* e = getenv("MNISTX_REFC1_FWD"); return (e && e[0] == '1') ? 1 : 2; }();
static int refc1_fwd_variant() { return g_refc1_fwd; }
void refc1_set_fwd_variant(int v) { g_refc1_fwd = v == 1 ? 1 : 2; }   // tests: A/B in one process
bool refc1_fwd_lrn_ok() { return refc1_band_enabled() && refc1_fwd_variant() == 2; }

static int refc1n_grid(int ntiles) {
  static int per_cu = -1, cus = 0;
  if (per_cu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
    cus = prop.multiProcessorCount;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, refc1n_fwd_k<true>, RNTH, 0) != hipSuccess) return -1;
    per_cu = nb > 0 ? nb : 1;
  }
  const int res = reserve_cut(per_cu * cus, per_cu);
  return cap_grid(ntiles < res ? ntiles : res);
}

static int refc1n3_grid(int ntiles) {
  static int per_cu = -1, cus = 0;
  if (per_cu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
    cus = prop.multiProcessorCount;
    for (auto k : {refc1n3_fwd_k<true>, refc1n3_fwd_k<false>})
      if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, R3_LDS * 2) != hipSuccess)
        return -1;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, refc1n3_fwd_k<true>, R3TH, R3_LDS * 2) != hipSuccess)
      return -1;
    per_cu = nb > 0 ? nb : 1;
  }
  const int res = reserve_cut(per_cu * cus, per_cu);
  return cap_grid(ntiles < res ? ntiles : res);
}

bool refc1_fwd3_ok() { return refc1_band_enabled() && refc1_fwd_variant() == 2; }

hipError_t refc1_band_fwd(const XSrc& x, const bf16_t* w, const float* b, int bn, int B, bf16_t* pooled,
                          uint8_t* arg, hipStream_t st, bf16_t* norm, float lrn_bias, float lrn_alpha,
                          float lrn_beta, int cin) {
  if (B <= 0) return hipSuccess;
  if (!x.x && !x.u8) return hipErrorInvalidValue;
  BandFwd a{x.u8 ? nullptr : x.x, x.u8, x.idx, x.idx ? x.n : B, w, b, bn, nullptr, nullptr, B, pooled, arg,
            nullptr, nullptr, nullptr, 0};
  const int ntiles = (B + BT - 1) / BT;
  if (cin == 3) {   // refc1n3_fwd_k: bf16 input only
    if (x.u8 || !x.x || refc1_fwd_variant() != 2) return hipErrorInvalidValue;
    const RefC1Lrn l{norm, lrn_bias, lrn_alpha, lrn_beta};
    const int grid = refc1n3_grid(ntiles);
    if (grid <= 0) return hipErrorInvalidValue;
    if (norm) hipLaunchKernelGGL(refc1n3_fwd_k<true>, dim3(grid), dim3(R3TH), R3_LDS * 2, st, a, l);
    else hipLaunchKernelGGL(refc1n3_fwd_k<false>, dim3(grid), dim3(R3TH), R3_LDS * 2, st, a, l);
    return hipGetLastError();
  }
  if (cin != 1) return hipErrorInvalidValue;
  if (refc1_fwd_variant() == 2) {
    const RefC1Lrn l{norm, lrn_bias, lrn_alpha, lrn_beta};
    const int grid = refc1n_grid(ntiles);
    if (grid <= 0) return hipErrorInvalidValue;
    if (norm) hipLaunchKernelGGL(refc1n_fwd_k<true>, dim3(grid), dim3(RNTH), 0, st, a, l);
    else hipLaunchKernelGGL(refc1n_fwd_k<false>, dim3(grid), dim3(RNTH), 0, st, a, l);
    return hipGetLastError();
  }
  if (norm) return hipErrorInvalidValue;   // the round-5 kernel writes no norm1
  const int grid = refc1_band_grid(ntiles);
  if (grid <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(refc1_band_fwd_k, dim3(grid), dim3(RNTH), 0, st, a);
  return hipGetLastError();
}

hipError_t lenet_band_fwd(const XSrc& x, const bf16_t* w1, const float* b1, int b1n, const bf16_t* w2,
                          const float* b2, int B, bf16_t* p1, uint8_t* arg1, bf16_t* p2, uint8_t* arg2,
                          hipStream_t st, unsigned long long* prof) {
  if (B <= 0) return hipSuccess;
  if (!x.x && !x.u8) return hipErrorInvalidValue;
  // conv1 (the busier role: ~90 % vs ~73 % of the iteration) at s_setprio 1 wins the
  // SIMD's issue arbitration against the conv2 waves: 219-222 -> 210-211 us, 0.61 -> 0.595
  // ms/step (profiles/r3/lenet/band_prio_ab.txt)
  BandFwd a{x.u8 ? nullptr : x.x, x.u8, x.idx, x.idx ? x.n : B, w1, b1, b1n, w2, b2, B, p1, arg1, p2, arg2, prof, 1};
  const int ntiles = (B + BT - 1) / BT;
  auto go = [&](auto ker, int grid) {
    if (grid <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(ker, dim3(grid), dim3(NTH), 0, st, a);
    return hipSuccess;
  };
  const hipError_t e = !p1    ? go(lenet_band_fwd_k<0>, fwd_grid<0>(ntiles))
                      : arg1 ? go(lenet_band_fwd_k<1>, fwd_grid<1>(ntiles))
                             : go(lenet_band_fwd_k<2>, fwd_grid<2>(ntiles));
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

}  // namespace mnistx
