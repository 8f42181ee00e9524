// LeNet-5 conv-stack backward as ONE persistent kernel, gfx950.
//
// Replaces the three backward launches of the LeNet conv blocks (conv2 dgrad, conv2
// weight gradient, conv1 weight gradient: SURVEY.md §2.3 N2/N3/N4/N6) with one pass per
// 8-image tile that keeps every intermediate in LDS: the unpooled conv2 gradient dY2, the
// pool1 gradient dP1 (never written to HBM) and the staged pool1 / input images.  Per
// block, the weight gradients accumulate in registers across all of its tiles and are
// written once as one split-K partial (deterministic: no atomics; splitk_reduce combines
// the blocks).  Reference: the backward of /root/reference/mnist_input.py:136-172 (conv
// blocks) produced by compute_gradients (mnist_input.py:262), on the LeNet-5 geometry of
// the BASELINE config (conv1 5x5 SAME 1->6, pool, conv2 5x5 VALID 6->16, pool).
//
// Every product is a v_mfma_f32_16x16x32_bf16 (lane l: A[l&15][8(l>>4)+j],
// B[8(l>>4)+j][l&15], C col l&15, rows 4(l>>4)+i):
//  * conv2 dgrad, banded: rows = (output column offset r, ci 8) of an output column pair,
//    K = (input column xs of an x pair, co 16), columns = (8 images, 2 output rows).  The
//    A fragment W2[dy][r + 4 - 2j - xs][ci][co] does not depend on the column pair, so the
//    15 fragments are formed once per block (LDS) and a row pair's 7 column pairs slide
//    over 5 B fragments (one 16-byte read each) per kernel row: 15 MFMAs per 8 LDS reads.
//    Kernel rows whose input row lies outside 0..9 for both output rows are skipped.
//  * conv2 weight gradient: rows = (2 taps, ci 8), columns = co 16, K = 32 dY2 pixels;
//    both operands are ds_read_b64_tr_b16 transposed reads of the NHWC tiles (one per
//    lane: 4 channels of one pixel); bias = a constant ones row read by the 13th tile.
//  * conv1 weight gradient, by pool-window phase: with dY1 = dP1 at the window position
//    d = 2a + b of each (window, channel)'s argmax, dW1[dy][dx][c] =
//    sum_d sum_w X[2yp+a+dy-2][2xp+b+dx-2] dP1[w][c] [code(w,c) == d], i.e. one GEMM
//    C[(ty, tx)][(c, d)] over the windows w (ty = a + dy, tx = b + dx in 0..5) folded at
//    the end.  A = input patches at (2yp + ty - 2, 2xp + tx - 2): a transposed read of 4
//    consecutive input pixels per lane (8-byte aligned because windows are taken by x
//    parity: even-xp windows cover tx -2..5, odd ones 0..7 -- two accumulator sets);
//    B = dP1 masked by the argmax code (VALU: code == d per column).
// Phases per tile (two barriers): [store X / codes of this tile, prefetch the next tile,
// dgrad (waves 0-6, one output row pair each) + conv2 wgrad k-steps (all waves)] ->
// [store dY2 / pool1 of the next tile, conv1 wgrad units].
#include "common.h"
#include "launchers.h"

namespace mnistx {
namespace {

DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

constexpr int NT = 512, NW = 8, T = 8;
constexpr int NPIX2 = 100, NWIN1 = 196;    // conv2 output pixels / pool1 windows per image
// ---- LDS layout (bytes).  Strides chosen with bench/lds_bwd.py (bank model): the dgrad
// B reads (ds_read_b128) are conflict-free with 11-pixel dY2 rows and 4288-byte images.
constexpr int AF_OFF = 0, AF_SZ = 15 * 64 * 16;           // dgrad A fragments [dy*3+j][lane] x 16 B
constexpr int DY2_RS = 352, DY2_IMG = 4288;               // dY2 [img][row -1..10][11 px][16 co] bf16
constexpr int DY2_OFF = AF_OFF + AF_SZ, DY2_SZ = T * DY2_IMG;
constexpr int P1_IMG = 3152;                              // pool1 [img][196][8] bf16
constexpr int P1_OFF = DY2_OFF + DY2_SZ, P1_SZ = T * P1_IMG;
constexpr int X_RS = 72, X_IMG = 2528;                    // input [img][row -2..29][col -4..31] bf16
constexpr int X_OFF = P1_OFF + P1_SZ, X_SZ = T * X_IMG;
constexpr int DP1_IMG = 3152;                             // dP1 [img][196][8] bf16
constexpr int DP1_OFF = X_OFF + X_SZ, DP1_SZ = T * DP1_IMG;
constexpr int CD_OFF = DP1_OFF + DP1_SZ, CD_SZ = T * DP1_IMG;   // argmax codes [img][196][8] u16
constexpr int ZERO_OFF = CD_OFF + CD_SZ;                  // 16 zero bytes (padded conv1 K)
constexpr int ONES_OFF = ZERO_OFF + 16;                   // bf16 {1, 0 x 7}: conv2 bias row
constexpr int LDS_BYTES = ONES_OFF + 16;
static_assert(LDS_BYTES <= 163840, "one workgroup per CU");
static_assert(12 * DY2_RS <= DY2_IMG && 32 * X_RS <= X_IMG && NWIN1 * 16 <= P1_IMG, "");
// epilogue scratch (aliases the tiles once the loop is done)
constexpr int E2_SZ = NW * 7 * 256 * 4, E1_SZ = NW * 6 * 256 * 4;
static_assert(E2_SZ <= LDS_BYTES && E1_SZ + NW * 64 * 16 <= LDS_BYTES, "");

// conv2 weight-gradient M tiles: two taps each; lanes of the second tap (p >= 2) add a
// constant byte offset to the first tap's pool1 address (bias tile: the ONES cell)
//   t 0..4: (0, t) & (4, t)   t 5..9: (1, t-5) & (2, t-5)   t 10, 11: (3, 2t-20) & (3, 2t-19)
//   t 12: (3, 4) & bias
DEV int c2_tap(int t, int h) {
  if (t < 5) return h ? 20 + t : t;
  if (t < 10) return h ? 10 + t - 5 : 5 + t - 5;
  if (t < 12) return 15 + 2 * (t - 10) + h;
  return h ? 25 : 19;
}
constexpr int c2_toff(int t) {   // pool1 byte offset of the tile's first tap
  return t < 5 ? 16 * t : t < 10 ? 16 * (14 + t - 5) : t < 12 ? 16 * (42 + 2 * (t - 10)) : 16 * (42 + 4);
}

// 0xffff in each 16-bit half of e that equals d, else 0
DEV uint32_t heq(uint32_t e, uint32_t d) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 x = __builtin_bit_cast(u16x2, e ^ (d * 0x00010001u));
  const u16x2 one = {1, 1};
  return __builtin_bit_cast(uint32_t, (u16x2)(__builtin_elementwise_min(x, one) - one));
}
// bytes b0, b1 of w -> u16 pair (b0 | b1 << 16)
DEV uint32_t bytes01(uint32_t w) { return (w & 0xffu) | ((w & 0xff00u) << 8); }
DEV uint32_t bytes23(uint32_t w) { return ((w >> 16) & 0xffu) | ((w >> 8) & 0xff0000u); }
DEV bf16x8 frag(s16x4 lo, s16x4 hi) { return join(lo, hi); }
DEV s16x4 tr4(const uint8_t* lds, int off) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + off)); }

struct BwdArgs {
  const bf16_t* x;        // input images [n][784] bf16 (or null with u8)
  const uint8_t* u8;      // input images [n][784] uint8, normalised while staging (or null)
  const int64_t* idx;     // per-sample row of x / u8 (null: sample b is row b)
  int n;
  const bf16_t* p1;       // pool1 [B][196][8] (channels 6, 7 zero)
  const uint8_t* arg1;    // pool1 argmax codes [B][196] x 4 bytes: byte k = code(k) | code(k + 4) << 4
  const bf16_t* dp2;      // dL/d pool2 [B][400] (NHWC 5x5x16)
  const uint8_t* arg2;    // pool2 argmax codes [B][400]
  const bf16_t* w2;       // conv2 weights [5][5][8][16]
  int B;
  float* slab1;           // [grid][32][8]: rows tap 0..24, 25 = bias
  float* slab2;           // [grid][208][16]: rows tap * 8 + ci, 200 = bias
  unsigned long long* prof;   // optional (experiments): per-phase clock sums [NPROF] over all waves
};
// phase clocks (s_memtime): 0 stage-in (X / codes + next-tile loads issue), 1 dgrad, 2 conv2
// wgrad, 3 barrier 1, 4 stage dY2 / pool1, 5 conv1 wgrad, 6 barrier 2 (loop top), 7 epilogue
constexpr int NPROF = 8;

// ------------------------------------------------------------------ staging (global -> regs -> LDS)
constexpr int NCH = (T * NWIN1 + NT - 1) / NT;   // 4: pool1 / input / code chunks per thread
struct Stage {
  u32x4 dp;               // dL/dpool2: 8 channels of one pooled pixel (threads < 400)
  u32x2 c2;               // their argmax codes
  u32x4 p1[NCH];          // pool1: one window (8 channels) per chunk
  u32x2 x[NCH];           // input: 4 pixels per chunk (uint8: x[i][0])
  uint32_t a1[NCH];       // pool1 argmax word per chunk

  DEV void load(const BwdArgs& a, int t0, int tid) {
    const int nimg = t0 < 0 ? 0 : min(T, a.B - t0);
    const int tb = t0 < 0 ? 0 : t0;
    const auto rdp = buf_rsrc(a.dp2 + (int64_t)tb * 400, (uint32_t)nimg * 800u);
    const auto ra2 = buf_rsrc(a.arg2 + (int64_t)tb * 400, (uint32_t)nimg * 400u);
    const auto rp1 = buf_rsrc(a.p1 + (int64_t)tb * NWIN1 * 8, (uint32_t)nimg * (NWIN1 * 16u));
    const auto ra1 = buf_rsrc(a.arg1 + (int64_t)tb * NWIN1 * 4, (uint32_t)nimg * (NWIN1 * 4u));
    const uint32_t esz = a.u8 ? 1u : 2u;
    const auto rx = a.u8 ? buf_rsrc(a.u8, (uint32_t)a.n * 784u) : buf_rsrc(a.x, (uint32_t)a.n * 1568u);
    // per-sample dataset rows (buffer loads: out-of-tile images read 0, no per-lane branch)
    const auto ridx = buf_rsrc(a.idx ? (const void*)(a.idx + tb) : (const void*)a.p1, a.idx ? (uint32_t)nimg * 8u : 0u);
    dp = buf_b128(rdp, tid < 400 ? 16u * tid : BUF_OOB);
    c2 = buf_b64(ra2, tid < 400 ? 8u * tid : BUF_OOB);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int e = tid + NT * i;
      const uint32_t ok = e < T * NWIN1 ? 0u : BUF_OOB;
      p1[i] = buf_b128(rp1, 16u * e + ok);
      a1[i] = buf_b32(ra1, 4u * e + ok);
      const int img = e / NWIN1, r = e - img * NWIN1;
      int row = tb + img;
      if (a.idx) {   // kernel argument: uniform
        const u32x2 rv = buf_b64(ridx, 8u * img);
        row = (int)rv[0];
        row = (rv[1] != 0u || row < 0) ? 0 : (row >= a.n ? a.n - 1 : row);
      }
      const uint32_t xo = (e < T * NWIN1 && img < nimg) ? (uint32_t)row * (784u * esz) + (uint32_t)r * 4u * esz
                                                        : BUF_OOB;
      if (a.u8) x[i] = u32x2{buf_b32(rx, xo), 0u};
      else x[i] = buf_b64(rx, xo);
    }
  }
  // input chunks + argmax codes (read by the conv1 weight gradient)
  DEV void store_x_codes(uint8_t* lds, int tid, bool u8) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int e = tid + NT * i;
      if (e < T * NWIN1) {
        const int img = e / NWIN1, r = e - img * NWIN1, y = r / 7, k = r - 7 * y;
        uint32_t lo = x[i][0], hi = x[i][1];
        if (u8) {
          const uint32_t b = x[i][0];
          lo = pack2(u8_norm(b & 0xff), u8_norm((b >> 8) & 0xff));
          hi = pack2(u8_norm((b >> 16) & 0xff), u8_norm(b >> 24));
        }
        *(u32x2*)(lds + X_OFF + img * X_IMG + (y + 2) * X_RS + (4 * k + 4) * 2) = u32x2{lo, hi};
        const uint32_t l4 = a1[i] & 0x0f0f0f0fu, h4 = (a1[i] >> 4) & 0x0f0f0f0fu;   // codes c 0..3 / 4..7
        *(u32x4*)(lds + CD_OFF + img * DP1_IMG + r * 16) = u32x4{bytes01(l4), bytes23(l4), bytes01(h4), bytes23(h4)};
      }
    }
  }
  // unpooled dY2 (ReLU mask folded in the codes) + pool1 (read by the conv2 kernels)
  DEV void store_dy2_p1(uint8_t* lds, int tid) const {
    if (tid < 400) {
      const int img = tid / 50, rr = tid - 50 * img, w = rr >> 1, hf = rr & 1;
      const int yp = w / 5, xp = w - 5 * yp;
      const uint32_t e0 = bytes01(c2[0]), e1 = bytes23(c2[0]), e2 = bytes01(c2[1]), e3 = bytes23(c2[1]);
      uint8_t* base = lds + DY2_OFF + img * DY2_IMG + (2 * yp + 1) * DY2_RS + 2 * xp * 32 + 16 * hf;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const u32x4 v = {dp[0] & heq(e0, d), dp[1] & heq(e1, d), dp[2] & heq(e2, d), dp[3] & heq(e3, d)};
        *(u32x4*)(base + (d >> 1) * DY2_RS + (d & 1) * 32) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int e = tid + NT * i;
      if (e < T * NWIN1) {
        const int img = e / NWIN1, r = e - img * NWIN1;
        *(u32x4*)(lds + P1_OFF + img * P1_IMG + r * 16) = p1[i];
      }
    }
  }
};

// Work split.  The weight-gradient accumulators are split between the two halves of the
// block (waves 0-3: conv2 M tiles 0-6 and the even-xp conv1 set; waves 4-7: tiles 7-12 and
// the odd set), so a wave holds 52 accumulator registers, not 100.  Phase 1: dgrad output
// row pair per wave (kernel-row counts 2, 4, 5, 5, 5, 4, 2 x 15 MFMAs; -1: none) and the
// range of conv2 k-steps each wave runs for its half's tiles (7 / 6 MFMAs each), balanced
// per SIMD (waves w, w + 4 share one).  Phase 2: each half's conv1 set, k-steps w % 4 + 4 i.
__constant__ int dg_row[NW] = {2, 3, 0, -1, 4, 1, 5, 6};
__constant__ int c2_ks0[NW] = {0, 2, 4, 12, 0, 4, 9, 15};
__constant__ int c2_ks1[NW] = {2, 4, 12, 25, 4, 9, 15, 25};
constexpr int C2T0 = 7;            // conv2 M tiles of the first half

__global__ __launch_bounds__(NT, 1) void lenet_bwd_k(const BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i16 = lane & 15, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ntiles = (a.B + T - 1) / T;
  const int nk = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  auto tile0 = [&](int k) { return ((int)blockIdx.x + k * (int)gridDim.x) * T; };

  // ---- prologue: zero the tiles (borders stay zero), ONES cell, dgrad A fragments
  for (int e = tid; e < (ZERO_OFF + 16) / 16; e += NT) *(u32x4*)(lds + 16 * e) = u32x4{0u, 0u, 0u, 0u};
  if (tid == 0) *(u32x4*)(lds + ONES_OFF) = u32x4{0x3f80u, 0u, 0u, 0u};
  __syncthreads();
  for (int e = tid; e < 15 * 64; e += NT) {
    const int f = e >> 6, l = e & 63, dy = f / 3, j = f - 3 * dy;
    const int r = (l & 15) >> 3, ci = l & 7, gg = l >> 4, xs = gg >> 1, co0 = 8 * (gg & 1);
    const int dx = r + 4 - 2 * j - xs;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (dx >= 0 && dx <= 4) v = *(const u32x4*)(a.w2 + ((dy * 5 + dx) * 8 + ci) * 16 + co0);
    *(u32x4*)(lds + AF_OFF + 16 * e) = v;
  }
  Stage st;
  st.load(a, nk > 0 ? tile0(0) : -1, tid);
  st.store_dy2_p1(lds, tid);

  const int half = wave >> 2;       // accumulator half (uniform)
  f32x4 acc2[C2T0];                  // conv2 M tiles half * 7 + t (t < 7 - half)
#pragma unroll
  for (int t = 0; t < C2T0; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1[3][2];                  // conv1 set sig = half: [M tile][N tile]
#pragma unroll
  for (int t = 0; t < 3; ++t) acc1[t][0] = acc1[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db1[4] = {0.f, 0.f, 0.f, 0.f};

  // per-lane constants of the transposed reads: MFMA K row 8g + 4rho + q is item kk[rho]
  // of the 32-item k-step (the 8 rows one 32-lane half reads together are consecutive items)
  const int kk0 = 16 * (g >> 1) + 4 * (g & 1) + q, kk1 = kk0 + 8;
  const int hA = p >> 1, pc = p & 1;
  const int hoff[3] = {hA ? 896 : 0, hA ? 224 : 0, hA ? 16 : 0};
  const uint32_t dsel = (uint32_t)(i16 >> 3);
  const auto rarg1 = buf_rsrc(a.arg1, (uint32_t)a.B * (NWIN1 * 4u));

  uint64_t pc_acc[NPROF] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tclk = __builtin_amdgcn_s_memtime();
  auto mark = [&](int ph) {
    if (a.prof) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      pc_acc[ph] += t - tclk;
      tclk = t;
    }
  };
  for (int k = 0; k < nk; ++k) {
    const int t0 = tile0(k);
    __syncthreads();   // dY2 / pool1 of this tile stored; the previous conv1 phase is done
    mark(6);
    st.store_x_codes(lds, tid, a.u8 != nullptr);
    st.load(a, k + 1 < nk ? tile0(k + 1) : -1, tid);
    mark(0);

    // ================================================ phase 1a: conv2 dgrad, one output row pair
    const int pr = dg_row[wave];
    if (pr >= 0) {
      const int img = i16 & 7, rr = i16 >> 3;
      const int dylo = max(0, 2 * pr - 9), dyhi = min(4, 2 * pr + 1);
      // argmax words of this lane's 7 windows (pool1 bias gradient: active windows only)
      uint32_t aw[7];
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const int w1 = (2 * pr + rr) * 14 + 2 * u + (g >> 1);
        aw[u] = buf_b32(rarg1, t0 + img < a.B ? 4u * ((uint32_t)(t0 + img) * NWIN1 + w1) : BUF_OOB);
      }
      f32x4 acc[7];
#pragma unroll
      for (int u = 0; u < 7; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int bB = DY2_OFF + img * DY2_IMG + (2 * pr + rr + 1) * DY2_RS + (g >> 1) * 32 + (g & 1) * 16;
#pragma unroll 1
      for (int dy = dylo; dy <= dyhi; ++dy) {
        bf16x8 A[3], Bv[5];
#pragma unroll
        for (int j = 0; j < 3; ++j) A[j] = *(const bf16x8*)(lds + AF_OFF + ((dy * 3 + j) * 64 + lane) * 16);
        const uint8_t* pb = lds + bB - dy * DY2_RS;
#pragma unroll
        for (int v = 0; v < 5; ++v) Bv[v] = *(const bf16x8*)(pb + 64 * v);
#pragma unroll
        for (int v = 0; v < 5; ++v)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[v + 2 - j] = mfma16(A[j], Bv[v], acc[v + 2 - j]);
      }
      // dP1 (bf16) for the conv1 weight gradient; the bias gradient of conv1 from the fp32
      // sums of the active windows (code != 4)
      const int sh = 4 * (g & 1);
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const int w1 = (2 * pr + rr) * 14 + 2 * u + (g >> 1);
        *(u32x2*)(lds + DP1_OFF + img * DP1_IMG + w1 * 16 + 8 * (g & 1)) =
            u32x2{pack2(acc[u][0], acc[u][1]), pack2(acc[u][2], acc[u][3])};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          db1[i] += ((aw[u] >> (8 * i + sh)) & 15u) != 4u ? acc[u][i] : 0.f;
      }
    }

    mark(1);
    // ================================================ phase 1b: conv2 weight gradient k-steps
    {
      const int s0 = c2_ks0[wave], s1 = c2_ks1[wave];
#pragma unroll 1
      for (int s = s0; s < s1; ++s) {
        int ab[2], bb[2];
#pragma unroll
        for (int rho = 0; rho < 2; ++rho) {
          const int kx = 32 * s + (rho ? kk1 : kk0);
          const int img = (kx * 5243) >> 19, pix = kx - 100 * img;
          const int y = (pix * 205) >> 11, x = pix - 10 * y;
          ab[rho] = P1_OFF + img * P1_IMG + (y * 14 + x) * 16 + 8 * pc;
          bb[rho] = DY2_OFF + img * DY2_IMG + (y + 1) * DY2_RS + x * 32 + 8 * p;
        }
        const bf16x8 Bf = frag(tr4(lds, bb[0]), tr4(lds, bb[1]));
        auto tile = [&](int t, f32x4& acc) {
          int o0, o1;
          if (t == 12 && hA) {
            o0 = o1 = ONES_OFF + 8 * pc;
          } else {
            const int ho = t == 12 ? 0 : hoff[t < 5 ? 0 : t < 10 ? 1 : 2];
            o0 = ab[0] + ho + c2_toff(t);
            o1 = ab[1] + ho + c2_toff(t);
          }
          acc = mfma16(frag(tr4(lds, o0), tr4(lds, o1)), Bf, acc);
        };
        if (half == 0) {
#pragma unroll
          for (int t = 0; t < C2T0; ++t) tile(t, acc2[t]);
        } else {
#pragma unroll
          for (int t = 0; t < 13 - C2T0; ++t) tile(C2T0 + t, acc2[t]);
        }
      }
    }

    mark(2);
    __syncthreads();   // dP1, input and codes of this tile visible; dY2 / pool1 no longer read
    mark(3);
    if (k + 1 < nk) st.store_dy2_p1(lds, tid);
    mark(4);

    // ================================================ phase 2: conv1 weight gradient
    const int sig = half;
#pragma unroll 1
    for (int s = wave & 3; s < 25; s += 4) {
      int ax[2], bx[2];
#pragma unroll
      for (int rho = 0; rho < 2; ++rho) {
        const int kx = 32 * s + (rho ? kk1 : kk0);
        const bool ok = kx < T * 98;
        const int kc = ok ? kx : T * 98 - 1;
        const int img = (kc * 669) >> 16, r = kc - 98 * img;
        const int yp = (r * 147) >> 10, xi = r - 7 * yp, xp = 2 * xi + sig;
        ax[rho] = X_OFF + img * X_IMG + (2 * yp + hA) * X_RS + (4 * xi + 4 * pc + 4 * sig) * 2;
        bx[rho] = ok ? img * DP1_IMG + (yp * 14 + xp) * 16 + 8 * pc : -1;
      }
      const s16x4 d0 = tr4(lds, bx[0] >= 0 ? DP1_OFF + bx[0] : ZERO_OFF + 8 * pc);
      const s16x4 d1 = tr4(lds, bx[1] >= 0 ? DP1_OFF + bx[1] : ZERO_OFF + 8 * pc);
      const s16x4 c0 = tr4(lds, bx[0] >= 0 ? CD_OFF + bx[0] : ZERO_OFF + 8 * pc);
      const s16x4 c1 = tr4(lds, bx[1] >= 0 ? CD_OFF + bx[1] : ZERO_OFF + 8 * pc);
      const u32x4 dv = __builtin_bit_cast(u32x4, frag(d0, d1)), cv = __builtin_bit_cast(u32x4, frag(c0, c1));
      bf16x8 Bm[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const uint32_t d = 2u * nt + dsel;
        Bm[nt] = __builtin_bit_cast(bf16x8, u32x4{dv[0] & heq(cv[0], d), dv[1] & heq(cv[1], d),
                                                  dv[2] & heq(cv[2], d), dv[3] & heq(cv[3], d)});
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const bf16x8 Af = frag(tr4(lds, ax[0] + 2 * t * X_RS), tr4(lds, ax[1] + 2 * t * X_RS));
        acc1[t][0] = mfma16(Af, Bm[0], acc1[t][0]);
        acc1[t][1] = mfma16(Af, Bm[1], acc1[t][1]);
      }
    }
    mark(5);
  }

  // ---- epilogue: the 8 waves' partials -> this block's slab rows (fixed summation order)
  __syncthreads();
  mark(6);
  // conv2: tile T of wave w = half(w) * 7 + t; partials [wave][t][col 16][row 16]
  float* e2 = (float*)lds;
#pragma unroll
  for (int t = 0; t < C2T0; ++t)
    *(f32x4*)(e2 + ((wave * C2T0 + t) * 16 + i16) * 16 + 4 * g) = acc2[t];
  __syncthreads();
  float* s2 = a.slab2 + (int64_t)blockIdx.x * 208 * 16;
  for (int e = tid; e < 13 * 256; e += NT) {
    const int tt = e >> 8, row = (e >> 4) & 15, col = e & 15;
    const int h = row >> 3, ci = row & 7, tap = c2_tap(tt, h);
    if (tap == 25 && ci != 0) continue;
    const int hw = tt < C2T0 ? 0 : 4, t = tt < C2T0 ? tt : tt - C2T0;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += e2[(((hw + w) * C2T0 + t) * 16 + col) * 16 + row];
    s2[(tap == 25 ? 200 : tap * 8 + ci) * 16 + col] = v;
  }
  __syncthreads();
  float* e1 = (float*)lds;                       // [wave][t][nt][col 16][row 16] (set = wave >> 2)
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      *(f32x4*)(e1 + (((wave * 3 + t) * 2 + nt) * 16 + i16) * 16 + 4 * g) = acc1[t][nt];
  float* eb = (float*)(lds + E1_SZ);             // [wave][lane][4]: conv1 bias partials
  *(f32x4*)(eb + (wave * 64 + lane) * 4) = f32x4{db1[0], db1[1], db1[2], db1[3]};
  __syncthreads();
  float* s1 = a.slab1 + (int64_t)blockIdx.x * 32 * 8;
  if (tid < 26 * 8) {
    const int tap = tid >> 3, c = tid & 7;
    float v = 0.f;
    if (tap < 25) {
      const int dy = tap / 5, dx = tap - 5 * dy;
      for (int w = 0; w < NW; ++w) {
        const int s = w >> 2;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int ty = dy + (d >> 1), tx = dx + (d & 1), txi = tx + (s ? 0 : 2);
          const int t = ty >> 1, row = 4 * (2 * (ty & 1) + (txi >> 2)) + (txi & 3);
          const int nt = d >> 1, col = c + 8 * (d & 1);
          v += e1[(((w * 3 + t) * 2 + nt) * 16 + col) * 16 + row];
        }
      }
    } else {
      // lane l holds channels 4 (l >> 4 & 1) + i of its windows (waves without a row pair: 0)
      for (int w = 0; w < NW; ++w)
        for (int l = 0; l < 64; ++l)
          if ((4 * ((l >> 4) & 1)) == (c & 4)) v += eb[(w * 64 + l) * 4 + (c & 3)];
    }
    s1[tap * 8 + c] = v;
  }
  if (a.prof) {
    mark(7);
    if (lane == 0)
      for (int i = 0; i < NPROF; ++i) atomicAdd(a.prof + i, (unsigned long long)pc_acc[i]);
  }
}

}  // namespace

int lenet_bwd_grid() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipFuncSetAttribute((const void*)lenet_bwd_k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lenet_bwd_k, NT, LDS_BYTES) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per <= 0)
      return -1;
    n = per * cus;
  }
  return n;
}

hipError_t lenet_bwd(const XSrc& x, const bf16_t* p1, const uint8_t* arg1, const bf16_t* dp2, const uint8_t* arg2,
                     const bf16_t* w2, int B, float* slab1, float* slab2, int grid, hipStream_t st,
                     unsigned long long* prof) {
  if (B <= 0) return hipSuccess;
  if ((!x.x && !x.u8) || grid <= 0) return hipErrorInvalidValue;
  const int res = lenet_bwd_grid();
  if (res <= 0) return hipErrorInvalidValue;
  BwdArgs a{x.u8 ? nullptr : x.x, x.u8, x.idx, x.idx ? x.n : B, p1, arg1, dp2, arg2, w2, B, slab1, slab2, prof};
  hipLaunchKernelGGL(lenet_bwd_k, dim3(grid), dim3(NT), LDS_BYTES, st, a);
  return hipGetLastError();
}

// the grid the executor sizes the slabs for: one block per CU (capped by the tile count)
int lenet_bwd_blocks(int B) {
  const int res = lenet_bwd_grid();
  if (res <= 0) return -1;
  const int ntiles = (B + T - 1) / T;
  return cap_grid(ntiles < res ? ntiles : res);
}

}  // namespace mnistx
