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
//    15 fragments are formed once per block (LDS) and the column pairs of a row pair slide
//    over the B fragments (one 16-byte read each) of a kernel row; kernel rows whose input
//    row lies outside 0..9 for both output rows are skipped.  A row pair is split in two
//    units (column pairs 0-3: 9 MFMAs per kernel row, 4-6: 6).
//  * conv2 weight gradient: rows = (2 taps, ci 8), columns = co 16, K = 32 (pixel, image)
//    items; both operands are ds_read_b64_tr_b16 transposed reads of the NHWC tiles (one
//    per lane: 4 channels of one pixel).  The bias needs no tile of its own: pool1 channel 6
//    (zero in HBM) is staged as 1.0, so row (tap 0, ci 6) sums dY2.
//  * conv1 weight gradient, by pool-window phase: with dY1 = dP1 at the window position
//    d = 2a + b of each (window, channel)'s argmax, dW1[dy][dx][c] =
//    sum_d sum_w X[2yp+a+dy-2][2xp+b+dx-2] dP1[w][c] [code(w,c) == d], i.e. one GEMM
//    C[(ty, tx)][(c, d)] over the windows w (ty = a + dy, tx = b + dx in 0..5) folded at
//    the end.  A = input patches at (2yp + ty - 2, 2xp + tx - 2): a transposed read of 4
//    consecutive input pixels per lane (8-byte aligned because windows are taken by x
//    parity: even-xp windows cover tx -2..5, odd ones 0..7 -- two accumulator sets);
//    B = dP1 masked by the argmax code (3 packed-u16 VALU per 2 columns).
//  * Weight-gradient K items are enumerated image-fastest (item = 8 * pixel + image) over
//    rows padded to a multiple of 4 pixels (dY2: 12, window sets: 8; the pad reads zeros),
//    so a k-step is one row segment: every lane address is a per-lane base plus a
//    wave-uniform step offset (one VALU add per operand per k-step, no index decode), the
//    32 lanes of one transposed read cover the 8 images of one pixel, and with the image
//    strides below the reads are conflict-free (bench/lds_bwd.py; conv2 tiles pair taps one
//    pixel or one 17-pixel row apart: 4 dwords mod 8 either way).
// 16 waves (4 per SIMD) share a tile in two phases (two barriers): [store input / codes of
// this tile, load the next tile's data, one dgrad unit + conv2 weight-gradient k-steps of
// the wave's tile group] -> [conv1 weight-gradient k-steps of the wave's parity set, store
// the next tile's dY2 / pool1].  The accumulators are split (a wave holds at
// most 4 conv2 tiles and one conv1 set: 40 registers) so the kernel fits 128 VGPRs.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "launchers.h"
#include "wgrad_tr.h"

namespace mnistx {
namespace {


constexpr int NT = 1024, NW = 16, T = 8;
constexpr int NWIN1 = 196;                                 // pool1 windows per image
// ---- LDS layout (bytes); image / row strides from bench/lds_bwd.py (bank model)
constexpr int AF_OFF = 0, AF_SZ = 15 * 64 * 16;            // dgrad A fragments [dy*3+j][lane] x 16 B
constexpr int DY2_RS = 384, DY2_IMG = 3872;                // dY2 [img][10 rows][12 px][16 co] bf16 (px 10, 11 zero)
constexpr int DY2_OFF = AF_OFF + AF_SZ, DY2_SZ = T * DY2_IMG;
constexpr int ZERO_OFF = DY2_OFF + DY2_SZ;                 // one zero dY2 row: the dgrad's rows -1 / 10
constexpr int P1_RS = 272, P1_IMG = 3808;                  // pool1 [img][14][17 px][8] bf16 (px 14.. zero)
constexpr int P1_OFF = ZERO_OFF + DY2_RS, P1_SZ = T * P1_IMG;
constexpr int X_RS = 80, X_IMG = 2592;                     // input [img][row -2..29][col -4..35] bf16
constexpr int X_OFF = P1_OFF + P1_SZ, X_SZ = T * X_IMG;
constexpr int D_RS = 280, D_IMG = 3920;                    // dP1 / codes [img][14][17.5 windows][8] x 2 B
constexpr int DP1_OFF = X_OFF + X_SZ, D_SZ = T * D_IMG;
constexpr int CD_OFF = DP1_OFF + D_SZ;                     // argmax codes (u16 per channel)
constexpr int LDS_BYTES = CD_OFF + D_SZ;
static_assert(LDS_BYTES <= 163840, "one workgroup per CU");
static_assert(10 * DY2_RS <= DY2_IMG && 32 * X_RS <= X_IMG && 14 * P1_RS <= P1_IMG && 14 * D_RS <= D_IMG, "");
static_assert((ZERO_OFF - DY2_OFF) % 256 == 0, "zero row bank-aligned with the dY2 rows (bench/lds_bwd.py)");
constexpr int C2MAX = 4;                                   // conv2 tiles per wave group (max)
static_assert(NW * C2MAX * 256 * 4 <= LDS_BYTES && NW * 6 * 256 * 4 + NW * 8 * 4 <= LDS_BYTES, "epilogue scratch");

// conv2 weight-gradient M tiles: rows h * 8 + ci are tap C2_TAP0[t] + h (tiles 0-9: taps one
// pixel apart) or C2_TAP0[t] + 5 h (tiles 10-12: one row apart; tap 29 = discarded rows).
// Tile groups: waves 4G .. 4G + 3 own the tiles of group G (G0: 0-3, G1: 4, 5, 10, G2: 6, 7,
// 11, G3: 8, 9, 12).
constexpr int C2_TAP0[13] = {0, 2, 5, 7, 10, 12, 15, 17, 20, 22, 4, 14, 24};
constexpr int C2_GT[4][C2MAX] = {{0, 1, 2, 3}, {4, 5, 10, -1}, {6, 7, 11, -1}, {8, 9, 12, -1}};
__constant__ int c2_gt[4][C2MAX] = {{0, 1, 2, 3}, {4, 5, 10, -1}, {6, 7, 11, -1}, {8, 9, 12, -1}};
__constant__ int c2_tap0[13] = {0, 2, 5, 7, 10, 12, 15, 17, 20, 22, 4, 14, 24};

struct BwdArgs {
  const bf16_t* x;        // input images [n][784] bf16 (or null with u8)
  const uint8_t* u8;      // input images [n][784] uint8, normalised while staging (or null)
  const int64_t* idx;     // per-sample row of x / u8 (null: sample b is row b)
  int n;
  const bf16_t* p1;       // pool1 records [B][196] x 16 bytes: channels 0-5 bf16, then the window's
                          // argmax code word (byte k = code(k) | code(k + 4) << 4) -- lenet_band.hip
  const bf16_t* dp2;      // dL/d pool2 [B][400] (NHWC 5x5x16)
  const uint8_t* arg2;    // pool2 argmax codes [B][400]
  const bf16_t* w2;       // conv2 weights [5][5][8][16]
  int B;
  float* slab1;           // [grid][32][8]: rows tap 0..24, 25 = bias
  float* slab2;           // [grid][208][16]: rows tap * 8 + ci, 200 = bias
  unsigned long long* prof;   // optional (experiments): per-phase clock sums [NPROF] over all waves
  int skip;               // experiments (prof launches only): work to skip, for time attribution
  int prof_waves;         // experiments: also per-wave sums prof[NPROF + wave * NPROF + phase]
  // the static work split (defaults below; MNISTX_BWD_SPLIT overrides it for experiments):
  // dgrad unit per wave, conv2 weight-gradient k-step range per wave (within its tile group),
  // conv1 weight-gradient k-step range per rank (wave >> 1)
  int8_t du[16], k20[16], k21[16], k10[8], k11[8];
};
// phase clocks (s_memtime): 0 store input / codes, 1 dgrad (+ next-tile input loads), 2 conv2
// wgrad, 3 barrier 1, 4 next-tile dY2 / pool1 loads issue, 5 conv1 wgrad + dY2 / pool1 store,
// 6 barrier 2 (loop top), 7 epilogue
constexpr int NPROF = 8;

// ------------------------------------------------------------------ staging (global -> regs -> LDS)
// Input, pool1 and codes: wave pair 2i stages image i, lane r of the pair windows / input
// quads r and r + 128 (< 196), so a wave's image and dataset row are wave-uniform (the
// batch-index entry is one uniform load, a tile ahead of the input it addresses).
// dL/dpool2 + codes: threads < 400, one pooled pixel (8 channels) each.  Everything for
// the next tile is loaded at the start of phase 1: the input + pool1 codes are stored at the
// next loop top, dY2 + pool1 at the end of phase 2.
constexpr int NCH = 2;
static_assert(NW == 2 * T && 2 * 128 >= NWIN1 && 128 <= NWIN1, "staging: one wave pair per image, 2 chunks");
template <bool U8, bool IDX>
struct Stage {
  u32x2 x[NCH];           // input: 4 pixels per chunk (uint8: x[i][0])
  u32x2 rowv;             // IDX: the batch-index entry of this wave's image, one tile ahead
  u32x4 dp;               // dL/dpool2: 8 channels of one pooled pixel (threads < 400)
  u32x2 c2;               // their argmax codes
  u32x4 p1[NCH];          // pool1 record: one window (channels 0-5 + its code word) per chunk; the
                          // codes are read by store_xc at the NEXT loop top, after store_dy

  DEV static int img_of(int wave) { return wave >> 1; }
  DEV void load_row(const BwdArgs& a, int t0, int wave) {
    if constexpr (IDX) {
      const int img = img_of(wave);
      const bool ok = t0 >= 0 && t0 + img < a.B;
      const auto ridx = buf_rsrc(a.idx + (ok ? t0 + img : 0), ok ? 8u : 0u);
      rowv = buf_b64(ridx, 0u);
    }
  }
  DEV void load_xc(const BwdArgs& a, int t0, int wave, int ln) {
    const int img = img_of(wave);
    const bool ok = t0 >= 0 && t0 + img < a.B;
    int row = ok ? t0 + img : 0;
    if constexpr (IDX) {
      const uint32_t lo = __builtin_amdgcn_readfirstlane(rowv[0]), hi = __builtin_amdgcn_readfirstlane(rowv[1]);
      row = (hi != 0u || (int)lo < 0) ? 0 : ((int)lo >= a.n ? a.n - 1 : (int)lo);
    }
    constexpr uint32_t esz = U8 ? 1u : 2u;
    const void* xb = U8 ? (const void*)(a.u8 + (int64_t)row * 784) : (const void*)(a.x + (int64_t)row * 784);
    const auto rx = buf_rsrc(xb, ok ? 784u * esz : 0u);
    const int r = ln + 64 * (wave & 1);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const uint32_t q = (uint32_t)(r + 128 * i);
      const uint32_t oob = q < NWIN1 ? 0u : BUF_OOB;
      if constexpr (U8) x[i] = u32x2{buf_b32(rx, 4u * q + oob), 0u};
      else x[i] = buf_b64(rx, 8u * q + oob);
    }
  }
  // input quads + argmax codes (read by the conv1 weight gradient; the codes ride in the pool1
  // records of this tile, still in p1 until load_dy fetches the next tile's)
  DEV void store_xc(uint8_t* lds, int wave, int ln) const {
    const int img = img_of(wave), r = ln + 64 * (wave & 1);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = r + 128 * i;
      if (i == 0 || q < NWIN1) {
        const int y = (q * 147) >> 10, k = q - 7 * y;          // input quad: row, 4-pixel group
        const int yp = (q * 147) >> 11, xp = q - 14 * yp;      // pool window
        uint32_t lo = x[i][0], hi = x[i][1];
        if constexpr (U8) {
          const uint32_t b = x[i][0];
          lo = pack2(u8_norm(b & 0xff), u8_norm((b >> 8) & 0xff));
          hi = pack2(u8_norm((b >> 16) & 0xff), u8_norm(b >> 24));
        }
        *(u32x2*)(lds + X_OFF + img * X_IMG + (y + 2) * X_RS + (4 * k + 4) * 2) = u32x2{lo, hi};
        const uint32_t a1 = p1[i][3];
        const uint32_t l4 = a1 & 0x0f0f0f0fu, h4 = (a1 >> 4) & 0x0f0f0f0fu;   // codes c 0..3 / 4..7
        uint8_t* cd = lds + CD_OFF + img * D_IMG + yp * D_RS + xp * 16;   // 8-byte aligned rows
        *(u32x2*)cd = u32x2{bytes01(l4), bytes23(l4)};
        *(u32x2*)(cd + 8) = u32x2{bytes01(h4), bytes23(h4)};
      }
    }
  }
  DEV void load_dy(const BwdArgs& a, int t0, int wave, int ln) {
    const int nimg = t0 < 0 ? 0 : min(T, a.B - t0);
    const int tb = t0 < 0 ? 0 : t0;
    const int tid = wave * 64 + ln;
    const auto rdp = buf_rsrc(a.dp2 + (int64_t)tb * 400, (uint32_t)nimg * 800u);
    const auto ra2 = buf_rsrc(a.arg2 + (int64_t)tb * 400, (uint32_t)nimg * 400u);
    dp = buf_b128(rdp, tid < 400 ? 16u * tid : BUF_OOB);
    c2 = buf_b64(ra2, tid < 400 ? 8u * tid : BUF_OOB);
    const int img = img_of(wave);
    const bool ok = t0 >= 0 && t0 + img < a.B;
    const auto rp1 = buf_rsrc(a.p1 + (int64_t)(ok ? t0 + img : 0) * NWIN1 * 8, ok ? NWIN1 * 16u : 0u);
    const int r = ln + 64 * (wave & 1);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const uint32_t q = (uint32_t)(r + 128 * i);
      p1[i] = a.skip & 32 ? u32x4{0u, 0u, 0u, 0u} : buf_b128(rp1, q < NWIN1 ? 16u * q : BUF_OOB);
    }
  }
  // unpooled dY2 (ReLU mask folded in the codes) and pool1 with channel 6 = 1.0 (the conv2
  // bias row), read by the conv2 kernels.  Called at the end of phase 2; the fence keeps the
  // compiler from hoisting the unpooling above the phase (it would wait for the loads there).
  DEV void store_dy(uint8_t* lds, int wave, int ln) {
    asm volatile("" : "+v"(dp), "+v"(c2), "+v"(p1[0]), "+v"(p1[1]));
    const int img = img_of(wave), r = ln + 64 * (wave & 1);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = r + 128 * i;
      if (i == 0 || q < NWIN1) {
        const int yp = (q * 147) >> 11, xp = q - 14 * yp;
        const u32x4 v = {p1[i][0], p1[i][1], p1[i][2], 0x3f80u};   // channel 6 = 1.0, 7 = 0
        *(u32x4*)(lds + P1_OFF + img * P1_IMG + yp * P1_RS + xp * 16) = v;
      }
    }
    const int tid = wave * 64 + ln;
    if (tid < 400) {
      const int im = tid / 50, rr = tid - 50 * im, w = rr >> 1, yp = w / 5, xp = w - 5 * yp;
      const int o = DY2_OFF + im * DY2_IMG + 2 * yp * DY2_RS + 2 * xp * 32 + 16 * (rr & 1);
      const uint32_t e[4] = {bytes01(c2[0]), bytes23(c2[0]), bytes01(c2[1]), bytes23(c2[1])};
      const int rot = (xp >> 1) & 1;   // window column of store i rotated per lane: 2-way -> 1.4 (bench/lds_bwd.py)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = i ^ rot;
        const uint32_t dd = (uint32_t)d * 0x00010001u;
        const u32x4 v = {sel_eq(dp[0], e[0], dd), sel_eq(dp[1], e[1], dd), sel_eq(dp[2], e[2], dd),
                         sel_eq(dp[3], e[3], dd)};
        *(u32x4*)(lds + o + (i >> 1) * DY2_RS + (d & 1) * 32) = v;
      }
    }
  }
};

// dgrad unit: column pairs 4H .. 4H + 3 (H = 1: 4..6) of one output row pair, kernel rows
// dylo..dyhi.  B fragment v (x pairs 2v, 2v + 1) and A fragment j feed column pair v + 2 - j.
template <int H>
DEV void dgrad_unit(const uint8_t* lds, int bB, int bZ, int orow, int lane, int dylo, int dyhi, f32x4 (&acc)[4]) {
  constexpr int VLO = H ? 2 : 0, VHI = H ? 4 : 3, NU = H ? 3 : 4;
#pragma unroll 2
  for (int dy = dylo; dy <= dyhi; ++dy) {
    bf16x8 Bv[VHI - VLO + 1];
    const int r = orow - dy;                                 // dY2 row; -1 / 10: the shared zero row
    const uint8_t* pb = lds + ((unsigned)r <= 9u ? bB - dy * DY2_RS : bZ);
#pragma unroll
    for (int v = VLO; v <= VHI; ++v) Bv[v - VLO] = *(const bf16x8*)(pb + 64 * v);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const bf16x8 A = *(const bf16x8*)(lds + AF_OFF + ((dy * 3 + j) * 64 + lane) * 16);
#pragma unroll
      for (int v = VLO; v <= VHI; ++v) {
        const int u = v + 2 - j - 4 * H;
        if (u >= 0 && u < NU) acc[u] = mfma16(A, Bv[v - VLO], acc[u]);
      }
    }
  }
}

// conv2 weight-gradient k-steps ks0 .. ks1 - 1 of tile group G (k-step s: dY2 row s / 3,
// pixels 4 (s % 3) .. + 3).  Lane bases: B (dY2), A for the pixel-apart tiles and A for the
// row-apart ones; a step adds one uniform offset to each.
template <int G>
DEV void c2w_steps(const uint8_t* lds, int ks0, int ks1, int ln, f32x4 (&acc2)[C2MAX]) {
  const int g = ln >> 4, q = (ln >> 2) & 3, p = ln & 3;
  const int img = 4 * (g & 1) + q, sub = 2 * (g >> 1), hA = p >> 1, pc = p & 1;
  const int bB = DY2_OFF + img * DY2_IMG + sub * 32 + 8 * p;
  const int aB = P1_OFF + img * P1_IMG + sub * 16 + 8 * pc;
  const int aP = aB + hA * 16, aR = aB + hA * P1_RS;        // second tap: next pixel / next row
  constexpr int NT2 = G == 0 ? 4 : 3;
#pragma unroll 2
  for (int s = ks0; s < ks1; ++s) {
    const int y = s / 3, x0 = 4 * (s - 3 * y);              // uniform
    const int sb = bB + y * DY2_RS + x0 * 32, sa = y * P1_RS + x0 * 16;
    const bf16x8 Bf = frag(tr4(lds, sb), tr4(lds, sb + 32));
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const int tile = C2_GT[G][t], tap = C2_TAP0[tile];
      const int base = (tile < 10 ? aP : aR) + sa + (tap / 5) * P1_RS + (tap % 5) * 16;
      acc2[t] = mfma16(frag(tr4(lds, base), tr4(lds, base + 16)), Bf, acc2[t]);
    }
  }
}

// ---- static work split.  Waves w, w + 4, w + 8, w + 12 share a SIMD (dgrad units: kernel-row
// counts 2, 4, 5, 5, 5, 4, 2 x 9 or 6 MFMAs; conv2 k-steps: 4 / 3 / 3 / 3 MFMAs in tile
// groups 0 / 1 / 2 / 3).
// dgrad unit of each wave (row pair * 2 + half, -1: none) and its conv2 k-step range
// (group wave >> 2; the group's 30 steps split end to end).
// Per-wave clocks (bench/micro_lenet_bwd.py, profiles/r5/lenet/bwd_per_wave/) showed the
// youngest waves of each SIMD (s, s+4, s+8, s+12) reaching the barriers last whatever their MFMA
// count; the split below moves dgrad units off waves 14 / 15 and the heavier ones (rows 2-4: 5
// taps) onto the oldest waves, evens tile group 0's k-steps and gives the conv1 ranks
// 4,4,4,4,4,4,2,2 steps: 201.8 -> 196.1 us (search round 3), -> 194.5 vs 196.9 us (rounds 4-5,
// eight interleaved rounds; bench/bwd_split_search.py, profiles/r5/lenet/bwd_split/; round-4
// split: 2,10,0,-1,... / 0,1,8,23 / ranks 4,4,4,4,3,3,3,3).
constexpr int8_t DG_UNIT[NW] = {7, 5, 9, 4, 6, 10, 3, 8, 2, 11, 0, 1, 12, 13, -1, -1};
constexpr int8_t C2_KS0[NW] = {0, 6, 13, 23, 0, 8, 16, 23, 0, 7, 15, 22, 0, 7, 14, 22};
constexpr int8_t C2_KS1[NW] = {6, 13, 23, 30, 8, 16, 23, 30, 7, 15, 22, 30, 7, 14, 22, 30};
// conv1 k-steps (s: window row s / 2, windows 4 (s % 2) .. + 3 of the set) of parity set
// w & 1: rank w >> 1 runs 4, 4, 4, 4, 4, 4, 2, 2 steps
constexpr int8_t C1_KS0[8] = {0, 4, 8, 12, 16, 20, 24, 26};
constexpr int8_t C1_KS1[8] = {4, 8, 12, 16, 20, 24, 26, 28};

template <bool PROF, bool U8, bool IDX>
__global__ __launch_bounds__(NT, 1) void lenet_bwd_k(const BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = (a.B + T - 1) / T;
  const int nk = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  auto tile0 = [&](int k) { return k < nk ? ((int)blockIdx.x + k * (int)gridDim.x) * T : -1; };

  // ---- prologue: zero the tiles (borders and pads stay zero), dgrad A fragments
  for (int e = tid; e < LDS_BYTES / 16; e += NT) *(u32x4*)(lds + 16 * e) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  if (tid < 15 * 64) {
    const int f = tid >> 6, dy = f / 3, j = f - 3 * dy;
    const int r = (lane & 15) >> 3, ci = lane & 7, xs = lane >> 5, co0 = 8 * ((lane >> 4) & 1);
    const int dx = r + 4 - 2 * j - xs;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (dx >= 0 && dx <= 4) v = *(const u32x4*)(a.w2 + ((dy * 5 + dx) * 8 + ci) * 16 + co0);
    *(u32x4*)(lds + AF_OFF + 16 * tid) = v;
  }
  Stage<U8, IDX> st;
  st.load_row(a, tile0(0), wave);
  st.load_xc(a, tile0(0), wave, lane);
  st.load_dy(a, tile0(0), wave, lane);
  st.load_row(a, tile0(1), wave);
  st.store_dy(lds, wave, lane);

  const int grp = wave >> 2, sig = wave & 1;          // conv2 tile group / conv1 parity set (uniform)
  f32x4 acc2[C2MAX];
#pragma unroll
  for (int t = 0; t < C2MAX; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1[3][2];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc1[t][0] = acc1[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db1[4] = {0.f, 0.f, 0.f, 0.f};
  const int du = a.du[wave];
  const int ks0 = a.k20[wave], ks1 = a.k21[wave];
  const int cs0 = a.k10[wave >> 1], cs1 = a.k11[wave >> 1];

  uint64_t pc_acc[NPROF] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tclk = __builtin_amdgcn_s_memtime();
  auto mark = [&](int ph) {
    if constexpr (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      pc_acc[ph] += t - tclk;
      tclk = t;
    }
  };

  for (int k = 0; k < nk; ++k) {
    const int t0 = tile0(k);
    if (!(PROF && (a.skip & 16))) __syncthreads();   // dY2 / pool1 of this tile stored; the previous conv1 phase is done
    mark(6);
    if (!(PROF && (a.skip & 8))) {
      const int ln = lane_now();
      st.store_xc(lds, wave, ln);
    }
    mark(0);

    // ================================================ phase 1a: conv2 dgrad unit
    if (du >= 0 && !(PROF && (a.skip & 1))) {
      const int ln = lane_now();
      const int i16 = ln & 15, g = ln >> 4;
      const int pr = du >> 1, hx = du & 1;
      const int img = i16 >> 1, rr = i16 & 1, orow = 2 * pr + rr;
      const int dylo = max(0, 2 * pr - 9), dyhi = min(4, 2 * pr + 1);
      const int u0 = 4 * hx;
      // this lane's windows' pool1 values (channels 4 (g & 1) .. + 3), from the LDS tile: the
      // conv1 bias gradient sums dP1 over the ACTIVE windows, and a window is active exactly
      // when its pooled ReLU output is > 0 (code != 4).  (Read from the records' code words in
      // HBM right in front of this unit, that latency was exposed whenever the records had
      // left the Infinity Cache.)  Padded channels 6 / 7 have dP1 = 0 (zero conv2 weights).
      u32x2 pv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        pv[u] = *(const u32x2*)(lds + P1_OFF + img * P1_IMG + orow * P1_RS + (2 * min(u0 + u, 6) + (g >> 1)) * 16 +
                                8 * (g & 1));
      if (!(PROF && (a.skip & 8))) st.load_xc(a, tile0(k + 1), wave, ln);
      f32x4 acc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int lo = (g >> 1) * 32 + (g & 1) * 16;
      const int bB = DY2_OFF + img * DY2_IMG + orow * DY2_RS + lo, bZ = ZERO_OFF + lo;
      if (hx) dgrad_unit<1>(lds, bB, bZ, orow, ln, dylo, dyhi, acc);
      else dgrad_unit<0>(lds, bB, bZ, orow, ln, dylo, dyhi, acc);
      // dP1 (bf16) for the conv1 weight gradient; the conv1 bias gradient from the fp32
      // sums of the active windows (code != 4, i.e. bit 2 of the nibble clear)
      const int wB = DP1_OFF + img * D_IMG + orow * D_RS + (2 * u0 + (g >> 1)) * 16 + 8 * (g & 1);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u0 + u < 7) {
          *(u32x2*)(lds + wB + 32 * u) = u32x2{pack2(acc[u][0], acc[u][1]), pack2(acc[u][2], acc[u][3])};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int16_t pvi = (int16_t)((pv[u][i >> 1] >> (16 * (i & 1))) & 0xffffu);   // bf16 > 0
            db1[i] = fmaf(acc[u][i], pvi > 0 ? 1.f : 0.f, db1[i]);
          }
        }
      }
    } else if (!(PROF && (a.skip & 8))) {
      st.load_xc(a, tile0(k + 1), wave, lane_now());
    }
    // the next tile's dY2 / pool1 (stored at the end of phase 2), issued apart from the input
    // loads so the 16 waves' load bursts do not queue behind each other
    if (!(PROF && (a.skip & 8))) st.load_dy(a, tile0(k + 1), wave, lane_now());
    mark(1);

    // ================================================ phase 1b: conv2 weight-gradient k-steps
    if (ks0 < ks1 && !(PROF && (a.skip & 2))) {
      const int ln = lane_now();
      switch (grp) {
        case 0: c2w_steps<0>(lds, ks0, ks1, ln, acc2); break;
        case 1: c2w_steps<1>(lds, ks0, ks1, ln, acc2); break;
        case 2: c2w_steps<2>(lds, ks0, ks1, ln, acc2); break;
        default: c2w_steps<3>(lds, ks0, ks1, ln, acc2); break;
      }
    }

    mark(2);
    if (!(PROF && (a.skip & 16))) __syncthreads();   // dP1, input and codes of this tile visible; dY2 / pool1 no longer read
    mark(3);
    if (!(PROF && (a.skip & 8))) st.load_row(a, tile0(k + 2), wave);
    mark(4);

    // ================================================ phase 2: conv1 weight gradient (set sig)
    {
      const int ln = lane_now(), g = ln >> 4, q = (ln >> 2) & 3, p = ln & 3;
      const int img = 4 * (g & 1) + q, sub = 2 * (g >> 1), hA = p >> 1, pc = p & 1;
      const uint32_t dsel = (uint32_t)((ln & 15) >> 3);
      const uint32_t dd0 = dsel * 0x00010001u, dd1 = (2u + dsel) * 0x00010001u;
      const int aB = X_OFF + img * X_IMG + hA * X_RS + (4 * sub + 4 * pc + 4 * sig) * 2;
      const int bB = DP1_OFF + img * D_IMG + (2 * sub + sig) * 16 + 8 * pc;
#pragma unroll 2
      for (int s = cs0; s < (PROF && (a.skip & 4) ? cs0 : cs1); ++s) {
        const int yp = s >> 1, xi0 = 4 * (s & 1);           // uniform
        const int sa = aB + 2 * yp * X_RS + 8 * xi0, sb = bB + yp * D_RS + 32 * xi0;
        const u32x4 dv = __builtin_bit_cast(u32x4, frag(tr4(lds, sb), tr4(lds, sb + 32)));
        const u32x4 cv = __builtin_bit_cast(u32x4, frag(tr4(lds, sb + (CD_OFF - DP1_OFF)),
                                                         tr4(lds, sb + (CD_OFF - DP1_OFF) + 32)));
        const bf16x8 B0 = __builtin_bit_cast(bf16x8, u32x4{sel_eq(dv[0], cv[0], dd0), sel_eq(dv[1], cv[1], dd0),
                                                           sel_eq(dv[2], cv[2], dd0), sel_eq(dv[3], cv[3], dd0)});
        const bf16x8 B1 = __builtin_bit_cast(bf16x8, u32x4{sel_eq(dv[0], cv[0], dd1), sel_eq(dv[1], cv[1], dd1),
                                                           sel_eq(dv[2], cv[2], dd1), sel_eq(dv[3], cv[3], dd1)});
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const bf16x8 Af = frag(tr4(lds, sa + 2 * t * X_RS), tr4(lds, sa + 2 * t * X_RS + 8));
          acc1[t][0] = mfma16(Af, B0, acc1[t][0]);
          acc1[t][1] = mfma16(Af, B1, acc1[t][1]);
        }
      }
    }
    if (k + 1 < nk && !(PROF && (a.skip & 8))) st.store_dy(lds, wave, lane_now());
    mark(5);
  }

  // ---- epilogue: the waves' partials -> this block's slab rows (fixed summation order)
  const int i16 = lane & 15, g = lane >> 4;
  __syncthreads();
  mark(6);
  // conv2: partials [wave][t][col 16][row 16]; tile c2_gt[G][t] is summed over waves 4G..4G+3
  float* e2 = (float*)lds;
#pragma unroll
  for (int t = 0; t < C2MAX; ++t) *(f32x4*)(e2 + ((wave * C2MAX + t) * 16 + i16) * 16 + 4 * g) = acc2[t];
  __syncthreads();
  float* s2 = a.slab2 + (int64_t)blockIdx.x * 208 * 16;
  for (int e = tid; e < 4 * C2MAX * 256; e += NT) {
    const int G = e >> 10, t = (e >> 8) & 3, row = (e >> 4) & 15, col = e & 15;
    const int tile = c2_gt[G][t];
    if (tile < 0) continue;
    const int h = row >> 3, ci = row & 7, tap = c2_tap0[tile] + h * (tile < 10 ? 1 : 5);
    const bool bias = tile == 0 && h == 0 && ci == 6;
    if (tap >= 25 || (ci >= 6 && !bias)) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += e2[(((4 * G + w) * C2MAX + t) * 16 + col) * 16 + row];
    s2[(bias ? 200 : tap * 8 + ci) * 16 + col] = v;
  }
  __syncthreads();
  float* e1 = (float*)lds;                       // [wave][t][nt][col 16][row 16] (set = wave & 1)
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      *(f32x4*)(e1 + (((wave * 3 + t) * 2 + nt) * 16 + i16) * 16 + 4 * g) = acc1[t][nt];
  // conv1 bias partials: lane l holds channels 4 ((l >> 4) & 1) + i of its windows; sum the
  // 32 lanes of each channel half (fixed shuffle tree), then [wave][8] (no dgrad unit: 0)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int m = 1; m <= 32; m = m == 8 ? 32 : 2 * m) db1[i] += __shfl_xor(db1[i], m);
  }
  float* eb = e1 + NW * 6 * 256;
  if (lane == 0 || lane == 16) *(f32x4*)(eb + wave * 8 + (lane >> 2)) = f32x4{db1[0], db1[1], db1[2], db1[3]};
  __syncthreads();
  float* s1 = a.slab1 + (int64_t)blockIdx.x * 32 * 8;
  if (tid < 26 * 8) {
    const int tap = tid >> 3, c = tid & 7;
    float v = 0.f;
    if (tap < 25) {
      const int dy = tap / 5, dx = tap - 5 * dy;
      for (int w = 0; w < NW; ++w) {
        const int s = w & 1;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int ty = dy + (d >> 1), tx = dx + (d & 1), txi = tx + (s ? 0 : 2);
          const int t = ty >> 1, row = 4 * (2 * (ty & 1) + (txi >> 2)) + (txi & 3);
          const int nt = d >> 1, col = c + 8 * (d & 1);
          v += e1[(((w * 3 + t) * 2 + nt) * 16 + col) * 16 + row];
        }
      }
    } else {
      for (int w = 0; w < NW; ++w) v += eb[w * 8 + c];
    }
    s1[tap * 8 + c] = v;
  }
  if constexpr (PROF) {   // one atomic per phase and block (the block's waves summed in LDS)
    mark(7);
    __syncthreads();
    unsigned long long* ep = (unsigned long long*)lds;
    if (lane == 0)
      for (int i = 0; i < NPROF; ++i) ep[wave * NPROF + i] = pc_acc[i];
    __syncthreads();
    if (tid < NPROF) {
      unsigned long long v = 0;
      for (int w = 0; w < NW; ++w) v += ep[w * NPROF + tid];
      atomicAdd(a.prof + tid, v);
    }
    if (a.prof_waves && tid < NW * NPROF) atomicAdd(a.prof + NPROF + tid, ep[tid]);   // [wave][phase]
  }
}

// The work split a launch uses: the defaults, or MNISTX_BWD_SPLIT = 64 comma-separated ints
// (du[16], k20[16], k21[16], k10[8], k11[8]) for balancing experiments
// (bench/micro_lenet_bwd_quick.py); an override is validated (every dgrad unit exactly once,
// each tile group's and the conv1 k-step ranges partitioning their steps) and refused if not.
struct BwdSplit {
  int8_t du[16], k20[16], k21[16], k10[8], k11[8];
  bool ok;
};
BwdSplit bwd_split() {
  BwdSplit s{};
  memcpy(s.du, DG_UNIT, 16);
  memcpy(s.k20, C2_KS0, 16);
  memcpy(s.k21, C2_KS1, 16);
  memcpy(s.k10, C1_KS0, 8);
  memcpy(s.k11, C1_KS1, 8);
  s.ok = true;
  const char* e = getenv("MNISTX_BWD_SPLIT");
  if (!e || !*e) return s;
  int v[64], n = 0;
  for (const char* p = e; *p && n < 64;) {
    char* end = nullptr;
    const long x = strtol(p, &end, 10);
    if (end == p) break;
    v[n++] = (int)x;
    p = *end == ',' ? end + 1 : end;
  }
  if (n != 64) return BwdSplit{{}, {}, {}, {}, {}, false};
  int seen[14] = {};
  for (int w = 0; w < 16; ++w) {
    if (v[w] < -1 || v[w] > 13) return BwdSplit{{}, {}, {}, {}, {}, false};
    if (v[w] >= 0) ++seen[v[w]];
  }
  for (int u = 0; u < 14; ++u)
    if (seen[u] != 1) return BwdSplit{{}, {}, {}, {}, {}, false};
  for (int G = 0; G < 4; ++G) {   // each group's ranges: a partition of [0, 30) in some wave order
    int cover[30] = {};
    for (int t = 0; t < 4; ++t) {
      const int w = 4 * G + t, k0 = v[16 + w], k1 = v[32 + w];
      if (k0 < 0 || k1 < k0 || k1 > 30) return BwdSplit{{}, {}, {}, {}, {}, false};
      for (int k = k0; k < k1; ++k) ++cover[k];
    }
    for (int k = 0; k < 30; ++k)
      if (cover[k] != 1) return BwdSplit{{}, {}, {}, {}, {}, false};
  }
  int cover1[28] = {};
  for (int r = 0; r < 8; ++r) {
    const int k0 = v[48 + r], k1 = v[56 + r];
    if (k0 < 0 || k1 < k0 || k1 > 28) return BwdSplit{{}, {}, {}, {}, {}, false};
    for (int k = k0; k < k1; ++k) ++cover1[k];
  }
  for (int k = 0; k < 28; ++k)
    if (cover1[k] != 1) return BwdSplit{{}, {}, {}, {}, {}, false};
  for (int i = 0; i < 16; ++i) {
    s.du[i] = (int8_t)v[i];
    s.k20[i] = (int8_t)v[16 + i];
    s.k21[i] = (int8_t)v[32 + i];
  }
  for (int i = 0; i < 8; ++i) {
    s.k10[i] = (int8_t)v[48 + i];
    s.k11[i] = (int8_t)v[56 + i];
  }
  return s;
}

using BwdKernel = void (*)(BwdArgs);
// [prof][u8][idx]
constexpr BwdKernel kBwd[8] = {lenet_bwd_k<false, false, false>, lenet_bwd_k<false, false, true>,
                               lenet_bwd_k<false, true, false>,  lenet_bwd_k<false, true, true>,
                               lenet_bwd_k<true, false, false>,  lenet_bwd_k<true, false, true>,
                               lenet_bwd_k<true, true, false>,   lenet_bwd_k<true, true, true>};

}  // namespace

int lenet_bwd_grid(int* per_cu = nullptr) {
  static int n = 0, per = 0;
  if (n == 0) {
    int dev = 0, cus = 0;
    for (BwdKernel k : kBwd)
      if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) != hipSuccess)
        return -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kBwd[0], NT, LDS_BYTES) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per <= 0)
      return -1;
    n = per * cus;
  }
  if (per_cu) *per_cu = per;
  return n;
}

hipError_t lenet_bwd(const XSrc& x, const bf16_t* p1, const bf16_t* dp2, const uint8_t* arg2, const bf16_t* w2,
                     int B, float* slab1, float* slab2, int grid, hipStream_t st, unsigned long long* prof) {
  if (B <= 0) return hipSuccess;
  if ((!x.x && !x.u8) || grid <= 0) return hipErrorInvalidValue;
  const int res = lenet_bwd_grid();
  if (res <= 0) return hipErrorInvalidValue;
  BwdArgs a{x.u8 ? nullptr : x.x, x.u8, x.idx, x.idx ? x.n : B, p1, dp2, arg2, w2, B, slab1, slab2, prof, 0, 0,
            {}, {}, {}, {}, {}};
  static const BwdSplit sp = bwd_split();
  if (!sp.ok) return hipErrorInvalidValue;
  memcpy(a.du, sp.du, 16);
  memcpy(a.k20, sp.k20, 16);
  memcpy(a.k21, sp.k21, 16);
  memcpy(a.k10, sp.k10, 8);
  memcpy(a.k11, sp.k11, 8);
  if (prof) {   // experiments only: skip bits 1 dgrad, 2 conv2 wgrad, 4 conv1 wgrad, 8 staging, 16 loop
                // barriers, 32 pool1 / code loads; MNISTX_BWD_PROF_WAVES=1: per-wave sums too
                // (the prof buffer then holds NPROF + NW * NPROF entries)
    const char* e = getenv("MNISTX_BWD_SKIP");
    a.skip = e ? atoi(e) : 0;
    const char* pw = getenv("MNISTX_BWD_PROF_WAVES");
    a.prof_waves = (pw && pw[0] == '1') ? 1 : 0;
  }
  const BwdKernel k = kBwd[(prof ? 4 : 0) + (x.u8 ? 2 : 0) + (x.idx ? 1 : 0)];
  void* args[] = {&a};
  return hipLaunchKernel((const void*)k, dim3(grid), dim3(NT), args, LDS_BYTES, st);
}

// one block per CU (capped by the tile count), less the reserved CUs; the executor sizes the
// slabs with it at construction and launches min(that, this) per step
int lenet_bwd_blocks(int B) {
  int per = 1;
  const int full = lenet_bwd_grid(&per);
  if (full <= 0) return -1;
  const int res = reserve_cut(full, per);
  const int ntiles = (B + T - 1) / T;
  return cap_grid(ntiles < res ? ntiles : res);
}

}  // namespace mnistx
