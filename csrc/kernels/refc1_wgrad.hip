// Reference-CNN conv1 weight gradient with the norm1 backward folded in, gfx950 (bf16).
//
// conv1 (5x5 SAME, 28x28x1 -> 32) -> ReLU -> pool1 (2x2/2) -> norm1 (LRN, radius 4):
// /root/reference/mnist_input.py:142-151, differentiated by compute_gradients (:262).  Per
// 2-image tile the kernel
//   1. applies the LRN backward to dL/d norm1 (with the pool1 activations, lrn_bwd8: the
//      same arithmetic and bf16 rounding as lrn_bwd_k) and keeps dP1 = dL/d pool1 in LDS,
//      with the pool argmax codes (one u16 per channel; 4 = ReLU output 0);
//   2. accumulates dW1 as the pool-window-phase GEMM of lenet_bwd.hip's conv1 part:
//      C[(ty, tx)][(c, d)] = sum over windows w of X[2yp + ty - 2][2xp + tx - 2] *
//      dP1[w][c] [code(w, c) == d], folded to dW1[dy][dx][c] = sum_d C[(dy + a, dx + b)][(c, d)]
//      at the end (d = 2a + b; tx taken by window x parity: two accumulator sets).
// Warp-specialised pipeline (one block of 16 waves per CU, persistent): waves 0-7 stage tile
// k (LRN backward, VALU) into one LDS buffer while waves 8-15 run tile k-1's GEMM (MFMA) from
// the other, one barrier per tile.  Measured at B = 16384 (bench/micro_refc1.py skip bits,
// profiles/r4/refcnn/micro_refc1_v*.txt): 152 us (the serial 4-image-tile version: 155-167).
// Without the LRN math and the GEMM it is 89 us -- the 0.54 GB of operands at ~6 TB/s, the
// floor -- and the LRN backward (~200 VALU + 16 transcendental + 16 DPP instructions per 8
// channels) and the GEMM are not fully hidden behind the loads (115 us without the GEMM).
// The bias moved off the producers (below) took 167 -> 152 us.
// Every product is a v_mfma_f32_16x16x32_bf16 on ds_read_b64_tr_b16 fragments.  A k-step is
// one window-row pair of one parity set: K row 8g + 4rho + q = (window 4(g>>1) + (g&1) +
// 2rho of the set, row 2r + (q >> 1), image q & 1), so a lane address is a per-lane base
// plus a uniform step, and with the strides below every read is bank-conflict-free
// (bench/lds_refc1.py).  Consumer wave w owns parity set w & 1 and channel group w >> 1 (8
// channels x 4 window positions = 2 N tiles) over all 7 row pairs.  The conv1 bias gradient
// is the sum of the active windows' dP1 (an all-ones A fragment on the consumers).  One
// deterministic split-K slab [grid][48][32] per launch in convpool_wgrad's layout (rows
// kh * 8 + kw, bias 40), so the executor's splitk_reduce is the same.
//
// Replaces convpool_wgrad_k<RefC1g> with its LRN fold (259.9 us at B = 16384, 6.8 % MFMA
// busy, VALU/MFMA 37.5: profiles/r4/refcnn/).
//
// CIN = 3 (the reference's own 3-channel DLI records, mnist_input.py:13-15,134): the same
// kernel with the input staged as 3 channel planes (de-interleaved from NHWC while staging)
// and the consumers' GEMM run once per plane against the SAME masked dP1 fragments -- the
// LRN backward, the expensive part, is shared by the 3 planes.  Slab [grid][80][32] in
// convpool_wgrad's Geo<3, 32, ...> layout (rows tap * 3 + ci, bias 75).  Replaces
// convpool_wgrad_k<Geo<ci3,...>> with its LRN fold (511 us at B = 16384, profiles/r5/ref3/).
#include "common.h"
#include "launchers.h"
#include "lrn_math.h"
#include "wgrad_tr.h"

#include <cstdlib>

namespace mnistx {
namespace {

constexpr int NT = 1024, NW = 16, NPW = 8, NPT = 64 * NPW, T = 2, C = 32, NWIN = 196;
// ---- LDS layout (bytes), two buffers
constexpr int X_RS = 96, X_IMG = 3192;                      // input [img][row -2..29][col -4..35] bf16
constexpr int D_RS = 1040, D_IMG = 14560;                   // dP1 / codes [img][14][16 windows][32] x 2 B
// per input-channel count: the input planes [img][ci] come first in each buffer
template <int CIN>
struct Lay {
  static constexpr int X_OFF = 0, DP1_OFF = T * CIN * X_IMG, CD_OFF = DP1_OFF + T * D_IMG;
  static constexpr int BUF = CD_OFF + T * D_IMG;             // one buffer
  static constexpr int LDS_BYTES = 2 * BUF;
  // slab rows = convpool_wgrad's layout for the geometry (splitk_reduce as for it): CIN 1
  // (RefC1g): kh * 8 + kw, bias 40; CIN 3: (kh * 5 + kw) * 3 + ci, bias 75
  static constexpr int SLAB_ROWS = CIN == 1 ? 48 : 80, BIAS_ROW = CIN == 1 ? 40 : 75;
  static_assert(32 * X_RS <= X_IMG && 14 * D_RS <= D_IMG && 16 * 64 <= D_RS && LDS_BYTES <= 163840, "");
  static_assert(BUF % 16 == 0 && DP1_OFF % 16 == 0, "");
  static_assert(NPW * CIN * 6 * 256 * 4 + NPW * 16 * 4 <= LDS_BYTES, "epilogue scratch");
};
constexpr int NTASK = T * NWIN * 4;                        // LRN tasks per tile: (window, 8 channels)
constexpr int PER = (NTASK + NPT - 1) / NPT;                // 4 rounds over the 512 producer lanes
static_assert((NTASK - (PER - 1) * NPT) % 16 == 0, "the partial round covers whole DPP rows");
static_assert(T * NWIN <= NPT, "one input quad per producer lane");

struct Args {
  const bf16_t* x;        // input images [n][784] bf16 (or null with u8)
  const uint8_t* u8;      // input images [n][784] uint8, normalised while staging (or null)
  const int64_t* idx;     // per-sample row of x / u8 (null: sample b is row b)
  int n;
  const bf16_t* dn;       // dL/d norm1 [B][196][32]
  const bf16_t* p1;       // pool1 = the LRN input [B][196][32]
  const uint8_t* arg;     // pool1 argmax codes [B][196][32] (4 = ReLU output 0)
  int B;
  float bias, alpha, beta;
  float* slab;            // [grid][48][32]
  int skip;               // experiments only (refc1_set_skip): 1 no GEMM, 2 no LRN math, 4 no next-tile loads
};

// producer registers of one tile: LRN task vectors (dL/d norm1, pool1, codes) and the input
template <bool U8, bool IDX, int CIN, bool PK3 = false>
struct Stage {
  using L = Lay<CIN>;
  u32x4 y[PER], p[PER];
  u32x2 a[PER];
  u32x2 x[CIN];           // one 4-pixel quad per lane: image t / 196, quad t % 196 (t < 392);
                          // CIN 3: the quad's 12 interleaved values (NHWC), 3 x 8 bytes
  u32x2 rowv;             // IDX: the batch-index entry of that image, one tile ahead

  static DEV int img_of(int t) { return (t * 669) >> 17; }   // t / 196 for t < 1024
  DEV void load_row(const Args& g, int t0, int t) {
    if constexpr (IDX) {
      const int img = img_of(t);
      const bool ok = t < T * NWIN && t0 >= 0 && t0 + img < g.B;
      rowv = buf_b64(buf_rsrc(g.idx, (uint32_t)g.B * 8u), ok ? (uint32_t)(t0 + img) * 8u : BUF_OOB);
    }
  }
  struct Rsrc {
    __amdgpu_buffer_rsrc_t y, p, a;
  };
  DEV Rsrc rsrc(const Args& g, int t0) const {
    const int nimg = t0 < 0 ? 0 : min(T, g.B - t0);
    const int tb = t0 < 0 ? 0 : t0;
    const uint32_t nb = (uint32_t)nimg * NWIN * C * 2u;
    return Rsrc{buf_rsrc(g.dn + (int64_t)tb * NWIN * C, nb), buf_rsrc(g.p1 + (int64_t)tb * NWIN * C, nb),
                buf_rsrc(g.arg + (int64_t)tb * NWIN * C, nb / 2u)};
  }
  // every producer lane issues the same loads (out of range: no memory access, zeros), so
  // the load count per tile is fixed and the compiler's vmcnt waits stay exact
  DEV void load_u(const Rsrc& r, int u, int t) {
    const int e = t + u * NPT;
    const uint32_t ok = e < NTASK ? 0u : BUF_OOB;
    y[u] = buf_b128(r.y, 16u * e + ok);
    p[u] = buf_b128(r.p, 16u * e + ok);
    a[u] = buf_b64(r.a, 8u * e + ok);
  }
  DEV void load_x(const Args& g, int t0, int t) {
    const int img = img_of(t), q = t - NWIN * img;
    const bool ok = t < T * NWIN && t0 >= 0 && t0 + img < g.B;
    constexpr uint32_t esz = U8 ? 1u : 2u;
    const void* base = U8 ? (const void*)g.u8 : (const void*)g.x;
    uint32_t off;
    if constexpr (IDX) {   // the dataset (< 2 GB, binding check) through the batch index
      const uint32_t lo = rowv[0], hi = rowv[1];
      const int row = (hi != 0u || (int)lo < 0) ? 0 : ((int)lo >= g.n ? g.n - 1 : (int)lo);
      off = ((uint32_t)row * 196u + (uint32_t)q) * 4u * esz;
    } else {
      off = ((uint32_t)(ok ? t0 + img : 0) * 196u + (uint32_t)q) * 4u * esz;
    }
    const auto rx = buf_rsrc(base, 0x7fffffffu);
    if constexpr (CIN == 3) {   // bf16 NHWC: the batch (x0) or, IDX, the dataset rows; 24 bytes per quad
      if constexpr (IDX) {
        const uint32_t lo = rowv[0], hi = rowv[1];
        const int row = (hi != 0u || (int)lo < 0) ? 0 : ((int)lo >= g.n ? g.n - 1 : (int)lo);
        off = ok ? ((uint32_t)row * 196u + (uint32_t)q) * 24u : BUF_OOB;
      } else {
        off = ok ? ((uint32_t)(t0 + img) * 196u + (uint32_t)q) * 24u : BUF_OOB;
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) x[c] = buf_b64(rx, off + 8u * c);
      return;
    }
    if (!ok) off = BUF_OOB;
    if constexpr (U8) x[0] = u32x2{buf_b32(rx, off), 0u};
    else x[0] = buf_b64(rx, off);
  }
  // (the same issue order as store_load's: the waitcnt pass merges the two at the loop head)
  DEV void load(const Args& g, int t0, int t) {
    load_x(g, t0, t);
    __builtin_amdgcn_sched_barrier(0);
    const Rsrc r = rsrc(g, t0);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      load_u(r, u, t);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  DEV void store_x(uint8_t* buf, int t) {
    if (t < T * NWIN) {
      const int img = img_of(t), q = t - NWIN * img, yy = (q * 147) >> 10, k = q - 7 * yy;
      uint8_t* dst = buf + L::X_OFF + img * CIN * X_IMG + (yy + 2) * X_RS + (4 * k + 4) * 2;
      if constexpr (CIN == 3) {
        // words w0..w5 hold values e = 3 * pixel + ci (e in word e >> 1, half e & 1): plane ci
        // gets e = ci, ci + 3, ci + 6, ci + 9
        const uint32_t w0 = x[0][0], w1 = x[0][1], w2 = x[1][0], w3 = x[1][1], w4 = x[2][0], w5 = x[2][1];
        auto lo_hi = [](uint32_t a, uint32_t b) { return (a & 0xffffu) | (b & 0xffff0000u); };   // a.lo, b.hi
        auto hi_lo = [](uint32_t a, uint32_t b) { return (a >> 16) | (b << 16); };               // a.hi, b.lo
        auto lo_lo = [](uint32_t a, uint32_t b) { return (a & 0xffffu) | (b << 16); };           // a.lo, b.lo
        auto hi_hi = [](uint32_t a, uint32_t b) { return (a >> 16) | (b & 0xffff0000u); };       // a.hi, b.hi
        *(u32x2*)(dst) = u32x2{lo_hi(w0, w1), lo_hi(w3, w4)};                 // e 0, 3 | 6, 9
        *(u32x2*)(dst + X_IMG) = u32x2{hi_lo(w0, w2), hi_lo(w3, w5)};         // e 1, 4 | 7, 10
        *(u32x2*)(dst + 2 * X_IMG) = u32x2{lo_hi(w1, w2), lo_hi(w4, w5)};     // e 2, 5 | 8, 11
        (void)lo_lo;
        (void)hi_hi;
      } else {
        uint32_t lo = x[0][0], hi = x[0][1];
        if constexpr (U8) {
          const uint32_t b = x[0][0];
          lo = pack2(u8_norm(b & 0xff), u8_norm((b >> 8) & 0xff));
          hi = pack2(u8_norm((b >> 16) & 0xff), u8_norm(b >> 24));
        }
        *(u32x2*)dst = u32x2{lo, hi};
      }
    }
  }
  // This tile into LDS buffer `buf` -- the input, then per round the LRN backward -> dP1
  // (bf16) and the codes (u16), with the bias sums of the active windows -- each part's
  // registers refilled with the next tile's data right after use.
  // LDS offset of round u's task (the same every tile; -1: no task)
  static DEV int task_off(int t, int u) {
    const int e = t + u * NPT;
    if (e >= NTASK) return -1;
    const int px = e >> 2, cg = e & 3, img = px / NWIN, w = px - img * NWIN, yp = w / 14, xp = w - 14 * yp;
    return img * D_IMG + yp * D_RS + xp * 64 + 16 * cg;
  }
  DEV void store_load(uint8_t* buf, const Args& g, int t_next, int t, const int (&off)[PER]) {
    if (g.skip & 4) t_next = -1;
    store_x(buf, t);
    load_x(g, t_next, t);
    const Rsrc r = rsrc(g, t_next);
    // rounds in pairs: the LRN backward of rounds u and u + 1 as one packed (v_pk) computation
    // (bitwise lrn_bwd8; the last round's lanes past the partial round compute on whatever
    // their registers hold and store nothing -- whole DPP rows either way)
    // (CIN 3 without PK3: one round at a time -- the pairs spill 20 bytes beside the 3 input planes)
    static_assert(PER % 2 == 0, "round pairs");
    if constexpr (CIN == 3 && !PK3) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        if (u < PER - 1 || t < NTASK - (PER - 1) * NPT) {   // whole DPP rows (lrn_bwd8's exchanges)
          const u32x4 d = (g.skip & 2) ? y[u] : lrn_bwd8<4, 4, true>(p[u], y[u], t & 3, g.bias, g.alpha, g.beta, 0);
          const uint32_t a0 = a[u][0], a1 = a[u][1];
          if (off[u] >= 0) {
            *(u32x4*)(buf + L::DP1_OFF + off[u]) = d;
            *(u32x4*)(buf + L::CD_OFF + off[u]) = u32x4{bytes01(a0), bytes23(a0), bytes01(a1), bytes23(a1)};
          }
        }
        load_u(r, u, t);
        __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < PER; u += 2) {
      u32x4 d0 = y[u], d1 = y[u + 1];
      if (!(g.skip & 2))
        lrn_bwd8x2_b075<4, 4>(p[u], y[u], p[u + 1], y[u + 1], t & 3, g.bias, g.alpha, g.beta, 0, d0, d1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int uu = u + h;
        const uint32_t a0 = a[uu][0], a1 = a[uu][1];
        if ((uu < PER - 1 || t < NTASK - (PER - 1) * NPT) && off[uu] >= 0) {
          *(u32x4*)(buf + L::DP1_OFF + off[uu]) = h ? d1 : d0;
          *(u32x4*)(buf + L::CD_OFF + off[uu]) = u32x4{bytes01(a0), bytes23(a0), bytes01(a1), bytes23(a1)};
        }
        load_u(r, uu, t);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
};

// one tile's GEMM (consumer wave w = parity set w & 1, channel group w >> 1) from `buf`
// The conv1 bias gradient (the active windows' dP1 summed) rides along as a product with an
// all-ones A fragment: every row of accb[nt] is sum_k B[k][n], so sum_d [code == d] dP1 over
// the tile -- two more MFMAs per k-step on the (hidden) consumer side instead of ~30 VALU
// per LRN task on the producers.
template <int CIN>
DEV void gemm_tile(const uint8_t* buf, int w, f32x4 (&acc)[CIN][3][2], f32x4 (&accb)[2]) {
  using L = Lay<CIN>;
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
  const int sig = w & 1, cg = w >> 1;
  const int ln = lane_now(), gg = ln >> 4, q = (ln >> 2) & 3, p = ln & 3;
  const int hA = p >> 1, pc = p & 1, xil = 4 * (gg >> 1) + (gg & 1), yr = q >> 1, im = q & 1;
  const uint32_t dsel = (uint32_t)((ln & 15) >> 3);
  const uint32_t dd0 = dsel * 0x00010001u, dd1 = (2u + dsel) * 0x00010001u;
  const int aB = L::X_OFF + im * CIN * X_IMG + (2 * yr + hA) * X_RS + (4 * xil + 4 * pc + 4 * sig) * 2;
  const int bB = L::DP1_OFF + im * D_IMG + yr * D_RS + (2 * xil + sig) * 64 + 16 * cg + 8 * pc;
#pragma unroll 2
  for (int r = 0; r < 7; ++r) {
    const int sa = aB + 4 * r * X_RS, sb = bB + 2 * r * D_RS;
    const u32x4 dv = __builtin_bit_cast(u32x4, frag(tr4(buf, sb), tr4(buf, sb + 256)));
    const u32x4 cv = __builtin_bit_cast(u32x4, frag(tr4(buf, sb + (L::CD_OFF - L::DP1_OFF)),
                                                     tr4(buf, sb + (L::CD_OFF - L::DP1_OFF) + 256)));
    const bf16x8 B0 = __builtin_bit_cast(bf16x8, u32x4{sel_eq(dv[0], cv[0], dd0), sel_eq(dv[1], cv[1], dd0),
                                                       sel_eq(dv[2], cv[2], dd0), sel_eq(dv[3], cv[3], dd0)});
    const bf16x8 B1 = __builtin_bit_cast(bf16x8, u32x4{sel_eq(dv[0], cv[0], dd1), sel_eq(dv[1], cv[1], dd1),
                                                       sel_eq(dv[2], cv[2], dd1), sel_eq(dv[3], cv[3], dd1)});
#pragma unroll
    for (int c = 0; c < CIN; ++c)
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int sc = sa + c * X_IMG + 2 * t * X_RS;
        const bf16x8 Af = frag(tr4(buf, sc), tr4(buf, sc + 16));
        acc[c][t][0] = mfma16(Af, B0, acc[c][t][0]);
        acc[c][t][1] = mfma16(Af, B1, acc[c][t][1]);
      }
    accb[0] = mfma16(ones, B0, accb[0]);
    accb[1] = mfma16(ones, B1, accb[1]);
  }
}

template <bool U8, bool IDX, int CIN = 1, bool PK3 = false>
__global__ __launch_bounds__(NT, 1) void refc1_wgrad_k(const Args g) {
  using L = Lay<CIN>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = (g.B + T - 1) / T;
  const int nk = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  auto tile0 = [&](int k) { return k < nk ? ((int)blockIdx.x + k * (int)gridDim.x) * T : -1; };

  for (int e = tid; e < L::LDS_BYTES / 16; e += NT) *(u32x4*)(lds + 16 * e) = u32x4{0u, 0u, 0u, 0u};
  f32x4 acc[CIN][3][2], accb[2];
#pragma unroll
  for (int c = 0; c < CIN; ++c)
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[c][t][0] = acc[c][t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  accb[0] = accb[1] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (wave < NPW) {
    // ======================================================== producers: LRN backward staging
    Stage<U8, IDX, CIN, PK3> st;
    int off[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) off[u] = Stage<U8, IDX, CIN, PK3>::task_off(tid, u);
    st.load_row(g, tile0(0), tid);
    st.load(g, tile0(0), tid);
    st.load_row(g, tile0(1), tid);
    for (int k = 0; k <= nk; ++k) {
      __syncthreads();   // buffer k & 1 is no longer read by the consumers (tile k - 2)
      if (k < nk) {
        const int t = wave * 64 + lane_now();
        st.store_load(lds + (k & 1) * L::BUF, g, tile0(k + 1), t, off);
        st.load_row(g, tile0(k + 2), t);
      }
    }
  } else {
    // ======================================================== consumers: the GEMM of tile k - 1
    for (int k = 0; k <= nk; ++k) {
      __syncthreads();   // buffer (k - 1) & 1 holds tile k - 1
      if (k > 0 && !(g.skip & 1)) gemm_tile<CIN>(lds + ((k - 1) & 1) * L::BUF, wave - NPW, acc, accb);
    }
  }

  // ---- epilogue: consumer accumulators -> one slab (fixed order)
  const int i16 = lane & 15, g4 = lane >> 4;
  __syncthreads();
  float* e1 = (float*)lds;                          // [consumer w][ci][t][nt][col 16][row 16]
  float* eb = e1 + NPW * CIN * 6 * 256;             // [consumer w][col 16]: bias partials
  if (wave >= NPW) {
    const int w = wave - NPW;
#pragma unroll
    for (int c = 0; c < CIN; ++c)
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          *(f32x4*)(e1 + ((((w * CIN + c) * 3 + t) * 2 + nt) * 16 + i16) * 16 + 4 * g4) = acc[c][t][nt];
    // accb rows are all equal: row 0 (lanes 0-15, register 0) = column n's sum over K
    if (lane < 16) eb[w * 16 + lane] = accb[0][0] + accb[1][0];
  }
  __syncthreads();
  float* s = g.slab + (int64_t)blockIdx.x * L::SLAB_ROWS * C;
  for (int e = tid; e < L::SLAB_ROWS * C; e += NT) {
    const int r = e >> 5, c = e & 31, cgc = c >> 3, cl = c & 7;
    // CIN 1: r = dy * 8 + dx; CIN 3: r = (dy * 5 + dx) * 3 + ci
    const int tap = CIN == 1 ? r : r / 3, ci = CIN == 1 ? 0 : r - 3 * tap;
    const int dy = CIN == 1 ? r >> 3 : tap / 5, dx = CIN == 1 ? r & 7 : tap - 5 * dy;
    float v = 0.f;
    if (r < L::BIAS_ROW && dx < 5) {
      for (int sg = 0; sg < 2; ++sg) {
        const int w = sg + 2 * cgc;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int ty = dy + (d >> 1), tx = dx + (d & 1), txi = tx + (sg ? 0 : 2);
          const int t = ty >> 1, row = 4 * (2 * (ty & 1) + (txi >> 2)) + (txi & 3);
          const int nt = d >> 1, col = cl + 8 * (d & 1);
          v += e1[((((w * CIN + ci) * 3 + t) * 2 + nt) * 16 + col) * 16 + row];
        }
      }
    } else if (r == L::BIAS_ROW) {   // columns cl / cl + 8 = window positions d even / odd
      for (int sg = 0; sg < 2; ++sg) v += eb[(sg + 2 * cgc) * 16 + cl] + eb[(sg + 2 * cgc) * 16 + cl + 8];
    }
    s[e] = v;
  }
}

using Kern = void (*)(Args);
constexpr Kern kRefc1[4] = {refc1_wgrad_k<false, false>, refc1_wgrad_k<false, true>, refc1_wgrad_k<true, false>,
                            refc1_wgrad_k<true, true>};
// 3 channels: bf16 NHWC, the batch (x0) or the resident dataset through the batch index;
// [packed LRN pairs][idx].  The pairs spill 20 bytes at the 128-VGPR cap and still win: 190.4 vs
// 197.4 us at B = 16384 (profiles/r6/refc1pk/wg3/; MNISTX_REFC1_PK3=0: one round at a time)
constexpr Kern kRefc1x3[2][2] = {{refc1_wgrad_k<false, false, 3>, refc1_wgrad_k<false, true, 3>},
                                 {refc1_wgrad_k<false, false, 3, true>, refc1_wgrad_k<false, true, 3, true>}};
static int g_pk3 = [] { const char* e = getenv("MNISTX_REFC1_PK3"); return (e && e[0] == '0') ? 0 : 1; }();

int g_skip = 0;

}  // namespace

void refc1_set_skip(int s) { g_skip = s; }

int refc1_wgrad_grid(int* per_cu = nullptr) {
  static int n = 0, per = 0;
  if (n == 0) {
    int dev = 0, cus = 0;
    for (Kern k : kRefc1)
      if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, Lay<1>::LDS_BYTES) !=
          hipSuccess)
        return -1;
    for (const auto& ks : kRefc1x3)
      for (Kern k : ks)
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, Lay<3>::LDS_BYTES) !=
            hipSuccess)
          return -1;
    // both channel counts hold one block per CU (LDS); the grid is the same
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kRefc1x3[0][0], NT, Lay<3>::LDS_BYTES) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per <= 0)
      return -1;
    n = per * cus;
  }
  if (per_cu) *per_cu = per;
  return n;
}

int refc1_wgrad_blocks(int B) {
  int per = 1;
  const int full = refc1_wgrad_grid(&per);
  if (full <= 0) return -1;
  const int res = reserve_cut(full, per);
  const int ntiles = (B + T - 1) / T;
  return cap_grid(ntiles < res ? ntiles : res);
}

hipError_t refc1_wgrad(const XSrc& x, const bf16_t* dn, const bf16_t* p1, const uint8_t* arg, int B, float bias,
                       float alpha, float beta, float* slab, int grid, hipStream_t st, int cin) {
  if (B <= 0) return hipSuccess;
  if ((!x.x && !x.u8) || grid <= 0 || refc1_wgrad_grid() <= 0) return hipErrorInvalidValue;
  if (beta != 0.75f) return hipErrorInvalidValue;   // the lrn_bwd8 fast path (the reference's beta)
  if (cin != 1 && !(cin == 3 && x.x && !x.u8)) return hipErrorInvalidValue;
  Args a{x.u8 ? nullptr : x.x, x.u8, x.idx, x.idx ? x.n : B, dn, p1, arg, B, bias, alpha, beta, slab, g_skip};
  const Kern k = cin == 3 ? kRefc1x3[g_pk3][x.idx ? 1 : 0] : kRefc1[(x.u8 ? 2 : 0) + (x.idx ? 1 : 0)];
  void* args[] = {&a};
  return hipLaunchKernel((const void*)k, dim3(grid), dim3(NT), args, cin == 3 ? Lay<3>::LDS_BYTES : Lay<1>::LDS_BYTES,
                         st);
}

}  // namespace mnistx
