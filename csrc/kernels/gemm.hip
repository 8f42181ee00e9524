// MFMA GEMM engine for gfx950 (CDNA4) — dense layers and implicit-GEMM convolutions.
//
// One templated kernel computes C[M,N] = sum_k A(m,k) B(k,n) with bf16 operands
// on v_mfma_f32_16x16x32_bf16 (fp32 accumulate).  Operands come through
// "loaders" that produce 16-byte (8 x bf16) vectors along the operand's
// contiguous memory direction, so the same engine serves
//   * dense fwd / dgrad / wgrad      (MatLoader in either orientation)
//   * conv fwd / dgrad (implicit im2col along K, Im2colK, WFlipK)
//   * conv wgrad (im2col transposed: pixels are the reduction dim, Im2colMN)
// without materialising im2col or transposes in HBM.
//
// LDS images keep the operand in its *memory* orientation:
//   K-contiguous image  [rows = m|n][48]   -> fragment by ONE ds_read_b128
//   MN-contiguous image [BK][cols = m|n]   -> fragment by 2 x ds_read_b64_tr_b16
// The fragment k-slot order is permuted identically for A and B
// (lane group g, element j -> k = 4g + (j&3) + 16(j>>2)), which makes the
// transposed reads bank-conflict-free with an odd-multiple-of-32B row stride
// (a plain 8g+j order puts rows r and r+8 of one 32-lane half on the same banks).
// K-contiguous images are stored in that permuted order (column c' = 8g + j), so a
// lane's 8 k-slots are 16 contiguous bytes; the staging store splits each 16-byte
// global vector into two 8-byte halves.  Row stride 48 elements (6 x 16 B): every
// ds_read_b128 lane group hits 16 distinct 16-byte bank groups (bench/lds_sim.py).
//
// Staging: register double-buffered (global -> VGPR for tile t+1 while the MFMAs
// of tile t run from LDS), one barrier per K step; split-K over blockIdx.y for
// the huge-K weight-gradient reductions (deterministic fp32 slabs, reduced by
// splitk_reduce in misc.hip).  Tiles are mapped XCD-aware (common.h).
//
// Replaces the reference's TF Conv2D / Conv2DBackprop* / MatMul kernels
// (call sites mnist_input.py:142,161,184,192,205).
#include "common.h"
#include "launchers.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace mnistx {
namespace {

constexpr int BK = 32;
// K rows staged per step by the weight-gradient GEMMs (both operands MN-contiguous,
// split-K).  128 was measured SLOWER on every wgrad shape (LeNet fc3/fc4/fc5 at
// B=65536: bench/micro_wgrad.py; reference conv2 wgrad 1.50 -> 1.74 ms): the 80 KB+
// LDS images halve the resident blocks.  The knob stays for future tiles.
constexpr int BK_WG = 32;
// K steps kept in flight (VGPR prefetch slots) by the weight-gradient GEMMs.
constexpr int WG_PF_DENSE = 4;
constexpr int WG_PF_IM2COL = 2;
template <bool AKC, bool BKC>
constexpr int kstep() { return (!AKC && !BKC) ? BK_WG : BK; }

// Row stride (elements) of an LDS image whose contiguous extent is COLS.
template <int COLS, bool KC, bool PAD48 = true>
struct ImgStride {
  static_assert(!KC || COLS == 32, "K-contiguous images assume BK = 32");
  // K-contiguous: 48 = conflict-free ds_read_b128.  Implicit-im2col tiles are bound
  // by their loader's index math and need the occupancy more: 40 (2-way reads).
  static constexpr int value = KC ? (PAD48 ? 48 : 40) : (((COLS / 16) % 2 == 0) ? COLS + 16 : COLS);
};

// permuted column of k (0 <= k < 32) inside a K-contiguous image row
constexpr int kc_col(int k) { return 8 * ((k & 15) >> 2) + (k & 3) + 4 * (k >> 4); }

// ---------------------------------------------------------------- loaders
// load(r, c): 8 bf16 at memory coordinates (row r, cols c..c+7); zero outside.

// Branch-free vector loads.  A loader whose result passes through a
// data-dependent select or a per-lane branch (zero-fill, the bias ones-column)
// makes the compiler wait for the load right there (s_waitcnt vmcnt(0) at the
// join), which serialises the K-step prefetch -- every weight-gradient GEMM was
// latency-bound on exactly that.  The vector loaders (V = true) issue ONE
// unconditional buffer_load_dwordx4 per vector: an out-of-range element gets a
// byte offset past the descriptor's num_records and the hardware returns zeros
// without touching memory (a shared zero vector in HBM would funnel every padded
// load onto one L2 channel).  The bias ones-column is OR-ed in by fix() at LDS
// store time, where the value is waited for anyway.
constexpr uint32_t OOB_OFF = 0x80000000u;   // > every num_records (vec_ok: < 2 GB)
DEV __amdgpu_buffer_rsrc_t rsrc_of(const void* base, int64_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
}
DEV u32x4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
constexpr int64_t VEC_MAX_BYTES = (int64_t)1 << 31;

template <bool V>
struct MatLoaderT {
  const bf16_t* p;
  int R, C, ld;
  int ones_col;  // virtual column holding 1.0 (bias-gradient row), -1 = none
  // whole 16-byte vectors; the ones column (if any) starts the vector past C
  __host__ __device__ bool vec_ok() const {
    return ((ld | C) & 7) == 0 && (ones_col < 0 || ones_col == C) && (int64_t)R * ld * 2 < VEC_MAX_BYTES;
  }
  DEV u32x4 load(int r, int c) const {
    if constexpr (V) {
      const bool in = r < R && c < C;
      return bload(rsrc_of(p, (int64_t)R * ld * 2), in ? (uint32_t)(r * ld + c) * 2u : OOB_OFF);
    } else {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (r >= R) return v;
      const bf16_t* row = p + (int64_t)r * ld;
      if (c + 8 <= C && (ld & 7) == 0) {
        v = *(const u32x4*)(row + c);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c + j < C) u4_set(v, j, row[c + j]);
      }
      if (ones_col >= c && ones_col < c + 8) u4_set(v, ones_col - c, (bf16_t)0x3f80);
      return v;
    }
  }
  // vector path: the ones column is the first element of the vector at c == C
  DEV void fix(u32x4& v, int r, int c) const {
    if constexpr (V) {
      if (c == ones_col && r < R) v[0] |= 0x3f80u;
    }
  }
};
using MatLoader = MatLoaderT<false>;
using MatLoaderV = MatLoaderT<true>;
template <class L> struct IsMat : std::false_type {};
template <bool V> struct IsMat<MatLoaderT<V>> : std::true_type {};

// Implicit im2col, K-contiguous: row m = output pixel (n, oh, ow), col k = (kh, kw, ci).
template <bool V>
struct Im2colKT {
  const bf16_t* x;
  int H, W, C;          // input NHWC (C = channel stride)
  int OH, OW;           // output spatial
  int KH, KW, ph, pw;   // stride 1
  int M, K;
  FastDiv fOHW, fOW, fC, fKW;
  __host__ __device__ int64_t nbytes() const { return (int64_t)(M / (OH * OW)) * H * W * C * 2; }
  __host__ __device__ bool vec_ok() const { return (C & 7) == 0 && nbytes() < VEC_MAX_BYTES; }
  DEV u32x4 load(int m, int k) const {
    u32x4 v = {0u, 0u, 0u, 0u};
    if constexpr (V) {                     // branch-free buffer load (see bload)
      const bool ok = m < M && k < K;
      m = ok ? m : 0;
      k = ok ? k : 0;
      const int n = fOHW.div(m);
      const int rem = fOHW.mod(m, n);
      const int oh = fOW.div(rem);
      const int ow = fOW.mod(rem, oh);
      const int tap = fC.div(k);
      const int ci = fC.mod(k, tap);
      const int kh = fKW.div(tap);
      const int kw = fKW.mod(tap, kh);
      const int ih = oh - ph + kh, iw = ow - pw + kw;
      const bool in = ok && ih >= 0 && ih < H && iw >= 0 && iw < W;
      return bload(rsrc_of(x, nbytes()), in ? (uint32_t)((((n * H + ih) * W + iw) * C + ci) * 2) : OOB_OFF);
    } else {
      if (m >= M || k >= K) return v;
      const int n = fOHW.div(m);
      const int rem = fOHW.mod(m, n);
      const int oh = fOW.div(rem);
      const int ow = fOW.mod(rem, oh);
      const bf16_t* img = x + (int64_t)n * H * W * C;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = k + j;
        if (kk < K) {
          const int tap = kk / C;
          const int ci = kk - tap * C;
          const int kh = tap / KW;
          const int kw = tap - kh * KW;
          const int ih = oh - ph + kh, iw = ow - pw + kw;
          if (ih >= 0 && ih < H && iw >= 0 && iw < W) u4_set(v, j, img[((int64_t)ih * W + iw) * C + ci]);
        }
      }
      return v;
    }
  }
  DEV void fix(u32x4&, int, int) const {}
};

// Implicit im2col, MN-contiguous (conv weight gradient): row = pixel p (reduction),
// col = m = (kh, kw, ci); column Mreal is a virtual 1.0 (bias gradient).
template <bool V>
struct Im2colMNT {
  const bf16_t* x;
  int H, W, C;
  int OH, OW;
  int KH, KW, ph, pw;
  int P, Mreal;
  int ones;  // 1: append the ones column at Mreal
  FastDiv fOHW, fOW, fC, fKW;
  __host__ __device__ int64_t nbytes() const { return (int64_t)(P / (OH * OW)) * H * W * C * 2; }
  __host__ __device__ bool vec_ok() const { return ((C | Mreal) & 7) == 0 && nbytes() < VEC_MAX_BYTES; }
  DEV u32x4 load(int p, int m) const {
    u32x4 v = {0u, 0u, 0u, 0u};
    if constexpr (V) {                     // branch-free buffer load; ones column: fix()
      const bool pin = p < P, min_ = m < Mreal;
      const int pp = pin ? p : 0, mm = min_ ? m : 0;
      const int n = fOHW.div(pp);
      const int rem = fOHW.mod(pp, n);
      const int oh = fOW.div(rem);
      const int ow = fOW.mod(rem, oh);
      const int tap = fC.div(mm);
      const int ci = fC.mod(mm, tap);
      const int kh = fKW.div(tap);
      const int kw = fKW.mod(tap, kh);
      const int ih = oh - ph + kh, iw = ow - pw + kw;
      const bool in = pin && min_ && ih >= 0 && ih < H && iw >= 0 && iw < W;
      return bload(rsrc_of(x, nbytes()), in ? (uint32_t)((((n * H + ih) * W + iw) * C + ci) * 2) : OOB_OFF);
    } else {
      if (p >= P) return v;
      const int n = fOHW.div(p);
      const int rem = fOHW.mod(p, n);
      const int oh = fOW.div(rem);
      const int ow = fOW.mod(rem, oh);
      const bf16_t* img = x + (int64_t)n * H * W * C;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int mm = m + j;
        if (mm < Mreal) {
          const int tap = mm / C;
          const int ci = mm - tap * C;
          const int kh = tap / KW;
          const int kw = tap - kh * KW;
          const int ih = oh - ph + kh, iw = ow - pw + kw;
          if (ih >= 0 && ih < H && iw >= 0 && iw < W) u4_set(v, j, img[((int64_t)ih * W + iw) * C + ci]);
        }
      }
      if (ones && Mreal >= m && Mreal < m + 8) u4_set(v, Mreal - m, (bf16_t)0x3f80);
      return v;
    }
  }
  DEV void fix(u32x4& v, int p, int m) const {
    if constexpr (V) {
      if (ones && m == Mreal && p < P) v[0] |= 0x3f80u;
    }
  }
};

// Conv data-gradient B operand, K-contiguous: row = ci (fwd input channel),
// col k = (tap', co); value W[KH*KW-1-tap'][ci][co]  (180-degree filter flip).
struct WFlipK {
  const bf16_t* w;  // [T][Cin_p][Cout_p]
  int T, Cin, Cout;
  FastDiv fCout;
  __host__ __device__ bool vec_ok() const { return (int64_t)T * Cin * Cout * 2 < VEC_MAX_BYTES; }
  DEV u32x4 load(int ci, int k) const {   // branch-free buffer load (see bload)
    const bool in = ci < Cin && k < T * Cout;
    k = in ? k : 0;
    const int tp = fCout.div(k);
    const int co = fCout.mod(k, tp);
    const int tap = T - 1 - tp;
    return bload(rsrc_of(w, (int64_t)T * Cin * Cout * 2), in ? (uint32_t)(((tap * Cin + ci) * Cout + co) * 2) : OOB_OFF);
  }
  DEV void fix(u32x4&, int, int) const {}
};
using Im2colK = Im2colKT<false>;
using Im2colKV = Im2colKT<true>;
using Im2colMN = Im2colMNT<false>;
using Im2colMNV = Im2colMNT<true>;

// ---------------------------------------------------------------- fragment reads

// K-contiguous image [rows][S] in permuted column order: lane i=l&15 row r0+i,
// k-slots 4g..4g+3 and 16+4g..16+4g+3 = columns 8g..8g+7 (one 16-byte read).
template <int S>
DEV bf16x8 frag_kc(const bf16_t* img, int r0, int kb, int lane) {
  const int i = lane & 15, g = lane >> 4;
  (void)kb;
  // 48-element rows: the 16-byte blocks of odd rows are stored swapped in pairs (kc_store;
  // r0 is a multiple of 16, so the row parity is i's)
  const int gs = S == 48 ? (g ^ (i & 1)) : g;
  return __builtin_bit_cast(bf16x8, *(const u32x4*)(img + (r0 + i) * S + 8 * gs));
}

// MN-contiguous image [BK][S]: transposed read of 4-row x 16-col blocks.
template <int S>
DEV bf16x8 frag_tr(const bf16_t* img, int c0, int kb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* a0 = img + (kb + 4 * g + q) * S + c0 + 4 * p;
  const bf16_t* a1 = a0 + 16 * S;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  return join(lo, hi);
}

// ---------------------------------------------------------------- kernel
// One (tile t, K split) of C = A.B; the kernels below only choose (t, split).
template <int BM, int BN, int WM, int WN, class LA, bool AKC, class LB, bool BKC, int PFO = 0>
DEV void gemm_body(const LA& la, const LB& lb, const GemmEpi& ep, int M, int N, int K, int kchunk, int tiles_n,
                   int t, int split) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave tile too small");
  constexpr bool DENSE = IsMat<LA>::value && IsMat<LB>::value;
  constexpr int KB = kstep<AKC, BKC>();                 // rows of K staged per step
  constexpr int SA = ImgStride<AKC ? BK : BM, AKC, DENSE>::value;
  constexpr int SB = ImgStride<BKC ? BK : BN, BKC, DENSE>::value;
  constexpr int A_ELEMS = AKC ? BM * SA : KB * SA;
  constexpr int B_ELEMS = BKC ? BN * SB : KB * SB;
  constexpr int A_VEC = BM * KB / 8, B_VEC = BN * KB / 8;
  constexpr int A_VPT = (A_VEC + NT - 1) / NT, B_VPT = (B_VEC + NT - 1) / NT;

  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (A_ELEMS + B_ELEMS)];
  // buffer b of A / B (computed, not a pointer table: a local array of LDS
  // addresses is lowered as a static initializer hipcc cannot emit)
#define As(b) (smem + (b) * A_ELEMS)
#define Bs(b) (smem + 2 * A_ELEMS + (b) * B_ELEMS)

  const int tid = threadIdx.x;
  if (tid >= NT) __builtin_unreachable();   // lets hipcc drop the v < A_VEC guards when A_VEC % NT == 0
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int m0 = (t / tiles_n) * BM;
  const int n0 = (t % tiles_n) * BN;
  const int kbeg = split * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int nsteps = (kend - kbeg + KB - 1) / KB;

  // Prefetch depth (K steps in flight in VGPRs).  Weight gradients have a small
  // output, so few workgroups per CU: with one step in flight a CU keeps only
  // ~4 x 8 KB of loads outstanding and the split-K GEMMs ran at a fraction of HBM
  // bandwidth, latency-bound.  PF slots let each block keep PF steps in flight.
  constexpr int PF = PFO > 0 ? PFO : (!AKC && !BKC) ? (DENSE ? WG_PF_DENSE : WG_PF_IM2COL) : 1;
  u32x4 ra[PF][A_VPT], rb[PF][B_VPT];

  // K index past the split's end: every loader returns zeros for it (out of range)
  constexpr int KOOB = 0x3fffffff;
  // Every load is unconditional (vectors past A_VEC/B_VEC re-load a valid one and
  // are simply not stored): a load under a per-lane branch leaves the compiler's
  // vmcnt bookkeeping with two paths to merge, and it falls back to waiting for
  // everything, which serialises the prefetch.
  auto gload = [&](int slot, int k0) {
#pragma unroll
    for (int u = 0; u < A_VPT; ++u) {
      const int v = (A_VEC % NT == 0) ? tid + u * NT : (tid + u * NT) % A_VEC;
      if (AKC) {
        const int r = v / (BK / 8), c = (v % (BK / 8)) * 8;
        ra[slot][u] = la.load(m0 + r, k0 + c < kend ? k0 + c : KOOB);
      } else {
        const int r = v / (BM / 8), c = (v % (BM / 8)) * 8;
        ra[slot][u] = la.load(k0 + r < kend ? k0 + r : KOOB, m0 + c);
      }
    }
#pragma unroll
    for (int u = 0; u < B_VPT; ++u) {
      const int v = (B_VEC % NT == 0) ? tid + u * NT : (tid + u * NT) % B_VEC;
      if (BKC) {
        const int r = v / (BK / 8), c = (v % (BK / 8)) * 8;
        rb[slot][u] = lb.load(n0 + r, k0 + c < kend ? k0 + c : KOOB);
      } else {
        const int r = v / (BN / 8), c = (v % (BN / 8)) * 8;
        rb[slot][u] = lb.load(k0 + r < kend ? k0 + r : KOOB, n0 + c);
      }
    }
  };
  // K-contiguous: the 8 k of a vector land in two 4-column runs of the permuted order
  // With 48-element rows the 4 rows x 4 vectors of a 16-lane store group hit every bank twice
  // (2-way; the staging stores were most of the 25-33 % LDS bank-conflict cycles of the
  // large dense GEMMs, profiles/r4/refcnn/pmc_refcnn_b16384_before.md): odd rows swap their
  // 16-byte blocks in pairs, which makes the stores conflict-free and keeps the fragment
  // reads (frag_kc) conflict-free (bench/lds_gemm_kc.py).
  auto kc_store = [&](bf16_t* img, int S, int v, const u32x4& x) {
    const int r = v / (BK / 8), vq = v % (BK / 8);
    bf16_t* row = img + r * S;
    // the stores split into two ds_write_b64 (a ds_write2_b64 needs one offset pair for all
    // lanes); swapping the data instead keeps the pair but measured slower (the selects)
    const int sw = S == 48 ? ((r & 1) << 3) : 0;
    *(u32x2*)(row + (kc_col(8 * vq) ^ sw)) = u32x2{x[0], x[1]};
    *(u32x2*)(row + (kc_col(8 * vq + 4) ^ sw)) = u32x2{x[2], x[3]};
  };
  // fix(): loader post-processing of a waited-for vector (the bias ones column)
  auto sstore = [&](int slot, int buf, int k0) {
#pragma unroll
    for (int u = 0; u < A_VPT; ++u) {
      const int v = tid + u * NT;
      if (v < A_VEC) {
        u32x4 x = ra[slot][u];
        if (AKC) {
          const int r = v / (BK / 8), c = (v % (BK / 8)) * 8;
          la.fix(x, m0 + r, k0 + c < kend ? k0 + c : KOOB);
          kc_store(As(buf), SA, v, x);
        } else {
          const int r = v / (BM / 8), c = (v % (BM / 8)) * 8;
          la.fix(x, k0 + r < kend ? k0 + r : KOOB, m0 + c);
          *(u32x4*)(As(buf) + r * SA + c) = x;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < B_VPT; ++u) {
      const int v = tid + u * NT;
      if (v < B_VEC) {
        u32x4 x = rb[slot][u];
        if (BKC) {
          const int r = v / (BK / 8), c = (v % (BK / 8)) * 8;
          lb.fix(x, n0 + r, k0 + c < kend ? k0 + c : KOOB);
          kc_store(Bs(buf), SB, v, x);
        } else {
          const int r = v / (BN / 8), c = (v % (BN / 8)) * 8;
          lb.fix(x, k0 + r < kend ? k0 + r : KOOB, n0 + c);
          *(u32x4*)(Bs(buf) + r * SB + c) = x;
        }
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsteps > 0) {
    // Steps are padded to a multiple of PF (the pad steps read zeros: KOOB) so the
    // loop body has no data-dependent exits; loads and LDS stores are issued
    // unconditionally, which keeps hipcc's vmcnt waits counted (it waits only for
    // the slot it is about to store, not for the loads just issued).
    const int nsp = (nsteps + PF - 1) / PF * PF;
    // slots 0..PF-1 <- steps 0..PF-1; step 0 -> LDS buffer 0
#pragma unroll
    for (int p = 0; p < PF; ++p) gload(p, kbeg + p * KB);
    sstore(0, 0, kbeg);
    __syncthreads();
    // step s = s0 + p lives in slot p (statically indexed: the loop is unrolled by PF).
    // Its slot was drained into LDS at the end of step s-1, so the load of step
    // s + PF reuses it before step s computes.
    for (int s0 = 0; s0 < nsp; s0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const int s = s0 + p;
        const int cur = s & 1;
        gload(p, kbeg + (s + PF) * KB);   // past the end: zeros (KOOB), never stored
#pragma unroll
        for (int kb = 0; kb < KB; kb += BK) {
          bf16x8 af[FM], bfr[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const int r0 = wm * TM + i * 16;
            af[i] = AKC ? frag_kc<SA>(As(cur), r0, kb, lane) : frag_tr<SA>(As(cur), r0, kb, lane);
          }
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int c0 = wn * TN + j * 16;
            bfr[j] = BKC ? frag_kc<SB>(Bs(cur), c0, kb, lane) : frag_tr<SB>(Bs(cur), c0, kb, lane);
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        sstore((p + 1) % PF, cur ^ 1, kbeg + (s + 1) * KB);
        __syncthreads();
      }
    }
  }

#undef As
#undef Bs
  // ---- epilogue.  Vector path (N, ldc, ldm multiples of 8): each wave stages a
  // 16 x TN block of its accumulators in LDS, then every lane owns 8 consecutive
  // columns of one row: bias / ReLU / mask on 8 values, one 16-byte bf16 store
  // (or 2 x 16-byte fp32 stores) instead of eight 2-byte stores.
  const int g = lane >> 4, li = lane & 15;
  const bool vec = (N % 8 == 0) && (ep.ldc % 8 == 0) && ((uintptr_t)ep.out % 16 == 0) &&
                   (ep.mask == nullptr || (ep.ldm % 8 == 0 && (uintptr_t)ep.mask % 16 == 0));
  if (vec) {
    constexpr int EP_LD = TN + 4;
    constexpr int VI = (16 * (TN / 8) + 63) / 64;   // 8-column vectors per lane per fragment row
    static_assert((NT / 64) * 16 * EP_LD * 4 <= 2 * (A_ELEMS + B_ELEMS) * 2, "epilogue staging must fit in smem");
    float* eb = (float*)smem + wave * 16 * EP_LD;
    // A lane's columns do not depend on the fragment row i: its bias values are loaded once,
    // and the mask of fragment row i + 1 is in flight while row i is staged and stored (loaded
    // inside the row loop, every wave stalled on each of the FM loads in turn).
    auto vrow = [&](int v) { return v / (TN / 8); };
    auto vcol = [&](int v) { return n0 + wn * TN + (v - vrow(v) * (TN / 8)) * 8; };
    float bv[VI][8];
#pragma unroll
    for (int k = 0; k < VI; ++k) {
      const int n = vcol(lane + 64 * k);
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[k][e] = (ep.bias && n + e < ep.bias_n) ? ep.bias[n + e] : 0.f;
    }
    auto mload = [&](int i, u32x4 (&mk)[VI]) {
#pragma unroll
      for (int k = 0; k < VI; ++k) {
        const int v = lane + 64 * k;
        const int m = m0 + wm * TM + i * 16 + vrow(v), n = vcol(v);
        const bool ok = ep.mask && v < 16 * (TN / 8) && m < M && n < N;
        mk[k] = ok ? *(const u32x4*)(ep.mask + (int64_t)m * ep.ldm + n) : u32x4{0u, 0u, 0u, 0u};
      }
    };
    u32x4 mkc[VI];
    mload(0, mkc);
    __syncthreads();   // the main loop's operand images are dead from here on
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      u32x4 mkn[VI];
      if (i + 1 < FM) mload(i + 1, mkn);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) eb[(4 * g + r) * EP_LD + j * 16 + li] = acc[i][j][r];
      // eb is this wave's own: LDS accesses of one wave complete in order, so only the
      // compiler needs fencing (no workgroup barrier)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < VI; ++k) {
        const int v = lane + 64 * k;
        const int rr = vrow(v), cv = v - rr * (TN / 8);
        const int m = m0 + wm * TM + i * 16 + rr, n = vcol(v);
        if (v < 16 * (TN / 8) && m < M && n < N) {
          f32x4 lo = *(const f32x4*)(eb + rr * EP_LD + 8 * cv), hi = *(const f32x4*)(eb + rr * EP_LD + 8 * cv + 4);
          if (ep.mode == EPI_SLAB) {
            float* o = (float*)ep.out + (int64_t)split * ep.slab_stride + (int64_t)m * ep.ldc + n;
            *(f32x4*)o = lo;
            *(f32x4*)(o + 4) = hi;
            continue;
          }
          float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] += bv[k][e];
          if (ep.relu)
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = fmaxf(x[e], 0.f);
          if (ep.mask) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (!(u4_get(mkc[k], e) > 0.f)) x[e] = 0.f;
          }
          if (ep.mode == EPI_F32) {
            float* o = (float*)ep.out + (int64_t)m * ep.ldc + n;
            *(f32x4*)o = f32x4{x[0], x[1], x[2], x[3]};
            *(f32x4*)(o + 4) = f32x4{x[4], x[5], x[6], x[7]};
          } else {
            *(u32x4*)((bf16_t*)ep.out + (int64_t)m * ep.ldc + n) =
                u32x4{pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(x[4], x[5]), pack2(x[6], x[7])};
          }
        }
      }
      // the next row's staging overwrites eb: this row's reads first (same wave: in order)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (i + 1 < FM)
#pragma unroll
        for (int k = 0; k < VI; ++k) mkc[k] = mkn[k];
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + j * 16 + li;
      if (n >= N) continue;
      float bias = 0.f;
      if (ep.bias && n < ep.bias_n) bias = ep.bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + 4 * g + r;
        if (m >= M) continue;
        float v = acc[i][j][r];
        if (ep.mode == EPI_SLAB) {
          float* o = (float*)ep.out + (int64_t)split * ep.slab_stride;
          o[(int64_t)m * ep.ldc + n] = v;
          continue;
        }
        v += bias;
        if (ep.relu) v = fmaxf(v, 0.f);
        if (ep.mask && !(bf2f(ep.mask[(int64_t)m * ep.ldm + n]) > 0.f)) v = 0.f;
        if (ep.mode == EPI_F32) ((float*)ep.out)[(int64_t)m * ep.ldc + n] = v;
        else ((bf16_t*)ep.out)[(int64_t)m * ep.ldc + n] = f2bf(v);
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, class LA, bool AKC, class LB, bool BKC, int PFO = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(LA la, LB lb, GemmEpi ep, int M, int N, int K,
                                                            int kchunk, int tiles_n) {
  const int tiles_mn = gridDim.x;
  // Split-K launches remap the whole 2-D grid: blocks are dealt round-robin over the
  // 8 XCDs by linear id, so a plain (tile, split) grid scatters the tiles of one split
  // -- which all read the same K rows of both operands -- over every XCD.  Remapped,
  // consecutive logical ids (the tiles of a split, then the next split) share one
  // XCD's L2 and each K slab is fetched from HBM about once instead of once per tile.
  int t, split;
  if (gridDim.y > 1) {
    const int lin = xcd_remap(blockIdx.y * tiles_mn + blockIdx.x, tiles_mn * gridDim.y);
    split = lin / tiles_mn;
    t = lin - split * tiles_mn;
  } else {
    t = xcd_remap(blockIdx.x, tiles_mn);
    split = 0;
  }
  gemm_body<BM, BN, WM, WN, LA, AKC, LB, BKC, PFO>(la, lb, ep, M, N, K, kchunk, tiles_n, t, split);
}

// Grouped weight gradients: up to WG_GROUP_MAX independent split-K problems in ONE
// launch (LeNet's fc3 / fc4 / fc5 run back to back otherwise, each too small to
// fill the GPU on its own and each paying a drain / ramp between kernels).  Blocks
// [start[p], start[p+1]) belong to problem p; the XCD remap keeps a problem's split
// on one L2.
constexpr int WG_GROUP_MAX = 4;
struct WgGroup {
  MatLoaderV a[WG_GROUP_MAX], b[WG_GROUP_MAX];
  GemmEpi ep[WG_GROUP_MAX];
  int M[WG_GROUP_MAX], N[WG_GROUP_MAX], K[WG_GROUP_MAX], kchunk[WG_GROUP_MAX], tiles_n[WG_GROUP_MAX],
      tiles_mn[WG_GROUP_MAX];
  int start[WG_GROUP_MAX + 1];
  int np;
};
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void gemm_wg_group_kernel(const WgGroup g) {
  // Problem ranges start at multiples of 8 blocks, so block b of problem p sits on
  // XCD b % 8 like any launch: the remap is applied WITHIN each problem (its splits
  // group on one L2) while every problem still spreads over all 8 XCDs.  Remapping
  // the whole grid instead put fc3's (heavy) blocks on 3 XCDs and fc5's on 2.
  const int b = blockIdx.x;
  int p = 0;
#pragma unroll
  for (int q = 1; q < WG_GROUP_MAX; ++q) p += (q < g.np && b >= g.start[q]) ? 1 : 0;
  p = __builtin_amdgcn_readfirstlane(p);
  const int n = g.tiles_mn[p] * ((g.K[p] + g.kchunk[p] - 1) / g.kchunk[p]);
  // bijective on the padded range: every logical block < n is produced exactly once
  const int local = xcd_remap(b - g.start[p], (n + 7) / 8 * 8);
  if (local >= n) return;                     // one of the <= 7 padding blocks
  const int split = local / g.tiles_mn[p];
  const int t = local - split * g.tiles_mn[p];
  gemm_body<BM, BN, WM, WN, MatLoaderV, false, MatLoaderV, false>(g.a[p], g.b[p], g.ep[p], g.M[p], g.N[p], g.K[p],
                                                                 g.kchunk[p], g.tiles_n[p], t, split);
}

// ---------------------------------------------------------------- dispatch
template <int BM, int BN, int WM, int WN, class LA, bool AKC, class LB, bool BKC, int PFO = 0>
hipError_t launch_cfg(const LA& la, const LB& lb, const GemmEpi& ep, int M, int N, int K, int splits,
                      hipStream_t st) {
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  if (splits < 1) splits = 1;
  int kchunk = (K + splits - 1) / splits;
  constexpr int KB = kstep<AKC, BKC>();
  kchunk = ((kchunk + KB - 1) / KB) * KB;
  splits = (K + kchunk - 1) / kchunk;
  if (splits < 1) splits = 1;
  dim3 grid(tm * tn, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, LA, AKC, LB, BKC, PFO>), grid, dim3(64 * WM * WN), 0, st, la, lb, ep,
                     M, N, K, kchunk, tn);
  return hipGetLastError();
}

// Tile choice (ops/functional.py::gemm_tile mirrors the weight-gradient rule).
//  * Weight gradients (A and B both MN-contiguous, K = batch or pixels) have a
//    small output and a huge K: small tiles give every split many workgroups,
//    so the deterministic fp32 split-K slab (splits x M x N) stays small.
//  * Everything else drops to 64-row tiles whenever the large tile would leave
//    the 256 CUs with fewer than 4 workgroups each.
enum TileCode { T256x16, T256x32, T128x64, T64x128, T128x128, T64x16, T64x32, T64x64, T256x128, T32x192, T64x192,
                T128x192 };

// 192-column tiles (reference CNN local4, N = 192): the whole output width in one column
// tile, so the M operand is read once (A/B switch set_tile192; MNISTX_TILE192=0 at load).
// local4 forward, bench/micro_local4.py: 32 x 192 20.8 us, 64 x 192 22.2, 64 x 128 22.5.
static int g_tile192 = [] { const char* e = getenv("MNISTX_TILE192"); return (e && e[0] == '0') ? 0 : 1; }();


int tile_code(int M, int N, bool wgrad) {
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  // (forward / data gradient only: the 128 x 192 weight-gradient tile measured slower than
  // 64 x 64 on local4, 31.6 vs 19.0 us, bench/micro_local4.py; it stays reachable by code)
  if (g_tile192 && !wgrad && N > 128 && N <= 192) return tiles(64, 192) >= 1024 ? T64x192 : T32x192;
  if (wgrad) {
    if (N <= 16) return T64x16;
    if (N <= 32) return T64x32;
    if (N <= 64) return T64x64;
    if (N <= 128) return M >= 256 ? T64x128 : T64x64;   // whole N per tile: M operand read once
    // 128x128 halves the operand traffic per MAC; from 128 tiles up it wins even with
    // few splits (reference local3 3137x1024xK16384: 64x64/S3 214 us -> 128x128/S2
    // 156 us incl. the split-K reduce, bench/micro_wgrad.py ref)
    if (tiles(128, 128) < 128) return T64x64;
    return T128x128;
  }
  if (N <= 16) return tiles(256, 16) >= 1024 ? T256x16 : T64x16;
  if (N <= 32) return tiles(256, 32) >= 1024 ? T256x32 : T64x32;
  if (N <= 64) return tiles(128, 64) >= 1024 ? T128x64 : T64x64;
  if (M <= 64 || tiles(128, 128) < 1024) return T64x128;
  return T128x128;
}

template <class LA, bool AKC, class LB, bool BKC>
hipError_t launch_any(const LA& la, const LB& lb, const GemmEpi& ep, int M, int N, int K, int splits,
                      hipStream_t st, int code = -1) {
  constexpr bool WG = !AKC && !BKC;
  int c = code >= 0 ? code : tile_code(M, N, WG);
  if constexpr (!WG) {
    // Large dense fwd / dgrad GEMMs (fully-connected layers at big batch): 256x128
    // tiles with 2 K-steps in flight, measured on MI355X (profiles/r1s3/gemm_sweep.md:
    // 16384x3136x1024 fwd 184 -> 151 us, dgrad 174 -> 153 us vs the 128x128 tile).
    constexpr bool DENSE = IsMat<LA>::value && IsMat<LB>::value;
    if (DENSE && code < 0 && N > 64 && M >= 4096 &&
        ((M + 255) / 256) * ((N + 127) / 128) >= 512)
      return launch_cfg<256, 128, 2, 2, LA, AKC, LB, BKC, 2>(la, lb, ep, M, N, K, splits, st);
    if (c == T256x128) return launch_cfg<256, 128, 2, 2, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
  }
  if constexpr (WG) {
    // explicit request only (bench/micro_wgrad.py): 256 x 128 weight-gradient tiles
    if (c == T256x128) return launch_cfg<256, 128, 2, 2, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
  }
  switch (c) {
    case T64x16: return launch_cfg<64, 16, 4, 1, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
    case T64x32: return launch_cfg<64, 32, 4, 1, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
    case T64x64: return launch_cfg<64, 64, 2, 2, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
    case T128x128: return launch_cfg<128, 128, 2, 2, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
    case T128x64: return launch_cfg<128, 64, 2, 2, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
    case T64x128: return launch_cfg<64, 128, 1, 4, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
    case T128x192: return launch_cfg<128, 192, 2, 2, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
    default: break;
  }
  if constexpr (!WG) {   // skinny dense outputs: 2 K steps in flight (latency-bound otherwise)
    switch (c) {
      case T32x192: return launch_cfg<32, 192, 1, 4, LA, AKC, LB, BKC, 2>(la, lb, ep, M, N, K, splits, st);
      case T64x192: return launch_cfg<64, 192, 1, 4, LA, AKC, LB, BKC, 2>(la, lb, ep, M, N, K, splits, st);
      default: break;
    }
  }
  if constexpr (!WG) {
    switch (c) {
      case T256x16: return launch_cfg<256, 16, 4, 1, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
      case T256x32: return launch_cfg<256, 32, 4, 1, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

// Vector loaders (VA/VB: same fields as LA/LB) when both operands qualify; the
// general loaders otherwise, with one fixed tile (odd shapes are not hot paths).
template <class VA, class VB, bool AKC, bool BKC, class LA, class LB>
hipError_t launch_pick(const LA& la, const LB& lb, const GemmEpi& ep, int M, int N, int K, int splits,
                       hipStream_t st, int code = -1) {
  if (la.vec_ok() && lb.vec_ok()) {
    VA va;
    VB vb;
    static_assert(sizeof(VA) == sizeof(LA) && sizeof(VB) == sizeof(LB), "vector loaders mirror the general ones");
    memcpy((void*)&va, (const void*)&la, sizeof(LA));
    memcpy((void*)&vb, (const void*)&lb, sizeof(LB));
    return launch_any<VA, AKC, VB, BKC>(va, vb, ep, M, N, K, splits, st, code);
  }
  return launch_cfg<64, 64, 2, 2, LA, AKC, LB, BKC>(la, lb, ep, M, N, K, splits, st);
}

}  // namespace

// ---------------------------------------------------------------- public launchers
void gemm_tile(int M, int N, int wgrad, int* bm, int* bn) {
  static const int BMS[] = {256, 256, 128, 64, 128, 64, 64, 64, 256, 32, 64, 128};
  static const int BNS[] = {16, 32, 64, 128, 128, 16, 32, 64, 128, 192, 192, 192};
  const int c = tile_code(M, N, wgrad != 0);
  *bm = BMS[c];
  *bn = BNS[c];
}

void set_tile192(int on) { g_tile192 = on; }

hipError_t dense_fwd(const bf16_t* x, const bf16_t* w, int M, int N, int K, int ldx, int ldw,
                     const GemmEpi& ep, hipStream_t st, int tile) {
  if (tile < 0 && gemm256_ok(M, N, K, ep)) return gemm256_fwd(x, w, M, N, K, ldx, ldw, ep, st);
  MatLoader a{x, M, K, ldx, -1};
  MatLoader b{w, K, N, ldw, -1};
  return launch_pick<MatLoaderV, MatLoaderV, true, false>(a, b, ep, M, N, K, 1, st, tile);
}

hipError_t dense_dgrad(const bf16_t* dy, const bf16_t* w, int M, int N, int K, int lddy, int ldw,
                       const GemmEpi& ep, hipStream_t st, int tile) {
  // dX[M, N=Din] = dY[M, K=Dout] . W[Din, Dout]^T  ; B(k, n) = W[n][k]  (K-contiguous rows n)
  if (tile < 0 && gemm256_ok(M, N, K, ep)) return gemm256_dgrad(dy, w, M, N, K, lddy, ldw, ep, st);
  MatLoader a{dy, M, K, lddy, -1};
  MatLoader b{w, N, K, ldw, -1};
  return launch_pick<MatLoaderV, MatLoaderV, true, true>(a, b, ep, M, N, K, 1, st, tile);
}

hipError_t dense_wgrad(const bf16_t* x, const bf16_t* dy, int Din, int Dout, int B, int ldx, int lddy,
                       int with_bias, int splits, const GemmEpi& ep, hipStream_t st, int tile, int* used) {
  // slab[Din(+1), Dout] = X^T dY ; A(m=din, k=b) = X[b][din] ; B(k=b, n) = dY[b][n]
  if (used) *used = splits;
  if (tile < 0 && used) {
    // the GEMMs that fill the GPU on 256 x 256 tiles: gemm256's own split count (one round
    // of blocks), when the caller's slab holds that many partials
    const int cus = gemm256_cus();
    const int s2 = cus > 0 ? gemm256_wgrad_splits(Din, Dout, B, with_bias, cus) : 0;
    if (s2 > 0 && s2 <= splits) {
      *used = s2;
      return gemm256_wgrad(x, dy, Din, Dout, B, ldx, lddy, with_bias, s2, ep, st);
    }
  }
  MatLoader a{x, B, Din, ldx, with_bias ? Din : -1};
  MatLoader b{dy, B, Dout, lddy, -1};
  const int M = Din + (with_bias ? 1 : 0);
  return launch_pick<MatLoaderV, MatLoaderV, false, false>(a, b, ep, M, Dout, B, splits, st, tile);
}

// Tile width of the grouped weight gradients: 128 columns cover LeNet's fc3 / fc4 outputs
// (120 / 88) in ONE column tile, so their input activations (fc3: the 52 MB pool2 at
// B = 65536) are read once instead of twice (64: profiles/r3/lenet/knobs/, slower); the
// split choice (ops/functional.py pick_splits, grouped=True) assumes the same width.
int wg_group_bn() { return 128; }

hipError_t dense_wgrad_group(int np, const bf16_t* const* x, const bf16_t* const* dy, const int* Din, const int* Dout,
                             int B, const int* ldx, const int* lddy, int* splits, const GemmEpi* ep, hipStream_t st) {
  constexpr int BM = 64;
  const int BN = wg_group_bn();
  if (np < 1 || np > WG_GROUP_MAX) return hipErrorInvalidValue;
  WgGroup g{};
  g.np = np;
  int total = 0;
  for (int p = 0; p < np; ++p) {
    MatLoader a{x[p], B, Din[p], ldx[p], Din[p]};
    MatLoader b{dy[p], B, Dout[p], lddy[p], -1};
    if (!a.vec_ok() || !b.vec_ok()) return hipErrorInvalidValue;   // callers fall back to dense_wgrad
    memcpy((void*)&g.a[p], (const void*)&a, sizeof(a));
    memcpy((void*)&g.b[p], (const void*)&b, sizeof(b));
    g.ep[p] = ep[p];
    g.M[p] = Din[p] + 1;
    g.N[p] = Dout[p];
    g.K[p] = B;
    int s = splits[p] < 1 ? 1 : splits[p];
    int kchunk = (B + s - 1) / s;
    kchunk = (kchunk + BK_WG - 1) / BK_WG * BK_WG;
    s = (B + kchunk - 1) / kchunk;
    splits[p] = s;
    g.kchunk[p] = kchunk;
    g.tiles_n[p] = (g.N[p] + BN - 1) / BN;
    g.tiles_mn[p] = ((g.M[p] + BM - 1) / BM) * g.tiles_n[p];
    g.start[p] = total;
    total += (g.tiles_mn[p] * s + 7) / 8 * 8;
  }
  g.start[np] = total;
  if (BN == 128) hipLaunchKernelGGL((gemm_wg_group_kernel<BM, 128, 1, 4>), dim3(total), dim3(256), 0, st, g);
  else hipLaunchKernelGGL((gemm_wg_group_kernel<BM, 64, 2, 2>), dim3(total), dim3(256), 0, st, g);
  return hipGetLastError();
}

// MNISTX_CONV_HALO=0 keeps the im2col GEMM for the geometries conv_halo.hip covers
bool conv_halo_enabled() {
  static const int on = [] { const char* e = getenv("MNISTX_CONV_HALO"); return (e && e[0] == '0') ? 0 : 1; }();
  return on != 0;
}
static bool halo_enabled() { return conv_halo_enabled(); }

hipError_t conv_fwd(const bf16_t* x, const bf16_t* w, int Nb, int H, int W, int C, int OH, int OW, int KH,
                    int KW, int ph, int pw, int Cout, const GemmEpi& ep, hipStream_t st, LrnParams lrn) {
  const bool halo = halo_enabled() && ep.mode == EPI_BF16 && ep.ldc == Cout && ep.mask == nullptr &&
                    conv5_halo_fwd_ok(H, W, C, OH, OW, KH, KW, ph, pw, Cout);
  if (halo) return conv5_halo_fwd(x, w, Nb, C, Cout, ep.bias, ep.bias_n, ep.relu, (bf16_t*)ep.out, st, lrn);
  if (lrn.on) return hipErrorInvalidValue;   // the LRN fold exists in the halo kernels only
  const int M = Nb * OH * OW, K = KH * KW * C;
  Im2colK a{x, H, W, C, OH, OW, KH, KW, ph, pw, M, K,
            FastDiv(OH * OW), FastDiv(OW), FastDiv(C), FastDiv(KW)};
  MatLoader b{w, K, Cout, Cout, -1};
  return launch_pick<Im2colKV, MatLoaderV, true, false>(a, b, ep, M, Cout, K, 1, st);
}

hipError_t conv_dgrad(const bf16_t* dy, const bf16_t* w, int Nb, int OH, int OW, int Cout, int H, int W,
                      int KH, int KW, int ph, int pw, int Cin, const GemmEpi& ep, hipStream_t st) {
  if (halo_enabled() && ep.mode == EPI_BF16 && ep.ldc == Cin && ep.bias == nullptr && !ep.relu &&
      (ep.mask == nullptr || ep.ldm == Cin) && conv5_halo_dgrad_ok(OH, OW, Cout, H, W, KH, KW, ph, pw, Cin))
    return conv5_halo_dgrad(dy, w, Nb, Cout, Cin, ep.mask, (bf16_t*)ep.out, st);
  // dX = conv(dY, flip(W)^T) with pad' = K-1-pad, over the dY image.
  const int M = Nb * H * W, K = KH * KW * Cout;
  Im2colK a{dy, OH, OW, Cout, H, W, KH, KW, KH - 1 - ph, KW - 1 - pw, M, K,
            FastDiv(H * W), FastDiv(W), FastDiv(Cout), FastDiv(KW)};
  WFlipK b{w, KH * KW, Cin, Cout, FastDiv(Cout)};
  return launch_pick<Im2colKV, WFlipK, true, true>(a, b, ep, M, Cin, K, 1, st);
}

hipError_t conv_wgrad(const bf16_t* x, const bf16_t* dy, int Nb, int H, int W, int C, int OH, int OW, int KH,
                      int KW, int ph, int pw, int Cout, int with_bias, int splits, const GemmEpi& ep,
                      hipStream_t st, LrnParams lrn) {
  // halo path: `splits` persistent blocks, one slab partial each (the binding sizes it)
  if (halo_enabled() && ep.mode == EPI_SLAB && ep.ldc == Cout &&
      conv5_halo_wgrad_ok(H, W, C, OH, OW, KH, KW, ph, pw, Cout, with_bias))
    return conv5_halo_wgrad(x, dy, Nb, splits, (float*)ep.out, st, lrn);
  if (lrn.on) return hipErrorInvalidValue;
  const int P = Nb * OH * OW, Mreal = KH * KW * C;
  Im2colMN a{x, H, W, C, OH, OW, KH, KW, ph, pw, P, Mreal, with_bias,
             FastDiv(OH * OW), FastDiv(OW), FastDiv(C), FastDiv(KW)};
  MatLoader b{dy, P, Cout, Cout, -1};
  return launch_pick<Im2colMNV, MatLoaderV, false, false>(a, b, ep, Mreal + (with_bias ? 1 : 0), Cout, P, splits,
                                                          st);
}

}  // namespace mnistx
