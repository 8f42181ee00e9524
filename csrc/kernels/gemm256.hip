// Large dense GEMMs on 256 x 256 tiles with LDS-DMA staging, gfx950.
//
// The reference CNN's local3 layer (/root/reference/mnist_input.py:175-184: 16384 x 3136
// -> 1024 at the BASELINE batch) is the one GEMM of the framework big enough to be bound by
// the MFMA engine itself; the register-staged 256 x 128 x 32 tiles of gemm.hip run it at
// ~0.75-0.9 PFLOP/s (MFMA busy ~33 %, profiles/r4/gemm_kc/).  This kernel is built the way
// the CDNA4 playbook's large-GEMM recipe reads (cdna_hip_programming.md §5):
//  * one 256 x 256 output tile per workgroup, 8 waves (2 along M x 4 along N), each wave
//    128 x 64 = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators;
//  * K steps of 64, staged global -> LDS by buffer_load_dwordx4 ... lds (no VGPR round trip,
//    no ds_write pass; an out-of-range 16-byte chunk reads zeros through the descriptor's
//    num_records, so tails need no branches), two LDS buffers (2 x 64 KB): the DMA of step
//    t + 1 runs under the MFMAs of step t, one vmcnt(0) + barrier per step;
//  * the LDS images are lane-linear (the DMA writes base + 16 lane), so the bank swizzle
//    is applied to the per-lane GLOBAL source chunk and undone on the read (rule 21):
//      K-contiguous operand  [256 rows][64 k]  (128 B rows): chunk c of row r at c ^ ((r >> 1) & 7)
//                                              -> every ds_read_b128 lane group conflict-free
//      MN-contiguous operand [64 k][256 cols]  (512 B rows): chunk c of row r at c ^ f(r),
//                            f(r) = 2 (r & 1) + 4 ((r >> 1) & 1) + 8 ((r >> 3) & 1)
//                                              -> every ds_read_b64_tr_b16 half-wave conflict-free
//    (both searched exhaustively over XOR-of-row-bit swizzles with the gfx950 lane-group
//    tables, bench/lds_gemm256.py);
//  * fragments in natural k order (lane l: k = 8 (l >> 4) + j), read by one ds_read_b128
//    (K-contiguous) or two ds_read_b64_tr_b16 (MN-contiguous) per fragment;
//  * XCD-aware tile order (the column tiles of one row panel share an L2);
//  * the epilogue of gemm.hip: bias / ReLU / ReLU-backward mask, bf16 or fp32 out, 16-byte
//    stores staged through LDS per wave.
// Operand orientations: forward (x K-contiguous, W [K][N] MN-contiguous) and data gradient
// (dY and W both K-contiguous).  The weight gradient stays on gemm.hip's split-K engine.
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace mnistx {
namespace {

constexpr int BM = 256, BN = 256, NTH = 512;
constexpr int WM = 2, WN = 4, TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
constexpr int LDS_BYTES = 128 * 1024;      // every stage ring: one workgroup per CU
static_assert(BM == BN, "one image size for both operands");

// K-step geometry.  BK = 64: two 64 KB stages (DMA of step t + 1 under the MFMAs of step t,
// vmcnt(0) each step).  BK = 32: four 32 KB stages, three steps of DMA in flight, each step
// waits only for its own stage (counted vmcnt), so an HBM miss has ~3 steps of MFMAs to land.
template <int BK>
struct Geo {
  static constexpr int IMG = BM * BK * 2;            // bytes of one operand image
  static constexpr int BUF = 2 * IMG;                // one stage: A image then B image
  static constexpr int STAGES = LDS_BYTES / BUF;
  static constexpr int NI = IMG / 1024 / 8;          // 1 KB DMA instructions per wave per image
  static constexpr int DPS = 2 * NI;                 // ... per stage (A + B)
  static constexpr int KC_RB = 2 * BK;               // K-contiguous image row bytes
  static constexpr int KC_RPI = 1024 / KC_RB;        // K-contiguous rows per DMA instruction
  static_assert(STAGES * BUF == LDS_BYTES && (BK == 32 || BK == 64), "");
};

// Bank swizzles (16-byte chunk XOR per row), bench/lds_gemm256.py:
//   K-contiguous, 128-byte rows (BK 64): c ^ ((r >> 1) & 7); 64-byte rows (BK 32): c ^ (2 ((r >> 3) & 1))
//   MN-contiguous, 512-byte rows: c ^ f(r)
template <int BK>
DEV int kc_swz(int r) { return BK == 64 ? (r >> 1) & 7 : ((r >> 3) & 1) << 1; }
DEV int mn_swz(int r) { return ((r & 1) << 1) | (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3); }

typedef __attribute__((address_space(3))) void lds_void;

// One operand: KC = K-contiguous rows [R][K] (ld >= K), else MN-contiguous [K][R] (ld >= R).
struct Opnd {
  const bf16_t* p;
  int ld, R, K;
  uint32_t nbytes;
};

// Block -> (tile, K split) schedule.  Data / forward GEMMs: one block per tile.  Weight
// gradients (split-K): the full-height row tiles take S splits and a partial last row tile
// (local3: rows 3072-3136 of 3137) its own S_p, so the grid fills the CUs once without the
// thin tiles holding full-size K chunks (local3: 48 x 5 + 4 x 4 = 256 blocks instead of
// 52 x 4 = 208); the last split of a partial tile zero-fills slabs S_p .. S - 1 of its rows,
// which the S-slab reduce then sums harmlessly.
struct Sched {
  int tiles_n;          // column tiles
  int tm_full;          // row tiles scheduled with S splits (all of them when not split)
  int S, kchunk;        // their splits and K chunk (1, K when not split)
  int np, S_p, kchunk_p;   // blocks / splits / K chunk of the partial last row tile (np = 0: none)
};
DEV void decode(const Sched& sc, int lin, int& m0, int& n0, int& split, int& kchunk, bool& zero_rest) {
  if (lin < sc.np) {
    split = lin / sc.tiles_n;
    m0 = sc.tm_full * BM;
    n0 = (lin - split * sc.tiles_n) * BN;
    kchunk = sc.kchunk_p;
    zero_rest = split == sc.S_p - 1;
  } else {
    const int l = lin - sc.np, per = sc.tm_full * sc.tiles_n;
    split = l / per;
    const int t = l - split * per;
    m0 = (t / sc.tiles_n) * BM;
    n0 = (t % sc.tiles_n) * BN;
    kchunk = sc.kchunk;
    zero_rest = false;
  }
}

// One LDS-DMA instruction (16 bytes per lane to lds_dst + 16 lane) issued from inline asm:
// through the builtin, hipcc sees an LDS write it cannot tell apart from the next step's
// ds_reads and waits vmcnt(0) in front of them, which serialises the DMA of step t + 1 with
// the MFMAs of step t.  Hidden in asm it is not counted by hipcc at all: the kernel waits
// for it with its own vmcnt before the barrier that publishes the image.  M0 (the DMA's LDS
// base) is compiler-reserved, so it is saved and restored inside the statement; s_nop 4
// covers a descriptor fresh from readfirstlane (cdna_hip_programming.md §5.7).
DEV void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds_dst), "s"(rs)
      : "memory");
}
// wait until at most N of this wave's DMA instructions are outstanding
template <int N>
DEV void wait_dma() {
  static_assert(N == 0 || N == 4 || N == 8 || N == 12 || N == 16, "");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

// Stage the BK-deep K slab k0 (rows past kend: zeros) of rows / cols r0 .. r0 + 255 into the
// image at byte offset img: IMG / 1 KB DMA instructions (KC_RPI K-contiguous rows or 2 MN rows
// each), NI per wave.
template <int BK, bool KC>
DEV void stage(uint32_t lds_base, int img, const Opnd& o, int r0, int k0, int kend, int wave, int lane) {
  using G = Geo<BK>;
  const auto rs = buf_rsrc(o.p, o.nbytes);
#pragma unroll
  for (int u = 0; u < G::NI; ++u) {
    const int i = wave + 8 * u;                                 // DMA instruction of the image
    uint32_t off;
    if constexpr (KC) {
      constexpr int CPR = BK / 8;                               // 16-byte chunks per row
      const int row = G::KC_RPI * i + lane / CPR, ch = (lane % CPR) ^ kc_swz<BK>(row);
      const int r = r0 + row, k = k0 + 8 * ch;
      off = (r < o.R && k < kend) ? (uint32_t)(r * o.ld + k) * 2u : BUF_OOB;
    } else {
      const int row = 2 * i + (lane >> 5), ch = (lane & 31) ^ mn_swz(row);
      const int k = k0 + row, c = r0 + 8 * ch;
      off = (k < kend && c < o.R) ? (uint32_t)(k * o.ld + c) * 2u : BUF_OOB;
    }
    dma16(rs, off, (uint32_t)__builtin_amdgcn_readfirstlane(lds_base + img + 1024 * i));
  }
}

// Fragment of rows / cols c0 .. c0 + 15 for k-half kh (k = 32 kh + 8 (lane >> 4) + j)
template <int BK, bool KC>
DEV bf16x8 frag(const uint8_t* lds, int img, int c0, int kh, int lane) {
  const int i = lane & 15, g = lane >> 4;
  if constexpr (KC) {
    const int r = c0 + i, ch = (4 * kh + g) ^ kc_swz<BK>(r);
    return __builtin_bit_cast(bf16x8, *(const u32x4*)(lds + img + r * Geo<BK>::KC_RB + 16 * ch));
  } else {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int r = 32 * kh + 8 * g + q;                          // k rows r (j 0-3) and r + 4 (j 4-7)
    const int cb = 2 * (c0 + 4 * p);                            // byte in the row before the swizzle
    const int lo = r * 512 + 16 * ((cb >> 4) ^ mn_swz(r)) + (cb & 15);
    const int hi = (r + 4) * 512 + 16 * ((cb >> 4) ^ mn_swz(r + 4)) + (cb & 15);
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + img + lo));
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + img + hi));
    return join(a, b);
  }
}

template <bool AKC, bool BKC, bool WG, int BK, int S, bool RP = false>
__global__ __launch_bounds__(NTH, 1) void gemm256_k(const Opnd a, const Opnd b, const GemmEpi ep, int M, int N,
                                                    int K, const Sched sc, int ones, int dbg) {
  using G = Geo<BK>;
  static_assert(S >= 2 && S * G::BUF <= 160 * 1024, "stage ring fits the LDS");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // split-K (weight gradients): consecutive logical ids are the tiles of one split, which
  // read the same K rows of both operands -- remapped onto one XCD's L2 (gemm.hip gemm_kernel)
  int m0, n0, split, kchunk;
  bool zero_rest;
  decode(sc, xcd_remap(blockIdx.x, gridDim.x), m0, n0, split, kchunk, zero_rest);
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg + BK - 1) / BK;
  // weight gradients: the A image column `ones` (Din, the bias row of the output) reads zeros
  // from the DMA (past the operand); the lanes that staged its chunk write 1.0 over it
  const bool has_ones = WG && ones >= m0 && ones < m0 + BM;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_void*)lds;
  auto issue = [&](int kt) {   // stage of step kt into ring slot kt % S
    const int buf = (kt % S) * G::BUF;
    stage<BK, AKC>(lds_base, buf, a, m0, kbeg + kt * BK, kend, wave, lane);
    stage<BK, BKC>(lds_base, buf + G::IMG, b, n0, kbeg + kt * BK, kend, wave, lane);
  };
  auto patch_ones = [&](int kt) {   // this wave's own DMA chunks of the ones column of stage kt
    if constexpr (WG) {
      if (has_ones) {
        const int buf = (kt % S) * G::BUF;
#pragma unroll
        for (int u = 0; u < G::NI; ++u) {
          const int i = wave + 8 * u, row = 2 * i + (lane >> 5), ch = (lane & 31) ^ mn_swz(row);
          if (m0 + 8 * ch == ones && kbeg + kt * BK + row < kend)
            *(bf16_t*)(lds + buf + 1024 * i + 16 * lane) = (bf16_t)0x3f80;   // the lane's DMA slot
        }
      }
    }
  };
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) issue(p);
  if constexpr (RP) {
    // Register-prefetch schedule (one 32-deep k-half per step): the fragments of step kt + 1
    // are read from LDS while the MFMAs of step kt run, so no step starts on a ds_read
    // latency.  At the top of step kt each wave waits for ITS DMA of stage kt + 1 (stage
    // kt + 2 may stay in flight), patches, and the barrier makes every wave's stage kt + 1
    // visible; the DMA of stage kt + 3 then refills the slot of stage kt - 1, whose
    // fragments were read during step kt - 2 and consumed before this barrier.
    static_assert(S == 4 && BK == 32, "register prefetch: the 4 x 32-deep ring");
    // prefetched per step: the B fragments and the first PH A fragments (2 x 24 VGPRs next to
    // the 128 accumulators; a full second fragment set spilled); the other A fragments are
    // read at the step's start, behind the PH x FN MFMAs that need none of them
    constexpr int PH = 2;
    bf16x8 pa0[PH], pb0[FN], pa1[PH], pb1[FN];
    auto rd = [&](int kt, bf16x8 (&pa)[PH], bf16x8 (&pb)[FN]) {
      const int buf = (kt % S) * G::BUF;
#pragma unroll
      for (int j = 0; j < FN; ++j) pb[j] = frag<BK, BKC>(lds, buf + G::IMG, wn * TN + 16 * j, 0, lane);
#pragma unroll
      for (int i = 0; i < PH; ++i) pa[i] = frag<BK, AKC>(lds, buf, wm * TM + 16 * i, 0, lane);
    };
    auto mm = [&](int kt, const bf16x8 (&pa)[PH], const bf16x8 (&pb)[FN]) {
      const int buf = (kt % S) * G::BUF;
      bf16x8 fa[FM];
#pragma unroll
      for (int i = PH; i < FM; ++i) fa[i] = frag<BK, AKC>(lds, buf, wm * TM + 16 * i, 0, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(i < PH ? pa[i < PH ? i : 0] : fa[i], pb[j], acc[i][j], 0, 0, 0);
    };
    // stages 0 and 1 landed (stage 2 may stay in flight), visible to every wave
    if (nk > 2) wait_dma<G::DPS>();
    else wait_dma<0>();
    patch_ones(0);
    if (nk > 1) patch_ones(1);
    __syncthreads();
    rd(0, pa0, pb0);
    // step kt: the barrier makes stage kt + 1 visible; the rest of step kt's A fragments
    // (its slot visible since step kt - 1's barrier) are read inside mm, after the prefetch
    auto step = [&](int kt, bf16x8 (&pa)[PH], bf16x8 (&pb)[FN], bf16x8 (&na)[PH], bf16x8 (&nb)[FN]) {
      if (kt + 1 < nk) {
        if (kt >= 1) {   // stage kt + 1 (issued two steps ago); kt + 2 may stay in flight
          if (kt + 2 < nk) wait_dma<G::DPS>();
          else wait_dma<0>();
          patch_ones(kt + 1);
        }
        __syncthreads();
        if (kt + 3 < nk && !(dbg & 1)) issue(kt + 3);
        rd(kt + 1, na, nb);
      }
      mm(kt, pa, pb);
    };
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      step(kt, pa0, pb0, pa1, pb1);
      step(kt + 1, pa1, pb1, pa0, pb0);
    }
    if (kt < nk) step(kt, pa0, pb0, pa1, pb1);
  } else
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = (kt % S) * G::BUF;
    // this wave's DMA of step kt done: the stages issued after it may stay in flight
    const int ahead = min(S - 2, nk - 1 - kt);
    if constexpr (S >= 5) {
      if (ahead >= 3) wait_dma<3 * G::DPS>();
      else if (ahead == 2) wait_dma<2 * G::DPS>();
      else if (ahead == 1) wait_dma<G::DPS>();
      else wait_dma<0>();
    } else if constexpr (S == 4) {
      if (ahead >= 2) wait_dma<2 * G::DPS>();
      else if (ahead == 1) wait_dma<G::DPS>();
      else wait_dma<0>();
    } else {
      wait_dma<0>();
    }
    patch_ones(kt);    // (its wait above ordered this wave's DMA)
    __syncthreads();   // step kt's images landed (every wave's DMA); step kt - 1's reads done
    if (kt + S - 1 < nk && !(dbg & 1)) issue(kt + S - 1);   // into the slot step kt - 1 read
#pragma unroll
    for (int kh = 0; kh < BK / 32; ++kh) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag<BK, BKC>(lds, cur + G::IMG, wn * TN + 16 * j, kh, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag<BK, AKC>(lds, cur, wm * TM + 16 * i, kh, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();   // operand images dead: the epilogue reuses the LDS

  // ---- epilogue (gemm.hip's vector path): a wave stages one 16-row fragment row of its
  // 128 x 64 block, then every lane owns 8 consecutive columns of a row (2 vectors per lane)
  const int g = lane >> 4, li = lane & 15;
  constexpr int EP_LD = TN + 4, VI = 16 * (TN / 8) / 64;
  float* eb = (float*)lds + wave * 16 * EP_LD;
  float bv[VI][8];
#pragma unroll
  for (int k = 0; k < VI; ++k) {
    const int v = lane + 64 * k, n = n0 + wn * TN + (v % (TN / 8)) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[k][e] = (ep.bias && n + e < ep.bias_n) ? ep.bias[n + e] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) eb[(4 * g + r) * EP_LD + j * 16 + li] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < VI; ++k) {
      const int v = lane + 64 * k, rr = v / (TN / 8), cv = v % (TN / 8);
      const int m = m0 + wm * TM + 16 * i + rr, n = n0 + wn * TN + 8 * cv;
      if (m < M && n < N) {
        const f32x4 lo = *(const f32x4*)(eb + rr * EP_LD + 8 * cv), hi = *(const f32x4*)(eb + rr * EP_LD + 8 * cv + 4);
        if constexpr (WG) {   // split-K partial: this split's fp32 slab (+ zeros in the slabs it skips)
          float* o = (float*)ep.out + (int64_t)split * ep.slab_stride + (int64_t)m * ep.ldc + n;
          *(f32x4*)o = lo;
          *(f32x4*)(o + 4) = hi;
          if (zero_rest)
            for (int z = split + 1; z < sc.S; ++z) {
              float* oz = o + (int64_t)(z - split) * ep.slab_stride;
              *(f32x4*)oz = f32x4{0.f, 0.f, 0.f, 0.f};
              *(f32x4*)(oz + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          continue;
        }
        float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] += bv[k][e];
        if (ep.relu)
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = fmaxf(x[e], 0.f);
        if (ep.mask) {
          const u32x4 mk = *(const u32x4*)(ep.mask + (int64_t)m * ep.ldm + n);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (!(u4_get(mk, e) > 0.f)) x[e] = 0.f;
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
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// experiments only (set_gemm256_debug): bit 0 skips the in-loop staging (timing, wrong
// results); bit 1 runs the 2-stage BK = 64 ring instead of the 4-stage BK = 32 one, bit 2 a
// 5-stage BK = 32 ring (160 KB), bit 3 the BK = 64 ring for the data gradient only, bit 4 the
// register-prefetch schedule (also MNISTX_GEMM256_BK=64 / MNISTX_GEMM256_STAGES=5 /
// MNISTX_GEMM256_DGRAD_BK=64 / MNISTX_GEMM256_RP=1 at load,
// for whole-step A/Bs)
int g_gemm256_dbg = [] {
  const char* e = getenv("MNISTX_GEMM256_BK");
  const char* s5 = getenv("MNISTX_GEMM256_STAGES");
  const char* dg = getenv("MNISTX_GEMM256_DGRAD_BK");
  const char* rp = getenv("MNISTX_GEMM256_RP");
  return ((e && e[0] == '6') ? 2 : 0) | ((s5 && s5[0] == '5') ? 4 : 0) | ((dg && dg[0] == '6') ? 8 : 0) |
         ((rp && rp[0] == '1') ? 16 : 0);
}();

// the CUs a launch can count on: all of them less the ones reserved for a collective running
// beside it (set_reserve_cus, data-parallel runs with world > 1).  A one-round grid of 256
// blocks on 248 free CUs would run as TWO rounds.
int num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = -1;
  }
  if (cus <= 0) return cus;
  const int r = reserve_cus();
  return (r > 0 && cus - r >= 1) ? cus - r : cus;
}

// fraction of the last round of `tiles` one-per-CU blocks that is busy
double round_fill(int64_t tiles, int cus) {
  const int64_t rounds = (tiles + cus - 1) / cus;
  return (double)tiles / (double)(rounds * cus);
}

// Schedule of an M x N x K launch; WG: `splits` for the full-height row tiles (the caller's
// slab count), the partial last row tile gets what fills the remaining CUs (<= splits).
// Returns the grid size, 0 if `splits` is not an exact chunking of K.
int make_sched(Sched& sc, int M, int N, int K, bool wg, int splits) {
  const int tn = (N + BN - 1) / BN, tm = (M + BM - 1) / BM;
  if (!wg) {
    sc = Sched{tn, tm, 1, K, 0, 0, 0};
    return tm * tn;
  }
  const int kchunk = ((K + splits - 1) / splits + 63) / 64 * 64;
  if ((K + kchunk - 1) / kchunk != splits) return 0;
  const int tm_full = M / BM;
  sc = Sched{tn, tm_full, splits, kchunk, 0, 0, 0};
  if (tm_full < tm) {
    const int cus = num_cus();
    int sp = cus > 0 ? (cus - tm_full * tn * splits) / tn : 1;
    sp = sp < 1 ? 1 : (sp > splits ? splits : sp);
    const int kcp = ((K + sp - 1) / sp + 63) / 64 * 64;
    sc.S_p = (K + kcp - 1) / kcp;
    sc.kchunk_p = kcp;
    sc.np = tn * sc.S_p;
  }
  return sc.np + tm_full * tn * splits;
}

template <bool AKC, bool BKC, bool WG, int BK, int S, bool RP = false>
hipError_t launch_bk(const Opnd& a, const Opnd& b, const GemmEpi& ep, int M, int N, int K, int splits, int ones,
                     hipStream_t st) {
  constexpr int bytes = S * Geo<BK>::BUF;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm256_k<AKC, BKC, WG, BK, S, RP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            bytes) != hipSuccess)
      return hipErrorInvalidValue;
    attr = true;
  }
  Sched sc;
  const int grid = make_sched(sc, M, N, K, WG, splits);   // WG: the caller's split count (its slab)
  if (grid <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm256_k<AKC, BKC, WG, BK, S, RP>), dim3(grid), dim3(NTH), bytes, st, a, b, ep, M, N, K, sc, ones,
                     g_gemm256_dbg);
  return hipGetLastError();
}

template <bool AKC, bool BKC, bool WG>
hipError_t launch256(const Opnd& a, const Opnd& b, const GemmEpi& ep, int M, int N, int K, int splits, int ones,
                     hipStream_t st) {
  if ((g_gemm256_dbg & 2) || ((g_gemm256_dbg & 8) && AKC && BKC))
    return launch_bk<AKC, BKC, WG, 64, 2>(a, b, ep, M, N, K, splits, ones, st);
  if (g_gemm256_dbg & 4) return launch_bk<AKC, BKC, WG, 32, 5>(a, b, ep, M, N, K, splits, ones, st);
  if (g_gemm256_dbg & 16) return launch_bk<AKC, BKC, WG, 32, 4, true>(a, b, ep, M, N, K, splits, ones, st);
  return launch_bk<AKC, BKC, WG, 32, 4>(a, b, ep, M, N, K, splits, ones, st);
}

bool sizes_ok(int64_t rows, int ld, int K, int R) {
  return (ld & 7) == 0 && (K & 7) == 0 && (R & 7) == 0 && rows * ld * 2 < ((int64_t)1 << 31);
}

// ---------------------------------------------------------------- fp32 (--precision fp32)
// The same tile, DMA ring and epilogue on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32
// sums: the reference trains in tf.float32, mnist_input.py:86,107).  16-deep K stages, four
// of them (4 x 32 KB), three in flight.  The 4 k-slots of an MFMA are k = 4 g + s for lane
// group g and MFMA s of the stage's 4 slices, so a lane's 4 k of one fragment row are one
// 16-byte chunk: a K-contiguous operand gives them in ONE ds_read_b128, an MN-contiguous one
// in 4 ds_read_b32 (rows 4 g .. 4 g + 3 at the lane's column).
constexpr int BKF = 16;
constexpr int IMGF = BM * BKF * 4;          // 16 KB per operand image
constexpr int BUFF = 2 * IMGF;
constexpr int SF = LDS_BYTES / BUFF;        // 4 stages
constexpr int NIF = IMGF / 1024 / 8;        // 1 KB DMA instructions per wave per image (2)
constexpr int DPSF = 2 * NIF;               // ... per stage (4)
static_assert(SF == 4 && DPSF == 4, "fp32 ring: 4 stages of 4 DMA instructions per wave");
// swizzles (bench/lds_gemm256.py): 64-byte K-contiguous rows read by ds_read_b128 (the
// bf16 32-deep geometry); 1 KB MN rows read by ds_read_b32: rows 4 apart in one half-wave
// are moved to the other 64-byte half of the bank line
DEV int kcs_f(int r) { return ((r >> 3) & 1) << 1; }
DEV int mns_f(int r) { return ((r >> 2) & 1) << 2; }

struct OpndF {
  const float* p;
  int ld, R, K;
  uint32_t nbytes;
};
struct EpiF32 {
  float* out;            // output, or the split-K slab base (WG)
  int ldc;
  const float* bias;     // + bias[n] (n < bias_n)
  int bias_n, relu;
  const float* mask;     // keep v where mask[m * ldm + n] > 0 (ReLU backward)
  int ldm;
  int64_t slab_stride;
};

template <bool KC>
DEV void stage_f(uint32_t lds_base, int img, const OpndF& o, int r0, int k0, int kend, int wave, int lane) {
  const auto rs = buf_rsrc(o.p, o.nbytes);
#pragma unroll
  for (int u = 0; u < NIF; ++u) {
    const int i = wave + 8 * u;
    uint32_t off;
    if constexpr (KC) {   // 16 rows of 64 bytes per instruction
      const int row = 16 * i + (lane >> 2), ch = (lane & 3) ^ kcs_f(row);
      const int r = r0 + row, k = k0 + 4 * ch;
      off = (r < o.R && k < kend) ? (uint32_t)(r * o.ld + k) * 4u : BUF_OOB;
    } else {              // one 1 KB row (256 columns) per instruction
      const int row = i, ch = lane ^ mns_f(row);
      const int k = k0 + row, c = r0 + 4 * ch;
      off = (k < kend && c < o.R) ? (uint32_t)(k * o.ld + c) * 4u : BUF_OOB;
    }
    dma16(rs, off, (uint32_t)__builtin_amdgcn_readfirstlane(lds_base + img + 1024 * i));
  }
}

// the 4 k (= 4 g .. 4 g + 3) of row / column c0 + (lane & 15) for the stage's 4 MFMAs
template <bool KC>
DEV f32x4 frag_f(const uint8_t* lds, int img, int c0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  if constexpr (KC) {
    const int r = c0 + i;
    return *(const f32x4*)(lds + img + r * 64 + 16 * (g ^ kcs_f(r)));
  } else {
    const int c = c0 + i;
    f32x4 v;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 4 * g + s;
      v[s] = *(const float*)(lds + img + k * 1024 + 16 * ((c >> 2) ^ mns_f(k)) + 4 * (c & 3));
    }
    return v;
  }
}

template <bool AKC, bool BKC, bool WG>
__global__ __launch_bounds__(NTH, 1) void gemm256f_k(const OpndF a, const OpndF b, const EpiF32 ep, int M, int N,
                                                     int K, const Sched sc, int ones) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  int m0, n0, split, kchunk;
  bool zero_rest;
  decode(sc, xcd_remap(blockIdx.x, gridDim.x), m0, n0, split, kchunk, zero_rest);
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg + BKF - 1) / BKF;
  const bool has_ones = WG && ones >= m0 && ones < m0 + BM;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_void*)lds;
  auto issue = [&](int kt) {
    const int buf = (kt % SF) * BUFF;
    stage_f<AKC>(lds_base, buf, a, m0, kbeg + kt * BKF, kend, wave, lane);
    stage_f<BKC>(lds_base, buf + IMGF, b, n0, kbeg + kt * BKF, kend, wave, lane);
  };
#pragma unroll
  for (int p = 0; p < SF - 1; ++p)
    if (p < nk) issue(p);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = (kt % SF) * BUFF;
    const int ahead = min(SF - 2, nk - 1 - kt);
    if (ahead >= 2) wait_dma<2 * DPSF>();
    else if (ahead == 1) wait_dma<DPSF>();
    else wait_dma<0>();
    if constexpr (WG) {
      if (has_ones) {   // this wave's own DMA chunks of the ones column
#pragma unroll
        for (int u = 0; u < NIF; ++u) {
          const int i = wave + 8 * u, ch = lane ^ mns_f(i);
          if (m0 + 4 * ch == ones && kbeg + kt * BKF + i < kend) *(float*)(lds + cur + 1024 * i + 16 * lane) = 1.f;
        }
      }
    }
    __syncthreads();
    if (kt + SF - 1 < nk) issue(kt + SF - 1);
    f32x4 fa[FM], fb[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = frag_f<BKC>(lds, cur + IMGF, wn * TN + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = frag_f<AKC>(lds, cur, wm * TM + 16 * i, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  }
  __syncthreads();

  // epilogue: the bf16 kernel's (8 consecutive columns of one row per lane and vector)
  const int g = lane >> 4, li = lane & 15;
  constexpr int EP_LD = TN + 4, VI = 16 * (TN / 8) / 64;
  float* eb = (float*)lds + wave * 16 * EP_LD;
  float bv[VI][8];
#pragma unroll
  for (int k = 0; k < VI; ++k) {
    const int v = lane + 64 * k, n = n0 + wn * TN + (v % (TN / 8)) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[k][e] = (!WG && ep.bias && n + e < ep.bias_n) ? ep.bias[n + e] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) eb[(4 * g + r) * EP_LD + j * 16 + li] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < VI; ++k) {
      const int v = lane + 64 * k, rr = v / (TN / 8), cv = v % (TN / 8);
      const int m = m0 + wm * TM + 16 * i + rr, n = n0 + wn * TN + 8 * cv;
      if (m < M && n < N) {
        f32x4 lo = *(const f32x4*)(eb + rr * EP_LD + 8 * cv), hi = *(const f32x4*)(eb + rr * EP_LD + 8 * cv + 4);
        float* o;
        if constexpr (WG) {
          o = ep.out + (int64_t)split * ep.slab_stride + (int64_t)m * ep.ldc + n;
          if (zero_rest)
            for (int z = split + 1; z < sc.S; ++z) {
              float* oz = o + (int64_t)(z - split) * ep.slab_stride;
              *(f32x4*)oz = f32x4{0.f, 0.f, 0.f, 0.f};
              *(f32x4*)(oz + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        } else {
          o = ep.out + (int64_t)m * ep.ldc + n;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            lo[e] += bv[k][e];
            hi[e] += bv[k][e + 4];
          }
          if (ep.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              lo[e] = fmaxf(lo[e], 0.f);
              hi[e] = fmaxf(hi[e], 0.f);
            }
          }
          if (ep.mask) {
            const f32x4 ml = *(const f32x4*)(ep.mask + (int64_t)m * ep.ldm + n);
            const f32x4 mh = *(const f32x4*)(ep.mask + (int64_t)m * ep.ldm + n + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if (!(ml[e] > 0.f)) lo[e] = 0.f;
              if (!(mh[e] > 0.f)) hi[e] = 0.f;
            }
          }
        }
        *(f32x4*)o = lo;
        *(f32x4*)(o + 4) = hi;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <bool AKC, bool BKC, bool WG>
hipError_t launch_f(const OpndF& a, const OpndF& b, const EpiF32& ep, int M, int N, int K, int splits, int ones,
                    hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm256f_k<AKC, BKC, WG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            LDS_BYTES) != hipSuccess)
      return hipErrorInvalidValue;
    attr = true;
  }
  Sched sc;
  const int grid = make_sched(sc, M, N, K, WG, splits);
  if (grid <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm256f_k<AKC, BKC, WG>), dim3(grid), dim3(NTH), LDS_BYTES, st, a, b, ep, M, N, K, sc, ones);
  return hipGetLastError();
}

bool sizes_ok_f(int64_t rows, int ld, int K, int R) {
  return (ld & 3) == 0 && (K & 3) == 0 && (R & 3) == 0 && rows * ld * 4 < ((int64_t)1 << 31);
}

bool fill_ok(int M, int N, int min_tiles) {
  const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  return tiles >= min_tiles && (double)M * N / ((double)tiles * BM * BN) >= 0.9;
}

}  // namespace

int gemm256_cus() { return num_cus(); }

// Routing switch (A/B): MNISTX_GEMM256=0 starts with every dense GEMM on gemm.hip;
// set_gemm256 flips it at run time (tests and benches compare both paths in one process).
static int g_gemm256 = -1;
bool gemm256_enabled() {
  if (g_gemm256 < 0) {
    const char* e = getenv("MNISTX_GEMM256");
    g_gemm256 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_gemm256 != 0;
}
void set_gemm256(bool on) { g_gemm256 = on ? 1 : 0; }
void set_gemm256_debug(int bits) { g_gemm256_dbg = bits; }

// The 256 x 256 path takes a GEMM when it fills the GPU at least once (>= 256 tiles of a
// mostly-full 256 x 256), the epilogue is a plain bf16 / fp32 store and every vector is whole.
bool gemm256_ok(int M, int N, int K, const GemmEpi& ep) {
  if (!gemm256_enabled() || ep.mode == EPI_SLAB || K < 512) return false;   // >= 8 K steps of 64
  const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const double fill = (double)M * N / ((double)tiles * BM * BN);
  const int cus = num_cus();
  // the last round >= 80 % busy (local3 dgrad: 832 tiles = 3.25 rounds of 256 measured faster
  // than gemm.hip; local3 forward, 256 tiles, would be 2 rounds on 248 free CUs)
  return tiles >= 256 && fill >= 0.9 && cus > 0 && round_fill(tiles, cus) >= 0.8 && (N & 7) == 0 &&
         (ep.ldc & 7) == 0 && ((uintptr_t)ep.out & 15) == 0 &&
         (ep.mask == nullptr || ((ep.ldm & 7) == 0 && ((uintptr_t)ep.mask & 15) == 0));
}

// y[M, N] = x[M, K] . W[K, N]   (x K-contiguous, W MN-contiguous)
hipError_t gemm256_fwd(const bf16_t* x, const bf16_t* w, int M, int N, int K, int ldx, int ldw, const GemmEpi& ep,
                       hipStream_t st) {
  if (!sizes_ok(M, ldx, K, 8) || !sizes_ok(K, ldw, 8, N)) return hipErrorInvalidValue;
  const Opnd a{x, ldx, M, K, (uint32_t)((int64_t)M * ldx * 2)};
  const Opnd b{w, ldw, N, K, (uint32_t)((int64_t)K * ldw * 2)};
  return launch256<true, false, false>(a, b, ep, M, N, K, 1, -1, st);
}

// dX[M, N] = dY[M, K] . W[N, K]^T   (both K-contiguous)
hipError_t gemm256_dgrad(const bf16_t* dy, const bf16_t* w, int M, int N, int K, int lddy, int ldw, const GemmEpi& ep,
                         hipStream_t st) {
  if (!sizes_ok(M, lddy, K, 8) || !sizes_ok(N, ldw, K, 8)) return hipErrorInvalidValue;
  const Opnd a{dy, lddy, M, K, (uint32_t)((int64_t)M * lddy * 2)};
  const Opnd b{w, ldw, N, K, (uint32_t)((int64_t)N * ldw * 2)};
  return launch256<true, true, false>(a, b, ep, M, N, K, 1, -1, st);
}

// Weight gradient slab[split][Din (+1)][Dout] = X^T dY over the split's K rows (X [B][Din],
// dY [B][Dout]: both MN-contiguous); with_bias: row Din sums dY (the ones column of X^T).
// The split count is the caller's (gemm256_wgrad_splits chose it).
hipError_t gemm256_wgrad(const bf16_t* x, const bf16_t* dy, int Din, int Dout, int B, int ldx, int lddy,
                         int with_bias, int splits, const GemmEpi& ep, hipStream_t st) {
  if (!sizes_ok(B, ldx, 8, Din) || !sizes_ok(B, lddy, 8, Dout) || ep.mode != EPI_SLAB || (ep.ldc & 7) != 0 ||
      ((uintptr_t)ep.out & 15) != 0 || (ep.slab_stride & 3) != 0)
    return hipErrorInvalidValue;
  const Opnd a{x, ldx, Din, B, (uint32_t)((int64_t)B * ldx * 2)};
  const Opnd b{dy, lddy, Dout, B, (uint32_t)((int64_t)B * lddy * 2)};
  return launch256<false, false, true>(a, b, ep, Din + (with_bias ? 1 : 0), Dout, B, splits, with_bias ? Din : -1, st);
}

// Split count of a gemm256 weight gradient: the most splits whose blocks still fit in one
// round of the CUs (a 257th block would run as a second round), chunks >= 8 steps; 0 when
// the shape does not belong on this path (too few tiles, partial vectors).
int gemm256_wgrad_splits(int Din, int Dout, int B, int with_bias, int cus) {
  if (!gemm256_enabled() || (Din & 7) || (Dout & 7) || B < 1024) return 0;
  const int M = Din + (with_bias ? 1 : 0);
  const int tiles = ((M + BM - 1) / BM) * ((Dout + BN - 1) / BN);
  const double fill = (double)M * Dout / ((double)tiles * BM * BN);
  if (tiles < 32 || tiles > cus || fill < 0.9) return 0;
  // splits of the full-height tiles (make_sched gives a partial last row tile the rest)
  const int full = (M / BM) * ((Dout + BN - 1) / BN);
  int s = cus / (full > 0 ? full : tiles);
  while (s > 1 && B / s < 512) --s;
  // the effective count of the chunking launch_bk uses
  const int kchunk = ((B + s - 1) / s + 63) / 64 * 64;
  return (B + kchunk - 1) / kchunk;
}

// ---- fp32: the f32.hip launchers route here (same conditions as the bf16 path; N % 8 for
// the 8-column epilogue vectors, 16-byte aligned operands)
// fp32 only: also require the last round of tiles to be >= 90 % full -- the fp32 data
// gradient of local3 (832 tiles = 3.25 rounds of 256 CUs) ran 993 us here vs 925 on
// f32.hip's 128 x 128 tiles (bench/micro_gemm256.py), its forward 761 vs 893 (1 round)
bool gemm256f_ok(int M, int N, int K) {
  if (!gemm256_enabled() || K < 256 || (N & 7) || !fill_ok(M, N, 256)) return false;
  const int cus = num_cus();
  if (cus <= 0) return false;
  return round_fill((int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN), cus) >= 0.9;
}

// y[M, N] = x[M, K] . W[K, N] (+ bias, ReLU)
hipError_t gemm256f_fwd(const float* x, const float* w, int M, int N, int K, const float* bias, int bias_n, int relu,
                        float* y, int ldy, hipStream_t st) {
  if (!sizes_ok_f(M, K, K, 4) || !sizes_ok_f(K, N, 4, N) || (ldy & 3) || ((uintptr_t)y & 15)) return hipErrorInvalidValue;
  const OpndF a{x, K, M, K, (uint32_t)((int64_t)M * K * 4)};
  const OpndF b{w, N, N, K, (uint32_t)((int64_t)K * N * 4)};
  return launch_f<true, false, false>(a, b, EpiF32{y, ldy, bias, bias_n, relu, nullptr, 0, 0}, M, N, K, 1, -1, st);
}

// dx[M, Din] = dy[M, Dout] . W[Din, Dout]^T (x mask > 0)
hipError_t gemm256f_dgrad(const float* dy, const float* w, int M, int Din, int Dout, const float* mask, float* dx,
                          hipStream_t st) {
  if (!sizes_ok_f(M, Dout, Dout, 4) || !sizes_ok_f(Din, Dout, Dout, 4) || (Din & 7) || ((uintptr_t)dx & 15) ||
      ((uintptr_t)mask & 15))
    return hipErrorInvalidValue;
  const OpndF a{dy, Dout, M, Dout, (uint32_t)((int64_t)M * Dout * 4)};
  const OpndF b{w, Dout, Din, Dout, (uint32_t)((int64_t)Din * Dout * 4)};
  return launch_f<true, true, false>(a, b, EpiF32{dx, Din, nullptr, 0, 0, mask, Din, 0}, M, Din, Dout, 1, -1, st);
}

int gemm256f_wgrad_splits(int Din, int Dout, int B, int cus) {
  if (!gemm256_enabled() || (Din & 3) || (Dout & 7) || B < 1024) return 0;
  const int M = Din + 1;
  const int tiles = ((M + BM - 1) / BM) * ((Dout + BN - 1) / BN);
  if (tiles < 32 || tiles > cus || !fill_ok(M, Dout, 32)) return 0;
  const int full = (M / BM) * ((Dout + BN - 1) / BN);
  int s = cus / (full > 0 ? full : tiles);
  while (s > 1 && B / s < 512) --s;
  const int kchunk = ((B + s - 1) / s + 63) / 64 * 64;
  return (B + kchunk - 1) / kchunk;
}

// slab[split][Din + 1][Dout]: rows < Din = x^T dy over the split's rows, row Din = sums of dy
hipError_t gemm256f_wgrad(const float* x, const float* dy, int B, int Din, int Dout, int splits, float* slab,
                          hipStream_t st) {
  if (!sizes_ok_f(B, Din, 4, Din) || !sizes_ok_f(B, Dout, 4, Dout) || ((uintptr_t)slab & 15)) return hipErrorInvalidValue;
  const OpndF a{x, Din, Din, B, (uint32_t)((int64_t)B * Din * 4)};
  const OpndF b{dy, Dout, Dout, B, (uint32_t)((int64_t)B * Dout * 4)};
  const int64_t stride = (int64_t)(Din + 1) * Dout;
  if (stride & 3) return hipErrorInvalidValue;
  return launch_f<false, false, true>(a, b, EpiF32{slab, Dout, nullptr, 0, 0, nullptr, 0, stride}, Din + 1, Dout, B,
                                      splits, Din, st);
}

}  // namespace mnistx
