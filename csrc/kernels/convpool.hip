// Fused small-channel conv blocks for gfx950: conv(5x5, stride 1) + bias + ReLU + 2x2/2 max-pool.
//
// The first conv layers of MNIST nets have tiny channel counts (Cin 1/3/8, Cout
// 8/16/32), so a generic implicit GEMM wastes its tiles and spends its time in
// index arithmetic.  These kernels are specialised at compile time on the
// layer geometry and keep whole padded input images as LDS tiles:
//
// * Pool-window-major GEMM rows: output pixel row r = 4*window + d with
//   d = (dy, dx) inside the 2x2 pooling window.  A v_mfma_f32_16x16x32_bf16
//   accumulator gives each lane rows 4g..4g+3 of one column, i.e. exactly one
//   pooling window of one channel -- bias + ReLU + max-pool + argmax happen in
//   registers and the full-resolution conv output never touches HBM.
// * im2col fragments are aligned vector LDS reads: Cin 8 -> one ds_read_b128 of
//   8 channels; Cin 1 -> K ordered (kh, kw padded to 8) and the image kept 4x in
//   LDS shifted by 0..3 elements, so every run of 4 pixels is one aligned
//   ds_read_b64.  Weight gradients read im2col^T with ds_read_b64_tr_b16.
// * Idle MFMA columns: with Cout 8 (LeNet conv1) / Cin 8 (LeNet conv2 dgrad) the
//   16-wide MFMA N dimension is half empty; the "pair" kernels fill columns
//   8..15 with the kw-shifted filter, i.e. the horizontally adjacent pixel.
// * Backward rebuilds dY from the pooled gradient and the argmax byte; the ReLU
//   mask is folded into the byte (ARG_OFF), so the pooled activations are never
//   re-read.  wgrad's bias gradient is a virtual ones-row; per-block fp32
//   partials go to a slab reduced deterministically by splitk_reduce.
// * Staging is software-pipelined: the next image group's global data is
//   loaded into VGPRs while the current group computes.
//
// Replaces: Conv2D + BiasAdd + Relu + MaxPool and
// their gradients at mnist_input.py:142-150 (conv1 -> pool1) and the LeNet-5
// conv blocks.
#include "common.h"
#include "launchers.h"
#include "lrn_math.h"

#include <cstdlib>
#include <type_traits>

namespace mnistx {
namespace {

// smallest column count >= c whose byte width (c * cin * 2) is a multiple of 16
constexpr int align_cols(int c, int cin) {
  while ((c * cin * 2) % 16 != 0) ++c;
  return c;
}

// Row width (columns) for tiles read with ds_read_b64 by 16 pixels spanning two
// image rows (pool-window-major): a row of 128 bytes mod 256 puts the second row
// in the other half of the 64 banks.
constexpr int bank_cols(int c, int cin) {
  c = align_cols(c, cin);
  if (cin % 4 != 0) return c;
  while ((c * cin * 2) % 256 != 128) c += align_cols(1, cin);
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
  static constexpr int WS = bank_cols(X0 + W + PAD, CIN);
  static constexpr int XOFF = X0 - PAD;
  static constexpr int ROWV = W * CIN / 4;            // 8-byte vectors per interior row
  static_assert((W * CIN) % 4 == 0, "interior rows must be whole 8-byte vectors");
  static constexpr int PH = OH / 2, PW = OW / 2;
  static constexpr int NWIN = PH * PW;
  static constexpr int NPIX = OH * OW;
  static constexpr int MF = (NPIX + 15) / 16;
  // im2col column order (K):
  //  MODE 0 (Cin == 1):     k = kh*8 + kw, kw padded to 8.  Four consecutive k are
  //                         four consecutive pixels of one input row; the image is
  //                         kept in LDS 4 times, shifted by 0..3 elements, so every
  //                         such run is ONE aligned 8-byte LDS read.
  //  MODE 1 (Cin % 8 == 0): k = (kh*KS + kw)*Cin + ci; a lane's 8 k-slots are the 8
  //                         consecutive channels of one tap (one ds_read_b128).
  //  MODE 2 (other Cin):    MODE 1 order with scalar 2-byte gathers.
  static constexpr int MODE = CIN == 1 ? 0 : (CIN % 8 == 0 ? 1 : 2);
  static constexpr int KC = KS * KS * CIN;             // real im2col columns
  static constexpr int KE = MODE == 0 ? KS * 8 : KC;   // im2col columns incl. kw padding
  static constexpr int KSTEPS = (KE + 31) / 32;
  static constexpr int NF = (COUT + 15) / 16;
  static constexpr int NCOL = NF * 16;
  static constexpr int TILE = HP * WS * CIN;
  static constexpr int NCOPY = MODE == 0 ? 4 : 1;
  static constexpr int TSTR = (TILE + 16 + 7) / 8 * 8;  // per-copy stride: zero slack for padded-k over-reads
  static constexpr int IMG_LDS = NCOPY * TSTR;
  static constexpr int INTERIOR = H * W * CIN;
  static constexpr int KM = ((KE + 1) + 15) / 16 * 16;  // wgrad rows incl. the bias (ones) row at KE
  static constexpr int MFW = KM / 16;
  static constexpr int RSTEPS = (NPIX + 31) / 32;
  // slab row layout for splitk_reduce: row = g * RED_IP + i, bias row KE
  static constexpr int RED_G = MODE == 0 ? KS : KS * KS;
  static constexpr int RED_IP = MODE == 0 ? 8 : CIN;
  static_assert(OH % 2 == 0 && OW % 2 == 0, "pool-window-major order needs an even conv output");
  static_assert(NPIX == 4 * NWIN, "");
  static_assert(MODE == 2 || KE % 4 == 0, "bias row must start a 4-column chunk");
  static_assert(MODE != 0 || WS % 4 == 0, "MODE 0 chunk deltas must keep the shifted-copy alignment");
  // Cout == 8 with Cin == 1: MFMA columns 8..15 compute the right-hand pixel of
  // each 2x2 pool window (weights shifted by one kw), see convpool_*_pair_k.
  static constexpr bool PAIR = MODE == 0 && COUT == 8;
  static_assert(MODE != 0 || ((OH - 1 + KS - 1) * WS + OW - 1 + XOFF + 7) < TSTR, "padded-kw over-read inside the copy");

  // LDS offset of im2col column k (MODE 1/2 order) relative to the pixel base
  static DEV int kdelta(int k) {
    const int tap = k / CIN, ci = k - (k / CIN) * CIN;
    const int kh = tap / KS, kw = tap - (tap / KS) * KS;
    return (kh * WS + kw) * CIN + ci;
  }
  // LDS offset of the 4-column chunk starting at k (k % 4 == 0, k < KE)
  static DEV int chunk_delta(int k) {
    if constexpr (MODE == 0) return (k >> 3) * WS + (k & 7);
    else return kdelta(k);
  }
  // LDS offset of the top-left input pixel feeding pool window w
  static DEV int wbase(int w) {
    const int ph = w / PW, pw = w - (w / PW) * PW;
    return ((2 * ph) * WS + 2 * pw + XOFF) * CIN;
  }
  static DEV int doff(int d) { return ((d >> 1) * WS + (d & 1)) * CIN; }
  // LDS element offset (within one image's region) of the 4 columns starting at
  // copy-0 offset a: MODE 0 picks the shifted copy that makes the read aligned.
  static DEV int aligned_off(int a) {
    if constexpr (MODE == 0) return a + (a & 3) * (TSTR - 1);
    else return a;
  }
  // im2col column of A/B fragment element j of lane group g in k-step s.
  // MODE 0: two runs of 4 (4g.., 16+4g..) = two aligned 8-byte reads;
  // MODE 1/2: one run of 8 (8g..) = one 16-byte read (MODE 1).
  static DEV int kslot(int s, int g, int j) {
    if constexpr (MODE == 0) return 32 * s + 4 * g + (j & 3) + 16 * (j >> 2);
    else return 32 * s + 8 * g + j;
  }
};

DEV __bf16 as_bf(bf16_t v) { return __builtin_bit_cast(__bf16, v); }

// Two 8-byte LDS reads at a constant distance are fused by the compiler into
// ds_read2_b64, which runs at HALF the rate of two ds_read_b64 on gfx950 (8 LDS
// cycles, 32-bank mapping: MI355X_MICROARCH.md LDS table).  Hiding the offset's
// value keeps them separate.
DEV int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Max-pool with the argmax riding in the value: the 2-bit window position d is
// written into the two low mantissa bits of the fp32 conv sum (a <= 3-ulp
// perturbation, far below bf16 resolution), so pooling is plain v_max_f32 and the
// winner's position is bits & 3.  ReLU(. + b) is monotone, so pooling the raw sums
// and applying bias + ReLU once is exact.
DEV float pos_embed(float v, uint32_t d) { return __uint_as_float((__float_as_uint(v) & ~3u) | d); }
DEV float vmax(float a, float b) {  // bare v_max_f32 (fmaxf adds NaN-canonicalising moves)
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
DEV uint32_t pos_of(float v) { return __float_as_uint(v) & 3u; }
// 0xffff in each 16-bit half of e that equals d (d < 0x10000), else 0:
// v_xor + v_pk_min_u16 + v_pk_sub_u16
DEV uint32_t half_eq_mask(uint32_t e, uint32_t d) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 x = __builtin_bit_cast(u16x2, e ^ (d * 0x00010001u));
  const u16x2 one = {1, 1};
  return __builtin_bit_cast(uint32_t, (u16x2)(__builtin_elementwise_min(x, one) - one));
}
DEV float pos_clear(float v) { return __uint_as_float(__float_as_uint(v) & ~3u); }

constexpr int NTH = 256;

// A following LRN folded into a weight gradient's dY staging (reference CNN norm1
// after conv1+pool1): the kernel reads dL/d(LRN output) and the LRN input (= the
// pooled activations) and applies the LRN backward while staging, so the pool-level
// gradient never goes to HBM.  p == nullptr: no fold.
struct LrnFold {
  const bf16_t* p;
  float bias, alpha, beta;
};
// Minimum waves per SIMD the register allocator must leave room for (the
// __launch_bounds__ second argument).  LeNet conv2 fwd: 104 VGPRs, 4 waves (a bound
// of 5 forces 96 with a spill and measured slower); its wgrad: 122 VGPRs, 4 waves,
// matching its 39 KB of LDS.  The reference conv1 variants spill under a bound, so
// they keep the default.
template <class G> constexpr int fwd_minw() { return (G::CIN == 8 && G::COUT == 16) ? 4 : 1; }
template <class G> constexpr int wgrad_minw() { return (G::CIN == 8 && G::COUT == 16) ? 4 : 1; }
// Argmax byte of a pool window whose ReLU output is 0: matches no position, so
// the backward kernels need only (dP, arg) -- the ReLU mask is folded in here
// and the pooled activations are never re-read.
constexpr uint32_t ARG_OFF = 4;
// LeNet conv1 (8 channels, quad forward): the argmax codes (0..3, ARG_OFF) are stored
// packed, 4 bits each: byte k of a window = code(c = k) | code(c = k + 4) << 4
// (4 bytes per window instead of 8).  Other geometries keep one byte per channel.
template <class G>
constexpr bool arg_packed() { return G::MODE == 0 && G::COUT == 8 && G::H == 28 && G::W == 28 && G::PAD == 2; }
template <class G>
constexpr int arg_bytes() { return arg_packed<G>() ? G::COUT / 2 : G::COUT; }

template <int N>
DEV void lds_zero(bf16_t* p, int tid) {
  static_assert(N % 8 == 0, "");
  for (int e = tid; e < N / 8; e += NTH) *(u32x4*)(p + 8 * e) = u32x4{0u, 0u, 0u, 0u};
}

// ------------------------------------------------------------------ staging
// Global data of the NEXT image group is loaded into VGPRs while the current
// group computes (software pipelining); store() moves it to LDS after the barrier.

// Input interiors (NHWC rows) -> copy 0 of the LDS image tiles, 8-byte vectors.
template <class G, int IMGS>
struct XStage {
  static constexpr int NV = IMGS * G::H * G::ROWV;
  static constexpr int VPI = G::H * G::ROWV;   // vectors per image
  static constexpr int NWV = NTH / 64;
  // dataset gathers (first layers only): 1-channel images, and the reference CNN's
  // 3-channel 28x28 records (mnist_input.py:13-15: NHWC rows, the layout of the batch x0)
  static constexpr bool U8 = G::CIN == 1 || (G::CIN == 3 && G::H == 28 && G::W == 28);
  // First-layer geometries: whole waves load one image (WPI waves per image), so the
  // image -- and, for dataset gathers, its row -- is wave-uniform: one index load per
  // wave per group and no per-vector row select (the select + 64-bit clamp cost
  // ~25 VALU per vector in the 4-image forward).
  static constexpr bool WIMG = U8 && IMGS <= NWV;
  static constexpr int WPI = WIMG ? NWV / IMGS : 1;
  static constexpr int TPI = 64 * WPI;
  static constexpr int PER = WIMG ? (VPI + TPI - 1) / TPI : (NV + NTH - 1) / NTH;
  // vector slot u of thread tid -> image-major vector index e (NV: no vector)
  static DEV int vec(int u, int tid) {
    if constexpr (WIMG) {
      const int im = (tid >> 6) / WPI, j = tid % TPI + u * TPI;
      return (im < IMGS && j < VPI) ? im * VPI + j : NV;
    } else {
      return min(tid + u * NTH, NV);
    }
  }
  u32x2 v[PER];
  // dataset gathers: row index of the group to load next, fetched one group ahead so
  // its load never stalls the data prefetch behind it.  WIMG: the wave's own image,
  // by a VECTOR load (a scalar load would share lgkmcnt with every LDS wait of the
  // compute phase); raw int64, clamped only when load() uses it.  Otherwise every
  // image's row by (uniform) scalar loads.
  u32x2 wrow;
  int64_t rows[WIMG ? 1 : IMGS];
  DEV void fetch_rows(const XSrc& src, int img0, int B) {
    if (!U8 || !src.idx || B <= 0) return;
    if constexpr (WIMG) {
      const int im = min((int)(threadIdx.x >> 6) / WPI, IMGS - 1);
      wrow = buf_b64(buf_rsrc(src.idx, (uint32_t)B * 8u), 8u * (uint32_t)max(0, min(img0 + im, B - 1)));
    } else {
#pragma unroll
      for (int im = 0; im < IMGS; ++im) rows[im] = src.idx[max(0, min(img0 + im, B - 1))];
    }
  }
  DEV int row_of(const XSrc& src, int k) const {
    return (int)min(max(rows[k], (int64_t)0), (int64_t)src.n - 1);
  }
  // byte offset of this wave's image in a dataset of EB-byte pixels (WIMG), wave-uniform
  template <int EB>
  DEV uint32_t wave_base(const XSrc& src) const {
    const int64_t r = (int64_t)(((uint64_t)wrow[1] << 32) | wrow[0]);
    const uint32_t row = (uint32_t)min(max(r, (int64_t)0), (int64_t)src.n - 1);
    return __builtin_amdgcn_readfirstlane(row * (uint32_t)(G::INTERIOR * EB));
  }
  // bf16 activations, or (first layer) a resident dataset gathered through the
  // batch index: uint8, normalised x/255 - 0.5 exactly like prep_images (K10 fused),
  // or bf16 already normalised (XSrc.x with idx set).
  // gathers: the row(s) of this group must have been fetched (fetch_rows one group earlier).
  // Branch-free buffer loads (common.h buf_*): invalid slots read zeros; the raw
  // uint8 words are converted only at store time, so no load is waited for here.
  bool u8mode = false;
  DEV void load(const XSrc& src, int img0, int B, int tid) {
    const int nimg = max(0, min(IMGS, B - img0));
    u8mode = U8 && src.u8 != nullptr;
    if constexpr (WIMG) {
      const int im = (tid >> 6) / WPI;
      const bool img_ok = im < nimg;
      if (src.u8) {
        const auto r = buf_rsrc(src.u8, (uint32_t)((int64_t)src.n * G::INTERIOR));
        const uint32_t base = wave_base<1>(src);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int j = tid % TPI + u * TPI;
          v[u] = u32x2{buf_b32(r, img_ok && j < VPI ? base + (uint32_t)j * 4u : BUF_OOB), 0u};
        }
      } else if (src.idx) {
        // resident bf16 dataset (already normalised): gathered 8-byte vectors, no conversion
        const auto r = buf_rsrc(src.x, (uint32_t)((int64_t)src.n * G::INTERIOR * 2));
        const uint32_t base = wave_base<2>(src);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int j = tid % TPI + u * TPI;
          v[u] = buf_b64(r, img_ok && j < VPI ? base + (uint32_t)j * 8u : BUF_OOB);
        }
      } else {
        const auto r = buf_rsrc(src.x + (int64_t)img0 * G::INTERIOR, (uint32_t)(nimg * G::INTERIOR * 2));
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = vec(u, tid);
          v[u] = buf_b64(r, e < NV ? (uint32_t)(e * 8) : BUF_OOB);
        }
      }
    } else if (U8 && src.u8) {
      const auto r = buf_rsrc(src.u8, (uint32_t)((int64_t)src.n * G::INTERIOR));
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = tid + u * NTH;
        const int im = e / VPI, rem = e - im * VPI;
        int row = row_of(src, 0);
#pragma unroll
        for (int k = 1; k < IMGS; ++k) row = im == k ? row_of(src, k) : row;
        const bool ok = e < NV && im < nimg;
        v[u] = u32x2{buf_b32(r, ok ? (uint32_t)(row * G::INTERIOR + rem * 4) : BUF_OOB), 0u};
      }
    } else if (U8 && src.idx) {
      const auto r = buf_rsrc(src.x, (uint32_t)((int64_t)src.n * G::INTERIOR * 2));
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = tid + u * NTH;
        const int im = e / VPI, rem = e - im * VPI;
        int row = row_of(src, 0);
#pragma unroll
        for (int k = 1; k < IMGS; ++k) row = im == k ? row_of(src, k) : row;
        const bool ok = e < NV && im < nimg;
        v[u] = buf_b64(r, ok ? (uint32_t)(row * G::INTERIOR * 2 + rem * 8) : BUF_OOB);
      }
    } else {
      const auto r = buf_rsrc(src.x + (int64_t)img0 * G::INTERIOR, (uint32_t)(nimg * G::INTERIOR * 2));
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = tid + u * NTH;
        v[u] = buf_b64(r, e < NV ? (uint32_t)(e * 8) : BUF_OOB);   // e*4 elements = the image-major interior
      }
    }
  }
  DEV u32x2 value(int u) const {
    if (!u8mode) return v[u];
    const uint32_t b4 = v[u][0];
    return u32x2{pack2(u8_norm(b4 & 0xff), u8_norm((b4 >> 8) & 0xff)),
                 pack2(u8_norm((b4 >> 16) & 0xff), u8_norm(b4 >> 24))};
  }
  // Called at the top of a group, where the previous group's prefetch loads (x, the
  // next row index, the dY staging) are all about to be consumed: one explicit
  // vmcnt(0) at this dominating point.  Without it the waitcnt pass, merging over the
  // per-lane staging branches, inserted full waits BEHIND the new gathered prefetch
  // loads (a whole memory latency per group in the gathered-input weight gradient).
  // NST: vector-memory STORES a thread issues after the prefetch loads (the previous
  // group's output copy-out): they may stay in flight (vmcnt counts loads and stores
  // in issue order).  NST < 0: no explicit wait.
  template <int NST = 0>
  static DEV void drain() {
    static_assert(NST < 64, "vmcnt is 6 bits");
    if constexpr (U8 && NST >= 0)   // vmcnt(NST), expcnt / lgkmcnt untouched
      __builtin_amdgcn_s_waitcnt((NST & 15) | ((NST >> 4) << 14) | 0x0F70);
  }
  // offset of vector e in the LDS tile
  static DEV int tile_off(int e) {
    const int im = e / VPI, rem = e - im * VPI;
    const int hh = rem / G::ROWV, vv = rem - hh * G::ROWV;
    return im * G::IMG_LDS + ((hh + G::PAD) * G::WS + G::X0) * G::CIN + 4 * vv;
  }
  // MODE 0 pair layouts (window-left pixels) read only the shifted copies 0 and 2 (the
  // window's column offset is even): each staged vector goes to copy 0 as one 8-byte
  // store and to copy 2 (copy2[j] = copy0[j + 2]) as two dword stores, so no
  // make_shifted pass -- its 2 reads + 3 writes per vector and one barrier per group.
  // c2off: LDS offset of copy 2 (2 * TSTR in the 4-copy layout).
  DEV void store_c02(bf16_t* tile, int tid, int c2off = 2 * G::TSTR) const {
    static_assert(G::MODE == 0 && G::X0 >= 2, "copy-2 writes start 2 elements before the interior");
    auto put = [&](int e, u32x2 val) {
      const int o = tile_off(e);
      *(u32x2*)(tile + o) = val;
      uint32_t* c2 = (uint32_t*)(tile + c2off + o - 2);
      c2[0] = val[0];
      c2[1] = val[1];
    };
    if (U8 && u8mode) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = vec(u, tid);
        if (e < NV) put(e, value(u));
      }
    } else {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = vec(u, tid);
        if (e < NV) put(e, v[u]);
      }
    }
  }
  // the uint8 conversion sits behind a uniform branch (a select made every bf16 staging
  // pay for it: ~10 VALU per vector)
  DEV void store(bf16_t* tile, int tid) const {
    if (U8 && u8mode) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = vec(u, tid);
        if (e < NV) *(u32x2*)(tile + tile_off(e)) = value(u);
      }
    } else {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = vec(u, tid);
        if (e < NV) *(u32x2*)(tile + tile_off(e)) = v[u];
      }
    }
  }
};

// MODE 0: derive the three shifted copies (copy_s[j] = copy_0[j + s]) of every image.
template <class G, int IMGS>
DEV void make_shifted(bf16_t* tile, int tid) {
  constexpr int NG = G::TSTR / 4;
  for (int e = tid; e < IMGS * NG; e += NTH) {
    const int im = e / NG, v = e - im * NG;
    bf16_t* src = tile + im * G::IMG_LDS;
    const u32x2 lo = *(const u32x2*)(src + 4 * v);
    const u32x2 hi = (v + 1 < NG) ? *(const u32x2*)(src + 4 * v + 4) : u32x2{0u, 0u};
    const uint32_t w0 = lo[0], w1 = lo[1], w2 = hi[0], w3 = hi[1];
    *(u32x2*)(src + 1 * G::TSTR + 4 * v) = u32x2{__builtin_amdgcn_alignbit(w1, w0, 16),
                                                 __builtin_amdgcn_alignbit(w2, w1, 16)};
    *(u32x2*)(src + 2 * G::TSTR + 4 * v) = u32x2{w1, w2};
    *(u32x2*)(src + 3 * G::TSTR + 4 * v) = u32x2{__builtin_amdgcn_alignbit(w2, w1, 16),
                                                 __builtin_amdgcn_alignbit(w3, w2, 16)};
  }
}

// Pooled gradient + argmax bytes ([img][window][Cout]), 8 channels per vector.
// LRNB: y is dL/d(LRN output) and p the LRN input (LrnFold); store() stages the
// LRN backward of them (bitwise lrn_bwd_k: same lrn_bwd8, same bf16 rounding).
template <class G, int IMGS, int LRNB = 0>   // LRNB: 0 no fold, 1 LRN fold, 2 LRN fold with beta = 0.75
struct DYStage {
  static constexpr int NWC = G::NWIN * G::COUT;
  static constexpr int NV = IMGS * NWC / 8;
  static constexpr int PER = (NV + NTH - 1) / NTH;
  static_assert(NWC % 8 == 0, "");
  static_assert(!LRNB || (G::COUT == 32 && NTH % (G::COUT / 8) == 0), "LRN fold: 4 lanes per pixel, radius 4");
  u32x4 y[PER];
  u32x2 a[PER];
  u32x4 p[LRNB ? PER : 1];
  DEV void load_lrn(const bf16_t* __restrict__ P, int img0, int B, int tid) {
    if constexpr (LRNB) {
      const int nimg = max(0, min(IMGS, B - img0));
      const auto rp = buf_rsrc(P + (int64_t)img0 * NWC, (uint32_t)(nimg * NWC * 2));
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int e = 8 * (tid + u * NTH);
        p[u] = buf_b128(rp, e < IMGS * NWC ? (uint32_t)(e * 2) : BUF_OOB);
      }
    }
  }
  // LRN backward in place (every lane takes part: the DPP exchanges read neighbours).
  // One vector at a time (scheduling barriers): interleaving all of them cost ~100
  // VGPRs of temporaries and two waves per SIMD.
  DEV void apply_lrn(const LrnFold& f, int tid) {
    if constexpr (LRNB) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        y[u] = lrn_bwd8<G::COUT / 8, 4, LRNB == 2>(p[u], y[u], tid % (G::COUT / 8), f.bias, f.alpha, f.beta, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // branch-free buffer loads: slots past the batch read dP = 0 and arg = 0, which
  // contribute nothing (every consumer multiplies / selects dP by the argmax)
  DEV void load(const bf16_t* __restrict__ dP, const uint8_t* __restrict__ arg, int img0, int B, int tid) {
    const int nimg = max(0, min(IMGS, B - img0));
    constexpr int AB = arg_bytes<G>();                 // arg bytes per window
    const auto ry = buf_rsrc(dP + (int64_t)img0 * NWC, (uint32_t)(nimg * NWC * 2));
    const auto ra = buf_rsrc(arg + (int64_t)img0 * G::NWIN * AB, (uint32_t)(nimg * G::NWIN * AB));
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = 8 * (tid + u * NTH);
      const bool ok = e < IMGS * NWC;
      y[u] = buf_b128(ry, ok ? (uint32_t)(e * 2) : BUF_OOB);
      if constexpr (arg_packed<G>())   // one window's 8 packed codes
        a[u] = u32x2{buf_b32(ra, ok ? (uint32_t)(e / 8 * AB) : BUF_OOB), 0u};
      else
        a[u] = buf_b64(ra, ok ? (uint32_t)e : BUF_OOB);
    }
  }
  DEV void store(bf16_t* dys, uint8_t* args, int tid) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = 8 * (tid + u * NTH);
      if (e < IMGS * NWC) {
        *(u32x4*)(dys + e) = y[u];
        *(u32x2*)(args + e) = a[u];
      }
    }
  }
};

// ------------------------------------------------------------------ forward
template <class G, int IMGS>
__global__ __launch_bounds__(NTH, fwd_minw<G>()) void convpool_fwd_k(const XSrc x, const bf16_t* __restrict__ w,
                                                      const float* __restrict__ bias, int bias_n, int B,
                                                      bf16_t* __restrict__ pooled, uint8_t* __restrict__ arg) {
  constexpr int LDS = (IMGS * G::IMG_LDS + 7) / 8 * 8;
  constexpr int OUTE = G::NWIN * G::COUT;              // pooled elements per image
  // small outputs (LeNet conv2: 400 per image) are staged in LDS and leave as 16-byte
  // vectors; wide ones (32 channels) keep direct 32-byte-per-row stores (LDS budget)
  constexpr bool STAGE = IMGS * OUTE * 3 <= 16384 && OUTE % 16 == 0;
  __shared__ __attribute__((aligned(16))) bf16_t tile[LDS];
  // staged: one spare window past the group absorbs the rows past the last pixel
  __shared__ __attribute__((aligned(16))) bf16_t pout[STAGE ? IMGS * OUTE + G::COUT : 8];
  __shared__ __attribute__((aligned(16))) uint8_t aout[STAGE ? IMGS * OUTE + G::COUT : 16];
  // small images (LeNet conv2: 112 fragment rows): fragment row -> pixel base offset from
  // an LDS table instead of ~20 VALU of window / position arithmetic per fragment
  constexpr bool PTAB = G::MF * 16 <= 128;
  __shared__ int ptab[PTAB ? G::MF * 16 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  lds_zero<LDS>(tile, tid);
  if constexpr (PTAB)
    for (int i = tid; i < G::MF * 16; i += NTH) {
      const int r = min(i, G::NPIX - 1);
      ptab[i] = G::wbase(r >> 2) + G::doff(r & 3);
    }

  // per-lane A-operand offsets: dd = run deltas (MODE 0: two 4-runs; MODE 1: one 8-run),
  // dl = scalar deltas (MODE 2)
  int dd[G::KSTEPS][2];
  int dl[G::MODE == 2 ? G::KSTEPS : 1][8];
  bf16x8 bfr[G::KSTEPS][G::NF];
#pragma unroll
  for (int s = 0; s < G::KSTEPS; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k0 = G::kslot(s, g, 4 * h);
      dd[s][h] = (G::MODE != 2 && k0 < G::KE) ? G::chunk_delta(k0) : 0;  // padded k: finite pixel, zero weight
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = G::kslot(s, g, j);
      if constexpr (G::MODE == 2) dl[s][j] = k < G::KC ? G::kdelta(k) : 0;
      bool valid;
      int wrow;
      if constexpr (G::MODE == 0) {
        valid = (k >> 3) < G::KS && (k & 7) < G::KS;
        wrow = (k >> 3) * G::KS + (k & 7);
      } else {
        valid = k < G::KC;
        wrow = k;
      }
#pragma unroll
      for (int nf = 0; nf < G::NF; ++nf) {
        const int n = nf * 16 + li;
        bfr[s][nf][j] = as_bf((valid && n < G::COUT) ? w[wrow * G::COUT + n] : (bf16_t)0);
      }
    }
  }
  float bs[G::NF];
#pragma unroll
  for (int nf = 0; nf < G::NF; ++nf) {
    const int n = nf * 16 + li;
    bs[nf] = n < bias_n ? bias[n] : 0.f;
  }

  const int stride = gridDim.x * IMGS;
  XStage<G, IMGS> xs;
  xs.fetch_rows(x, blockIdx.x * IMGS, B);
  xs.load(x, blockIdx.x * IMGS, B, tid);
  xs.fetch_rows(x, blockIdx.x * IMGS + stride, B);
  // staged outputs leave in the NEXT group's staging phase, before its prefetch loads
  // (see convpool_fwd_quad_k: stores pending behind a load make every wait vmcnt(0))
  auto copy_out = [&](int g0) {
    if constexpr (STAGE) {
      const int nimg = min(IMGS, B - g0);
      bf16_t* pg = pooled + (int64_t)g0 * OUTE;
      uint8_t* ag = arg + (int64_t)g0 * OUTE;
      constexpr int PV = IMGS * OUTE / 8, AV = IMGS * OUTE / 16;
#pragma unroll
      for (int u = 0; u < (PV + NTH - 1) / NTH; ++u) {
        const int e = tid + u * NTH;
        if (e < nimg * OUTE / 8) *(u32x4*)(pg + 8 * e) = *(const u32x4*)(pout + 8 * e);
      }
#pragma unroll
      for (int u = 0; u < (AV + NTH - 1) / NTH; ++u) {
        const int e = tid + u * NTH;
        if (e < nimg * OUTE / 16) *(u32x4*)(ag + 16 * e) = *(const u32x4*)(aout + 16 * e);
      }
    }
  };
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += stride) {
    __syncthreads();
    xs.store(tile, tid);
    if (img0 != (int)blockIdx.x * IMGS) copy_out(img0 - stride);   // the previous group's outputs
    __syncthreads();
    if constexpr (G::MODE == 0) {
      make_shifted<G, IMGS>(tile, tid);
      __syncthreads();
    }
    {   // unconditional prefetch (past the batch: buffer loads of nothing return 0), so
        // every path issues the same loads and the waitcnt pass keeps its counts exact
      xs.load(x, img0 + stride, B, tid);
      xs.fetch_rows(x, img0 + 2 * stride, B);
    }
    for (int f = wave; f < IMGS * G::MF; f += NTH / 64) {
      const int im = f / G::MF, fm = f - im * G::MF;
      const bf16_t* tb = tile + im * G::IMG_LDS;
      int pb;
      if constexpr (PTAB) {
        pb = ptab[fm * 16 + li];
      } else {
        const int r = min(fm * 16 + li, G::NPIX - 1);
        pb = G::wbase(r >> 2) + G::doff(r & 3);
      }
      f32x4 acc[G::NF];
#pragma unroll
      for (int nf = 0; nf < G::NF; ++nf) acc[nf] = f32x4{0.f, 0.f, 0.f, 0.f};
      // every A fragment of the chain is read before the first MFMA (a read-then-wait per
      // MFMA serialised the chain on LDS latency)
      bf16x8 a[G::KSTEPS];
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) {
        if constexpr (G::MODE == 2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) a[s][j] = as_bf(tb[pb + dl[s][j]]);
        } else if constexpr (G::MODE == 1) {
          a[s] = __builtin_bit_cast(bf16x8, *(const u32x4*)(tb + pb + dd[s][0]));
        } else {
          const s16x4 lo = *(const s16x4*)(tb + G::aligned_off(pb + dd[s][0]));
          const s16x4 hi = *(const s16x4*)(tb + G::aligned_off(pb + opaque(dd[s][1])));
          a[s] = join(lo, hi);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s)
#pragma unroll
        for (int nf = 0; nf < G::NF; ++nf)
          acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], bfr[s][nf], acc[nf], 0, 0, 0);
      // staged: windows past the last one (their rows are clamped copies of pixel
      // NPIX-1, not a real window) go to the spare window -- a select, not a branch
      const int win = (STAGE && fm * 4 + g >= G::NWIN) ? G::NWIN * (IMGS - im) : fm * 4 + g;
      if (STAGE || (win < G::NWIN && img0 + im < B)) {
        bf16_t* pimg = STAGE ? pout + im * OUTE : pooled + (int64_t)(img0 + im) * OUTE;
        uint8_t* aimg = STAGE ? aout + im * OUTE : arg + (int64_t)(img0 + im) * OUTE;
#pragma unroll
        for (int nf = 0; nf < G::NF; ++nf) {
          const int n = nf * 16 + li;
          if (n < G::COUT) {
            // relu(. + b) is monotone: pool the raw sums, then bias + ReLU once
            const f32x4 v = acc[nf];
            const float best = vmax(vmax(pos_embed(v[0], 0u), pos_embed(v[1], 1u)),
                                    vmax(pos_embed(v[2], 2u), pos_embed(v[3], 3u)));
            const float o = pos_clear(best) + bs[nf];
            pimg[win * G::COUT + n] = f2bf(vmax(o, 0.f));
            aimg[win * G::COUT + n] = (uint8_t)(o > 0.f ? pos_of(best) : ARG_OFF);
          }
        }
      }
    }
  }
  if constexpr (STAGE) {   // the last group's outputs
    __syncthreads();
    if ((int)blockIdx.x * IMGS < B) copy_out(blockIdx.x * IMGS + (B - 1 - (int)blockIdx.x * IMGS) / stride * stride);
  }
}

DEV float swap_half_row(float v) {  // lane i <-> lane i^8 within each 16-lane row (DPP row_ror:8)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false));
}
DEV int swap_half_row(int v) { return __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false); }

// ------------------------------------------------------------------ forward, Cin 1 / Cout 8 pair layout
// MFMA row i of a fragment = (pool window fm*8 + i/2, window row dy = i&1) at the
// window's LEFT column; column n = (channel c = n&7, side sx = n>>3).  Side 1 uses
// the weights shifted by one kw, i.e. it convolves the RIGHT-hand pixel, so one
// 16x16x32 MFMA chain produces a whole 2x2 window per (row pair, channel).  The
// pool max over dy stays in the lane, the max over dx is one DPP half-row swap,
// and every lane stores one (window, channel): 16 contiguous bf16 per row group.
template <class G, int IMGS>
__global__ __launch_bounds__(NTH) void convpool_fwd_pair_k(const XSrc x, const bf16_t* __restrict__ w,
                                                           const float* __restrict__ bias, int bias_n, int B,
                                                           bf16_t* __restrict__ pooled, uint8_t* __restrict__ arg) {
  static_assert(G::PAIR, "");
  constexpr int LDS = (IMGS * G::IMG_LDS + 7) / 8 * 8;
  constexpr int MFP = (G::NWIN + 7) / 8;  // fragments per image (8 windows each)
  __shared__ __attribute__((aligned(16))) bf16_t tile[LDS];
  __shared__ int wtab[G::NWIN];            // window -> aligned LDS offset of its top-left pixel
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int c = li & 7, sx = li >> 3;
  lds_zero<LDS>(tile, tid);
  for (int w = tid; w < G::NWIN; w += NTH) wtab[w] = G::aligned_off(G::wbase(w));

  int dd[G::KSTEPS][2];
  bf16x8 bfr[G::KSTEPS];
#pragma unroll
  for (int s = 0; s < G::KSTEPS; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k0 = 32 * s + 16 * h + 4 * g;
      dd[s][h] = k0 < G::KE ? G::chunk_delta(k0) : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 4 * g + (j & 3) + 16 * (j >> 2);
      const int kh = k >> 3, kw = (k & 7) - sx;
      const bool valid = kh < G::KS && kw >= 0 && kw < G::KS;
      bfr[s][j] = as_bf(valid ? w[(kh * G::KS + kw) * 8 + c] : (bf16_t)0);
    }
  }
  const float bs = c < bias_n ? bias[c] : 0.f;

  const int stride = gridDim.x * IMGS;
  XStage<G, IMGS> xs;
  xs.fetch_rows(x, blockIdx.x * IMGS, B);
  xs.load(x, blockIdx.x * IMGS, B, tid);
  xs.fetch_rows(x, blockIdx.x * IMGS + stride, B);
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += stride) {
    xs.template drain<-1>();
    __syncthreads();
    xs.store(tile, tid);
    __syncthreads();
    make_shifted<G, IMGS>(tile, tid);
    __syncthreads();
    {   // unconditional prefetch (past the batch: buffer loads of nothing return 0), so
        // every path issues the same loads and the waitcnt pass keeps its counts exact
      xs.load(x, img0 + stride, B, tid);
      xs.fetch_rows(x, img0 + 2 * stride, B);
    }
#pragma unroll 1
    for (int im = 0; im < IMGS; ++im) {
      const bf16_t* timg = tile + im * G::IMG_LDS;
      const bool img_ok = img0 + im < B;
      bf16_t* pimg = pooled + (int64_t)(img0 + im) * (G::NWIN * 8);
      uint8_t* aimg = arg + (int64_t)(img0 + im) * (G::NWIN * 8);
      for (int fm = wave; fm < MFP; fm += NTH / 64) {
        // dy = li&1 adds WS (a multiple of 4): same shifted copy as the window base
        const bf16_t* tb = timg + wtab[min(fm * 8 + (li >> 1), G::NWIN - 1)] + (li & 1) * G::WS;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < G::KSTEPS; ++s) {
          const bf16x8 a = join(*(const s16x4*)(tb + dd[s][0]), *(const s16x4*)(tb + opaque(dd[s][1])));
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[s], acc, 0, 0, 0);
        }
        // rows 4g+r: r=0,1 -> window 2g (dy 0,1); r=2,3 -> window 2g+1
        // one compare per pair feeds both the max and the argmax (no NaN-canonicalising fmaxf)
        const bool t0 = acc[1] > acc[0], t1 = acc[3] > acc[2];
        const float m0 = t0 ? acc[1] : acc[0], m1 = t1 ? acc[3] : acc[2];
        const int d0 = t0 ? 2 : 0, d1 = t1 ? 2 : 0;
        // side 0 owns window 2g, side 1 owns window 2g+1: trade the other window's column max
        const float oth = swap_half_row(sx ? m0 : m1);
        const int doth = swap_half_row(sx ? d0 : d1);
        const float L = sx ? oth : m0, R = sx ? m1 : oth;
        const int dL = sx ? doth : d0, dR = sx ? d1 : doth;
        const bool right = R > L;
        const int wo = fm * 8 + 2 * g + sx;
        if (wo < G::NWIN && img_ok) {
          const float o = (right ? R : L) + bs;
          pimg[wo * 8 + c] = f2bf(fmaxf(o, 0.f));
          aimg[wo * 8 + c] = (uint8_t)(o > 0.f ? (right ? dR + 1 : dL) : (int)ARG_OFF);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ forward, Cin 1 / Cout 8 quad layout (32x32x16)
// v_mfma_f32_32x32x16_bf16 with column n = (shift s = n>>3 in 0..3, channel c = n&7):
// one A row = 8 consecutive input pixels per kernel row (K = kh*8 + kw', kw' 0..7),
// and shift s convolves output column ow0 + s, so a row produces 4 horizontally
// adjacent outputs = 2 pool windows.  Row r = (quad qw = r/2, window row dy = r&1),
// quad = (pooled row ph, column pair pq): output columns 4pq..4pq+3.  The image sits
// in LDS ONCE with its interior at column X0 = 10, so every A run (input column
// 4pq - 2 + 10) is 8-byte aligned: two ds_read_b64, no shifted copies.
// Epilogue: dy max in-lane (accumulator rows 2m, 2m+1), dx max across lanes n, n^8
// (DPP half-row swap); each lane finalises 4 (window, channel) outputs.
struct QuadGeo {
  static constexpr int CIN = 1, H = 28, W = 28, PAD = 2, KS = 5, COUT = 8;
  static constexpr int HP = 32, X0 = 10, WS = 40;
  static constexpr int ROWV = W * CIN / 4;          // 4-pixel vectors per interior row
  static constexpr int INTERIOR = H * W;
  static constexpr int IMG_LDS = HP * WS;
  static constexpr int PW = 14, NWIN = 196, PQ = 7, NQUAD = 14 * 7;
  static_assert(PW == 2 * PQ, "window = 2 * quad + side");
  static constexpr int MFQ = (NQUAD + 15) / 16;     // 32-row fragments per image
  static_assert(4 * (PQ - 1) - PAD + X0 + 7 < WS, "A runs stay inside the row");
  static_assert((X0 - PAD) % 4 == 0 && WS % 4 == 0, "A runs are 8-byte aligned");
};

template <int IMGS>
__global__ __launch_bounds__(NTH) void convpool_fwd_quad_k(const XSrc x, const bf16_t* __restrict__ w,
                                                           const float* __restrict__ bias, int bias_n, int B,
                                                           bf16_t* __restrict__ pooled, uint8_t* __restrict__ arg) {
  using Q = QuadGeo;
  // one zero row past the last image: the kh = 5 A run (zero weight) of the bottom window row
  constexpr int LDS = IMGS * Q::IMG_LDS + Q::WS;
  constexpr int OUTE = Q::NWIN * 8;                 // pooled elements per image (16-byte multiple)
  constexpr int OUTS = Q::MFQ * 32 * 8;             // LDS stride per image: every fragment slot
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  __shared__ __attribute__((aligned(16))) bf16_t tile[LDS];
  // quad slot (fragment row pair) -> tile offset of its window row 0 A run; slots past
  // the last quad repeat it (their outputs are rewritten with identical values)
  __shared__ int qtab[Q::MFQ * 16];
  // STAGE_OUT: outputs of the block's image group are staged in LDS and written as
  // 16-byte vectors; otherwise each lane stores its (window, channel) directly
  constexpr bool STAGE_OUT = true;
  __shared__ __attribute__((aligned(16))) bf16_t pout[STAGE_OUT ? IMGS * OUTS : 8];
  __shared__ __attribute__((aligned(16))) uint8_t aout[STAGE_OUT ? IMGS * OUTS : 16];
  static_assert((OUTE * 2) % 16 == 0 && OUTE % 16 == 0 && STAGE_OUT, "");
  // wave index in an SGPR: the fragment / image bookkeeping below runs on the scalar unit
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 31, h = lane >> 5;
  const int s = n >> 3, c = n & 7, sp = s & 1, wp = s >> 1;
  lds_zero<LDS>(tile, tid);
  for (int i = tid; i < Q::MFQ * 16; i += NTH) {
    const int quad = min(i, Q::NQUAD - 1), ph = quad / Q::PQ, pq = quad - ph * Q::PQ;
    qtab[i] = 2 * ph * Q::WS + 4 * pq - Q::PAD + Q::X0;
  }

  // B operand: k = 16q + 8h + j -> (kh = 2q + h, kw' = j); shift s uses tap kw = kw' - s
  bf16x8 bfr[3];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kh = 2 * q + h, kw = j - s;
      const bool valid = kh < Q::KS && kw >= 0 && kw < Q::KS;
      bfr[q][j] = as_bf(valid ? w[(kh * Q::KS + kw) * Q::COUT + c] : (bf16_t)0);
    }
  const float bs = c < bias_n ? bias[c] : 0.f;
  // this lane's A row: r = lane & 31 -> quad qw = r >> 1, dy = r & 1
  const int r = lane & 31, qw = r >> 1, dyr = r & 1;

  const int stride = gridDim.x * IMGS;
  XStage<Q, IMGS> xs;
  xs.fetch_rows(x, blockIdx.x * IMGS, B);
  xs.load(x, blockIdx.x * IMGS, B, tid);
  xs.fetch_rows(x, blockIdx.x * IMGS + stride, B);
  // Copy-out of a group's staged outputs (pout / aout): 16-byte stores, the group's
  // outputs being contiguous in HBM.  It runs in the NEXT group's staging phase, before
  // that group's prefetch loads are issued: the waitcnt pass treats vmcnt as out of
  // order once loads and stores are both pending and waits vmcnt(0) for any load, so
  // stores issued after the prefetch (at the end of the group) were waited for at the
  // next loop top; issued before it, they drain during the compute phase.
  auto copy_out = [&](int g0) {
    const int nimg = min(IMGS, B - g0);
    bf16_t* pg = pooled + (int64_t)g0 * OUTE;
    uint8_t* ag = arg + (int64_t)g0 * (Q::NWIN * 4);
    constexpr int PV = IMGS * OUTE / 8;
#pragma unroll
    for (int u = 0; u < (PV + NTH - 1) / NTH; ++u) {
      const int e = tid + u * NTH, im = e / (OUTE / 8);
      if (e < nimg * (OUTE / 8))
        *(u32x4*)(pg + 8 * e) = *(const u32x4*)(pout + im * OUTS + 8 * (e - im * (OUTE / 8)));
    }
    // argmax codes packed 4 bits each (arg_packed<LeNetC1>): 16 output bytes = 4
    // windows (32 LDS bytes)
    constexpr int AV4 = IMGS * Q::NWIN / 4;
    static_assert(Q::NWIN % 4 == 0, "");
#pragma unroll
    for (int u = 0; u < (AV4 + NTH - 1) / NTH; ++u) {
      const int e = tid + u * NTH, im = e / (Q::NWIN / 4);
      if (e < nimg * (Q::NWIN / 4)) {
        const uint8_t* src = aout + im * OUTS + 32 * (e - im * (Q::NWIN / 4));
        const u32x4 lo = *(const u32x4*)src, hi = *(const u32x4*)(src + 16);
        *(u32x4*)(ag + 16 * e) = u32x4{lo[0] | lo[1] << 4, lo[2] | lo[3] << 4, hi[0] | hi[1] << 4, hi[2] | hi[3] << 4};
      }
    }
  };
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += stride) {
    __syncthreads();
    // interior rows at column X0 = 10 (4-byte aligned): two 4-byte stores per vector;
    // the uint8 conversion behind a uniform branch (not a per-vector select)
    auto stage = [&](auto conv) {
#pragma unroll
      for (int u = 0; u < XStage<Q, IMGS>::PER; ++u) {
        const int e = XStage<Q, IMGS>::vec(u, tid);
        if (e < XStage<Q, IMGS>::NV) {
          const int im = e / (Q::H * Q::ROWV), rem = e - im * (Q::H * Q::ROWV);
          const int hh = rem / Q::ROWV, vv = rem - hh * Q::ROWV;
          bf16_t* dst = tile + im * Q::IMG_LDS + (hh + Q::PAD) * Q::WS + Q::X0 + 4 * vv;
          const u32x2 val = conv(u);
          *(uint32_t*)dst = val[0];
          *(uint32_t*)(dst + 2) = val[1];
        }
      }
    };
    if (xs.u8mode) stage([&](int u) { return xs.value(u); });
    else stage([&](int u) { return xs.v[u]; });
    if (img0 != (int)blockIdx.x * IMGS) copy_out(img0 - stride);   // the previous group's outputs
    __syncthreads();
    {   // unconditional prefetch (past the batch: buffer loads of nothing return 0), so
        // every path issues the same loads and the waitcnt pass keeps its counts exact
      xs.load(x, img0 + stride, B, tid);
      xs.fetch_rows(x, img0 + 2 * stride, B);
    }
    // the group's IMGS x MFQ fragments are dealt over the waves as one flat list (a
    // per-image loop left wave 3 with 1 of every 7 fragments).  Measured neutral, as
    // were two MFMA chains per iteration and other grids (profiles/r2/conv1_fwd_experiments.md)
    constexpr int NFR = IMGS * Q::MFQ, NWV = NTH / 64;
    auto frag_base = [&](int f) {
      const int im = f / Q::MFQ, fm = f - im * Q::MFQ;
      // tile row of (oh + kh) for kh = h (+2q): oh = 2ph + dy; column 4pq - PAD + X0
      return tile + im * Q::IMG_LDS + qtab[fm * 16 + qw] + (dyr + h) * Q::WS;
    };
    auto epilogue = [&](int f, const f32x16& acc) {
      const int im = f / Q::MFQ, fm = f - im * Q::MFQ;
      bf16_t* pimg = pout + im * OUTS;
      uint8_t* aimg = aout + im * OUTS;
      // acc[i]: row (i&3) + 8(i>>2) + 4h -> quad t-slot t = i/2 (qw = (t&1) + 4(t>>1) + 2h),
      // dy = i&1; this lane's pixel column within the window is sp: position 2dy + sp
      float m[8];
#pragma unroll
      for (int t = 0; t < 8; ++t)
        m[t] = vmax(pos_embed(acc[2 * t], (uint32_t)sp), pos_embed(acc[2 * t + 1], 2u + sp));
      // lanes n and n^8 hold the left / right pixel of the same window; the even-s lane
      // finalises even t-slots, the odd-s lane odd ones
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float oth = swap_half_row(sp ? m[2 * u] : m[2 * u + 1]);
        const int t = 2 * u + sp;
        const float best = vmax(sp ? m[2 * u + 1] : m[2 * u], oth);
        // quad slot qt = fm*16 + (t&1) + 4(t>>1) + 2h = fm*16 + 4u + sp + 2h, window 2qt + wp
        // (ph*14 + 2pq + wp with qt = ph*7 + pq, PW == 2*PQ) = 32 fm (scalar) + 8u
        // (immediate) + a lane constant.
        // Slots past the last quad land in the per-image LDS padding (never copied out).
        const int win = 32 * fm + 8 * u + (2 * sp + 4 * h + wp);
        (void)t;
        const float o = pos_clear(best) + bs;
        pimg[win * 8 + c] = f2bf(vmax(o, 0.f));
        aimg[win * 8 + c] = (uint8_t)(o > 0.f ? pos_of(best) : ARG_OFF);
      }
    };
    auto afrag = [&](const bf16_t* tb, int q) {
      // kh = 2q + h; the padded kh = 5 (zero weight) reads the next row: finite, or the zero row
      const int rowoff = 2 * q * Q::WS;
      return join(*(const s16x4*)(tb + rowoff), *(const s16x4*)(tb + opaque(rowoff + 4)));
    };
    for (int f = wave; f < NFR; f += NWV) {
      const bf16_t* tb = frag_base(f);
      f32x16 acc = {};
#pragma unroll
      for (int q = 0; q < 3; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afrag(tb, q), bfr[q], acc, 0, 0, 0);
      epilogue(f, acc);
    }
  }
  // the last group's outputs
  __syncthreads();
  if ((int)blockIdx.x * IMGS < B) copy_out(blockIdx.x * IMGS + (B - 1 - (int)blockIdx.x * IMGS) / stride * stride);
}

// ------------------------------------------------------------------ weight gradient
// dW[k][n] = sum over pixels of im2col[pixel][k] * dY[pixel][n]: M = k, N = Cout,
// reduction = pixels (pool-window-major).  MODE 0/1 read the im2col^T operand
// with ds_read_b64_tr_b16: each lane supplies one pixel row and one 4-column
// chunk; the bias row (k = KE) reads a constant [1,0,0,0] LDS cell.  dY is
// rebuilt from (dP, arg): position d of a window gets dP iff arg == d.
template <class G, int IMGS, int LRNB = 0, bool PRIO = false>
__global__ __launch_bounds__(NTH, wgrad_minw<G>()) void convpool_wgrad_k(const XSrc x, const bf16_t* __restrict__ dP,
                                                        const uint8_t* __restrict__ arg, int B,
                                                        float* __restrict__ slab, const LrnFold lrn) {
  constexpr int CELL = IMGS * G::IMG_LDS;             // [1,0,0,0] then [0,0,0,0]
  constexpr int LDS = (CELL + 8 + 7) / 8 * 8;
  // FAST (LeNet conv2, 16 channels x 8-channel taps): dY is max-unpooled ONCE per group
  // into U2[img][channel][window] = the window's 4 positions (8 bytes), so a step's B
  // operand is two ds_read_b64 with no per-step select arithmetic; the A reads use
  // two per-window base registers + compile-time tap offsets (see below).  Row stride
  // 34 windows = 68 dwords (4 mod 64): the 16 channels x 2 lane groups of a half-wave
  // hit distinct bank pairs.  The cross-wave reduction reuses U2.
  constexpr bool FAST = G::MODE == 1 && G::COUT == 16 && G::CIN == 8 && !LRNB;
  constexpr int URW = 34, NWPAD = G::RSTEPS * 8;
  static_assert(!FAST || (URW >= NWPAD && (2 * URW) % 64 == 4), "U2 row stride");
  constexpr int U2E = FAST ? IMGS * G::COUT * URW * 4 : 4;   // bf16 elements
  __shared__ __attribute__((aligned(16))) bf16_t tile[LDS];
  __shared__ __attribute__((aligned(16))) bf16_t dys[FAST ? 8 : IMGS * G::NWIN * G::COUT];
  __shared__ __attribute__((aligned(16))) uint8_t args[FAST ? 16 : IMGS * G::NWIN * G::COUT];
  __shared__ __attribute__((aligned(16))) bf16_t U2[U2E];
  __shared__ float red_own[FAST ? 1 : G::KM * G::NCOL];
  __shared__ int wtab[FAST ? NWPAD : 1];
  static_assert(!FAST || U2E * 2 >= G::KM * G::NCOL * 4, "reduction reuses U2");
  float* const red = FAST ? (float*)U2 : red_own;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  lds_zero<LDS>(tile, tid);
  if constexpr (FAST) {
    lds_zero<U2E>(U2, tid);                        // windows >= NWIN stay zero
    for (int w = tid; w < NWPAD; w += NTH) wtab[w] = G::wbase(min(w, G::NWIN - 1));
  }
  __syncthreads();
  if (tid == 0) tile[CELL] = (bf16_t)0x3f80;

  // MODE 0/1: per-lane chunk delta of the tr-read column chunk (-1: bias cell, -2: zero cell)
  // MODE 2: per-lane scalar delta of im2col column k = mf*16 + li
  const int q = (lane >> 2) & 3, p = lane & 3;
  int cd[G::MFW];
  int kind[G::MFW];  // MODE 2: 0 im2col column, 1 bias ones-row, 2 zero pad
#pragma unroll
  for (int mf = 0; mf < G::MFW; ++mf) {
    if constexpr (G::MODE != 2) {
      const int k0 = mf * 16 + 4 * p;
      cd[mf] = k0 < G::KE ? G::chunk_delta(k0) : (k0 == G::KE ? -1 : -2);
      kind[mf] = 0;
    } else {
      const int k = mf * 16 + li;
      cd[mf] = k < G::KC ? G::kdelta(k) : 0;
      kind[mf] = k < G::KC ? 0 : (k == G::KC ? 1 : 2);
    }
  }
  f32x4 acc[G::MFW][G::NF];
#pragma unroll
  for (int mf = 0; mf < G::MFW; ++mf)
#pragma unroll
    for (int nf = 0; nf < G::NF; ++nf) acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int stride = gridDim.x * IMGS;
  XStage<G, IMGS> xs;
  DYStage<G, IMGS, LRNB> ys;
  xs.fetch_rows(x, blockIdx.x * IMGS, B);
  xs.load(x, blockIdx.x * IMGS, B, tid);
  xs.fetch_rows(x, blockIdx.x * IMGS + stride, B);
  ys.load(dP, arg, blockIdx.x * IMGS, B, tid);
  ys.load_lrn(lrn.p, blockIdx.x * IMGS, B, tid);
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += stride) {
    xs.drain();
    __syncthreads();
    xs.store(tile, tid);
    ys.apply_lrn(lrn, tid);
    if constexpr (FAST) {
      constexpr int NWC = G::NWIN * G::COUT;
#pragma unroll
      for (int u = 0; u < DYStage<G, IMGS, LRNB>::PER; ++u) {
        const int e = 8 * (tid + u * NTH);
        if (e < IMGS * NWC) {
          const int im = e / NWC, rem = e - im * NWC;
          const int win = rem / G::COUT, co0 = rem - win * G::COUT;
          bf16_t* urow = U2 + ((im * G::COUT + co0) * URW + win) * 4;
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            // y_c in both halves, d_c in all four bytes; byte b of a mask = table[d + k_b]
            // (0xff only at byte 3): positions (0, 1) -> k = (3, 3, 2, 2), (2, 3) -> (1, 1, 0, 0)
            const uint32_t y2 = __builtin_amdgcn_perm(0u, ys.y[u][c >> 1], (c & 1) ? 0x03020302u : 0x01000100u);
            const uint32_t r = __builtin_amdgcn_perm(0u, ys.a[u][c >> 2], 0x01010101u * (c & 3));
            *(u32x2*)(urow + c * URW * 4) = u32x2{y2 & __builtin_amdgcn_perm(0u, 0xff000000u, r + 0x02020303u),
                                                   y2 & __builtin_amdgcn_perm(0u, 0xff000000u, r + 0x00000101u)};
          }
        }
      }
    } else {
      ys.store(dys, args, tid);
    }
    __syncthreads();
    if constexpr (G::MODE == 0) {
      make_shifted<G, IMGS>(tile, tid);
      __syncthreads();
    }
    {   // unconditional prefetch (past the batch: buffer loads of nothing return 0), so
        // every path issues the same loads and the waitcnt pass keeps its counts exact
      xs.load(x, img0 + stride, B, tid);
      xs.fetch_rows(x, img0 + 2 * stride, B);
      ys.load(dP, arg, img0 + stride, B, tid);
      ys.load_lrn(lrn.p, img0 + stride, B, tid);
    }
    if constexpr (FAST) {
      // A operand: chunk k0 = 16 mf + 4p is tap t = 2mf + e (e = p >> 1), channels 4(p&1)..+3;
      // its LDS offset is off(2mf) (compile time) + 4(p&1) + e * 8, except when 2mf is the
      // last tap of a kernel row (2mf % KS == KS-1): then tap 2mf+1 starts the next row,
      // e * (WS - KS + 1) * 8 -- two base registers per window, every read an immediate.
      const int e1 = p >> 1;
      const int lane_a = 4 * (p & 1) + e1 * G::CIN;
      const int lane_b = 4 * (p & 1) + e1 * (G::WS - G::KS + 1) * G::CIN;
      auto toff = [](int t) constexpr { return ((t / G::KS) * G::WS + t % G::KS) * G::CIN; };
      // RSTEPS == waves (LeNet conv2: 4): every step of a wave has s = wave, so its window
      // bases are fixed -- computed here, not looked up in wtab ahead of each step's tr reads
      constexpr bool FIXS = G::RSTEPS == NTH / 64;
      const int fb0 = G::wbase(min(8 * wave + g, G::NWIN - 1)) + G::doff(q);
      const int fb1 = G::wbase(min(8 * wave + g + 4, G::NWIN - 1)) + G::doff(q);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      for (int it = wave; it < IMGS * G::RSTEPS; it += NTH / 64) {
        const int im = it / G::RSTEPS, s = FIXS ? wave : it - im * G::RSTEPS;
        const int w0 = 8 * s + g;
        const bf16_t* ub = U2 + ((im * G::COUT + li) * URW + w0) * 4;
        const bf16x8 bfr = join(*(const s16x4*)ub, *(const s16x4*)(ub + opaque(16)));
        // rows supplied by this lane: pixel q of windows w0 / w0 + 4 (clamped; dY is zero there)
        const bf16_t* t0 = tile + im * G::IMG_LDS + (FIXS ? fb0 : wtab[w0] + G::doff(q));
        const bf16_t* t1 = tile + im * G::IMG_LDS + (FIXS ? fb1 : wtab[w0 + 4] + G::doff(q));
#pragma unroll
        for (int mf = 0; mf < G::MFW; ++mf) {
          const bool rowend = (2 * mf) % G::KS == G::KS - 1;
          const int lo = rowend ? lane_b : lane_a;
          const bf16_t* a0 = t0 + lo + toff(2 * mf);
          const bf16_t* a1 = t1 + lo + toff(2 * mf);
          if (16 * mf + 16 > G::KE) {     // the fragment holding the bias / zero cells
            const int k0 = 16 * mf + 4 * p;
            if (k0 >= G::KE) a0 = a1 = tile + CELL + (k0 == G::KE ? 0 : 4);
          }
          const bf16x8 a = join(lds_tr4(a0), lds_tr4(a1));
          acc[mf][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr, acc[mf][0], 0, 0, 0);
        }
      }
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      continue;
    }
    for (int it = wave; it < IMGS * G::RSTEPS; it += NTH / 64) {
      const int im = it / G::RSTEPS, s = it - im * G::RSTEPS;
      // this lane's two pool windows for the 8 reduction slots
      const int w0 = 8 * s + g, w1 = w0 + 4;
      const bool v0 = w0 < G::NWIN, v1 = w1 < G::NWIN;
      const bf16_t* tb = tile + im * G::IMG_LDS;
      bf16x8 bfr[G::NF];
#pragma unroll
      for (int nf = 0; nf < G::NF; ++nf) {
        const int n = nf * 16 + li;
        const bool nv = n < G::COUT;
        const int i0 = (im * G::NWIN + w0) * G::COUT + n, i1 = (im * G::NWIN + w1) * G::COUT + n;
        const bf16_t y0 = (nv && v0) ? dys[i0] : (bf16_t)0, y1 = (nv && v1) ? dys[i1] : (bf16_t)0;
        const int a0 = (nv && v0) ? args[i0] : (int)ARG_OFF, a1 = (nv && v1) ? args[i1] : (int)ARG_OFF;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bfr[nf][d] = as_bf(a0 == d ? y0 : (bf16_t)0);
          bfr[nf][4 + d] = as_bf(a1 == d ? y1 : (bf16_t)0);
        }
      }
      if constexpr (G::MODE != 2) {
        // rows supplied by this lane: pixel q of windows w0 / w1 (clamped; dY is zero there)
        const int pb0 = G::wbase(min(w0, G::NWIN - 1)) + G::doff(q);
        const int pb1 = G::wbase(min(w1, G::NWIN - 1)) + G::doff(q);
#pragma unroll
        for (int mf = 0; mf < G::MFW; ++mf) {
          const int c = cd[mf];
          const int cell = CELL + (c == -1 ? 0 : 4);
          const int o0 = c >= 0 ? im * G::IMG_LDS + G::aligned_off(pb0 + c) : cell;
          const int o1 = c >= 0 ? im * G::IMG_LDS + G::aligned_off(pb1 + c) : cell;
          const bf16x8 a = join(lds_tr4(tile + o0), lds_tr4(tile + o1));
#pragma unroll
          for (int nf = 0; nf < G::NF; ++nf)
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[nf], acc[mf][nf], 0, 0, 0);
        }
      } else {
        const int b0 = v0 ? G::wbase(w0) : 0, b1 = v1 ? G::wbase(w1) : 0;
#pragma unroll
        for (int mf = 0; mf < G::MFW; ++mf) {
          bf16x8 a;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            bf16_t e0 = 0, e1 = 0;
            if (kind[mf] == 0) {
              e0 = v0 ? tb[b0 + G::doff(d) + cd[mf]] : (bf16_t)0;
              e1 = v1 ? tb[b1 + G::doff(d) + cd[mf]] : (bf16_t)0;
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

// ------------------------------------------------------------------ weight gradient, Cin 1 / Cout 8 pair layout
// Reduction slot t of a 32-slot step = (window 16*s + t/2, window row dy = t&1) at
// the window's LEFT column; output column (c, sx) pairs that left-pixel patch with
// the dY of pixel (dy, sx).  The right pixel's patch is the left one shifted by one
// kw, so R[kh*8+kw'][8+c] accumulates dW[kh][kw'-1][c]: the fold
// dW[m][c] = R[m][c] + R[m+1][8+c] is applied to the block partials, and the slab
// has the plain MODE 0 layout [KM][8].
//
// The unpooled dY lives in LDS as U[sx*8 + c][window][dy] (one dword per window),
// built once per image group from the (dP, arg) vectors, so the MFMA B operand of a
// step is two aligned ds_read_b64 (windows 16s+2g.. and +8) with no per-step unpool
// arithmetic.  Row stride 212 dwords (4 x odd): the 16 rows x 2 lane groups of a
// ds_read_b64 half-wave hit 64 distinct banks.  The unpool is byte-select arithmetic:
// v_perm replicates y_c into both halves and d_c into all four bytes, and a second
// v_perm turns (d_c + k) per byte into a 0xff/0x00 byte mask from a one-entry table
// (8 VALU per channel, no compares).  The bias gradient comes out of the MFMA: the
// lanes supplying im2col^T rows KE..KE+3 read a constant [1,0,0,0] cell, so row KE
// accumulates sum(dY) per column (deterministic MFMA order, no staging VALU).
template <class G, int IMGS, bool PRIO = false>
__global__ __launch_bounds__(NTH, 7) void convpool_wgrad_pair_k(const XSrc x,
                                                             const bf16_t* __restrict__ dP,
                                                             const uint8_t* __restrict__ arg, int B,
                                                             float* __restrict__ slab) {
  static_assert(G::PAIR, "");
  constexpr int RS = (2 * G::NWIN + 31) / 32;        // reduction steps per image
  constexpr int NWP = RS * 16;                        // windows incl. the zero tail of the last step
  constexpr int URS = 212;                            // U row stride in dwords (4 x odd, >= NWP)
  static_assert(URS >= NWP && URS % 8 == 4, "U row stride");
  constexpr int UIMG = 16 * URS;                      // dwords per image
  constexpr int NWC = G::NWIN * 8;
  // Only copies 0 and 2 are read (window-left columns are even: XOFF even, WS % 4 == 0).
  // One image per group: the tile holds just those two, copy 2 right after copy 0
  // (LDS 24.0 -> 19.5 KB per workgroup: 7 instead of 6 per CU); more images keep the
  // 4-copy stride.
  static_assert(G::XOFF % 2 == 0 && G::WS % 4 == 0, "window-left offsets are even");
  constexpr bool CMP = IMGS == 1;
  constexpr int C2OFF = CMP ? G::TSTR : 2 * G::TSTR;
  constexpr int TILE_E = CMP ? (2 * G::TSTR + 7) / 8 * 8 : (IMGS * G::IMG_LDS + 7) / 8 * 8;
  __shared__ __attribute__((aligned(16))) bf16_t tile[TILE_E];
  __shared__ __attribute__((aligned(16))) uint32_t U[IMGS * UIMG];   // also the bias combine at the end
  __shared__ int wtab[G::NWIN];            // window -> aligned LDS offset of its top-left pixel
  __shared__ __attribute__((aligned(8))) bf16_t one_cell[4];   // [1, 0, 0, 0]: im2col^T rows KE..KE+3
  // the cross-wave reduction reuses the image tile (written only after the barrier
  // that ends the main loop): 2 KB less LDS -> 6 instead of 5 workgroups per CU
  float* const red = (float*)tile;
  static_assert(TILE_E * 2 >= G::KM * 16 * 4, "reduction reuses the tile");
  static_assert(G::KE % 4 == 0 && G::KE + 4 <= G::KM, "bias chunk");
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  lds_zero<TILE_E>(tile, tid);
  lds_zero<IMGS * UIMG * 2>((bf16_t*)U, tid);          // windows >= NWIN stay zero
  for (int w = tid; w < G::NWIN; w += NTH) {
    const int a = G::wbase(w);                 // a & 3 is 0 or 2: copy 0, or copy 2 at C2OFF
    wtab[w] = (a & 3) ? a - 2 + C2OFF : a;
  }
  if (tid < 4) one_cell[tid] = tid == 0 ? (bf16_t)0x3f80 : (bf16_t)0;

  const int q = (lane >> 2) & 3, p = lane & 3;
  int cd[G::MFW];
#pragma unroll
  for (int mf = 0; mf < G::MFW; ++mf) {
    const int k0 = mf * 16 + 4 * p;
    cd[mf] = k0 < G::KE ? G::chunk_delta(k0) : 0;   // rows > KE+3: any valid pixel (never read back)
  }
  constexpr int MFB = G::KE / 16;                     // the fragment holding the bias chunk
  const bool bias_lane = 4 * p == G::KE % 16;
  f32x4 acc[G::MFW];
#pragma unroll
  for (int mf = 0; mf < G::MFW; ++mf) acc[mf] = f32x4{0.f, 0.f, 0.f, 0.f};

  // IMGS == 1: pixel bases of this wave's steps (wtab's values, computed in registers)
  constexpr int NSW = (RS + NTH / 64 - 1) / (NTH / 64);
  int pbs[NSW][2];
#pragma unroll
  for (int k = 0; k < NSW; ++k)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int w = min(16 * (wave + k * (NTH / 64)) + 2 * g + (q >> 1) + 8 * h, G::NWIN - 1);
      const int a = G::wbase(w);
      pbs[k][h] = ((a & 3) ? a - 2 + C2OFF : a) + (q & 1) * G::WS;
    }

  const int stride = gridDim.x * IMGS;
  XStage<G, IMGS> xs;
  DYStage<G, IMGS> ys;
  xs.fetch_rows(x, blockIdx.x * IMGS, B);
  xs.load(x, blockIdx.x * IMGS, B, tid);
  xs.fetch_rows(x, blockIdx.x * IMGS + stride, B);
  ys.load(dP, arg, blockIdx.x * IMGS, B, tid);
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += stride) {
    xs.drain();
    __syncthreads();
    xs.store_c02(tile, tid, C2OFF);   // copies 0 and 2 only: this layout reads no others
    // max-unpool into U: U[sx*8+c][w] = (dy0: arg==sx ? dP : 0, dy1: arg==2+sx ? dP : 0)
#pragma unroll
    for (int u = 0; u < DYStage<G, IMGS>::PER; ++u) {
      const int e = 8 * (tid + u * NTH);
      if (e < IMGS * NWC) {
        const int im = e / NWC, win = (e - im * NWC) >> 3;
        uint32_t* urow = U + im * UIMG + win;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          // y_c in both halves, d_c (0..3, ARG_OFF = 4) in all four bytes (packed codes:
          // byte c & 3, nibble c >> 2)
          const uint32_t y2 = __builtin_amdgcn_perm(0u, ys.y[u][c >> 1], (c & 1) ? 0x03020302u : 0x01000100u);
          uint32_t r;
          if constexpr (arg_packed<G>()) {
            const uint32_t t = __builtin_amdgcn_perm(0u, ys.a[u][0], 0x01010101u * (c & 3));
            r = ((c >> 2) ? t >> 4 : t) & 0x0f0f0f0fu;
          } else {
            r = __builtin_amdgcn_perm(0u, ys.a[u][c >> 2], 0x01010101u * (c & 3));
          }
          // byte b of the mask = table[d + k_b] with 0xff only at byte 3: set iff d == 3 - k_b.
          // side 0: (dy0, dy1) = positions (0, 2) -> k = (3, 3, 1, 1); side 1: (1, 3) -> (2, 2, 0, 0)
          urow[c * URS] = y2 & __builtin_amdgcn_perm(0u, 0xff000000u, r + 0x01010303u);
          urow[(8 + c) * URS] = y2 & __builtin_amdgcn_perm(0u, 0xff000000u, r + 0x00000202u);
        }
      }
    }
    __syncthreads();
    {   // unconditional prefetch (past the batch: buffer loads of nothing return 0), so
        // every path issues the same loads and the waitcnt pass keeps its counts exact
      xs.load(x, img0 + stride, B, tid);
      xs.fetch_rows(x, img0 + 2 * stride, B);
      ys.load(dP, arg, img0 + stride, B, tid);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    // one reduction step: dY operand from U, im2col^T rows at this lane's pixel bases pb0 / pb1
    auto step = [&](int im, int s, int pb0, int pb1) {
      // dY operand: element j <-> window 16s + 2g + ((j>>1)&1) + 8(j>>2), dy = j&1
      const uint32_t* ub = U + im * UIMG + li * URS + 16 * s + 2 * g;
      const bf16x8 bfr = join(*(const s16x4*)ub, *(const s16x4*)(ub + opaque(8)));
#pragma unroll
      for (int mf = 0; mf < G::MFW; ++mf) {
        const bf16_t* a0 = tile + pb0 + cd[mf];
        const bf16_t* a1 = tile + pb1 + cd[mf];
        if (mf == MFB) {
          a0 = bias_lane ? one_cell : a0;
          a1 = bias_lane ? one_cell : a1;
        }
        const bf16x8 a = join(lds_tr4(a0), lds_tr4(a1));
        acc[mf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr, acc[mf], 0, 0, 0);
      }
    };
    if constexpr (IMGS == 1) {
      // one image per group: a wave's steps s = wave + 4k are the same every group, so the
      // pixel bases were computed once (pbs) -- no wtab lookup ahead of the tr reads
#pragma unroll
      for (int k = 0; k < NSW; ++k)
        if (wave + k * (NTH / 64) < RS) step(0, wave + k * (NTH / 64), pbs[k][0], pbs[k][1]);
    } else {
      for (int it = wave; it < IMGS * RS; it += NTH / 64) {
        const int im = it / RS, s = it - im * RS;
        // im2col^T operand rows supplied by this lane: slot 4g+q (+16): window 16s + 2g + q/2 (+8), dy = q&1
        // (dy adds WS and the chunk deltas are multiples of 4: the copy is the window's)
        const int wq = 16 * s + 2 * g + (q >> 1);
        step(im, s, im * G::IMG_LDS + wtab[min(wq, G::NWIN - 1)] + (q & 1) * G::WS,
             im * G::IMG_LDS + wtab[min(wq + 8, G::NWIN - 1)] + (q & 1) * G::WS);
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  for (int wv = 0; wv < NTH / 64; ++wv) {
    __syncthreads();
    if (wave == wv) {
#pragma unroll
      for (int mf = 0; mf < G::MFW; ++mf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float& dst = red[(mf * 16 + 4 * g + r) * 16 + li];
          dst = (wv == 0) ? acc[mf][r] : dst + acc[mf][r];
        }
    }
  }
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * G::KM * 8;
  for (int e = tid; e < G::KM * 8; e += NTH) {
    const int m = e >> 3, cc = e & 7;
    float v = 0.f;
    if (m == G::KE) v = red[m * 16 + cc] + red[m * 16 + 8 + cc];   // left + right pixels' dY sums
    else if (m < G::KE) v = red[m * 16 + cc] + red[(m + 1) * 16 + 8 + cc];
    out[e] = v;
  }
}

// ------------------------------------------------------------------ data gradient, Cin 8 pair layout
// Row i of a fragment = input-pixel PAIR (ih = 2*mf + i/8, iw = 2*(i&7)): two
// image rows of 8 pairs (the 8th pair is padding for a 14-wide image), so with
// 48-byte pixels (a pair = 6 x 16 B) and a 256-byte-multiple row stride every
// ds_read_b128 lane group reads 16 distinct 16-byte bank groups.  Column n =
// (ci = n&7, side sx = n>>3): the dY patch row spans kw' = 0..KS (one extra tap)
// and side 1 uses the flipped filter shifted by one kw, i.e. it produces dx at
// (ih, iw + 1).  K-slot order: lane group g, element j -> tap 2s + g/2, co 8(g&1)+j,
// so each A fragment is ONE ds_read_b128.  The unpooled dY image lives in LDS
// with a KS-1-PAD halo.
//
// LA > 0 (A-row reuse): the A fragment of (fragment mf, k-step s) is the dY tile at
// row R = 2mf + kh(s) and tap pair c = s mod 3, so fragments mf and mf+1 share
// every row but their first / last two.  Each wave owns F consecutive fragments of
// one image and streams the rows R once (LA rows read ahead), issuing for each the
// MFMAs of every fragment it feeds: 3(2F+3) ds_read_b128 per wave instead of 15F --
// the kernel is LDS-bandwidth bound (105 x 1 KB of A reads per image otherwise).
// PRIO (default; MNISTX_DGRAD_PRIO=0 off): s_setprio 1 around each wave's MFMA phase, so the
// workgroups co-resident on a CU that are in their staging phase do not take the SIMD's
// issue slots from the ones feeding the matrix pipe (cdna_hip_programming.md T5)
template <class G, int IMGS, int DB = 0, int MINW = 1, int LA = 0, bool PRIO = false>
__global__ __launch_bounds__(NTH, MINW) void convpool_dgrad_pair_k(const bf16_t* __restrict__ dP,
                                                             const uint8_t* __restrict__ arg,
                                                             const bf16_t* __restrict__ w, int B,
                                                             bf16_t* __restrict__ dx) {
  static_assert(G::CIN == 8 && G::COUT == 16 && G::W % 2 == 0 && G::H % 2 == 0 && G::W <= 16, "pair dgrad layout");
  constexpr int Q = G::KS - 1 - G::PAD;
  constexpr int OHQ = G::OH + 2 * Q, OWQ = G::OW + 2 * Q;
  constexpr int DPS = G::COUT + 8;                    // 48-byte pixels: a pixel pair is 6 x 16 B
  // row stride = a multiple of 256 B: with 6-unit pixel pairs every ds_read_b128 lane
  // group ({0-3,12-15,20-27}, ...: MI355X_MICROARCH.md LDS table) hits 16 distinct
  // 16-byte bank groups (checked with bench/lds_sim.py)
  constexpr int RSE = (OWQ * DPS * 2 + 255) / 256 * 128;
  constexpr int DT = OHQ * RSE;
  constexpr int KWQ = G::KS + 1;
  constexpr int NTAP = G::KS * KWQ;
  constexpr int KSD = (NTAP + 1) / 2;                 // 2 taps x 16 co per 32-wide k-step
  constexpr int MFD = G::H / 2;                       // 2 image rows per fragment
  constexpr int NWC = G::NWIN * G::COUT;
  static_assert((IMGS * DT) % 8 == 0, "");
  static_assert(2 * 7 + KWQ - 1 < RSE / DPS, "padding pair's patch row stays inside the row stride");
  constexpr int OUTE = G::H * G::W * 8;              // dx elements per image
  static_assert(OUTE % 8 == 0, "");
  __shared__ __attribute__((aligned(16))) bf16_t dyt[IMGS * DT];
  __shared__ __attribute__((aligned(16))) bf16_t outs[IMGS * OUTE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int ci = li & 7, sx = li >> 3;
  lds_zero<IMGS * DT>(dyt, tid);

  // A-fragment tap of k-step s: tp = 2s + g/2; KWQ is even, so kh = (2s)/KWQ for both
  // g/2 and the tap offset is dtap_c(s) (compile time: a ds_read immediate) + the lane's
  // (g/2)*DPS + 8(g&1) (the padded last tap, tp = NTAP, reads a finite in-tile pixel
  // against a zero filter)
  static_assert(KWQ % 2 == 0 && 2 * (KSD - 1) + 1 <= NTAP, "tap split");
  auto dtap_c = [](int s) constexpr { return (2 * s / KWQ) * RSE + (2 * s % KWQ) * DPS; };
  const int lane_tap = (g >> 1) * DPS + 8 * (g & 1);
  bf16x8 bw[KSD];
#pragma unroll
  for (int s = 0; s < KSD; ++s) {
    const int tp = 2 * s + (g >> 1);
    const int kh = tp / KWQ, kwq = tp - kh * KWQ;
    const int kw = kwq - sx;
    const bool valid = tp < NTAP && kw >= 0 && kw < G::KS;
    const int tap = valid ? (G::KS - 1 - kh) * G::KS + (G::KS - 1 - kw) : 0;
    // the 8 co of one (tap, ci) are contiguous: one 16-byte load, zeroed for padded taps
    const u32x4 v = *(const u32x4*)(w + (tap * G::CIN + ci) * G::COUT + 8 * (g & 1));
    bw[s] = __builtin_bit_cast(bf16x8, valid ? v : u32x4{0u, 0u, 0u, 0u});
  }
  const int stride = gridDim.x * IMGS;
  DYStage<G, IMGS> ys;
  ys.load(dP, arg, blockIdx.x * IMGS, B, tid);
  // dx of a group leaves in the NEXT group's staging phase, before its prefetch loads
  // (see convpool_fwd_quad_k: stores pending behind a load make every wait vmcnt(0))
  auto copy_out = [&](int g0) {
    const int nimg = min(IMGS, B - g0);
    bf16_t* dg = dx + (int64_t)g0 * OUTE;
    constexpr int PV = IMGS * OUTE / 8;   // compile-time store count
#pragma unroll
    for (int u = 0; u < (PV + NTH - 1) / NTH; ++u) {
      const int e = tid + u * NTH;
      if (e < nimg * OUTE / 8) *(u32x4*)(dg + 8 * e) = *(const u32x4*)(outs + 8 * e);
    }
  };
  for (int img0 = blockIdx.x * IMGS; img0 < B; img0 += stride) {
    __syncthreads();
    // max-unpool: position d of a window receives dP where arg == d (arg 4: ReLU off)
#pragma unroll
    for (int u = 0; u < DYStage<G, IMGS>::PER; ++u) {
      const int e = 8 * (tid + u * NTH);
      if (e < IMGS * NWC) {
        const int im = e / NWC, rem = e - im * NWC;
        const int win = rem / G::COUT, co = rem - win * G::COUT;
        const int ph = win / G::PW, pw = win - ph * G::PW;
        // packed select: arg bytes 2k, 2k+1 spread to the two 16-bit halves of E[k]
        // (one v_perm), then per position d the halves equal to d become 0xffff
        // masks with two packed u16 ops -- 4 ops per word instead of a compare and a
        // select per element
        uint32_t E[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          E[k] = __builtin_amdgcn_perm(0u, ys.a[u][k >> 1], (k & 1) ? 0x0c030c02u : 0x0c010c00u);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int oh = 2 * ph + (d >> 1) + Q, ow = 2 * pw + (d & 1) + Q;
          u32x4 o;
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = ys.y[u][k] & half_eq_mask(E[k], (uint32_t)d);
          *(u32x4*)(dyt + im * DT + oh * RSE + ow * DPS + co) = o;
        }
      }
    }
    // the previous group's dx: after the staging consumed the prefetched loads (a wait
    // for them behind pending stores would be vmcnt(0)), before the next prefetch
    if (img0 != (int)blockIdx.x * IMGS) copy_out(img0 - stride);
    __syncthreads();
    ys.load(dP, arg, img0 + stride, B, tid);   // unconditional: past the batch loads return 0
    if constexpr (LA > 0) {
      static_assert(KWQ == 6 && KSD == 15 && (NTH / 64) % IMGS == 0, "row reuse: 5 tap rows x 3 tap pairs");
      constexpr int WPI = (NTH / 64) / IMGS;          // waves per image
      const int im = wave / WPI, k = wave - im * WPI;
      const int mf0 = k * MFD / WPI, F = (k + 1) * MFD / WPI - mf0;
      const bf16_t* tb0 = dyt + im * DT + (2 * mf0 + (li >> 3)) * RSE + 2 * (li & 7) * DPS + lane_tap;
      bf16_t* oimg = outs + im * OUTE;
      auto run = [&](auto FC) {
        constexpr int FF = decltype(FC)::value;
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
        constexpr int NR = 2 * FF + 3;                 // rows R' = kh + 2j, kh 0..4, j < FF
        f32x4 acc[FF];
#pragma unroll
        for (int j = 0; j < FF; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        bf16x8 a[LA + 1][3];
        auto load_row = [&](int r) {
#pragma unroll
          for (int c = 0; c < 3; ++c)
            a[r % (LA + 1)][c] = __builtin_bit_cast(bf16x8, *(const u32x4*)(tb0 + r * RSE + 2 * c * DPS));
        };
#pragma unroll
        for (int r = 0; r < LA; ++r) load_row(r);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          if (r + LA < NR) load_row(r + LA);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int j = 0; j < FF; ++j) {
              const int kh = r - 2 * j;
              if (kh >= 0 && kh < G::KS)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r % (LA + 1)][c], bw[3 * kh + c], acc[j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < FF; ++j) {
          const int ih = 2 * (mf0 + j) + (g >> 1);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int jr = 4 * (g & 1) + r;
            if (2 * jr < G::W) oimg[(ih * G::W + 2 * jr + sx) * 8 + ci] = f2bf(acc[j][r]);
          }
        }
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      };
      constexpr int FMAX = (MFD + WPI - 1) / WPI, FMIN = MFD / WPI;
      static_assert(FMAX - FMIN <= 1, "");
      if (F == FMAX) run(std::integral_constant<int, FMAX>{});
      else run(std::integral_constant<int, FMIN>{});
    }
    // the group's 2 x MFD fragments are dealt over the 4 waves together (balance)
    for (int f = wave; LA == 0 && f < IMGS * MFD; f += NTH / 64) {
      const int im = f / MFD, mf = f - im * MFD;
      const bf16_t* tb = dyt + im * DT + (2 * mf + (li >> 3)) * RSE + 2 * (li & 7) * DPS + lane_tap;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      // all A fragments (DB = 0) or batches of DB in flight before their MFMAs: one read
      // ahead left every MFMA waiting out a full LDS latency (wait_any 57 %, MFMA busy 38 %)
      constexpr int NB = DB == 0 ? KSD : DB;
#pragma unroll
      for (int b = 0; b < KSD; b += NB) {
        bf16x8 a[NB];
#pragma unroll
        for (int s = 0; s < NB; ++s)
          if (b + s < KSD) a[s] = __builtin_bit_cast(bf16x8, *(const u32x4*)(tb + dtap_c(b + s)));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < NB; ++s)
          if (b + s < KSD) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], bw[b + s], acc, 0, 0, 0);
      }
      // accumulator rows 4g + r: image row 2mf + g/2, pair jr = 4(g&1) + r -> LDS staging
      const int ih = 2 * mf + (g >> 1);
      bf16_t* oimg = outs + im * OUTE;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int jr = 4 * (g & 1) + r;
        if (2 * jr < G::W) oimg[(ih * G::W + 2 * jr + sx) * 8 + ci] = f2bf(acc[r]);
      }
    }
  }
  __syncthreads();   // the last group's dx
  if ((int)blockIdx.x * IMGS < B) copy_out(blockIdx.x * IMGS + (B - 1 - (int)blockIdx.x * IMGS) / stride * stride);
}

int grid_for(int B, int imgs, int cap) {
  int n = (B + imgs - 1) / imgs;
  return cap_grid(n < cap ? (n < 1 ? 1 : n) : cap);
}

// Workgroups that fill every CU exactly once (occupancy API, cached per kernel):
// the persistent grid-stride kernels get one resident wave and no partial last round.
template <auto KER>   // the kernel itself is the key: kernels with one signature share a type
int resident_grid() {
  static int n = 0;
  if (n == 0) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, KER, NTH, 0) == hipSuccess &&
        hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && per_cu > 0)
      n = per_cu * cus;
    else
      n = 2048;
  }
  return n;
}

template <class G, int IMGS>
hipError_t run_fwd(const XSrc& x, const bf16_t* w, const float* bias, int bias_n, int B, bf16_t* pooled, uint8_t* arg,
                   hipStream_t st) {
  if constexpr (G::PAIR && G::H == 28 && G::W == 28 && G::PAD == 2) {
    // two resident rounds (2048 blocks) measured 5 % faster than one for this kernel (same-box
    // A/B); 3 images per group (LDS 29.1 -> 21.8 KB, 5 -> 7 WGs/CU) measured no faster
    hipLaunchKernelGGL((convpool_fwd_quad_k<4>), dim3(grid_for(B, 4, 2048)), dim3(NTH), 0, st, x, w, bias, bias_n, B,
                       pooled, arg);
  } else if constexpr (G::PAIR) {
    hipLaunchKernelGGL((convpool_fwd_pair_k<G, IMGS>), dim3(grid_for(B, IMGS, 2048)), dim3(NTH), 0, st, x, w, bias,
                       bias_n, B, pooled, arg);
  } else {
    hipLaunchKernelGGL((convpool_fwd_k<G, IMGS>), dim3(grid_for(B, IMGS, resident_grid<convpool_fwd_k<G, IMGS>>())),
                       dim3(NTH), 0, st, x, w, bias, bias_n,
                       B, pooled, arg);
  }
  return hipGetLastError();
}

template <class G, int IMGS>
hipError_t run_wgrad(const XSrc& x, const bf16_t* dP, const uint8_t* arg, int B, float* slab, int grid,
                     hipStream_t st, const LrnFold& lrn = LrnFold{nullptr, 0.f, 0.f, 0.f}) {
  // s_setprio 1 around the MFMA phase (see convpool_dgrad_pair_k; backward phase 348 ->
  // 338-339 us, profiles/r3/lenet/bwd_prio_ab.txt)
  if constexpr (G::PAIR) {
    if (lrn.p) return hipErrorInvalidValue;
    hipLaunchKernelGGL((convpool_wgrad_pair_k<G, IMGS, true>), dim3(grid), dim3(NTH), 0, st, x, dP, arg, B, slab);
  } else if constexpr (G::COUT == 32) {
    if (lrn.p && lrn.beta == 0.75f)   // the reference's beta: pow_beta<true> (lrn_math.h)
      hipLaunchKernelGGL((convpool_wgrad_k<G, IMGS, 2>), dim3(grid), dim3(NTH), 0, st, x, dP, arg, B, slab, lrn);
    else if (lrn.p)
      hipLaunchKernelGGL((convpool_wgrad_k<G, IMGS, 1>), dim3(grid), dim3(NTH), 0, st, x, dP, arg, B, slab, lrn);
    else
      hipLaunchKernelGGL((convpool_wgrad_k<G, IMGS>), dim3(grid), dim3(NTH), 0, st, x, dP, arg, B, slab, lrn);
  } else {
    if (lrn.p) return hipErrorInvalidValue;
    hipLaunchKernelGGL((convpool_wgrad_k<G, IMGS, 0, true>), dim3(grid), dim3(NTH), 0, st, x, dP, arg, B, slab, lrn);
  }
  return hipGetLastError();
}

template <class G, int IMGS>
hipError_t run_dgrad(const bf16_t* dP, const uint8_t* arg, const bf16_t* w, int B, bf16_t* dx, int grid_cap,
                     hipStream_t st) {
  // grid_cap > 0: fewer persistent blocks than one resident wave, leaving CU slots
  // for a kernel running concurrently on another stream (overlapped backward).
  // Two images per group, A-row reuse with one row read ahead (158 VGPRs, 3 waves/SIMD):
  // 120 us at B = 65536; one image with the 15 A fragments in batches of 8 (122 VGPRs,
  // 4 waves) measured 134 us, two images with all 15 in flight 143-149 us.  MFMA-phase
  // priority on (backward phase 348 -> 338-339 us, profiles/r3/lenet/bwd_prio_ab.txt).
  int cap = resident_grid<convpool_dgrad_pair_k<G, 2, 0, 3, 1, true>>();
  if (grid_cap > 0 && grid_cap < cap) cap = grid_cap;
  cap = cap_grid(cap);
  hipLaunchKernelGGL((convpool_dgrad_pair_k<G, 2, 0, 3, 1, true>), dim3(grid_for(B, 2, cap)), dim3(NTH), 0, st, dP, arg,
                     w, B, dx);
  return hipGetLastError();
}

using LeNetC1 = Geo<1, 8, 5, 2, 28, 28>;
// conv1 wgrad: one image per group (LDS 25.7 KB -> 6 workgroups / CU); two images per
// group (~52 KB, 3 workgroups / CU) measured slower (profiles/r3/lenet/knobs/)
constexpr int WG_IMGS_C1 = 1;
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

template <class G>
void reduce_layout(int* out) {
  out[0] = G::RED_G;
  out[1] = G::RED_IP;
  out[2] = G::MODE == 0 ? G::KS : -1;  // real inner count (-1: the layer's real Cin)
  out[3] = G::KE;
}

int convpool_reduce_layout(int cfg, int* out) {
  switch (cfg) {
    case 0: reduce_layout<LeNetC1>(out); return 0;
    case 1: reduce_layout<LeNetC2>(out); return 0;
    case 2: reduce_layout<RefC1g>(out); return 0;
    case 3: reduce_layout<RefC1c>(out); return 0;
  }
  return -1;
}

hipError_t convpool_fwd(int cfg, const XSrc& x, const bf16_t* w, const float* bias, int bias_n, int B,
                        bf16_t* pooled, uint8_t* arg, hipStream_t st) {
  switch (cfg) {
    case 0: return run_fwd<LeNetC1, 2>(x, w, bias, bias_n, B, pooled, arg, st);
    case 1: return run_fwd<LeNetC2, 4>(x, w, bias, bias_n, B, pooled, arg, st);
    case 2:
      if (refc1_band_enabled()) return refc1_band_fwd(x, w, bias, bias_n, B, pooled, arg, st);
      return run_fwd<RefC1g, 2>(x, w, bias, bias_n, B, pooled, arg, st);
    case 3:
      if (refc1_fwd3_ok() && !x.u8) return refc1_band_fwd(x, w, bias, bias_n, B, pooled, arg, st, nullptr, 0.f, 0.f, 0.f, 3);
      return run_fwd<RefC1c, 4>(x, w, bias, bias_n, B, pooled, arg, st);
  }
  return hipErrorInvalidValue;
}

hipError_t convpool_wgrad(int cfg, const XSrc& x, const bf16_t* dP, const uint8_t* arg, int B, float* slab,
                          int grid, hipStream_t st, const bf16_t* lrn_p, float lrn_bias, float lrn_alpha,
                          float lrn_beta) {
  const LrnFold lrn{lrn_p, lrn_bias, lrn_alpha, lrn_beta};
  if (lrn_p && cfg != 2 && cfg != 3) return hipErrorInvalidValue;
  switch (cfg) {
    case 0:
      return run_wgrad<LeNetC1, WG_IMGS_C1>(x, dP, arg, B, slab, grid, st);
    case 1: return run_wgrad<LeNetC2, 4>(x, dP, arg, B, slab, grid, st);
    // the LRN fold stages one image per group (its LRN input vectors and temporaries
    // would push the 2-image variant past 256 VGPRs: one wave per SIMD)
    case 2: return lrn_p ? run_wgrad<RefC1g, 1>(x, dP, arg, B, slab, grid, st, lrn)
                         : run_wgrad<RefC1g, 2>(x, dP, arg, B, slab, grid, st);
    case 3: return lrn_p ? run_wgrad<RefC1c, 1>(x, dP, arg, B, slab, grid, st, lrn)
                         : run_wgrad<RefC1c, 2>(x, dP, arg, B, slab, grid, st);
  }
  return hipErrorInvalidValue;
}

template <class G, int IMGS>
int wgrad_grid_for() {
  int per_cu = 0, dev = 0, cus = 0;
  if constexpr (G::PAIR) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, convpool_wgrad_pair_k<G, IMGS>, NTH, 0) != hipSuccess)
      return -1;
  } else {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, convpool_wgrad_k<G, IMGS>, NTH, 0) != hipSuccess)
      return -1;
  }
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  return per_cu * cus;
}

// One resident wave of wgrad workgroups (every CU full, nothing queued): the
// persistent grid-stride loop then gives every block the same image count, and
// the slab has exactly one partial per resident block.
int convpool_wgrad_grid(int cfg) {
  switch (cfg) {
    case 0:
      return wgrad_grid_for<LeNetC1, WG_IMGS_C1>();
    case 1: return wgrad_grid_for<LeNetC2, 4>();
    case 2: return wgrad_grid_for<RefC1g, 2>();
    case 3: return wgrad_grid_for<RefC1c, 2>();
  }
  return -1;
}

int convpool_has_dgrad(int cfg) { return cfg == 1 ? 1 : 0; }

int convpool_arg_bytes(int cfg) {
  switch (cfg) {
    case 0: return arg_bytes<LeNetC1>();
    case 1: return arg_bytes<LeNetC2>();
    case 2: return arg_bytes<RefC1g>();
    case 3: return arg_bytes<RefC1c>();
    default: return -1;
  }
}

// first layers that gather a resident dataset: Cin == 1 (LeNet / reference conv1) and the
// reference conv1 on 3-channel records
int convpool_u8_input(int cfg) { return (cfg == 0 || cfg == 2 || cfg == 3) ? 1 : 0; }

hipError_t convpool_dgrad(int cfg, const bf16_t* dP, const uint8_t* arg, const bf16_t* w, int B, bf16_t* dx,
                          int grid_cap, hipStream_t st) {
  switch (cfg) {
    case 1: return run_dgrad<LeNetC2, 2>(dP, arg, w, B, dx, grid_cap, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace mnistx
