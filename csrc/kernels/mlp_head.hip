// Fused dense head of LeNet-5: fc3 (400->120, ReLU), fc4 (120->84, ReLU), fc5
// (84->10), softmax cross-entropy, and the whole data-gradient chain
// (dlogits -> dh4 -> dh3 -> dX) in ONE kernel.  The layered path runs the same
// math as 8 launches (3 dense fwd, softmax-CE, 3 dense dgrad) that re-read every
// activation from HBM; here each activation is written once (the weight
// gradients and eval need them) and never read back.
//
// Reference: the LeNet-5 head of models (SURVEY.md §2 model families; the TF
// graph's fully-connected layers + tf.nn.sparse_softmax_cross_entropy_with_logits,
// mnist_input.py:185-205 for the reference CNN's equivalent head).
//
// CDNA4 mapping
//  * One 512-thread block per 256 batch rows; each wave owns 32 rows.  All three
//    weight matrices stay resident in LDS (137 KB) as natural W^T images (row =
//    output unit), copied once per block from W^T bf16 copies that the fused
//    optimizer keeps next to the normal ones (no transposes in this kernel).
//  * Every product is computed transposed, h^T = W^T . x^T, with
//    v_mfma_f32_32x32x16_bf16: the batch row is the lane (column) and features are
//    the accumulator registers, so an accumulator tile is directly the B operand
//    of the next product (k-slot j of lane half h at step s = feature
//    16s + 8(j>>2) + 4h + (j&3); cdna_hip_programming.md "accumulator as the next
//    MFMA's operand").  No LDS round trip between layers, forward or backward.
//  * Forward A fragments are row reads of the images (one ds_read_b128; the fc4 /
//    fc5 images store columns with bits 2 and 3 swapped so the permuted k-slots are
//    contiguous); backward A fragments (W instead of W^T) are ds_read_b64_tr_b16
//    transposed reads of the SAME images.  16-byte-chunk XOR swizzles (chosen with
//    bench/lds_sim.py) make both kinds of read conflict-free.
//  * ReLU masks for the backward come from the bf16 activations still held in
//    registers; CE statistics use the deterministic block/ticket combine.
//  * Outputs leave through a per-wave 2 KB LDS tile, so each lane stores 16
//    contiguous bytes of a batch row instead of 8-byte feature fragments.
//  Measured (B = 65536, bench/micro_mlp_head.py): 48 us for ~164 MB of HBM traffic,
//  vs ~130 us for the 8 layered launches it replaces.
#include "ce_stats.h"
#include "common.h"
#include "launchers.h"

#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace mnistx {
namespace {

constexpr int NTH = 512, NWAVE = NTH / 64, ROWS = 32 * NWAVE;
constexpr int D0 = 400;                  // fc3 input (5x5x16 NHWC flatten)
constexpr int LD1 = 120, LD2 = 88, LD3 = 16;  // storage widths of h3, h4, logits
constexpr int T1 = 4, T2 = 3, TX = 13;   // 32-row tiles of fc3 out (128), fc4 out (96), dX (416)
constexpr int K1 = D0 / 16;              // k-steps of fc3
// LDS images (bf16 elements): rows x stride
constexpr int R3 = 32 * T1, S3 = 32 * TX;  // fc3 W^T: 128 x 416 (832-byte rows)
constexpr int R4 = 32 * T2, S4 = 160;      // fc4 W^T:  96 x 128 (320-byte rows), columns permuted
constexpr int R5 = LD3, S5 = 32 * T2;      // fc5 W^T:  16 x 96 (192-byte rows), columns permuted
static_assert(D0 % 16 == 0 && 32 * TX >= D0 && 32 * T1 >= LD1 && 32 * T2 >= LD2, "head geometry");

DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }

// 16-byte-chunk XOR swizzle per image (bench/lds_sim.py: conflict-free row reads
// AND transposed reads); `col` and the result are in elements.
template <int IMG>
DEV int swz(int r) { return IMG == 4 ? (r & 15) : ((r >> 2) & 3); }
template <int IMG>
DEV int ioff(int r, int col) {
  constexpr int S = IMG == 3 ? S3 : IMG == 4 ? S4 : S5;
  return r * S + ((((col >> 3) ^ swz<IMG>(r)) << 3) | (col & 7));
}
// column permutation of the fc4 / fc5 images: swap bits 2 and 3
DEV int p23(int c) { return (c & ~12) | ((c >> 1) & 4) | ((c << 1) & 8); }

DEV uint32_t half16(const u32x4& v, int f) { return (f & 1) ? (v[f >> 1] >> 16) : (v[f >> 1] & 0xffffu); }

// The LDS images are filled from the optimizer-maintained transposed bf16 copies
// W^T [R][C] (zero-padded; FlatParams.enable_transposed): straight 16-byte chunk
// copies, chunk k of row n to its swizzled (and, for PERM images, bit-2/3-permuted)
// place.  load_img issues the global loads, store_img writes them.
template <int R, int C, int NT>
struct ImgChunks {
  static constexpr int N = R * C / 8, PER = (N + NT - 1) / NT;
  u32x4 v[PER];
};
template <int R, int C, int NT>
DEV void load_img(ImgChunks<R, C, NT>& ch, const bf16_t* __restrict__ WT, int tid) {
#pragma unroll
  for (int i = 0; i < ImgChunks<R, C, NT>::PER; ++i) {
    const int b = tid + i * NT;
    if (b < ImgChunks<R, C, NT>::N) ch.v[i] = *(const u32x4*)(WT + (int64_t)b * 8);
  }
}
template <int IMG, bool PERM, int R, int C, int NT>
DEV void store_img(bf16_t* img, const ImgChunks<R, C, NT>& ch, int tid) {
#pragma unroll
  for (int i = 0; i < ImgChunks<R, C, NT>::PER; ++i) {
    const int b = tid + i * NT;
    if (b >= ImgChunks<R, C, NT>::N) break;
    const int r = b / (C / 8), c = (b % (C / 8)) * 8;
    const u32x4 o = ch.v[i];
    if constexpr (!PERM) {
      *(u32x4*)(img + ioff<IMG>(r, c)) = o;
    } else {
      *(u32x2*)(img + ioff<IMG>(r, p23(c))) = u32x2{o[0], o[1]};
      *(u32x2*)(img + ioff<IMG>(r, p23(c + 4))) = u32x2{o[2], o[3]};
    }
  }
}

DEV bf16x8 as_frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(bf16x8, u32x4{a, b, c, d});
}

// bf16 activation (low / high half of a packed word) > 0, as the layered path's mask test
DEV bool pos_lo(uint32_t w) { return __uint_as_float(w << 16) > 0.f; }
DEV bool pos_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u) > 0.f; }

// Per-wave 32 x 32 bf16 staging tile (64-byte rows, chunk ^= (row>>1)&3: conflict-free
// reads, 2-way writes -- bench/lds_sim.py).  An accumulator tile holds a FEATURE
// column per lane; staged, each lane stores 16 contiguous bytes of a batch row.
constexpr int STG = 32 * 32;
DEV int soff(int row, int col) { return row * 32 + ((((col >> 3) ^ ((row >> 1) & 3)) << 3) | (col & 7)); }

// pk[w] = packed features 8(w>>1) + 4h + 2(w&1) + {0,1} of batch row lane&31 (the
// packed accumulator layout); writes out[m0 + row][c0 + j] for j < ncols.
DEV void store_tile(bf16_t* stg, const uint32_t* pk, bf16_t* __restrict__ out, int ld, int m0, int nb, int c0,
                    int ncols, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int q = 0; q < 4; ++q) *(u32x2*)(stg + soff(r, 8 * q + 4 * h)) = u32x2{pk[2 * q], pk[2 * q + 1]};
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = 16 * p + (lane >> 2), ch = lane & 3;
    const u32x4 v = *(const u32x4*)(stg + soff(row, 8 * ch));
    if (m0 + row < nb && 8 * ch < ncols) *(u32x4*)(out + (int64_t)(m0 + row) * ld + c0 + 8 * ch) = v;
  }
}

// fc3 dgrad for NT consecutive 32-feature tiles of dX^T: NT independent accumulator
// chains (a single chain serialises on the MFMA latency), A = W3 by transposed reads
// of the fc3 image, B = dh3^T straight from the accumulator registers.
template <int NT>
DEV void dx_tiles(int v0, const bf16_t* i3, const uint32_t (&d3p)[T1][8], bf16_t* stg, bf16_t* __restrict__ dx,
                  int m0, int nb, int lane) {
  const int h = lane >> 5, q4 = (lane >> 2) & 3, c16 = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  f32x16 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x16{};
#pragma unroll
  for (int s = 0; s < 2 * T1; ++s) {
    const uint32_t* dp = &d3p[s >> 1][4 * (s & 1)];
    const bf16x8 b = as_frag(dp[0], dp[1], dp[2], dp[3]);
    const int r0 = 16 * s + 4 * h + q4;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = 32 * (v0 + j) + c16;
      const s16x4 lo = lds_tr4(i3 + ioff<3>(r0, col));
      const s16x4 hi = lds_tr4(i3 + ioff<3>(r0 + 8, col));
      acc[j] = mfma32(join(lo, hi), b, acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    uint32_t pk[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) pk[w] = pack2(acc[j][2 * w], acc[j][2 * w + 1]);
    store_tile(stg, pk, dx, D0, m0, nb, 32 * (v0 + j), D0 - 32 * (v0 + j), lane);
  }
}

// NW waves per block, TPW 32-row tiles per wave.  The launch uses TPW = 1 (every wave's
// load / compute / store phases in lockstep); TPW = 2 with 4 waves (the next tile's X
// loads under the current tile's backward chain) measured slower (0.540 vs 0.53 ms/step,
// profiles/r3/lenet/knobs/).
template <bool GRADS, int NW = NWAVE, int TPW = 1>
__global__ __launch_bounds__(64 * NW) void mlp_head_k(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W3t,
                                                  const float* __restrict__ b3, int n1, const bf16_t* __restrict__ W4t,
                                                  const float* __restrict__ b4, int n2, const bf16_t* __restrict__ W5t,
                                                  const float* __restrict__ b5, int nc,
                                                  const int32_t* __restrict__ labels, int nb, float scale,
                                                  bf16_t* __restrict__ h3, bf16_t* __restrict__ h4,
                                                  float* __restrict__ logits, bf16_t* __restrict__ dl,
                                                  bf16_t* __restrict__ dh4, bf16_t* __restrict__ dh3,
                                                  bf16_t* __restrict__ dx, float* __restrict__ stats,
                                                  float* __restrict__ work, int defer_stats,
                                                  float* __restrict__ dbias) {
  __shared__ __attribute__((aligned(16))) bf16_t i3[R3 * S3];
  __shared__ __attribute__((aligned(16))) bf16_t i4[R4 * S4];
  __shared__ __attribute__((aligned(16))) bf16_t i5[R5 * S5];
  __shared__ __attribute__((aligned(16))) float bias[32 * T1 + 32 * T2 + LD3];
  constexpr int NT = 64 * NW;
  __shared__ __attribute__((aligned(16))) bf16_t stage[NW * STG];
  float* bias3 = bias;
  float* bias4 = bias + 32 * T1;
  float* bias5 = bias4 + 32 * T2;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  auto tile_m0 = [&](int t) { return ((int)(blockIdx.x * TPW + t) * NW + wave) * 32; };
  bf16_t* stg = stage + wave * STG;

  // 1. weight chunks, then the wave's whole 32 x 400 input tile and its labels, are
  // requested up front: the weight loads are older in the in-order vmcnt queue, so the
  // LDS staging below waits only for them while X is still in flight.
  ImgChunks<R3, S3, NT> c3;
  ImgChunks<R4, 32 * T1, NT> c4;
  ImgChunks<R5, S5, NT> c5;
  load_img(c3, W3t, tid);
  load_img(c4, W4t, tid);
  load_img(c5, W5t, tid);
  // (rows past nb load row nb-1: MFMA columns are independent and invalid ones are never stored)
  u32x4 xr[K1];
  auto load_x = [&](int mt) {       // the wave's 32 x 400 tile at row mt; returns the label
    int lb = -1;
    if (mt < nb) {
      const int mc = min(mt + r, nb - 1);
      const bf16_t* xrow = X + (int64_t)mc * D0 + 8 * h;
#pragma unroll
      for (int c = 0; c < K1; ++c) xr[c] = *(const u32x4*)(xrow + 16 * c);
      lb = labels[mc];
    } else {
#pragma unroll
      for (int c = 0; c < K1; ++c) xr[c] = u32x4{0u, 0u, 0u, 0u};
    }
    return lb;
  };
  int lab = load_x(tile_m0(0));
  // 2. weights -> LDS images, biases (zero beyond each layer's width)
  store_img<3, false>(i3, c3, tid);
  store_img<4, true>(i4, c4, tid);
  store_img<5, true>(i5, c5, tid);
  for (int i = tid; i < 32 * T1 + 32 * T2 + LD3; i += NT) {
    float v = 0.f;
    if (i < 32 * T1) v = i < n1 ? b3[i] : 0.f;
    else if (i < 32 * (T1 + T2)) v = (i - 32 * T1) < n2 ? b4[i - 32 * T1] : 0.f;
    else v = (i - 32 * (T1 + T2)) < nc ? b5[i - 32 * (T1 + T2)] : 0.f;
    bias[i] = v;
  }
  __syncthreads();

  float loss = 0.f, corr = 0.f, bad = 0.f;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // fp32 dlogits column sums (dbias)
#pragma unroll
  for (int ti = 0; ti < TPW; ++ti) {
  const int m0 = tile_m0(ti);
  const int m = m0 + r;
  const bool valid = m < nb;
  const bool active = m0 < nb;  // wave-uniform
  int lab_next = -1;
  if (active) {
    // ---------------- fc3: h3^T[128 x 32] = W3^T . X^T
    f32x16 a1[T1];
#pragma unroll
    for (int t = 0; t < T1; ++t) a1[t] = f32x16{};
#pragma unroll
    for (int c = 0; c < K1; ++c) {
      const bf16x8 xb = __builtin_bit_cast(bf16x8, xr[c]);
#pragma unroll
      for (int t = 0; t < T1; ++t) {
        const bf16x8 wa = *(const bf16x8*)(i3 + ioff<3>(32 * t + r, 16 * c + 8 * h));
        a1[t] = mfma32(wa, xb, a1[t]);
      }
    }
    if constexpr (!GRADS)   // forward only: xr is consumed, the next tile's X streams in now
      if (ti + 1 < TPW) lab_next = load_x(tile_m0(ti + 1));
    // bias + ReLU -> packed bf16 (register w of tile t = features 2w, 2w+1 of its slot list)
    uint32_t h3p[T1][8];
#pragma unroll
    for (int t = 0; t < T1; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = 32 * t + 8 * q + 4 * h;
        const f32x4 bb = *(const f32x4*)(bias3 + n);
        h3p[t][2 * q] = pack2(fmaxf(a1[t][4 * q] + bb[0], 0.f), fmaxf(a1[t][4 * q + 1] + bb[1], 0.f));
        h3p[t][2 * q + 1] = pack2(fmaxf(a1[t][4 * q + 2] + bb[2], 0.f), fmaxf(a1[t][4 * q + 3] + bb[3], 0.f));
      }
#pragma unroll
      for (int t = 0; t < T1; ++t) store_tile(stg, h3p[t], h3, LD1, m0, nb, 32 * t, LD1 - 32 * t, lane);

    // ---------------- fc4: h4^T[96 x 32] = W4^T . h3^T (h3 accumulators are the B operand)
    f32x16 a2[T2];
#pragma unroll
    for (int u = 0; u < T2; ++u) a2[u] = f32x16{};
#pragma unroll
    for (int s = 0; s < 2 * T1; ++s) {
      const uint32_t* hp = &h3p[s >> 1][4 * (s & 1)];
      const bf16x8 hb = as_frag(hp[0], hp[1], hp[2], hp[3]);
#pragma unroll
      for (int u = 0; u < T2; ++u) {
        const bf16x8 wa = *(const bf16x8*)(i4 + ioff<4>(32 * u + r, 16 * s + 8 * h));
        a2[u] = mfma32(wa, hb, a2[u]);
      }
    }
    uint32_t h4p[T2][8];
#pragma unroll
    for (int u = 0; u < T2; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = 32 * u + 8 * q + 4 * h;
        const f32x4 bb = *(const f32x4*)(bias4 + n);
        h4p[u][2 * q] = pack2(fmaxf(a2[u][4 * q] + bb[0], 0.f), fmaxf(a2[u][4 * q + 1] + bb[1], 0.f));
        h4p[u][2 * q + 1] = pack2(fmaxf(a2[u][4 * q + 2] + bb[2], 0.f), fmaxf(a2[u][4 * q + 3] + bb[3], 0.f));
      }
#pragma unroll
      for (int u = 0; u < T2; ++u) store_tile(stg, h4p[u], h4, LD2, m0, nb, 32 * u, LD2 - 32 * u, lane);

    // ---------------- fc5: logits^T[32 (16 real) x 32] = W5^T . h4^T
    f32x16 a3 = f32x16{};
#pragma unroll
    for (int s = 0; s < 2 * T2; ++s) {
      const uint32_t* hp = &h4p[s >> 1][4 * (s & 1)];
      const bf16x8 hb = as_frag(hp[0], hp[1], hp[2], hp[3]);
      bf16x8 wa = *(const bf16x8*)(i5 + ioff<5>(r & 15, 16 * s + 8 * h));
      if (r >= 16) wa = bf16x8{};
      a3 = mfma32(wa, hb, a3);
    }
    // registers 0..7 hold classes (i&3) + 8(i>>2) + 4h
    float lg[8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const f32x4 bb = *(const f32x4*)(bias5 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) lg[4 * q + e] = a3[4 * q + e] + bb[e];
      if (valid) *(f32x4*)(logits + (int64_t)m * LD3 + 8 * q + 4 * h) = f32x4{lg[4 * q], lg[4 * q + 1], lg[4 * q + 2], lg[4 * q + 3]};
    }
    // ---------------- softmax cross-entropy (a row's classes live in lanes r and r + 32)
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if ((i & 3) + 8 * (i >> 2) + 4 * h < nc) mx = fmaxf(mx, lg[i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float e[8], se = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      e[i] = ((i & 3) + 8 * (i >> 2) + 4 * h < nc) ? __expf(lg[i] - mx) : 0.f;
      se += e[i];
    }
    se += __shfl_xor(se, 32, 64);
    if (!valid) lab = -1;
    float ll = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) ll = ((i & 3) + 8 * (i >> 2) + 4 * h == lab) ? lg[i] : ll;
    ll += __shfl_xor(ll, 32, 64);
    if (valid && h == 0) {
      const float lo = -(ll - mx - __logf(se));
      loss += lo;
      corr += (ll >= mx) ? 1.f : 0.f;
      bad = isfinite(lo) ? bad : 1.f;
    }
    if constexpr (GRADS) {
      const float inv = 1.f / se;
      uint32_t dlp[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        float g2[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int i = 2 * w + k, cls = (i & 3) + 8 * (i >> 2) + 4 * h;
          g2[k] = cls < nc ? (e[i] * inv - (cls == lab ? 1.f : 0.f)) * scale : 0.f;
          cs[i] += valid ? g2[k] : 0.f;
        }
        dlp[w] = pack2(g2[0], g2[1]);
      }
      if (valid)
#pragma unroll
        for (int q = 0; q < 2; ++q) *(u32x2*)(dl + (int64_t)m * LD3 + 8 * q + 4 * h) = u32x2{dlp[2 * q], dlp[2 * q + 1]};

      // transposed-read coordinates: group g = lane>>4 supplies rows 4h+q4 (+8), columns 16(g&1)+4p4
      const int q4 = (lane >> 2) & 3, c16 = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);

      // ---------------- fc5 dgrad: dh4^T[96 x 32] = W5 . dlogits^T, masked by h4 > 0
      const bf16x8 db = as_frag(dlp[0], dlp[1], dlp[2], dlp[3]);
      uint32_t d4p[T2][8];
#pragma unroll
      for (int u = 0; u < T2; ++u) {
        const int col = p23(32 * u + c16);
        const s16x4 lo = lds_tr4(i5 + ioff<5>(4 * h + q4, col));
        const s16x4 hi = lds_tr4(i5 + ioff<5>(8 + 4 * h + q4, col));
        const f32x16 acc = mfma32(join(lo, hi), db, f32x16{});
#pragma unroll
        for (int w = 0; w < 8; ++w) {
          const float v0 = pos_lo(h4p[u][w]) ? acc[2 * w] : 0.f;
          const float v1 = pos_hi(h4p[u][w]) ? acc[2 * w + 1] : 0.f;
          d4p[u][w] = pack2(v0, v1);
        }
        store_tile(stg, d4p[u], dh4, LD2, m0, nb, 32 * u, LD2 - 32 * u, lane);
      }

      // ---------------- fc4 dgrad: dh3^T[128 x 32] = W4 . dh4^T, masked by h3 > 0
      f32x16 d3[T1];
#pragma unroll
      for (int t = 0; t < T1; ++t) d3[t] = f32x16{};
#pragma unroll
      for (int s = 0; s < 2 * T2; ++s) {
        const uint32_t* dp = &d4p[s >> 1][4 * (s & 1)];
        const bf16x8 b = as_frag(dp[0], dp[1], dp[2], dp[3]);
        const int r0 = 16 * s + 4 * h + q4;
#pragma unroll
        for (int t = 0; t < T1; ++t) {
          const int col = p23(32 * t + c16);
          const s16x4 lo = lds_tr4(i4 + ioff<4>(r0, col));
          const s16x4 hi = lds_tr4(i4 + ioff<4>(r0 + 8, col));
          d3[t] = mfma32(join(lo, hi), b, d3[t]);
        }
      }
      uint32_t d3p[T1][8];
#pragma unroll
      for (int t = 0; t < T1; ++t) {
#pragma unroll
        for (int w = 0; w < 8; ++w) {
          const float v0 = pos_lo(h3p[t][w]) ? d3[t][2 * w] : 0.f;
          const float v1 = pos_hi(h3p[t][w]) ? d3[t][2 * w + 1] : 0.f;
          d3p[t][w] = pack2(v0, v1);
        }
        store_tile(stg, d3p[t], dh3, LD1, m0, nb, 32 * t, LD1 - 32 * t, lane);
      }

      // ---------------- fc3 dgrad: dX^T[416 x 32] = W3 . dh3^T (no mask: the conv block's
      // pooled output is post-ReLU and its backward applies the mask itself)
      // the next tile's X streams in under this tile's fc3 data gradient (issued here, where
      // the forward activations are dead: right after fc3 the 100 live VGPRs spilled)
      if (ti + 1 < TPW) lab_next = load_x(tile_m0(ti + 1));
      dx_tiles<4>(0, i3, d3p, stg, dx, m0, nb, lane);
      dx_tiles<4>(4, i3, d3p, stg, dx, m0, nb, lane);
      dx_tiles<4>(8, i3, d3p, stg, dx, m0, nb, lane);
      dx_tiles<1>(12, i3, d3p, stg, dx, m0, nb, lane);
    }
  }
  lab = lab_next;
  }
  if (GRADS && dbias) {
    // the softmax_linear bias gradient in fp32 (the reference's tf.float32,
    // mnist_input.py:203-205): this block's column sums, lanes of a half in a fixed xor
    // tree, then the waves in order
    __shared__ float dbs[NW][16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) cs[i] += __shfl_xor(cs[i], o, 64);
    }
    if (r == 0)
#pragma unroll
      for (int i = 0; i < 8; ++i) dbs[wave][(i & 3) + 8 * (i >> 2) + 4 * h] = cs[i];
    __syncthreads();
    if (tid < 16) {
      float v = dbs[0][tid];
#pragma unroll
      for (int w = 1; w < NW; ++w) v += dbs[w][tid];
      dbias[(int64_t)blockIdx.x * 16 + tid] = v;
    }
  }
  if (stats) ce_block_stats<NW>(loss, corr, bad, stats, work, defer_stats != 0);
}

// ---------------------------------------------------------------------------- softmax tail
// The reference CNN's last layer (softmax_linear 192 -> 10, mnist_input.py:200-205) with the
// softmax cross-entropy and its data gradient as ONE kernel -- the fc5 / CE / fc5-dgrad part of
// mlp_head_k on a 192-wide input: logits^T = W5^T . h4^T (v_mfma_f32_32x32x16_bf16, batch rows
// as the lanes), CE statistics and dlogits in registers, then dh4^T = W5 . dlogits^T masked by
// h4 > 0 (local4's ReLU: the layered path's dgrad mask).  Replaces three launches (the fc5 GEMM,
// softmax_ce_rows_k, the fc5 data-gradient GEMM).  The input's k-slots are loaded in the order
// of the dgrad accumulator (lane half h: features 16 s + 4 h .. + 3 and 16 s + 8 + 4 h .. + 3 of
// chunk s; the W5^T image stores its columns with bits 2 and 3 swapped to match, as mlp_head's
// fc4 / fc5 images), so the ReLU mask of every dgrad register is already in the lane.
constexpr int TD0 = 192, TK = TD0 / 16, TU = TD0 / 32;
DEV int toff(int r, int col) { return r * TD0 + ((((col >> 3) ^ ((r >> 2) & 3)) << 3) | (col & 7)); }

template <int TNW, bool GRADS>
__global__ __launch_bounds__(64 * TNW) void ce_tail_k(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W5t,
                                                     const float* __restrict__ b5, int nc,
                                                     const int32_t* __restrict__ labels, int nb, float scale,
                                                     float* __restrict__ logits, bf16_t* __restrict__ dl,
                                                     bf16_t* __restrict__ dx, float* __restrict__ stats,
                                                     float* __restrict__ work, int defer_stats,
                                                     float* __restrict__ dbias) {
  __shared__ __attribute__((aligned(16))) bf16_t i5[16 * TD0];
  __shared__ __attribute__((aligned(16))) float bias5[LD3];
  __shared__ __attribute__((aligned(16))) bf16_t stage[TNW * STG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int m0 = ((int)blockIdx.x * TNW + wave) * 32, m = m0 + r;
  const bool valid = m < nb, active = m0 < nb;
  bf16_t* stg = stage + wave * STG;
  // W5^T [16][192] -> the swizzled, bit-2/3-permuted image (two 8-byte halves per chunk)
  for (int b = tid; b < 16 * TD0 / 8; b += 64 * TNW) {
    const int rr = b / (TD0 / 8), c = (b % (TD0 / 8)) * 8;
    const u32x4 o = *(const u32x4*)(W5t + (int64_t)b * 8);
    *(u32x2*)(i5 + toff(rr, p23(c))) = u32x2{o[0], o[1]};
    *(u32x2*)(i5 + toff(rr, p23(c + 4))) = u32x2{o[2], o[3]};
  }
  if (tid < LD3) bias5[tid] = tid < nc ? b5[tid] : 0.f;
  // the wave's 32 x 192 input tile in the permuted k-slot order (rows past nb: row nb - 1)
  u32x4 xr[TK];
  int lab = -1;
  if (active) {
    const int mc = min(m, nb - 1);
    const bf16_t* xrow = X + (int64_t)mc * TD0 + 4 * h;
#pragma unroll
    for (int c = 0; c < TK; ++c) {
      const u32x2 a = *(const u32x2*)(xrow + 16 * c), b = *(const u32x2*)(xrow + 16 * c + 8);
      xr[c] = u32x4{a[0], a[1], b[0], b[1]};
    }
    lab = labels[mc];
  }
  __syncthreads();
  float loss = 0.f, corr = 0.f, bad = 0.f;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    f32x16 a3 = f32x16{};
#pragma unroll
    for (int s = 0; s < TK; ++s) {
      bf16x8 wa = *(const bf16x8*)(i5 + toff(r & 15, 16 * s + 8 * h));
      if (r >= 16) wa = bf16x8{};
      a3 = mfma32(wa, __builtin_bit_cast(bf16x8, xr[s]), a3);
    }
    // softmax cross-entropy: mlp_head_k's (registers 0..7 hold classes (i&3) + 8(i>>2) + 4h)
    float lg[8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const f32x4 bb = *(const f32x4*)(bias5 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) lg[4 * q + e] = a3[4 * q + e] + bb[e];
      if (valid) *(f32x4*)(logits + (int64_t)m * LD3 + 8 * q + 4 * h) = f32x4{lg[4 * q], lg[4 * q + 1], lg[4 * q + 2], lg[4 * q + 3]};
    }
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if ((i & 3) + 8 * (i >> 2) + 4 * h < nc) mx = fmaxf(mx, lg[i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float e[8], se = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      e[i] = ((i & 3) + 8 * (i >> 2) + 4 * h < nc) ? __expf(lg[i] - mx) : 0.f;
      se += e[i];
    }
    se += __shfl_xor(se, 32, 64);
    if (!valid) lab = -1;
    float ll = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) ll = ((i & 3) + 8 * (i >> 2) + 4 * h == lab) ? lg[i] : ll;
    ll += __shfl_xor(ll, 32, 64);
    if (valid && h == 0) {
      const float lo = -(ll - mx - __logf(se));
      loss += lo;
      corr += (ll >= mx) ? 1.f : 0.f;
      bad = isfinite(lo) ? bad : 1.f;
    }
    if constexpr (GRADS) {
      const float inv = 1.f / se;
      uint32_t dlp[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        float g2[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int i = 2 * w + k, cls = (i & 3) + 8 * (i >> 2) + 4 * h;
          g2[k] = cls < nc ? (e[i] * inv - (cls == lab ? 1.f : 0.f)) * scale : 0.f;
          cs[i] += valid ? g2[k] : 0.f;
        }
        dlp[w] = pack2(g2[0], g2[1]);
      }
      if (valid)
#pragma unroll
        for (int q = 0; q < 2; ++q) *(u32x2*)(dl + (int64_t)m * LD3 + 8 * q + 4 * h) = u32x2{dlp[2 * q], dlp[2 * q + 1]};
      // dh4^T[192 x 32] = W5 . dlogits^T, masked by h4 > 0: register k of tile u = feature
      // 32 u + 8 (k >> 2) + 4 h + (k & 3) = chunk 2 u + (k >> 3), word 2 ((k >> 2) & 1) + ((k & 3) >> 1)
      const int q4 = (lane >> 2) & 3, c16 = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      const bf16x8 db = as_frag(dlp[0], dlp[1], dlp[2], dlp[3]);
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int col = p23(32 * u + c16);
        const s16x4 lo = lds_tr4(i5 + toff(4 * h + q4, col));
        const s16x4 hi = lds_tr4(i5 + toff(8 + 4 * h + q4, col));
        const f32x16 acc = mfma32(join(lo, hi), db, f32x16{});
        uint32_t pk[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
          const uint32_t xw = xr[2 * u + (w >> 2)][w & 3];   // features of registers 2w, 2w + 1
          const float v0 = pos_lo(xw) ? acc[2 * w] : 0.f;
          const float v1 = pos_hi(xw) ? acc[2 * w + 1] : 0.f;
          pk[w] = pack2(v0, v1);
        }
        store_tile(stg, pk, dx, TD0, m0, nb, 32 * u, TD0 - 32 * u, lane);
      }
    }
  }
  if (GRADS && dbias) {
    __shared__ float dbs[TNW][16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) cs[i] += __shfl_xor(cs[i], o, 64);
    }
    if (r == 0)
#pragma unroll
      for (int i = 0; i < 8; ++i) dbs[wave][(i & 3) + 8 * (i >> 2) + 4 * h] = cs[i];
    __syncthreads();
    if (tid < 16) {
      float v = dbs[0][tid];
#pragma unroll
      for (int w = 1; w < TNW; ++w) v += dbs[w][tid];
      dbias[(int64_t)blockIdx.x * 16 + tid] = v;
    }
  }
  if (stats) ce_block_stats<TNW>(loss, corr, bad, stats, work, defer_stats != 0);
}

}  // namespace

// waves per block (32 rows each): 2, or more when the block count would exceed the CE partial
// slots; MNISTX_CE_TAIL_NW overrides (1, 2 or 4).  At B = 16384 2 waves (256 blocks) measured
// 9.9 us, 1 wave 11.6 us, 4 waves 10.9 us (profiles/r6/cetail/README.md)
int ce_tail_nw(int nb) {
  static const int forced = [] {
    const char* e = getenv("MNISTX_CE_TAIL_NW");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? v : 0;
  }();
  int nw = forced ? forced : 2;
  while (nw < 4 && (nb + 32 * nw - 1) / (32 * nw) > CE_MAXB) nw *= 2;
  return nw;
}
int ce_tail_blocks(int nb) { const int r = 32 * ce_tail_nw(nb); return (nb + r - 1) / r; }
bool ce_tail_supported(int d0, int nc, int B) { return d0 == TD0 && nc > 0 && nc <= LD3 && B > 0 && ce_tail_blocks(B) <= CE_MAXB; }

hipError_t ce_tail(const bf16_t* x, const bf16_t* w5t, const float* b5, int nc, const int32_t* labels, int nb,
                   float scale, float* logits, bf16_t* dl, bf16_t* dx, float* stats, float* work, hipStream_t st,
                   int defer_stats, float* dbias) {
  if (nb <= 0) return hipSuccess;
  const dim3 grid(ce_tail_blocks(nb));
  const int nw = ce_tail_nw(nb);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(64 * nw), 0, st, x, w5t, b5, nc, labels, nb, scale, logits, dl, dx, stats,
                       work, defer_stats, dl ? dbias : nullptr);
  };
  if (dl) {
    if (nw == 1) go(ce_tail_k<1, true>);
    else if (nw == 2) go(ce_tail_k<2, true>);
    else go(ce_tail_k<4, true>);
  } else {
    if (nw == 1) go(ce_tail_k<1, false>);
    else if (nw == 2) go(ce_tail_k<2, false>);
    else go(ce_tail_k<4, false>);
  }
  return hipGetLastError();
}

int mlp_head_blocks(int nb) { return (nb + ROWS - 1) / ROWS; }

bool mlp_head_supported(int d0, int ld1, int ld2, int ld3, int n1, int n2, int nc, int B) {
  return d0 == D0 && ld1 == LD1 && ld2 == LD2 && ld3 == LD3 && n1 <= LD1 && n2 <= LD2 && nc <= LD3 && nc > 0 &&
         B > 0 && (B + ROWS - 1) / ROWS <= CE_MAXB;
}

hipError_t mlp_head(const bf16_t* x, const bf16_t* w3t, const float* b3, int n1, const bf16_t* w4t, const float* b4,
                    int n2, const bf16_t* w5t, const float* b5, int nc, const int32_t* labels, int nb, float scale,
                    bf16_t* h3, bf16_t* h4, float* logits, bf16_t* dl, bf16_t* dh4, bf16_t* dh3, bf16_t* dx,
                    float* stats, float* work, hipStream_t st, int defer_stats, float* dbias) {
  if (nb <= 0) return hipSuccess;
  const dim3 grid((nb + ROWS - 1) / ROWS);   // ROWS rows per block
  if (dl)
    hipLaunchKernelGGL(mlp_head_k<true>, grid, dim3(NTH), 0, st, x, w3t, b3, n1, w4t, b4, n2, w5t, b5, nc, labels, nb,
                       scale, h3, h4, logits, dl, dh4, dh3, dx, stats, work, defer_stats, dbias);
  else
    hipLaunchKernelGGL(mlp_head_k<false>, grid, dim3(NTH), 0, st, x, w3t, b3, n1, w4t, b4, n2, w5t, b5, nc, labels, nb,
                       scale, h3, h4, logits, dl, dh4, dh3, dx, stats, work, defer_stats, nullptr);
  return hipGetLastError();
}

}  // namespace mnistx
