// Common CDNA4 (gfx950) helpers for the MNIST kernels.
// Wave = 64 lanes; MFMA operands are bf16x8 fragments, fp32 accumulators.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

typedef uint16_t bf16_t;  // raw bf16 storage in global memory / LDS
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

DEV float bf2f(uint32_t v) { return __uint_as_float(v << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN stays NaN: hipcc emits v_cvt_pk_bf16_f32).
DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// uint8 pixel -> x/255 - 0.5 (mnist_input.py:37-39); fmaf so every kernel rounds identically
DEV float u8_norm(uint32_t b) { return fmaf((float)b, 1.f / 255.f, -0.5f); }

// Two floats -> a packed bf16 pair in ONE v_cvt_pk_bf16_f32 (RNE, bitwise the two f2bf
// conversions).  Packing two scalar conversions instead costs 4 VALU: hipcc converts each
// value alone (v_cvt_pk_bf16_f32 v, x, 0) and merges with a shift and an SDWA or.
DEV uint32_t pack2(float lo, float hi) {
  typedef __bf16 pk_bf16x2 __attribute__((ext_vector_type(2)));
  typedef float pk_f32x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(pk_f32x2{lo, hi}, pk_bf16x2));
}

// 8 bf16 in a 16-byte vector: element j lives in word j/2, half j%2.
DEV float u4_get(const u32x4& v, int j) {
  uint32_t w = v[j >> 1];
  return (j & 1) ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
}

DEV void u4_set(u32x4& v, int j, bf16_t x) {
  uint32_t w = v[j >> 1];
  w = (j & 1) ? ((w & 0x0000ffffu) | ((uint32_t)x << 16)) : ((w & 0xffff0000u) | x);
  v[j >> 1] = w;
}

DEV float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

DEV int warp_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware block-id remap (guide §5 "XCD swizzle must be bijective"):
// consecutive *logical* tiles land on one XCD so they share its L2.
DEV int xcd_remap(int bid, int nwg) {
  const int NX = 8;
  if (nwg <= NX) return bid;
  int xcd = bid % NX, loc = bid / NX;
  int q = nwg / NX, r = nwg % NX;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}

// Exact division by a runtime-invariant divisor for 0 <= n < 2^31
// (round-up multiplier, Granlund-Montgomery): q = mulhi(n, m) >> (l - 1),
// l = ceil(log2 d).  Replaces ~40-instruction integer divides in index math.
struct FastDiv {
  uint32_t d, m, sh;
  __host__ __device__ FastDiv() : d(1), m(0), sh(0) {}
  __host__ explicit FastDiv(uint32_t div) : d(div), m(0), sh(0) {
    if (div <= 1) return;
    uint32_t l = 0;
    while ((1ull << l) < div) ++l;
    m = (uint32_t)(((1ull << (31 + l)) + div - 1) / div);
    sh = l - 1;
  }
  DEV int div(int n) const { return m ? (int)(__umulhi((uint32_t)n, m) >> sh) : n; }
  DEV int mod(int n, int q) const { return n - q * (int)d; }
};

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

DEV bf16x8 join(s16x4 lo, s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// Transposed LDS read (ds_read_b64_tr_b16): in each 16-lane group, lane 4q+p
// supplies the address of 4 consecutive bf16 (row q, columns 4p..4p+3); lane i
// of the group receives column i of the 4 rows.  Addresses must be 8-byte aligned.
DEV s16x4 lds_tr4(const bf16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p); }

// Branch-free global loads through a buffer resource (raw buffer loads): an offset
// at or past num_records returns zeros without touching memory, so a tile's tail
// needs no per-lane branch.  A per-lane `if` (or a select) around a plain global
// load makes the compiler wait for the load at the control-flow join
// (s_waitcnt vmcnt(0)), which serialises a software-prefetch of several loads into
// one full memory latency each.
constexpr uint32_t BUF_OOB = 0x80000000u;   // > any num_records used here (< 2 GB)
// base and nbytes must be wave-uniform (every caller's are: a block's or a wave's image
// group, a kernel argument).  readfirstlane makes that visible to the compiler, which
// otherwise wraps each load whose descriptor it cannot prove uniform (e.g. one built
// from a loop-carried group index) in a waterfall loop: 4 readfirstlane, 2 compares and
// an exec-mask loop per load (the conv2 weight gradient had 9 of them).
DEV __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t nbytes) {
  const uint64_t b = (uint64_t)base;
  const uint64_t ub = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)ub, (short)0, (int)__builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
}
DEV uint32_t buf_b32(__amdgpu_buffer_rsrc_t r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0); }
DEV u32x2 buf_b64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
DEV u32x4 buf_b128(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
