// Helpers shared by the pool-window-phase weight-gradient kernels (lenet_bwd.hip,
// refc1_wgrad.hip): transposed LDS reads, argmax-code masks on packed bf16, the lane id
// as an opaque value.
#pragma once
#include "common.h"

namespace mnistx {
namespace {

DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

// packed u16: dv where the code half equals d, else 0 (3 VALU: xor, saturating 1 - x, mul)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
DEV uint32_t sel_eq(uint32_t dv, uint32_t codes, uint32_t dd) {
  const u16x2 x = __builtin_bit_cast(u16x2, codes ^ dd);
  const u16x2 one = {1, 1};
  const u16x2 m = __builtin_elementwise_sub_sat(one, x);
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, dv) * m);
}
// bytes b0, b1 of w -> u16 pair (b0 | b1 << 16)
DEV uint32_t bytes01(uint32_t w) { return (w & 0xffu) | ((w & 0xff00u) << 8); }
DEV uint32_t bytes23(uint32_t w) { return ((w >> 16) & 0xffu) | ((w >> 8) & 0xff0000u); }
DEV bf16x8 frag(s16x4 lo, s16x4 hi) { return join(lo, hi); }
DEV s16x4 tr4(const uint8_t* lds, int off) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + off)); }
// the lane id, re-read where it is needed: per-lane addressing constants derived from it are
// recomputed each tile (a few VALU) instead of being hoisted out of the tile loop, where they
// would pin registers of a kernel that must fit 128
DEV int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

}  // namespace
}  // namespace mnistx
