// Deterministic per-step cross-entropy statistics (loss sum, correct count, NaN
// flag) shared by the softmax-CE kernel (misc.hip) and the fused dense head
// (mlp_head.hip).  Each block reduces its threads in a fixed tree, writes one
// partial to `work`, and the last block to finish (ticket counter at
// work[4 * CE_MAXB]) combines the partials in block order: bitwise identical
// results across runs and between hipGraph replay and eager execution.
#pragma once
#include "common.h"

constexpr int CE_MAXB = 1024;  // max blocks per launch (work holds 4 floats per block + ticket)

// Every thread of the block must call this (it synchronises the block).
// With work == nullptr each block adds its partial atomically (order-dependent).
// defer: only write the block's partial; finalize_k combines them in block order in
// the step's last launch (no agent-scope fence here: each one writes back the L2,
// 11 us of the LeNet-5 head at B = 65536).
template <int NW>
DEV void ce_block_stats(float loss, float corr, float bad, float* __restrict__ stats, float* __restrict__ work,
                        bool defer = false) {
  __shared__ float red[3][NW];
  __shared__ int last;
  loss = warp_sum(loss);
  corr = warp_sum(corr);
  bad = warp_sum(bad);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = loss;
    red[1][wave] = corr;
    red[2][wave] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    loss = red[0][0];
    corr = red[1][0];
    bad = red[2][0];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      loss += red[0][w];
      corr += red[1][w];
      bad += red[2][w];
    }
    if (!work) {
      atomicAdd(&stats[0], loss);
      atomicAdd(&stats[1], corr);
      if (bad > 0.f) stats[2] = 1.f;
    } else {
      work[4 * blockIdx.x] = loss;
      work[4 * blockIdx.x + 1] = corr;
      work[4 * blockIdx.x + 2] = bad;
      if (defer) {
        last = 0;
      } else {
        __threadfence();
        unsigned* ticket = (unsigned*)(work + 4 * CE_MAXB);
        last = atomicAdd(ticket, 1u) == gridDim.x - 1;
      }
    }
  }
  if (!work) return;
  __syncthreads();
  if (!last) return;
  __threadfence();
  // last block: combine the partials in block order (64 lanes of wave 0, fixed tree)
  if (wave != 0) return;
  const volatile float* wv = work;
  float a = 0.f, b = 0.f, c = 0.f;
  for (int i = lane; i < (int)gridDim.x; i += 64) {
    a += wv[4 * i];
    b += wv[4 * i + 1];
    c += wv[4 * i + 2];
  }
  a = warp_sum(a);
  b = warp_sum(b);
  c = warp_sum(c);
  if (lane == 0) {
    stats[0] += a;
    stats[1] += b;
    if (c > 0.f) stats[2] = 1.f;
    *(unsigned*)(work + 4 * CE_MAXB) = 0u;
  }
}

// Deterministic per-block column sums of fp32 values (the last layer's bias gradient =
// sum over rows of dlogits, kept in fp32 as the reference's tf.float32 graph does:
// mnist_input.py:203-205 / 224-226): v[c] of every thread -> wave (fixed xor tree) ->
// waves in order -> out[c].  Every thread of the block must call this.
template <int NW, int LD>
DEV void block_colsum(const float (&v)[LD], float* __restrict__ out) {
  __shared__ float red[NW][LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < LD; ++c) {
    const float s = warp_sum(v[c]);
    if (lane == 0) red[wave][c] = s;
  }
  __syncthreads();
  if (threadIdx.x < LD) {
    float s = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; ++w) s += red[w][threadIdx.x];
    out[threadIdx.x] = s;
  }
}
