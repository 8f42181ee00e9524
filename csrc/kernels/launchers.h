// Host-callable launchers for the MNIST HIP kernels (no torch dependency).
// All pointers are device pointers; every launcher is asynchronous on `st`
// and graph-capturable (no allocation, no synchronisation).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mnistx {

typedef uint16_t bf16_t;

// Test hook (binding set_grid_cap, never set in production): an upper bound on the grid of
// every persistent grid-stride kernel, so the oracle tests run the multi-iteration paths
// (several tiles / images per block: ring reuse, next-tile prefetch) at small batches.
// 0 = no cap.
int grid_cap();
void set_grid_cap(int n);
inline int cap_grid(int g) {
  const int c = grid_cap();
  return (c > 0 && g > c) ? c : g;
}
// CUs kept free of the persistent (one-resident-wave) kernels so that a collective launched
// on another stream can start while they run (binding set_reserve_cus; parallel/dp.py sets
// it when a gradient bucket's all-reduce is issued before such a kernel and world > 1;
// profiles/r5/dp_coresidency/).  A resident grid of per_cu * cus blocks becomes
// per_cu * (cus - reserve).  0 = every CU (the default and the one-GPU setting).
int reserve_cus();
void set_reserve_cus(int n);
inline int reserve_cut(int resident, int per_cu) {
  const int r = reserve_cus() * (per_cu > 0 ? per_cu : 1);
  return (r > 0 && resident - r >= 1) ? resident - r : resident;
}

// ---- probe.hip (tests / measurements only): wall-clock marks and an RCCL-footprint probe
hipError_t clock_mark(uint64_t* out, int slot, hipStream_t st);
hipError_t coresidency_probe(uint64_t* out, int blocks, int threads, int lds_bytes, int spin_ticks, hipStream_t st);

enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_SLAB = 2 };

struct GemmEpi {
  void* out;              // bf16 / f32 output, or f32 split-K slab base
  int ldc;                // output row stride (elements)
  int mode;               // EPI_*
  const float* bias;      // fp32 bias (master weights), may be null
  int bias_n;             // bias valid for n < bias_n (zero-padded columns beyond)
  int relu;               // apply ReLU after bias
  const bf16_t* mask;     // ReLU-backward mask source: keep v where mask > 0
  int ldm;
  int64_t slab_stride;    // elements between split-K slabs
};

// An LRN (radius 4, across channels) applied to a conv's input while the conv stages it
// (reference CNN norm1 -> conv2): x is then the LRN's INPUT.  on == 0: none.
struct LrnParams {
  float bias, alpha, beta;
  int on;
};

// ---- gemm256.hip: 256 x 256 LDS-DMA tiles for the GEMMs that fill the GPU (dense_fwd /
// dense_dgrad route to it when gemm256_ok)
bool gemm256_enabled();              // MNISTX_GEMM256 != 0, or set_gemm256
void set_gemm256(bool on);
void set_gemm256_debug(int bits);     // experiments: bit 0 = skip the in-loop DMA (wrong results)
bool gemm256_ok(int M, int N, int K, const GemmEpi& ep);
hipError_t gemm256_fwd(const bf16_t* x, const bf16_t* w, int M, int N, int K, int ldx, int ldw, const GemmEpi& ep,
                       hipStream_t st);
hipError_t gemm256_dgrad(const bf16_t* dy, const bf16_t* w, int M, int N, int K, int lddy, int ldw, const GemmEpi& ep,
                         hipStream_t st);
int gemm256_cus();   // CUs a gemm256 grid can count on (all less reserve_cus())
int gemm256_wgrad_splits(int Din, int Dout, int B, int with_bias, int cus);   // 0: not this path
// fp32 twins (f32_dense_* route here when gemm256f_ok / gemm256f_wgrad_splits > 0)
bool gemm256f_ok(int M, int N, int K);
hipError_t gemm256f_fwd(const float* x, const float* w, int M, int N, int K, const float* bias, int bias_n, int relu,
                        float* y, int ldy, hipStream_t st);
hipError_t gemm256f_dgrad(const float* dy, const float* w, int M, int Din, int Dout, const float* mask, float* dx,
                          hipStream_t st);
int gemm256f_wgrad_splits(int Din, int Dout, int B, int cus);
hipError_t gemm256f_wgrad(const float* x, const float* dy, int B, int Din, int Dout, int splits, float* slab,
                          hipStream_t st);
hipError_t gemm256_wgrad(const bf16_t* x, const bf16_t* dy, int Din, int Dout, int B, int ldx, int lddy,
                         int with_bias, int splits, const GemmEpi& ep, hipStream_t st);

// ---- gemm.hip
// tile (BM, BN) launch_any picks for an M x N output (wgrad: both operands MN-contiguous)
void gemm_tile(int M, int N, int wgrad, int* bm, int* bn);
// tile >= 0: that launch_any tile code (benches / tests), skipping the gemm256 route
hipError_t dense_fwd(const bf16_t* x, const bf16_t* w, int M, int N, int K, int ldx, int ldw,
                     const GemmEpi& ep, hipStream_t st, int tile = -1);
hipError_t dense_dgrad(const bf16_t* dy, const bf16_t* w, int M, int N, int K, int lddy, int ldw,
                       const GemmEpi& ep, hipStream_t st, int tile = -1);
void set_tile192(int on);   // A/B switch of the 192-column tiles (MNISTX_TILE192)
// used (optional): the split count actually written -- the 256 x 256 path (tile < 0, used set)
// may write fewer partials than `splits` (the slab's capacity); the reduce must use *used
hipError_t dense_wgrad(const bf16_t* x, const bf16_t* dy, int Din, int Dout, int B, int ldx, int lddy,
                       int with_bias, int splits, const GemmEpi& ep, hipStream_t st, int tile = -1,
                       int* used = nullptr);
// np (<= 4) dense weight gradients in one launch (64x64 tiles; splits[] in: requested, out: effective)
hipError_t dense_wgrad_group(int np, const bf16_t* const* x, const bf16_t* const* dy, const int* Din, const int* Dout,
                             int B, const int* ldx, const int* lddy, int* splits, const GemmEpi* ep, hipStream_t st);
// conv_halo.hip: LDS-halo 5x5 convolutions (reference conv2 geometry); conv_fwd /
// conv_dgrad route there when *_ok() holds
void set_halo_variants(int fwd, int dgrad);
bool conv5_halo_fwd_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout);
bool conv5_halo_dgrad_ok(int OH, int OW, int Cout, int H, int W, int KH, int KW, int ph, int pw, int Cin);
hipError_t conv5_halo_fwd(const bf16_t* x, const bf16_t* w, int Nb, int C, int Cout, const float* bias, int bias_n,
                          int relu, bf16_t* out, hipStream_t st, LrnParams lrn = LrnParams{0.f, 0.f, 0.f, 0});
hipError_t conv5_halo_dgrad(const bf16_t* dy, const bf16_t* w, int Nb, int Cout, int Cin, const bf16_t* mask,
                            bf16_t* dx, hipStream_t st);
bool conv5_halo_wgrad_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout,
                         int with_bias);
int conv5_halo_wgrad_grid(int Nb);   // persistent blocks (= slab partials) for Nb images
hipError_t conv5_halo_wgrad(const bf16_t* x, const bf16_t* dy, int Nb, int grid, float* slab, hipStream_t st,
                            LrnParams lrn = LrnParams{0.f, 0.f, 0.f, 0});
bool conv_halo_enabled();            // MNISTX_CONV_HALO != 0
hipError_t conv_fwd(const bf16_t* x, const bf16_t* w, int Nb, int H, int W, int C, int OH, int OW, int KH,
                    int KW, int ph, int pw, int Cout, const GemmEpi& ep, hipStream_t st,
                    LrnParams lrn = LrnParams{0.f, 0.f, 0.f, 0});
hipError_t conv_dgrad(const bf16_t* dy, const bf16_t* w, int Nb, int OH, int OW, int Cout, int H, int W,
                      int KH, int KW, int ph, int pw, int Cin, const GemmEpi& ep, hipStream_t st);
hipError_t conv_wgrad(const bf16_t* x, const bf16_t* dy, int Nb, int H, int W, int C, int OH, int OW, int KH,
                      int KW, int ph, int pw, int Cout, int with_bias, int splits, const GemmEpi& ep,
                      hipStream_t st, LrnParams lrn = LrnParams{0.f, 0.f, 0.f, 0});

// ---- convpool.hip (fused small-channel conv + bias + ReLU + 2x2 max-pool)
// Input of a fused conv: bf16 NHWC activations x[B], or (Cin == 1 first layer) a
// resident dataset [n][H*W] gathered through the per-sample index idx[B]: uint8
// (u8 set, normalised in the kernel) or bf16 already normalised (x set, u8 null).
struct XSrc {
  const bf16_t* x;
  const uint8_t* u8;
  const int64_t* idx;
  int n;
};
int convpool_u8_input(int cfg);
int convpool_config(int cin, int cout, int ks, int pad, int h, int w);  // -1: unsupported
int convpool_wgrad_rows(int cfg);                                      // KM (slab rows incl. bias row)
// slab -> dW layout for splitk_reduce: {G, Ipad, I (-1: real Cin), bias_row}
int convpool_reduce_layout(int cfg, int* out);
hipError_t convpool_fwd(int cfg, const XSrc& x, const bf16_t* w, const float* bias, int bias_n, int B,
                        bf16_t* pooled, uint8_t* arg, hipStream_t st);
// backward needs only (dP, arg): arg == 4 marks a window whose ReLU output is 0
// workgroups that fill every CU once for this geometry's wgrad kernel (occupancy API)
int convpool_wgrad_grid(int cfg);
// lrn_p != nullptr (Cout 32 geometries): dP is dL/d(LRN output) of an LRN (radius 4)
// applied to the pooled output lrn_p; the LRN backward is applied while staging
hipError_t convpool_wgrad(int cfg, const XSrc& x, const bf16_t* dP, const uint8_t* arg, int B, float* slab,
                          int grid, hipStream_t st, const bf16_t* lrn_p = nullptr, float lrn_bias = 0.f,
                          float lrn_alpha = 0.f, float lrn_beta = 0.f);
int convpool_has_dgrad(int cfg);
// argmax bytes per pool window (LeNet conv1: 8 codes packed 4 bits each)
int convpool_arg_bytes(int cfg);
hipError_t convpool_dgrad(int cfg, const bf16_t* dP, const uint8_t* arg, const bf16_t* w, int B, bf16_t* dx,
                          int grid_cap, hipStream_t st);

// ---- lenet_bwd.hip: LeNet-5 conv-stack backward (conv2 dgrad + both weight gradients) as ONE
// persistent kernel; slab1 [grid][32][8] (rows tap 0..24, bias 25), slab2 [grid][208][16]
// (rows tap * 8 + ci, bias 200) -- the split-K partials splitk_reduce combines
// p1c: the band forward's combined pool1 records [B][196] x 16 bytes (channels 0-5 bf16 + the
// window's argmax code word; lenet_band_fwd with p1 and no arg1)
int lenet_bwd_blocks(int B);         // the grid for a batch (one block per CU, <= tiles); <= 0: error
hipError_t lenet_bwd(const XSrc& x, const bf16_t* p1c, const bf16_t* dp2, const uint8_t* arg2, const bf16_t* w2,
                     int B, float* slab1, float* slab2, int grid, hipStream_t st, unsigned long long* prof = nullptr);

// ---- refc1_wgrad.hip: reference-CNN conv1 weight gradient with the norm1 (LRN, radius 4, beta
// 0.75) backward folded in: dn = dL/d norm1, p1 = pool1 (the LRN input), arg = pool1 codes (one
// byte per channel), all [B][196][32].  slab [grid][48][32] in convpool_wgrad's RefC1g layout.
int refc1_wgrad_blocks(int B);       // the grid for a batch (one block per CU, <= tiles); <= 0: error
void refc1_set_skip(int s);          // experiments (bench/micro_refc1.py): parts of the kernel left out
// cin 3: the bf16 NHWC batch only (x.x, no index); slab [grid][80][32] (convpool's Geo<3, 32> layout)
hipError_t refc1_wgrad(const XSrc& x, const bf16_t* dn, const bf16_t* p1, const uint8_t* arg, int B, float bias,
                       float alpha, float beta, float* slab, int grid, hipStream_t st, int cin = 1);

// ---- lenet_band.hip: LeNet-5 conv1+pool1+conv2+pool2 forward on banded MFMA tiles
// (one persistent kernel; bf16 images only).  x.x = [n][784] images (x.idx: per-sample
// rows, else sample b = row b).  p1/arg1 (convpool cfg-0 layouts) are written only when
// p1 != nullptr; p1 without arg1 = the combined records lenet_bwd reads; p2/arg2 use the
// convpool cfg-1 layouts.
bool refc1_band_enabled();
// norm (optional): norm1 = LRN(pool1) (radius 4, the given bias / alpha / beta) [B][196][32], written by
// the same launch (refc1n_fwd_k) when refc1_fwd_lrn_ok()
bool refc1_fwd_lrn_ok();
void refc1_set_fwd_variant(int v);   // 1: the round-5 refc1_band_fwd_k, 2: refc1n_fwd_k (default)
// cin 3 (refc1n3_fwd_k, when refc1_fwd3_ok()): bf16 input only (x.x: the NHWC batch or the bf16
// dataset [n][2352] through x.idx)
bool refc1_fwd3_ok();
hipError_t refc1_band_fwd(const XSrc& x, const bf16_t* w, const float* b, int bn, int B, bf16_t* pooled,
                          uint8_t* arg, hipStream_t st, bf16_t* norm = nullptr, float lrn_bias = 0.f,
                          float lrn_alpha = 0.f, float lrn_beta = 0.f, int cin = 1);
hipError_t lenet_band_fwd(const XSrc& x, const bf16_t* w1, const float* b1, int b1n, const bf16_t* w2,
                          const float* b2, int B, bf16_t* p1, uint8_t* arg1, bf16_t* p2, uint8_t* arg2,
                          hipStream_t st, unsigned long long* prof = nullptr);

// ---- f32.hip: reference-precision (fp32) path, v_mfma_f32_16x16x4_f32
hipError_t f32_dense_fwd(const float* x, const float* w, int M, int N, int K, const float* bias, int bias_n, int relu,
                         float* y, int ldy, hipStream_t st);
hipError_t f32_dense_dgrad(const float* dy, const float* w, int M, int Din, int Dout, const float* mask, float* dx,
                           hipStream_t st);
// used (optional): the split count written (the 256 x 256 path may write fewer than `splits`)
hipError_t f32_dense_wgrad(const float* x, const float* dy, int B, int Din, int Dout, int splits, float* slab,
                           hipStream_t st, int* used = nullptr);
int f32_wgrad_splits_cap(int Din, int Dout, int B);   // slabs the 256 x 256 path may write (0: none)
// conv_halo_f32.hip: LDS-halo fp32 conv2 of the reference CNN (fwd / dgrad), routed to by f32_conv_*
bool f32_halo_fwd_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout);
bool f32_halo_dgrad_ok(int OH, int OW, int Cout, int H, int W, int KH, int KW, int ph, int pw, int Cin);
void set_f32_halo_fwd_variant(int v);   // 1: the pre-balance 7-group forward (A/B, tests)
hipError_t f32_halo_fwd(const float* x, const float* w, int Nb, int C, int Cout, const float* bias, int relu, float* y,
                        hipStream_t st);
hipError_t f32_halo_dgrad(const float* dy, const float* w, int Nb, int Cout, int Cin, const float* mask, float* dx,
                          hipStream_t st);
// conv1_f32.hip: fp32 28x28x1 -> 32, 5x5 SAME (reference CNN / fp32 conv1), routed to by f32_conv_*
bool f32_conv1_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout);
int f32_conv1_wgrad_grid();
hipError_t f32_conv1_fwd(const float* x, const float* w, int Nb, const float* bias, int relu, float* y,
                         hipStream_t st);
hipError_t f32_conv1_wgrad(const float* x, const float* dy, int Nb, int splits, float* slab, hipStream_t st);
// fused with the following 2x2 max-pool: pooled output [Nb][14][14][32] + codes (one byte per
// channel: window position 0..3, 4 = ReLU output 0); the weight gradient from dL/d pool + codes
hipError_t f32_conv1_fwd_pool(const float* x, const float* w, int Nb, const float* bias, float* y, uint8_t* arg,
                              hipStream_t st);
int f32_conv1_wgrad_unpool_grid();
hipError_t f32_conv1_wgrad_unpool(const float* x, const float* dp, const uint8_t* codes, int Nb, int splits,
                                  float* slab, hipStream_t st);
// the same with norm1's backward (LRN radius 4 over the 32 channels) folded in: dn = dL/d norm1,
// p1 = pool1 (the LRN input); dL/d pool1 is never written
int f32_conv1_wgrad_lrn_grid();
hipError_t f32_conv1_wgrad_lrn(const float* x, const float* dn, const float* p1, const uint8_t* codes, int Nb,
                               int splits, float bias, float alpha, float beta, float* slab, hipStream_t st);
bool f32_halo_wgrad_ok(int H, int W, int C, int OH, int OW, int KH, int KW, int ph, int pw, int Cout);
int f32_halo_wgrad_grid();
hipError_t f32_halo_wgrad(const float* x, const float* dy, int Nb, int splits, float* slab, hipStream_t st);
hipError_t f32_conv_fwd(const float* x, const float* w, int Nb, int H, int W, int C, int OH, int OW, int KH, int KW,
                        int ph, int pw, int Cout, const float* bias, int relu, float* y, hipStream_t st);
hipError_t f32_conv_dgrad(const float* dy, const float* w, int Nb, int OH, int OW, int Cout, int H, int W, int KH,
                          int KW, int ph, int pw, int Cin, const float* mask, float* dx, hipStream_t st);
hipError_t f32_conv_wgrad(const float* x, const float* dy, int Nb, int H, int W, int C, int OH, int OW, int KH,
                          int KW, int ph, int pw, int Cout, int splits, float* slab, hipStream_t st);
hipError_t f32_maxpool_fwd(const float* x, int Nb, int H, int W, int C, int OH, int OW, float* y, uint8_t* arg,
                           hipStream_t st);
hipError_t f32_maxpool_bwd(const float* dy, const uint8_t* arg, const float* y, int relu_mask, int Nb, int H, int W,
                           int C, int OH, int OW, float* dx, hipStream_t st);
hipError_t f32_lrn_fwd(const float* x, int64_t P, int C, int r, float bias, float alpha, float beta, float* y,
                       hipStream_t st);
hipError_t f32_lrn_bwd(const float* x, const float* dy, int64_t P, int C, int r, float bias, float alpha, float beta,
                       int relu_mask, float* dx, hipStream_t st);
// LRN then 2x2/2 max-pool fused (fp32; the pool's codes: first-maximum window position per
// channel), and its backward straight to dL/d(LRN input)
bool f32_lrn_pool_ok(int H, int W, int C, int r);
hipError_t f32_lrn_pool_fwd(const float* x, int Nb, int H, int W, int C, int r, float bias, float alpha, float beta,
                            float* y, uint8_t* arg, hipStream_t st);
hipError_t f32_lrn_pool_bwd(const float* x, const float* dy, const uint8_t* arg, int Nb, int H, int W, int C, int r,
                            float bias, float alpha, float beta, int relu_mask, float* dx, hipStream_t st);
hipError_t f32_softmax_ce(const float* logits, int ldl, const int32_t* labels, int B, int NC, float scale, float* dl,
                          int ldd, float* stats, float* probs, float* work, hipStream_t st);
hipError_t f32_prep_images(const uint8_t* src, const int64_t* idx, const int32_t* lab_src, int B, int HW, int Csrc,
                           int Cdst, float* out, int32_t* lab_out, hipStream_t st);

// ---- misc.hip
hipError_t perm_positions(int64_t* out, int64_t start, int n, int64_t N, uint32_t seed, int h, hipStream_t st,
                          const int32_t* lab_src = nullptr, int32_t* lab_out = nullptr);
// 28x28x1 batch gather + normalise with the Feistel epoch shuffle fused in (rows are
// perm_positions(start + b)): no index array, no separate permutation launch
hipError_t prep_images_perm(const uint8_t* src, const int32_t* lab_src, int B, int64_t start, int64_t N,
                            uint32_t seed, int h, bf16_t* out, int32_t* lab_out, hipStream_t st);
hipError_t prep_images(const uint8_t* src, const int64_t* idx, const int32_t* lab_src, int B, int HW, int Csrc,
                       int Cdst, bf16_t* out, int32_t* lab_out, hipStream_t st);
hipError_t maxpool_fwd(const bf16_t* x, int Nb, int H, int W, int C, int OH, int OW, bf16_t* y, uint8_t* arg,
                       hipStream_t st);
hipError_t maxpool_bwd(const bf16_t* dy, const uint8_t* arg, const bf16_t* y, int relu_mask, int Nb, int H,
                       int W, int C, int OH, int OW, bf16_t* dx, hipStream_t st);
hipError_t lrn_fwd(const bf16_t* x, int P, int C, int r, float bias, float alpha, float beta, bf16_t* y,
                   hipStream_t st);
hipError_t lrn_bwd(const bf16_t* x, const bf16_t* dy, int P, int C, int r, float bias, float alpha, float beta,
                   int relu_mask, bf16_t* dx, hipStream_t st);
// fused LRN -> 2x2/2 max-pool (even H, W; C 32/64, radius 4): pooled y + argmax bytes,
// and its backward from the pooled gradient
bool lrn_pool_supported(int H, int W, int C, int r);
hipError_t lrn_pool_fwd(const bf16_t* x, int Nb, int H, int W, int C, int r, float bias, float alpha, float beta,
                        bf16_t* y, uint8_t* arg, hipStream_t st, int nonneg = 0);
// nonneg: the input is >= 0 (post-ReLU), which the packed 14 x 14 x 64 forward needs
void lrn_set_packed(int on);
hipError_t lrn_pool_bwd(const bf16_t* x, const bf16_t* dP, const uint8_t* arg, int Nb, int H, int W, int C, int r,
                        float bias, float alpha, float beta, int relu_mask, bf16_t* dx, hipStream_t st);
// work (optional): >= 4*1024+1 floats, zero-initialised once; makes the loss /
// accuracy sums deterministic (per-block partials combined in block order)
// defer_blocks (optional out): with it, the row kernel writes per-block partials only and
// reports its block count there (0 when the fallback kernel ran: plain atomics); the
// caller's finalize_step combines them (ce_stats.h defer)
// dbias (optional, with dlogits): per-block fp32 column sums of dlogits [blocks][ldl]
// (blocks = softmax_ce_dbias_blocks; only the row kernel, ldl 16 / 32, writes them)
hipError_t softmax_ce(const float* logits, int ldl, const int32_t* labels, int B, int NC, float scale,
                      bf16_t* dlogits, int ldd, float* stats, float* probs, float* work, hipStream_t st,
                      int* defer_blocks = nullptr, float* dbias = nullptr);
int softmax_ce_dbias_blocks(int B, int ldl);
// Fused LeNet-5 dense head (mlp_head.hip): fc3/fc4/fc5 + softmax-CE (+ with dl:
// the data-gradient chain dlogits -> dh4 -> dh3 -> dx).  Writes h3, h4, logits
// always; dl, dh4, dh3, dx when dl != nullptr.  Same work-buffer contract as softmax_ce.
bool mlp_head_supported(int d0, int ld1, int ld2, int ld3, int n1, int n2, int nc, int B);
// w3t / w4t / w5t: zero-padded W^T copies [128][416], [96][128], [16][96].
hipError_t mlp_head(const bf16_t* x, const bf16_t* w3t, const float* b3, int n1, const bf16_t* w4t, const float* b4,
                    int n2, const bf16_t* w5t, const float* b5, int nc, const int32_t* labels, int nb, float scale,
                    bf16_t* h3, bf16_t* h4, float* logits, bf16_t* dl, bf16_t* dh4, bf16_t* dh3, bf16_t* dx,
                    float* stats, float* work, hipStream_t st, int defer_stats = 0, float* dbias = nullptr);
// blocks of one mlp_head launch (its per-block CE partials when defer_stats is set)
int mlp_head_blocks(int nb);
// the reference CNN's softmax_linear (192 -> nc <= 16) + softmax CE + its data gradient (masked by
// x > 0) in one launch; w5t = W^T [16][192] (the optimizer's transposed copy); dbias: fp32 per-block
// column sums [ce_tail_blocks][16]
bool ce_tail_supported(int d0, int nc, int B);
int ce_tail_blocks(int nb);
hipError_t ce_tail(const bf16_t* x, const bf16_t* w5t, const float* b5, int nc, const int32_t* labels, int nb,
                   float scale, float* logits, bf16_t* dl, bf16_t* dx, float* stats, float* work, hipStream_t st,
                   int defer_stats, float* dbias);
// NOTE: many splits over a small output are pre-summed IN PLACE (the slab is scratch).
hipError_t splitk_reduce(float* slab, int splits, int M, int N, int G, int Ipad, int I, int J,
                         int bias_row, float* wdst, float* bdst, float scale, hipStream_t st);
// Several layers' slabs in one launch per pass (descriptors are copied into the
// kernel arguments, so the call is hipGraph-capturable).
struct RedSpec {
  float* slab;
  float* wdst;
  float* bdst;           // nullptr: no bias row
  int splits, M, N, G, Ipad, I, J, bias_row;
  float scale;
};
hipError_t splitk_reduce_multi(const RedSpec* specs, int n, hipStream_t st);
// one launch for the partial and reduce passes (default; MNISTX_REDUCE_FUSED=0: two launches)
void set_reduce_fused(int on);
int reduce_fused_enabled();

struct OptSeg {          // one trainable tensor inside the flat buffers
  int64_t off;           // offset in the flat fp32 buffers
  int64_t n;             // elements
  int G, I, J;           // master shape [G][I][J]
  int Ip, Jp;            // padded bf16 copy shape [G][Ip][Jp]
  int64_t bf_off;        // offset of the bf16 copy (-1: none)
  float wd;              // L2 weight decay (0: none)
  int track_l2;          // accumulate sum(w^2) into l2[seg]
  int64_t bft_off;       // offset of a transposed bf16 copy [Jt][It] (G == 1; -1: none)
  int Jt, It;
};

struct OptParams {
  float lr0, decay_rate;
  int64_t decay_steps;   // staircase exponential_decay; <=0: constant
  float momentum;
  int nesterov;          // 0/1
  int use_momentum;
  float grad_scale;      // e.g. 1/world_size
  float ema_max;         // 0.9999 ; <0 disables EMA
  // push guard (PS mode, optional): skip the whole update unless *guard == guard_want;
  // a skipped update writes guard_id into *guard_err
  const int64_t* guard;
  int64_t guard_want;
  int* guard_err;
  int guard_id;
};

// l2 (optional): [l2n per-tensor sums | fused_optimizer_blocks() per-block partials]
int fused_optimizer_blocks(const OptSeg* segs, int nseg);
// finalize_step's arguments (finalize_k, or the last block of fused_opt_k: ticket != nullptr)
struct FinArgs {
  int64_t* step;
  float* stats;
  float* l2;
  const int* l2r;
  int l2base;
  const float* wds;
  int nw;
  float* loss_ema;
  int n_ema, batch, increment;
  const float* ce_work;
  int ce_nblk;
  int* ticket;
};
// fin (optional): the step's finalize_step, run by the optimizer launch's last block when the
// grid is small (<= 1024 blocks: one ticket address per launch) and no PS guard is set, else
// launched right after it (MNISTX_OPT_FIN_FUSED=0: always separate)
// the next batch's epoch-shuffle rows + labels (perm_positions), computed by extra blocks of the
// optimizer launch instead of a launch of their own at the next step's start (blk0: set by
// the launcher)
struct PermJob {
  int64_t* out;
  const int32_t* lab_src;
  int32_t* lab_out;
  int64_t start, N;
  uint32_t seed;
  int h, n, blk0;
};
// perm (optional): run that job in the same launch
hipError_t fused_optimizer(float* params, const float* grads, float* mom, float* ema, bf16_t* bf, const OptSeg* segs,
                           int nseg, int64_t total, const int64_t* step, OptParams op, float* l2, int l2n, hipStream_t st,
                           const FinArgs* fin = nullptr, const PermJob* perm = nullptr);
void set_opt_fin_fused(int on);
int opt_fin_fused_enabled();
// l2r (optional, device int32 [nw][3] = {weight index, first block, end block}): sum the
// fused optimizer's per-block partials at l2[l2base + block] for each weight
// ce_work / ce_nblk: per-block CE partials of a deferred-stats mlp_head launch, added to
// stats[0..2] in block order before anything reads them
hipError_t finalize_step(const FinArgs& f, hipStream_t st);
hipError_t cast_f32_bf16_padded(const float* src, bf16_t* dst, int G, int I, int J, int Ip, int Jp,
                                hipStream_t st);

}  // namespace mnistx
