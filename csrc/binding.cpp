#include <algorithm>
// Python bindings for the MNIST HIP kernels (torch extension `_kernels`).
//
// Every entry point validates device, dtype, contiguity and that each buffer is
// large enough for the indices the kernel will form, BEFORE launching: a
// mis-sized operand must raise here, never fault on the GPU.  Launches go to
// the caller's current HIP stream (so they are hipGraph-capturable and honour
// torch.cuda.stream contexts).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers.h"

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(const Tensor& t, at::ScalarType dt, int64_t need, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, ": must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected dtype ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": must be contiguous");
  TORCH_CHECK(need >= 0 && t.numel() >= need, name, ": needs ", need, " elements, has ", t.numel());
}

int64_t span(int64_t rows, int64_t ld, int64_t cols) { return rows <= 0 ? 0 : (rows - 1) * ld + cols; }

template <class T>
T* P(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
const mnistx::bf16_t* BF(const Tensor& t) { return reinterpret_cast<const mnistx::bf16_t*>(t.data_ptr()); }
mnistx::bf16_t* BFm(const Tensor& t) { return reinterpret_cast<mnistx::bf16_t*>(t.data_ptr()); }

void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " launch failed: ", hipGetErrorString(e));
}

mnistx::GemmEpi make_epi(const Tensor& out, int64_t M, int64_t N, int64_t ldc, const optional<Tensor>& bias,
                         int64_t bias_n, bool relu, const optional<Tensor>& mask, int64_t ldm) {
  TORCH_CHECK(ldc >= N, "ldc < N");
  mnistx::GemmEpi ep{};
  if (out.scalar_type() == at::kBFloat16) {
    check(out, at::kBFloat16, span(M, ldc, N), "out");
    ep.mode = mnistx::EPI_BF16;
  } else {
    check(out, at::kFloat, span(M, ldc, N), "out");
    ep.mode = mnistx::EPI_F32;
  }
  ep.out = out.data_ptr();
  ep.ldc = (int)ldc;
  ep.bias = nullptr;
  ep.bias_n = 0;
  if (bias.has_value() && bias->defined()) {
    check(*bias, at::kFloat, bias_n, "bias");
    ep.bias = P<const float>(*bias);
    ep.bias_n = (int)bias_n;
  }
  ep.relu = relu ? 1 : 0;
  ep.mask = nullptr;
  ep.ldm = 0;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(ldm >= N, "ldm < N");
    check(*mask, at::kBFloat16, span(M, ldm, N), "mask");
    ep.mask = BF(*mask);
    ep.ldm = (int)ldm;
  }
  ep.slab_stride = 0;
  return ep;
}

mnistx::GemmEpi make_slab(const Tensor& slab, int64_t splits, int64_t M, int64_t N) {
  check(slab, at::kFloat, splits * M * N, "slab");
  mnistx::GemmEpi ep{};
  ep.out = slab.data_ptr();
  ep.ldc = (int)N;
  ep.mode = mnistx::EPI_SLAB;
  ep.slab_stride = M * N;
  return ep;
}

// Effective split count the launcher will use (kchunk rounded to BK=32).
// split-K count the weight-gradient launch really uses: chunks round up to its
// K step (gemm.hip BK_WG = 32)
int64_t eff_splits(int64_t K, int64_t splits) {
  if (splits < 1) splits = 1;
  int64_t kchunk = (K + splits - 1) / splits;
  kchunk = ((kchunk + 31) / 32) * 32;
  if (kchunk < 32) kchunk = 32;
  return (K + kchunk - 1) / kchunk;
}

void dense_fwd(Tensor x, Tensor w, Tensor out, int64_t M, int64_t N, int64_t K, int64_t ldx, int64_t ldw,
               int64_t ldc, optional<Tensor> bias, int64_t bias_n, bool relu, optional<Tensor> mask, int64_t ldm,
               int64_t tile) {
  check(x, at::kBFloat16, span(M, ldx, K), "x");
  check(w, at::kBFloat16, span(K, ldw, N), "w");
  TORCH_CHECK(ldx >= K && ldw >= N, "bad leading dims");
  auto ep = make_epi(out, M, N, ldc, bias, bias_n, relu, mask, ldm);
  hip_ok(mnistx::dense_fwd(BF(x), BF(w), (int)M, (int)N, (int)K, (int)ldx, (int)ldw, ep, cur_stream(), (int)tile),
         "dense_fwd");
}

void dense_dgrad(Tensor dy, Tensor w, Tensor out, int64_t M, int64_t N, int64_t K, int64_t lddy, int64_t ldw,
                 int64_t ldc, optional<Tensor> mask, int64_t ldm, int64_t tile) {
  // out[M, N=Din] = dy[M, K=Dout] . W[Din, Dout]^T
  check(dy, at::kBFloat16, span(M, lddy, K), "dy");
  check(w, at::kBFloat16, span(N, ldw, K), "w");
  TORCH_CHECK(lddy >= K && ldw >= K, "bad leading dims");
  auto ep = make_epi(out, M, N, ldc, c10::nullopt, 0, false, mask, ldm);
  hip_ok(mnistx::dense_dgrad(BF(dy), BF(w), (int)M, (int)N, (int)K, (int)lddy, (int)ldw, ep, cur_stream(),
                             (int)tile),
         "dense_dgrad");
}

int64_t dense_wgrad(Tensor x, Tensor dy, Tensor slab, int64_t Din, int64_t Dout, int64_t B, int64_t ldx, int64_t lddy,
                    bool with_bias, int64_t splits, int64_t tile) {
  check(x, at::kBFloat16, span(B, ldx, Din), "x");
  check(dy, at::kBFloat16, span(B, lddy, Dout), "dy");
  TORCH_CHECK(ldx >= Din && lddy >= Dout, "bad leading dims");
  const int64_t M = Din + (with_bias ? 1 : 0);
  const int64_t S = eff_splits(B, splits);
  auto ep = make_slab(slab, S, M, Dout);
  int used = (int)S;
  hip_ok(mnistx::dense_wgrad(BF(x), BF(dy), (int)Din, (int)Dout, (int)B, (int)ldx, (int)lddy, with_bias ? 1 : 0,
                             (int)S, ep, cur_stream(), (int)tile, &used),
         "dense_wgrad");
  return used;   // the reduce sums exactly the partials written
}

// Split count the conv weight gradient prefers (slab sizing): the halo kernel's
// persistent grid when it covers the geometry, else -1 (use the GEMM rule).
int64_t conv_wgrad_pref_splits(int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW, int64_t KH,
                               int64_t KW, int64_t ph, int64_t pw, int64_t Cout, bool with_bias) {
  if (mnistx::conv_halo_enabled() &&
      mnistx::conv5_halo_wgrad_ok((int)H, (int)W, (int)C, (int)OH, (int)OW, (int)KH, (int)KW, (int)ph, (int)pw,
                                  (int)Cout, with_bias ? 1 : 0))
    return mnistx::conv5_halo_wgrad_grid((int)Nb);
  return -1;
}

// Grouped dense weight gradients (with bias rows) in one launch; returns the
// effective split counts.  Every problem must take the vector loader path
// (leading dims and widths multiples of 8): the executor checks dense_wgrad_group_ok.
std::vector<int64_t> dense_wgrad_group(std::vector<Tensor> x, std::vector<Tensor> dy, std::vector<Tensor> slab,
                                       std::vector<int64_t> Din, std::vector<int64_t> Dout, int64_t B,
                                       std::vector<int64_t> splits) {
  const size_t n = x.size();
  TORCH_CHECK(n >= 1 && n <= 4 && dy.size() == n && slab.size() == n && Din.size() == n && Dout.size() == n &&
                  splits.size() == n,
              "dense_wgrad_group: 1-4 problems, matching lists");
  const mnistx::bf16_t* xp[4];
  const mnistx::bf16_t* dp[4];
  int din[4], dout[4], ldx[4], lddy[4], sp[4];
  mnistx::GemmEpi ep[4];
  for (size_t p = 0; p < n; ++p) {
    TORCH_CHECK(x[p].dim() == 2 && dy[p].dim() == 2, "dense_wgrad_group: 2-D operands");
    const int64_t lx = x[p].size(1), ly = dy[p].size(1);
    TORCH_CHECK(Din[p] % 8 == 0 && Dout[p] % 8 == 0 && lx % 8 == 0 && ly % 8 == 0 && lx >= Din[p] && ly >= Dout[p],
                "dense_wgrad_group: widths must be multiples of 8");
    check(x[p], at::kBFloat16, span(B, lx, Din[p]), "x");
    check(dy[p], at::kBFloat16, span(B, ly, Dout[p]), "dy");
    const int64_t S = eff_splits(B, splits[p]);
    ep[p] = make_slab(slab[p], S, Din[p] + 1, Dout[p]);
    xp[p] = BF(x[p]);
    dp[p] = BF(dy[p]);
    din[p] = (int)Din[p];
    dout[p] = (int)Dout[p];
    ldx[p] = (int)lx;
    lddy[p] = (int)ly;
    sp[p] = (int)S;
  }
  hip_ok(mnistx::dense_wgrad_group((int)n, xp, dp, din, dout, (int)B, ldx, lddy, sp, ep, cur_stream()),
         "dense_wgrad_group");
  return std::vector<int64_t>(sp, sp + n);
}

mnistx::LrnParams lrn_params(int64_t lrn_r, double b, double a, double be) {
  TORCH_CHECK(lrn_r == 0 || lrn_r == 4, "LRN fold: depth_radius 4 only");
  return mnistx::LrnParams{(float)b, (float)a, (float)be, lrn_r == 4 ? 1 : 0};
}

void conv_fwd(Tensor x, Tensor w, Tensor out, int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW,
              int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t Cout, optional<Tensor> bias, int64_t bias_n,
              bool relu, int64_t lrn_r, double lrn_bias, double lrn_alpha, double lrn_beta) {
  check(x, at::kBFloat16, Nb * H * W * C, "x");
  check(w, at::kBFloat16, KH * KW * C * Cout, "w");
  TORCH_CHECK(Cout % 8 == 0, "Cout must be padded to a multiple of 8");
  auto ep = make_epi(out, Nb * OH * OW, Cout, Cout, bias, bias_n, relu, c10::nullopt, 0);
  hip_ok(mnistx::conv_fwd(BF(x), BF(w), (int)Nb, (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)KH, (int)KW, (int)ph,
                          (int)pw, (int)Cout, ep, cur_stream(), lrn_params(lrn_r, lrn_bias, lrn_alpha, lrn_beta)),
         "conv_fwd");
}

void conv_dgrad(Tensor dy, Tensor w, Tensor out, int64_t Nb, int64_t OH, int64_t OW, int64_t Cout, int64_t H,
                int64_t W, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t Cin, optional<Tensor> mask) {
  check(dy, at::kBFloat16, Nb * OH * OW * Cout, "dy");
  check(w, at::kBFloat16, KH * KW * Cin * Cout, "w");
  TORCH_CHECK(Cout % 8 == 0 && Cin % 8 == 0, "channels must be padded to multiples of 8");
  auto ep = make_epi(out, Nb * H * W, Cin, Cin, c10::nullopt, 0, false, mask, Cin);
  hip_ok(mnistx::conv_dgrad(BF(dy), BF(w), (int)Nb, (int)OH, (int)OW, (int)Cout, (int)H, (int)W, (int)KH, (int)KW,
                            (int)ph, (int)pw, (int)Cin, ep, cur_stream()),
         "conv_dgrad");
}

int64_t conv_wgrad(Tensor x, Tensor dy, Tensor slab, int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t OH,
                   int64_t OW, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t Cout, bool with_bias,
                   int64_t splits, int64_t lrn_r, double lrn_bias, double lrn_alpha, double lrn_beta) {
  check(x, at::kBFloat16, Nb * H * W * C, "x");
  check(dy, at::kBFloat16, Nb * OH * OW * Cout, "dy");
  TORCH_CHECK(Cout % 8 == 0, "Cout must be padded to a multiple of 8");
  const int64_t M = KH * KW * C + (with_bias ? 1 : 0);
  const bool halo = mnistx::conv_halo_enabled() &&
                    mnistx::conv5_halo_wgrad_ok((int)H, (int)W, (int)C, (int)OH, (int)OW, (int)KH, (int)KW, (int)ph,
                                                (int)pw, (int)Cout, with_bias ? 1 : 0);
  // halo weight gradient: one partial per persistent block (at most `splits`)
  const int64_t S = halo ? std::max<int64_t>(1, std::min<int64_t>(splits, mnistx::conv5_halo_wgrad_grid((int)Nb)))
                         : eff_splits(Nb * OH * OW, splits);
  auto ep = make_slab(slab, S, M, Cout);
  hip_ok(mnistx::conv_wgrad(BF(x), BF(dy), (int)Nb, (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)KH, (int)KW,
                            (int)ph, (int)pw, (int)Cout, with_bias ? 1 : 0, (int)S, ep, cur_stream(),
                            lrn_params(lrn_r, lrn_bias, lrn_alpha, lrn_beta)),
         "conv_wgrad");
  return S;
}

// lab_src [N] / lab_out [n] (optional, int32): gather the chosen rows' labels in the same launch
void perm_positions(Tensor out, int64_t start, int64_t N, int64_t seed, int64_t h, optional<Tensor> lab_src,
                    optional<Tensor> lab_out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous(), "perm_positions: out");
  TORCH_CHECK(N > 0 && h >= 1 && h <= 31 && (1ll << (2 * h)) >= N, "perm_positions: bad domain");
  const bool labs = lab_src.has_value() && lab_src->defined();
  TORCH_CHECK(labs == (lab_out.has_value() && lab_out->defined()), "perm_positions: lab_src and lab_out together");
  if (labs) {
    check(*lab_src, at::kInt, N, "lab_src");
    check(*lab_out, at::kInt, out.numel(), "lab_out");
  }
  hip_ok(mnistx::perm_positions(out.data_ptr<int64_t>(), start, (int)out.numel(), N, (uint32_t)seed, (int)h,
                                cur_stream(), labs ? P<const int32_t>(*lab_src) : nullptr,
                                labs ? P<int32_t>(*lab_out) : nullptr),
         "perm_positions");
}

void prep_images_perm(Tensor src, Tensor lab_src, Tensor out, Tensor lab_out, int64_t B, int64_t start, int64_t seed,
                      int64_t h) {
  TORCH_CHECK(src.dim() == 2 && src.size(1) == 784, "prep_images_perm: [N, 784] uint8 dataset");
  const int64_t N = src.size(0);
  check(src, at::kByte, N * 784, "src");
  check(lab_src, at::kInt, N, "lab_src");
  check(out, at::kBFloat16, B * 784, "out");
  check(lab_out, at::kInt, B, "lab_out");
  TORCH_CHECK(N > 0 && h >= 1 && h <= 31 && (1ll << (2 * h)) >= N, "prep_images_perm: bad domain");
  hip_ok(mnistx::prep_images_perm(P<const uint8_t>(src), P<const int32_t>(lab_src), (int)B, start, N, (uint32_t)seed,
                                  (int)h, BFm(out), P<int32_t>(lab_out), cur_stream()),
         "prep_images_perm");
}

void prep_images(Tensor src, Tensor idx, Tensor lab_src, Tensor out, Tensor lab_out, int64_t HW, int64_t Csrc,
                 int64_t Cdst) {
  const int64_t B = idx.numel();
  TORCH_CHECK((HW * Cdst) % 8 == 0, "HW*C must be a multiple of 8");
  check(idx, at::kLong, B, "idx");
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.is_contiguous(), "src: uint8 GPU tensor");
  TORCH_CHECK(src.numel() % (HW * Csrc) == 0, "src size");
  check(lab_src, at::kInt, src.numel() / (HW * Csrc), "lab_src");
  check(out, at::kBFloat16, B * HW * Cdst, "out");
  check(lab_out, at::kInt, B, "lab_out");
  hip_ok(mnistx::prep_images(P<const uint8_t>(src), P<const int64_t>(idx), P<const int32_t>(lab_src), (int)B,
                             (int)HW, (int)Csrc, (int)Cdst, BFm(out), P<int32_t>(lab_out), cur_stream()),
         "prep_images");
}

void maxpool_fwd(Tensor x, Tensor y, Tensor arg, int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t OH,
                 int64_t OW) {
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  TORCH_CHECK(OH == (H + 1) / 2 && OW == (W + 1) / 2, "2x2/2 SAME pooling shape");
  check(x, at::kBFloat16, Nb * H * W * C, "x");
  check(y, at::kBFloat16, Nb * OH * OW * C, "y");
  check(arg, at::kByte, Nb * OH * OW * C, "arg");
  hip_ok(mnistx::maxpool_fwd(BF(x), (int)Nb, (int)H, (int)W, (int)C, (int)OH, (int)OW, BFm(y), P<uint8_t>(arg),
                             cur_stream()),
         "maxpool_fwd");
}

void maxpool_bwd(Tensor dy, Tensor arg, Tensor y, bool relu_mask, Tensor dx, int64_t Nb, int64_t H, int64_t W,
                 int64_t C, int64_t OH, int64_t OW) {
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  TORCH_CHECK(OH == (H + 1) / 2 && OW == (W + 1) / 2, "2x2/2 SAME pooling shape");
  check(dy, at::kBFloat16, Nb * OH * OW * C, "dy");
  check(arg, at::kByte, Nb * OH * OW * C, "arg");
  check(y, at::kBFloat16, Nb * OH * OW * C, "y");
  check(dx, at::kBFloat16, Nb * H * W * C, "dx");
  hip_ok(mnistx::maxpool_bwd(BF(dy), P<const uint8_t>(arg), BF(y), relu_mask ? 1 : 0, (int)Nb, (int)H, (int)W,
                             (int)C, (int)OH, (int)OW, BFm(dx), cur_stream()),
         "maxpool_bwd");
}

void lrn_fwd(Tensor x, Tensor y, int64_t P_, int64_t C, int64_t r, double bias, double alpha, double beta) {
  check(x, at::kBFloat16, P_ * C, "x");
  check(y, at::kBFloat16, P_ * C, "y");
  hip_ok(mnistx::lrn_fwd(BF(x), (int)P_, (int)C, (int)r, (float)bias, (float)alpha, (float)beta, BFm(y),
                         cur_stream()),
         "lrn_fwd");
}

void lrn_bwd(Tensor x, Tensor dy, Tensor dx, int64_t P_, int64_t C, int64_t r, double bias, double alpha,
             double beta, bool relu_mask) {
  check(x, at::kBFloat16, P_ * C, "x");
  check(dy, at::kBFloat16, P_ * C, "dy");
  check(dx, at::kBFloat16, P_ * C, "dx");
  hip_ok(mnistx::lrn_bwd(BF(x), BF(dy), (int)P_, (int)C, (int)r, (float)bias, (float)alpha, (float)beta,
                         relu_mask ? 1 : 0, BFm(dx), cur_stream()),
         "lrn_bwd");
}

bool lrn_pool_supported(int64_t H, int64_t W, int64_t C, int64_t r) {
  return mnistx::lrn_pool_supported((int)H, (int)W, (int)C, (int)r);
}

void lrn_pool_fwd(Tensor x, Tensor y, Tensor arg, int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t r,
                  double bias, double alpha, double beta, bool nonneg) {
  TORCH_CHECK(mnistx::lrn_pool_supported((int)H, (int)W, (int)C, (int)r), "lrn_pool: unsupported geometry");
  check(x, at::kBFloat16, Nb * H * W * C, "x");
  check(y, at::kBFloat16, Nb * (H / 2) * (W / 2) * C, "y");
  check(arg, at::kByte, Nb * (H / 2) * (W / 2) * C, "arg");
  hip_ok(mnistx::lrn_pool_fwd(BF(x), (int)Nb, (int)H, (int)W, (int)C, (int)r, (float)bias, (float)alpha,
                              (float)beta, BFm(y), P<uint8_t>(arg), cur_stream(), nonneg ? 1 : 0),
         "lrn_pool_fwd");
}

void lrn_pool_bwd(Tensor x, Tensor dP, Tensor arg, Tensor dx, int64_t Nb, int64_t H, int64_t W, int64_t C,
                  int64_t r, double bias, double alpha, double beta, bool relu_mask) {
  TORCH_CHECK(mnistx::lrn_pool_supported((int)H, (int)W, (int)C, (int)r), "lrn_pool: unsupported geometry");
  check(x, at::kBFloat16, Nb * H * W * C, "x");
  check(dP, at::kBFloat16, Nb * (H / 2) * (W / 2) * C, "dP");
  check(arg, at::kByte, Nb * (H / 2) * (W / 2) * C, "arg");
  check(dx, at::kBFloat16, Nb * H * W * C, "dx");
  hip_ok(mnistx::lrn_pool_bwd(BF(x), BF(dP), P<const uint8_t>(arg), (int)Nb, (int)H, (int)W, (int)C, (int)r,
                              (float)bias, (float)alpha, (float)beta, relu_mask ? 1 : 0, BFm(dx), cur_stream()),
         "lrn_pool_bwd");
}

int64_t softmax_ce(Tensor logits, int64_t ldl, optional<Tensor> labels, int64_t B, int64_t NC, double scale,
                   optional<Tensor> dlogits, int64_t ldd, optional<Tensor> stats, optional<Tensor> probs,
                   optional<Tensor> work, bool defer_stats, optional<Tensor> dbias) {
  TORCH_CHECK(ldl >= NC, "ldl < NC");
  check(logits, at::kFloat, B * ldl, "logits");   // whole padded rows (vector loads)
  const int32_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    check(*labels, at::kInt, B, "labels");
    lab = P<const int32_t>(*labels);
  }
  mnistx::bf16_t* dl = nullptr;
  if (dlogits.has_value() && dlogits->defined()) {
    TORCH_CHECK(lab != nullptr, "dlogits needs labels");
    TORCH_CHECK(ldd >= NC, "ldd < NC");
    check(*dlogits, at::kBFloat16, B * ldd, "dlogits");
    TORCH_CHECK(ldd == ldl || ldd >= NC, "ldd");
    dl = BFm(*dlogits);
  }
  float* st = nullptr;
  if (stats.has_value() && stats->defined()) {
    check(*stats, at::kFloat, 8, "stats");
    st = P<float>(*stats);
  }
  float* pr = nullptr;
  if (probs.has_value() && probs->defined()) {
    check(*probs, at::kFloat, B * NC, "probs");
    pr = P<float>(*probs);
  }
  float* wk = nullptr;
  if (work.has_value() && work->defined()) {
    check(*work, at::kFloat, 4 * 1024 + 1, "work");
    wk = P<float>(*work);
  }
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(dl != nullptr, "dbias needs dlogits");
    const int nblk = mnistx::softmax_ce_dbias_blocks((int)B, (int)ldl);
    TORCH_CHECK(nblk > 0, "dbias: only the row kernel (ldl 16 / 32) writes bias partials");
    check(*dbias, at::kFloat, (int64_t)nblk * ldl, "dbias");
    db = P<float>(*dbias);
  }
  int deferred = 0;
  hip_ok(mnistx::softmax_ce(P<const float>(logits), (int)ldl, lab, (int)B, (int)NC, (float)scale, dl, (int)ldd, st, pr,
                            wk, cur_stream(), defer_stats ? &deferred : nullptr, db),
         "softmax_ce");
  return deferred;   // blocks whose CE partials the caller's finalize_step must combine
}

bool mlp_head_supported(int64_t d0, int64_t ld1, int64_t ld2, int64_t ld3, int64_t n1, int64_t n2, int64_t nc,
                        int64_t B) {
  return mnistx::mlp_head_supported((int)d0, (int)ld1, (int)ld2, (int)ld3, (int)n1, (int)n2, (int)nc, (int)B);
}

// Fused LeNet-5 dense head.  x [>=nb, 400] bf16; w3t [128,416], w4t [96,128], w5t [16,96]
// zero-padded transposed bf16 weights (FlatParams.bf16t_view); outputs h3 [nb,120], h4 [nb,88] bf16, logits [nb,16] fp32;
// with dl: dl [nb,16], dh4 [nb,88], dh3 [nb,120], dx [nb,400] bf16.
bool ce_tail_supported(int64_t d0, int64_t nc, int64_t B) { return mnistx::ce_tail_supported((int)d0, (int)nc, (int)B); }

// the reference CNN's softmax_linear + softmax CE (+ data gradient masked by x > 0): mlp_head.hip ce_tail_k
void ce_tail(Tensor x, Tensor w5t, Tensor b5, int64_t nc, Tensor labels, int64_t nb, double scale, Tensor logits,
             optional<Tensor> dl, optional<Tensor> dx, Tensor stats, optional<Tensor> work, bool defer_stats,
             optional<Tensor> dbias) {
  TORCH_CHECK(mnistx::ce_tail_supported(192, (int)nc, (int)std::max<int64_t>(nb, 1)), "ce_tail: unsupported geometry");
  check(x, at::kBFloat16, nb * 192, "x");
  check(w5t, at::kBFloat16, 16 * 192, "w5t");
  check(b5, at::kFloat, nc, "b5");
  check(labels, at::kInt, nb, "labels");
  check(logits, at::kFloat, nb * 16, "logits");
  check(stats, at::kFloat, 8, "stats");
  for (const Tensor* t : {&x, &w5t, &logits})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "ce_tail: operands must be 16-byte aligned");
  const bool has_work = work.has_value() && work->defined();
  if (has_work) check(*work, at::kFloat, 4 * 1024 + 1, "work");
  mnistx::bf16_t *pdl = nullptr, *pdx = nullptr;
  if (dl.has_value() && dl->defined()) {
    TORCH_CHECK(dx.has_value() && dx->defined(), "ce_tail: dl needs dx");
    check(*dl, at::kBFloat16, nb * 16, "dl");
    check(*dx, at::kBFloat16, nb * 192, "dx");
    for (const Tensor* t : {&*dl, &*dx})
      TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "ce_tail: gradients must be 16-byte aligned");
    pdl = BFm(*dl);
    pdx = BFm(*dx);
  }
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(pdl != nullptr, "ce_tail: dbias needs dl");
    check(*dbias, at::kFloat, (int64_t)mnistx::ce_tail_blocks((int)nb) * 16, "dbias");
    db = P<float>(*dbias);
  }
  hip_ok(mnistx::ce_tail(BF(x), BF(w5t), P<const float>(b5), (int)nc, P<const int32_t>(labels), (int)nb, (float)scale,
                         P<float>(logits), pdl, pdx, P<float>(stats), has_work ? P<float>(*work) : nullptr, cur_stream(),
                         defer_stats ? 1 : 0, db),
         "ce_tail");
}

void mlp_head(Tensor x, Tensor w3t, Tensor b3, int64_t n1, Tensor w4t, Tensor b4, int64_t n2, Tensor w5t, Tensor b5,
              int64_t nc, Tensor labels, int64_t nb, double scale, Tensor h3, Tensor h4, Tensor logits,
              optional<Tensor> dl, optional<Tensor> dh4, optional<Tensor> dh3, optional<Tensor> dx, Tensor stats,
              optional<Tensor> work, bool defer_stats, optional<Tensor> dbias) {
  TORCH_CHECK(mnistx::mlp_head_supported(400, 120, 88, 16, (int)n1, (int)n2, (int)nc, (int)std::max<int64_t>(nb, 1)),
              "mlp_head: unsupported geometry");
  check(x, at::kBFloat16, nb * 400, "x");
  check(w3t, at::kBFloat16, 128 * 416, "w3t");
  check(w4t, at::kBFloat16, 96 * 128, "w4t");
  check(w5t, at::kBFloat16, 16 * 96, "w5t");
  check(b3, at::kFloat, n1, "b3");
  check(b4, at::kFloat, n2, "b4");
  check(b5, at::kFloat, nc, "b5");
  check(labels, at::kInt, nb, "labels");
  check(h3, at::kBFloat16, nb * 120, "h3");
  check(h4, at::kBFloat16, nb * 88, "h4");
  check(logits, at::kFloat, nb * 16, "logits");
  check(stats, at::kFloat, 8, "stats");
  const bool has_work = work.has_value() && work->defined();   // none: order-dependent atomics
  if (has_work) check(*work, at::kFloat, 4 * 1024 + 1, "work");
  for (const Tensor* t : {&x, &w3t, &w4t, &w5t, &h3, &h4, &logits})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "mlp_head: operands must be 16-byte aligned");
  mnistx::bf16_t *pdl = nullptr, *pdh4 = nullptr, *pdh3 = nullptr, *pdx = nullptr;
  if (dl.has_value() && dl->defined()) {
    TORCH_CHECK(dh4.has_value() && dh3.has_value() && dx.has_value(), "mlp_head: dl needs dh4, dh3, dx");
    check(*dl, at::kBFloat16, nb * 16, "dl");
    check(*dh4, at::kBFloat16, nb * 88, "dh4");
    check(*dh3, at::kBFloat16, nb * 120, "dh3");
    check(*dx, at::kBFloat16, nb * 400, "dx");
    for (const Tensor* t : {&*dl, &*dh4, &*dh3, &*dx})
      TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 8 == 0, "mlp_head: gradients must be 8-byte aligned");
    pdl = BFm(*dl);
    pdh4 = BFm(*dh4);
    pdh3 = BFm(*dh3);
    pdx = BFm(*dx);
  }
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(pdl != nullptr, "mlp_head: dbias needs dl");
    check(*dbias, at::kFloat, (int64_t)mnistx::mlp_head_blocks((int)nb) * 16, "dbias");
    db = P<float>(*dbias);
  }
  hip_ok(mnistx::mlp_head(BF(x), BF(w3t), P<const float>(b3), (int)n1, BF(w4t), P<const float>(b4), (int)n2, BF(w5t),
                          P<const float>(b5), (int)nc, P<const int32_t>(labels), (int)nb, (float)scale, BFm(h3),
                          BFm(h4), P<float>(logits), pdl, pdh4, pdh3, pdx, P<float>(stats), has_work ? P<float>(*work) : nullptr,
                          cur_stream(), (defer_stats && has_work) ? 1 : 0, db),
         "mlp_head");
}

mnistx::RedSpec red_spec(Tensor slab, int64_t splits, int64_t M, int64_t N, int64_t G, int64_t Ipad, int64_t I,
                         int64_t J, int64_t bias_row, Tensor wdst, const Tensor* bdst, double scale) {
  check(slab, at::kFloat, splits * M * N, "slab");
  TORCH_CHECK(I <= Ipad && J <= N && G * Ipad <= M, "reduce geometry");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(slab.data_ptr()) % 16 == 0, "slab must be 16-byte aligned");
  check(wdst, at::kFloat, G * I * J, "wdst");
  float* b = nullptr;
  if (bdst != nullptr && bdst->defined() && bdst->numel() > 0) {
    TORCH_CHECK(bias_row >= 0 && bias_row < M, "bias_row");
    check(*bdst, at::kFloat, J, "bdst");
    b = P<float>(*bdst);
  }
  return mnistx::RedSpec{P<float>(slab), P<float>(wdst), b, (int)splits, (int)M, (int)N, (int)G, (int)Ipad, (int)I,
                         (int)J, (int)bias_row, (float)scale};
}

void splitk_reduce(Tensor slab, int64_t splits, int64_t M, int64_t N, int64_t G, int64_t Ipad, int64_t I, int64_t J,
                   int64_t bias_row, Tensor wdst, optional<Tensor> bdst, double scale) {
  const Tensor* bp = (bdst.has_value() && bdst->defined()) ? &*bdst : nullptr;
  const mnistx::RedSpec r = red_spec(slab, splits, M, N, G, Ipad, I, J, bias_row, wdst, bp, scale);
  hip_ok(mnistx::splitk_reduce_multi(&r, 1, cur_stream()), "splitk_reduce");
}

// Several split-K slabs reduced by one launch per pass.  geo: int64 [n, 8] on CPU =
// (splits, M, N, G, Ipad, I, J, bias_row) per tensor; bdsts[i] empty = no bias.
void splitk_reduce_multi(std::vector<Tensor> slabs, std::vector<Tensor> wdsts, std::vector<Tensor> bdsts, Tensor geo,
                         std::vector<double> scales) {
  const int64_t n = (int64_t)slabs.size();
  TORCH_CHECK((int64_t)wdsts.size() == n && (int64_t)bdsts.size() == n && (int64_t)scales.size() == n,
              "splitk_reduce_multi: list lengths differ");
  TORCH_CHECK(geo.device().is_cpu() && geo.scalar_type() == at::kLong && geo.dim() == 2 && geo.size(0) == n &&
                  geo.size(1) == 8 && geo.is_contiguous(),
              "splitk_reduce_multi: geo must be a contiguous CPU int64 [n, 8] tensor");
  const int64_t* g = geo.data_ptr<int64_t>();
  std::vector<mnistx::RedSpec> specs;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t* r = g + 8 * i;
    specs.push_back(red_spec(slabs[i], r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], wdsts[i], &bdsts[i],
                             scales[i]));
  }
  hip_ok(mnistx::splitk_reduce_multi(specs.data(), (int)n, cur_stream()), "splitk_reduce_multi");
}

// segs: int64 tensor [nseg, 14] on CPU:
//   off, n, G, I, J, Ip, Jp, bf_off, wd_bits(float32 as int), track_l2, bft_off, Jt, It, 0
mnistx::FinArgs prep_fin(Tensor step, Tensor stats, optional<Tensor> l2, optional<Tensor> wds, int64_t nw,
                         optional<Tensor> loss_ema, int64_t n_ema, int64_t batch, bool increment,
                         optional<Tensor> l2_ranges, optional<Tensor> ce_work, int64_t ce_nblk);

void fused_optimizer(Tensor params, Tensor grads, Tensor mom, Tensor ema, Tensor bf, Tensor segs, Tensor step,
                     double lr0, double decay_rate, int64_t decay_steps, double momentum, bool nesterov,
                     bool use_momentum, double grad_scale, double ema_max, optional<Tensor> l2,
                     optional<Tensor> guard, int64_t guard_want, optional<Tensor> guard_err, int64_t guard_id,
                     optional<py::tuple> fin, optional<py::tuple> perm) {
  const int64_t total = params.numel();
  check(params, at::kFloat, total, "params");
  check(grads, at::kFloat, total, "grads");
  if (use_momentum) check(mom, at::kFloat, total, "mom");
  if (ema_max >= 0) check(ema, at::kFloat, total, "ema");
  check(step, at::kLong, 1, "step");
  TORCH_CHECK(!segs.is_cuda() && segs.scalar_type() == at::kLong && segs.dim() == 2 && segs.size(1) == 14,
              "segs: CPU int64 [n,14]");
  const int nseg = (int)segs.size(0);
  std::vector<mnistx::OptSeg> sv(nseg);
  auto a = segs.accessor<int64_t, 2>();
  int64_t expect_off = 0;
  int max_l2 = 0;
  for (int i = 0; i < nseg; ++i) {
    auto& s = sv[i];
    s.off = a[i][0];
    s.n = a[i][1];
    s.G = (int)a[i][2];
    s.I = (int)a[i][3];
    s.J = (int)a[i][4];
    s.Ip = (int)a[i][5];
    s.Jp = (int)a[i][6];
    s.bf_off = a[i][7];
    int32_t wb = (int32_t)a[i][8];
    std::memcpy(&s.wd, &wb, 4);
    s.track_l2 = (int)a[i][9];
    s.bft_off = a[i][10];
    s.Jt = (int)a[i][11];
    s.It = (int)a[i][12];
    TORCH_CHECK(s.off == expect_off, "segments must tile the flat buffer in order");
    TORCH_CHECK(s.n == (int64_t)s.G * s.I * s.J, "segment size mismatch");
    TORCH_CHECK(s.Ip >= s.I && s.Jp >= s.J, "padding");
    if (s.bf_off >= 0)
      TORCH_CHECK(s.bf_off + (int64_t)s.G * s.Ip * s.Jp <= bf.numel(), "bf16 copy out of range");
    if (s.bft_off >= 0) {
      TORCH_CHECK(s.bf_off >= 0 && s.G == 1 && s.Jt >= s.J && s.It >= s.I, "transposed copy geometry");
      TORCH_CHECK(s.bft_off + (int64_t)s.Jt * s.It <= bf.numel(), "transposed bf16 copy out of range");
    }
    if (s.track_l2 > max_l2) max_l2 = s.track_l2;
    expect_off += s.n;
  }
  TORCH_CHECK(expect_off == total, "segments do not cover the parameters");
  check(bf, at::kBFloat16, 0, "bf");
  float* l2p = nullptr;
  const int l2n = max_l2;
  if (l2.has_value() && l2->defined()) {
    // [max_l2 per-tensor sums | one partial per optimizer block]
    check(*l2, at::kFloat, (int64_t)max_l2 + mnistx::fused_optimizer_blocks(sv.data(), nseg), "l2");
    l2p = P<float>(*l2);
  }
  mnistx::OptParams op{};
  op.lr0 = (float)lr0;
  op.decay_rate = (float)decay_rate;
  op.decay_steps = decay_steps;
  op.momentum = (float)momentum;
  op.nesterov = nesterov ? 1 : 0;
  op.use_momentum = use_momentum ? 1 : 0;
  op.grad_scale = (float)grad_scale;
  op.ema_max = (float)ema_max;
  if (guard.has_value() && guard->defined()) {   // PS push guard: int64 stamp on the device
    check(*guard, at::kLong, 1, "guard");
    TORCH_CHECK(guard_err.has_value() && guard_err->defined(), "guard needs guard_err");
    check(*guard_err, at::kInt, 1, "guard_err");
    TORCH_CHECK(guard->device() == params.device() && guard_err->device() == params.device(),
                "guard / guard_err: on the parameters' device");
    op.guard = P<const int64_t>(*guard);
    op.guard_want = guard_want;
    op.guard_err = P<int>(*guard_err);
    op.guard_id = (int)guard_id;
  }
  // fin: finalize_step's arguments after `step` (the same step tensor), run in this launch
  mnistx::FinArgs fa{};
  const bool has_fin = fin.has_value() && !fin->is_none();
  if (has_fin) {
    const py::tuple& t = *fin;
    TORCH_CHECK(t.size() == 11, "fin: (stats, l2, wds, nw, loss_ema, n_ema, batch, increment, l2_ranges, ce_work, ce_nblk)");
    auto ot = [&](int i) { return t[i].is_none() ? optional<Tensor>() : optional<Tensor>(t[i].cast<Tensor>()); };
    fa = prep_fin(step, t[0].cast<Tensor>(), ot(1), ot(2), t[3].cast<int64_t>(), ot(4), t[5].cast<int64_t>(),
                  t[6].cast<int64_t>(), t[7].cast<bool>(), ot(8), ot(9), t[10].cast<int64_t>());
  }
  // perm: (out, lab_src, lab_out, start, N, seed, h) -- perm_positions of the next batch, run by
  // extra blocks of this launch
  mnistx::PermJob pj{};
  const bool has_perm = perm.has_value() && !perm->is_none();
  if (has_perm) {
    const py::tuple& t = *perm;
    TORCH_CHECK(t.size() == 7, "perm: (out, lab_src, lab_out, start, N, seed, h)");
    Tensor out = t[0].cast<Tensor>(), ls = t[1].cast<Tensor>(), lo = t[2].cast<Tensor>();
    const int64_t start = t[3].cast<int64_t>(), N = t[4].cast<int64_t>(), seed = t[5].cast<int64_t>(),
                  h = t[6].cast<int64_t>();
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous() &&
                    out.device() == params.device(), "perm: out");
    TORCH_CHECK(N > 0 && h >= 1 && h <= 31 && (1ll << (2 * h)) >= N, "perm: bad domain");
    TORCH_CHECK(out.numel() < (1ll << 31), "perm: too many rows");
    check(ls, at::kInt, N, "perm lab_src");
    check(lo, at::kInt, out.numel(), "perm lab_out");
    pj.out = out.data_ptr<int64_t>();
    pj.lab_src = P<const int32_t>(ls);
    pj.lab_out = P<int32_t>(lo);
    pj.start = start;
    pj.N = N;
    pj.seed = (uint32_t)seed;
    pj.h = (int)h;
    pj.n = (int)out.numel();
  }
  hip_ok(mnistx::fused_optimizer(P<float>(params), P<const float>(grads), use_momentum ? P<float>(mom) : nullptr,
                                 ema_max >= 0 ? P<float>(ema) : nullptr, BFm(bf), sv.data(), nseg, total,
                                 P<const int64_t>(step), op, l2p, l2n, cur_stream(), has_fin ? &fa : nullptr,
                                 has_perm ? &pj : nullptr),
         "fused_optimizer");
}

mnistx::FinArgs prep_fin(Tensor step, Tensor stats, optional<Tensor> l2, optional<Tensor> wds, int64_t nw,
                         optional<Tensor> loss_ema, int64_t n_ema, int64_t batch, bool increment,
                         optional<Tensor> l2_ranges, optional<Tensor> ce_work, int64_t ce_nblk) {
  check(step, at::kLong, 1, "step");
  check(stats, at::kFloat, 8, "stats");
  TORCH_CHECK(nw <= 64, "finalize: at most 64 weight-decay entries");
  mnistx::FinArgs f{};
  f.step = P<int64_t>(step);
  f.stats = P<float>(stats);
  if (nw > 0) {
    TORCH_CHECK(l2.has_value() && wds.has_value(), "l2/wds needed when nw > 0");
    check(*l2, at::kFloat, nw, "l2");
    check(*wds, at::kFloat, nw, "wds");
    f.l2 = P<float>(*l2);
    f.wds = P<const float>(*wds);
  }
  f.nw = (int)nw;
  if (loss_ema.has_value() && loss_ema->defined()) {
    check(*loss_ema, at::kFloat, 3 * n_ema, "loss_ema");
    f.loss_ema = P<float>(*loss_ema);
    f.n_ema = (int)n_ema;
  }
  if (nw > 0 && l2_ranges.has_value() && l2_ranges->defined()) {
    check(*l2_ranges, at::kInt, 3 * nw, "l2_ranges");
    f.l2r = P<const int>(*l2_ranges);
    // partials follow the nw per-weight slots (binding fused_optimizer: l2n = max track index)
  }
  f.l2base = (int)nw;
  if (ce_nblk > 0) {
    TORCH_CHECK(ce_work.has_value() && ce_work->defined() && ce_nblk <= 1024, "ce_work needed for ce_nblk > 0");
    check(*ce_work, at::kFloat, 4 * 1024 + 1, "ce_work");
    f.ce_work = P<const float>(*ce_work);
    f.ce_nblk = (int)ce_nblk;
  }
  f.batch = (int)batch;
  f.increment = increment ? 1 : 0;
  return f;
}

void finalize_step(Tensor step, Tensor stats, optional<Tensor> l2, optional<Tensor> wds, int64_t nw,
                   optional<Tensor> loss_ema, int64_t n_ema, int64_t batch, bool increment,
                   optional<Tensor> l2_ranges, optional<Tensor> ce_work, int64_t ce_nblk) {
  const auto f = prep_fin(step, stats, l2, wds, nw, loss_ema, n_ema, batch, increment, l2_ranges, ce_work, ce_nblk);
  hip_ok(mnistx::finalize_step(f, cur_stream()), "finalize_step");
}

void cast_f32_bf16_padded(Tensor src, Tensor dst, int64_t G, int64_t I, int64_t J, int64_t Ip, int64_t Jp) {
  check(src, at::kFloat, G * I * J, "src");
  check(dst, at::kBFloat16, G * Ip * Jp, "dst");
  TORCH_CHECK(Ip >= I && Jp >= J, "padding");
  hip_ok(mnistx::cast_f32_bf16_padded(P<const float>(src), BFm(dst), (int)G, (int)I, (int)J, (int)Ip, (int)Jp,
                                      cur_stream()),
         "cast_f32_bf16_padded");
}

struct CPGeo {
  int cfg, OH, OW, PH, PW, KM;
};

CPGeo cp_geo(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w) {
  CPGeo g{};
  g.cfg = mnistx::convpool_config((int)cin, (int)cout, (int)ks, (int)pad, (int)h, (int)w);
  TORCH_CHECK(g.cfg >= 0, "convpool: unsupported geometry cin=", cin, " cout=", cout, " k=", ks, " pad=", pad,
              " ", h, "x", w);
  g.OH = (int)(h + 2 * pad - ks + 1);
  g.OW = (int)(w + 2 * pad - ks + 1);
  g.PH = g.OH / 2;
  g.PW = g.OW / 2;
  g.KM = mnistx::convpool_wgrad_rows(g.cfg);
  return g;
}

int64_t convpool_supported(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w) {
  return mnistx::convpool_config((int)cin, (int)cout, (int)ks, (int)pad, (int)h, (int)w);
}

int64_t convpool_rows(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w) {
  return cp_geo(cin, cout, ks, pad, h, w).KM;
}

std::vector<int64_t> gemm_tile(int64_t M, int64_t N, bool wgrad) {
  int bm, bn;
  mnistx::gemm_tile((int)M, (int)N, wgrad ? 1 : 0, &bm, &bn);
  return {bm, bn};
}

// (G, Ipad, I, bias_row) arguments of splitk_reduce for this geometry's wgrad slab
std::vector<int64_t> convpool_reduce_args(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w,
                                          int64_t cin_real) {
  auto g = cp_geo(cin, cout, ks, pad, h, w);
  int o[4];
  TORCH_CHECK(mnistx::convpool_reduce_layout(g.cfg, o) == 0, "convpool_reduce_args");
  return {o[0], o[1], o[2] < 0 ? cin_real : (int64_t)o[2], o[3]};
}

// Input of a fused conv: bf16 x, or the uint8 dataset + per-sample index (Cin == 1 geometries)
mnistx::XSrc cp_src(const Tensor& x, const optional<Tensor>& u8, const optional<Tensor>& idx, int cfg, int64_t B,
                    int64_t hwc) {
  mnistx::XSrc src{nullptr, nullptr, nullptr, 0};
  if (u8.has_value() && u8->defined()) {
    TORCH_CHECK(mnistx::convpool_u8_input(cfg), "convpool: uint8 input only for first layers (Cin 1, or 3 at 28x28)");
    TORCH_CHECK(idx.has_value() && idx->defined(), "convpool: uint8 input needs idx");
    check(*u8, at::kByte, hwc, "u8");
    TORCH_CHECK(u8->numel() % hwc == 0 && u8->numel() < (int64_t)INT32_MAX,
                "u8: [n, H*W*C] images, < 2 GB (the kernels address it through one buffer resource)");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(u8->data_ptr()) % 4 == 0, "u8 must be 4-byte aligned");
    check(*idx, at::kLong, B, "idx");
    src.u8 = P<const uint8_t>(*u8);
    src.idx = P<const int64_t>(*idx);
    src.n = (int)(u8->numel() / hwc);       // the kernel clamps every index into [0, n)
  } else if (idx.has_value() && idx->defined()) {
    // x is the resident bf16 dataset [n, H*W*C] (normalised once), gathered through idx
    TORCH_CHECK(mnistx::convpool_u8_input(cfg), "convpool: dataset input only for first layers (Cin 1, or 3 at 28x28)");
    check(x, at::kBFloat16, hwc, "x (dataset)");
    TORCH_CHECK(x.numel() % hwc == 0 && x.numel() * 2 < (int64_t)INT32_MAX,
                "x (dataset): [n, H*W*C] bf16 images, < 2 GB (one buffer resource)");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 8 == 0, "x (dataset) must be 8-byte aligned");
    check(*idx, at::kLong, B, "idx");
    src.x = BF(x);
    src.idx = P<const int64_t>(*idx);
    src.n = (int)(x.numel() / hwc);
  } else {
    check(x, at::kBFloat16, B * hwc, "x");
    src.x = BF(x);
  }
  return src;
}

void convpool_fwd(Tensor x, Tensor w, Tensor bias, int64_t bias_n, Tensor pooled, Tensor arg, int64_t B, int64_t cin,
                  int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t wd, optional<Tensor> u8,
                  optional<Tensor> idx, optional<Tensor> lrn_out, double lrn_bias, double lrn_alpha,
                  double lrn_beta, int64_t lrn_r) {
  auto g = cp_geo(cin, cout, ks, pad, h, wd);
  const auto src = cp_src(x, u8, idx, g.cfg, B, h * wd * cin);
  check(w, at::kBFloat16, ks * ks * cin * cout, "w");
  check(bias, at::kFloat, bias_n, "bias");
  check(pooled, at::kBFloat16, B * g.PH * g.PW * cout, "pooled");
  check(arg, at::kByte, B * g.PH * g.PW * mnistx::convpool_arg_bytes(g.cfg), "arg");
  if (lrn_out.has_value() && lrn_out->defined()) {
    // the following LRN (radius 4) written by the same launch (refc1n_fwd_k): reference conv1 only
    TORCH_CHECK(lrn_r == 4 && ((g.cfg == 2 && mnistx::refc1_fwd_lrn_ok()) ||
                               (g.cfg == 3 && mnistx::refc1_fwd3_ok() && !src.u8)),
                "convpool_fwd: lrn_out only for the reference conv1 (1 or 3 -> 32, SAME; 3 channels: bf16 input) "
                "with norm1 radius 4");
    check(*lrn_out, at::kBFloat16, B * g.PH * g.PW * cout, "lrn_out");
    hip_ok(mnistx::refc1_band_fwd(src, BF(w), P<const float>(bias), (int)bias_n, (int)B, BFm(pooled), P<uint8_t>(arg),
                                  cur_stream(), BFm(*lrn_out), (float)lrn_bias, (float)lrn_alpha, (float)lrn_beta,
                                  g.cfg == 3 ? 3 : 1),
           "convpool_fwd (+ norm1)");
    return;
  }
  hip_ok(mnistx::convpool_fwd(g.cfg, src, BF(w), P<const float>(bias), (int)bias_n, (int)B, BFm(pooled),
                              P<uint8_t>(arg), cur_stream()),
         "convpool_fwd");
}

void convpool_wgrad(Tensor x, Tensor dP, Tensor arg, Tensor slab, int64_t grid, int64_t B, int64_t cin, int64_t cout,
                    int64_t ks, int64_t pad, int64_t h, int64_t wd, optional<Tensor> u8, optional<Tensor> idx,
                    optional<Tensor> lrn_p, double lrn_bias, double lrn_alpha, double lrn_beta, int64_t lrn_r) {
  auto g = cp_geo(cin, cout, ks, pad, h, wd);
  TORCH_CHECK(grid >= 1 && grid <= 65535, "grid");
  const int64_t np = B * g.PH * g.PW * cout;
  const auto src = cp_src(x, u8, idx, g.cfg, B, h * wd * cin);
  check(dP, at::kBFloat16, np, "dP");
  check(arg, at::kByte, B * g.PH * g.PW * mnistx::convpool_arg_bytes(g.cfg), "arg");
  check(slab, at::kFloat, grid * g.KM * cout, "slab");
  const mnistx::bf16_t* lp = nullptr;
  if (lrn_p.has_value() && lrn_p->defined()) {
    TORCH_CHECK(lrn_r == 4 && cout == 32 && (g.cfg == 2 || g.cfg == 3), "LRN fold: reference conv1 (Cout 32), radius 4");
    check(*lrn_p, at::kBFloat16, np, "lrn_p");
    lp = BF(*lrn_p);
  }
  hip_ok(mnistx::convpool_wgrad(g.cfg, src, BF(dP), P<const uint8_t>(arg), (int)B, P<float>(slab), (int)grid,
                                cur_stream(), lp, (float)lrn_bias, (float)lrn_alpha, (float)lrn_beta),
         "convpool_wgrad");
}

bool convpool_u8_input(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w) {
  return mnistx::convpool_u8_input(cp_geo(cin, cout, ks, pad, h, w).cfg) != 0;
}

int64_t convpool_wgrad_grid(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w) {
  const int n = mnistx::convpool_wgrad_grid(cp_geo(cin, cout, ks, pad, h, w).cfg);
  TORCH_CHECK(n > 0, "convpool_wgrad_grid: occupancy query failed");
  return n;
}

int64_t convpool_arg_bytes(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w) {
  return mnistx::convpool_arg_bytes(cp_geo(cin, cout, ks, pad, h, w).cfg);
}

bool convpool_has_dgrad(int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w) {
  return mnistx::convpool_has_dgrad(cp_geo(cin, cout, ks, pad, h, w).cfg) != 0;
}

void convpool_dgrad(Tensor dP, Tensor arg, Tensor w, Tensor dx, int64_t B, int64_t cin, int64_t cout, int64_t ks,
                    int64_t pad, int64_t h, int64_t wd, int64_t grid_cap) {
  auto g = cp_geo(cin, cout, ks, pad, h, wd);
  TORCH_CHECK(mnistx::convpool_has_dgrad(g.cfg), "convpool_dgrad: no fused dgrad for this geometry");
  const int64_t np = B * g.PH * g.PW * cout;
  check(dP, at::kBFloat16, np, "dP");
  check(arg, at::kByte, B * g.PH * g.PW * mnistx::convpool_arg_bytes(g.cfg), "arg");
  check(w, at::kBFloat16, ks * ks * cin * cout, "w");
  check(dx, at::kBFloat16, B * h * wd * cin, "dx");
  hip_ok(mnistx::convpool_dgrad(g.cfg, BF(dP), P<const uint8_t>(arg), BF(w), (int)B, BFm(dx), (int)grid_cap,
                                cur_stream()),
         "convpool_dgrad");
}

// LeNet-5 conv1+pool1+conv2+pool2 forward on banded MFMA tiles (lenet_band.hip).
// x: bf16 images [n, 784] gathered through idx, or the batch itself [B, 784] (idx None).
void lenet_band_fwd(Tensor x, Tensor w1, Tensor b1, int64_t b1n, Tensor w2, Tensor b2, int64_t B, Tensor p2,
                    Tensor arg2, optional<Tensor> p1, optional<Tensor> arg1, optional<Tensor> idx,
                    optional<Tensor> prof) {
  mnistx::XSrc src{nullptr, nullptr, nullptr, 0};
  if (x.scalar_type() == at::kByte) {   // uint8 images, normalised x/255 - 0.5 in the kernel
    check(x, at::kByte, 784, "x");
    TORCH_CHECK(x.numel() % 784 == 0 && x.numel() < (int64_t)INT32_MAX, "x: [n, 784] uint8 images, < 2 GB");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 4 == 0, "x must be 4-byte aligned");
    src.u8 = P<const uint8_t>(x);
  } else {
    check(x, at::kBFloat16, 784, "x");
    TORCH_CHECK(x.numel() % 784 == 0 && x.numel() * 2 < (int64_t)INT32_MAX, "x: [n, 784] bf16 images, < 2 GB");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "x must be 16-byte aligned");
    src.x = BF(x);
  }
  src.n = (int)(x.numel() / 784);
  if (idx.has_value() && idx->defined()) {
    check(*idx, at::kLong, B, "idx");
    src.idx = P<const int64_t>(*idx);
  } else {
    TORCH_CHECK(src.n >= B, "x: needs B images without idx");
  }
  check(w1, at::kBFloat16, 5 * 5 * 8, "w1");
  check(b1, at::kFloat, b1n, "b1");
  TORCH_CHECK(b1n >= 0 && b1n <= 8, "b1n");
  check(w2, at::kBFloat16, 5 * 5 * 8 * 16, "w2");
  check(b2, at::kFloat, 16, "b2");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w1.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w2.data_ptr()) % 16 == 0,
              "w1 / w2 must be 16-byte aligned");
  check(p2, at::kBFloat16, B * 400, "p2");
  check(arg2, at::kByte, B * 400, "arg2");
  mnistx::bf16_t* pp1 = nullptr;
  uint8_t* pa1 = nullptr;
  if (p1.has_value() && p1->defined()) {   // with arg1: the convpool layouts; without: combined records
    check(*p1, at::kBFloat16, B * 14 * 14 * 8, "p1");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(p1->data_ptr()) % 16 == 0, "p1 must be 16-byte aligned");
    pp1 = BFm(*p1);
    if (arg1.has_value() && arg1->defined()) {
      check(*arg1, at::kByte, B * 14 * 14 * 4, "arg1");
      pa1 = P<uint8_t>(*arg1);
    }
  }
  unsigned long long* pr = nullptr;
  if (prof.has_value() && prof->defined()) {   // experiments: int64[4] clock sums
    check(*prof, at::kLong, 4, "prof");
    pr = P<unsigned long long>(*prof);
  }
  hip_ok(mnistx::lenet_band_fwd(src, BF(w1), P<const float>(b1), (int)b1n, BF(w2), P<const float>(b2), (int)B, pp1,
                                pa1, BFm(p2), P<uint8_t>(arg2), cur_stream(), pr),
         "lenet_band_fwd");
}

// LeNet-5 conv-stack backward as one kernel (lenet_bwd.hip): conv2 dgrad + both weight
// gradients; x as for lenet_band_fwd (the forward's input), p1c (the combined pool1 records:
// lenet_band_fwd with p1 and no arg1) / arg2 from it, dp2 = dL/d pool2 [B, 400].
// slab1 [grid, 32, 8], slab2 [grid, 208, 16] (split-K partials).
void lenet_bwd(Tensor x, Tensor p1, Tensor dp2, Tensor arg2, Tensor w2, int64_t B, Tensor slab1, Tensor slab2,
               int64_t grid, optional<Tensor> idx, optional<Tensor> prof) {
  mnistx::XSrc src{nullptr, nullptr, nullptr, 0};
  if (x.scalar_type() == at::kByte) {
    check(x, at::kByte, 784, "x");
    TORCH_CHECK(x.numel() % 784 == 0 && x.numel() < (int64_t)INT32_MAX, "x: [n, 784] uint8 images, < 2 GB");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 4 == 0, "x must be 4-byte aligned");
    src.u8 = P<const uint8_t>(x);
  } else {
    check(x, at::kBFloat16, 784, "x");
    TORCH_CHECK(x.numel() % 784 == 0 && x.numel() * 2 < (int64_t)INT32_MAX, "x: [n, 784] bf16 images, < 2 GB");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 8 == 0, "x must be 8-byte aligned");
    src.x = BF(x);
  }
  src.n = (int)(x.numel() / 784);
  if (idx.has_value() && idx->defined()) {
    check(*idx, at::kLong, B, "idx");
    src.idx = P<const int64_t>(*idx);
  } else {
    TORCH_CHECK(src.n >= B, "x: needs B images without idx");
  }
  TORCH_CHECK(B >= 1 && B * 196 * 16 < (int64_t)INT32_MAX, "B");
  check(p1, at::kBFloat16, B * 196 * 8, "p1");
  check(dp2, at::kBFloat16, B * 400, "dp2");
  check(arg2, at::kByte, B * 400, "arg2");
  check(w2, at::kBFloat16, 5 * 5 * 8 * 16, "w2");
  for (const Tensor* t : {&p1, &dp2, &w2})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "p1 / dp2 / w2 must be 16-byte aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(arg2.data_ptr()) % 8 == 0, "arg2 alignment");
  const int res = mnistx::lenet_bwd_blocks((int)B);
  TORCH_CHECK(res > 0, "lenet_bwd: occupancy query failed");
  TORCH_CHECK(grid >= 1 && grid <= res, "lenet_bwd: grid must be in [1, ", res, "] (one block per CU, <= tiles)");
  check(slab1, at::kFloat, grid * 32 * 8, "slab1");
  check(slab2, at::kFloat, grid * 208 * 16, "slab2");
  unsigned long long* pr = nullptr;
  if (prof.has_value() && prof->defined()) {
    const char* pw = getenv("MNISTX_BWD_PROF_WAVES");
    check(*prof, at::kLong, (pw && pw[0] == '1') ? 8 + 16 * 8 : 8, "prof");
    pr = P<unsigned long long>(*prof);
  }
  hip_ok(mnistx::lenet_bwd(src, BF(p1), BF(dp2), P<const uint8_t>(arg2), BF(w2), (int)B, P<float>(slab1),
                           P<float>(slab2), (int)grid, cur_stream(), pr),
         "lenet_bwd");
}

// Reference-CNN conv1 weight gradient with the norm1 backward folded in (refc1_wgrad.hip).
// x / u8 / idx as for convpool_wgrad (cfg RefC1g); dn = dL/d norm1, p1 = pool1, arg = pool1 codes.
void refc1_wgrad(Tensor x, Tensor dn, Tensor p1, Tensor arg, Tensor slab, int64_t grid, int64_t B, double lrn_bias,
                 double lrn_alpha, double lrn_beta, optional<Tensor> u8, optional<Tensor> idx, int64_t cin) {
  TORCH_CHECK(cin == 1 || cin == 3, "refc1_wgrad: 1 or 3 input channels");
  const int cfg = mnistx::convpool_config((int)cin, 32, 5, 2, 28, 28);
  TORCH_CHECK(cfg >= 0, "refc1_wgrad: no RefC1 geometry");
  TORCH_CHECK(B >= 1 && B * 784 * cin * 2 < (int64_t)INT32_MAX, "B: the batch (and its index) must stay < 2 GB");
  TORCH_CHECK(cin == 1 || !(u8.has_value() && u8->defined()),
              "refc1_wgrad: 3 channels read bf16 (the batch, or the dataset through idx) only");
  const auto src = cp_src(x, u8, idx, cfg, B, 784 * cin);
  if (src.x) TORCH_CHECK(reinterpret_cast<uintptr_t>(src.x) % 8 == 0, "x must be 8-byte aligned");
  const int64_t np = B * 196 * 32;
  check(dn, at::kBFloat16, np, "dn");
  check(p1, at::kBFloat16, np, "p1");
  check(arg, at::kByte, np, "arg");
  for (const Tensor* t : {&dn, &p1})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "dn / p1 must be 16-byte aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(arg.data_ptr()) % 8 == 0, "arg must be 8-byte aligned");
  TORCH_CHECK(lrn_beta == 0.75, "refc1_wgrad: LRN beta 0.75 only");
  const int res = mnistx::refc1_wgrad_blocks((int)B);
  TORCH_CHECK(res > 0, "refc1_wgrad: occupancy query failed");
  TORCH_CHECK(grid >= 1 && grid <= res, "refc1_wgrad: grid must be in [1, ", res, "] (one block per CU, <= tiles)");
  check(slab, at::kFloat, grid * (cin == 1 ? 48 : 80) * 32, "slab");
  hip_ok(mnistx::refc1_wgrad(src, BF(dn), BF(p1), P<const uint8_t>(arg), (int)B, (float)lrn_bias, (float)lrn_alpha,
                             (float)lrn_beta, P<float>(slab), (int)grid, cur_stream(), (int)cin),
         "refc1_wgrad");
}

// ---------------------------------------------------------------- fp32 (reference precision) path
const float* Fo(const optional<Tensor>& t, int64_t need, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check(*t, at::kFloat, need, name);
  return P<const float>(*t);
}

void f32_dense_fwd(Tensor x, Tensor w, Tensor y, int64_t M, int64_t N, int64_t K, int64_t ldy, optional<Tensor> bias,
                   bool relu) {
  check(x, at::kFloat, M * K, "x");
  check(w, at::kFloat, K * N, "w");
  TORCH_CHECK(ldy >= N, "ldy");
  check(y, at::kFloat, span(M, ldy, N), "y");
  hip_ok(mnistx::f32_dense_fwd(P<const float>(x), P<const float>(w), (int)M, (int)N, (int)K, Fo(bias, N, "bias"),
                               (int)N, relu ? 1 : 0, P<float>(y), (int)ldy, cur_stream()),
         "f32_dense_fwd");
}

void f32_dense_dgrad(Tensor dy, Tensor w, Tensor dx, int64_t M, int64_t Din, int64_t Dout, optional<Tensor> mask) {
  check(dy, at::kFloat, M * Dout, "dy");
  check(w, at::kFloat, Din * Dout, "w");
  check(dx, at::kFloat, M * Din, "dx");
  hip_ok(mnistx::f32_dense_dgrad(P<const float>(dy), P<const float>(w), (int)M, (int)Din, (int)Dout,
                                 Fo(mask, M * Din, "mask"), P<float>(dx), cur_stream()),
         "f32_dense_dgrad");
}

// returns the split count written (the reduce must sum exactly those partials)
int64_t f32_dense_wgrad(Tensor x, Tensor dy, Tensor slab, int64_t B, int64_t Din, int64_t Dout, int64_t splits) {
  check(x, at::kFloat, B * Din, "x");
  check(dy, at::kFloat, B * Dout, "dy");
  TORCH_CHECK(splits >= 1 && splits <= 65535, "splits");
  check(slab, at::kFloat, splits * (Din + 1) * Dout, "slab");
  int used = (int)splits;
  hip_ok(mnistx::f32_dense_wgrad(P<const float>(x), P<const float>(dy), (int)B, (int)Din, (int)Dout, (int)splits,
                                 P<float>(slab), cur_stream(), &used),
         "f32_dense_wgrad");
  return used;
}

void f32_conv_fwd(Tensor x, Tensor w, Tensor y, int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW,
                  int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t Cout, optional<Tensor> bias, bool relu) {
  check(x, at::kFloat, Nb * H * W * C, "x");
  check(w, at::kFloat, KH * KW * C * Cout, "w");
  check(y, at::kFloat, Nb * OH * OW * Cout, "y");
  hip_ok(mnistx::f32_conv_fwd(P<const float>(x), P<const float>(w), (int)Nb, (int)H, (int)W, (int)C, (int)OH,
                              (int)OW, (int)KH, (int)KW, (int)ph, (int)pw, (int)Cout, Fo(bias, Cout, "bias"),
                              relu ? 1 : 0, P<float>(y), cur_stream()),
         "f32_conv_fwd");
}

void f32_conv_dgrad(Tensor dy, Tensor w, Tensor dx, int64_t Nb, int64_t OH, int64_t OW, int64_t Cout, int64_t H,
                    int64_t W, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t Cin, optional<Tensor> mask) {
  check(dy, at::kFloat, Nb * OH * OW * Cout, "dy");
  check(w, at::kFloat, KH * KW * Cin * Cout, "w");
  check(dx, at::kFloat, Nb * H * W * Cin, "dx");
  hip_ok(mnistx::f32_conv_dgrad(P<const float>(dy), P<const float>(w), (int)Nb, (int)OH, (int)OW, (int)Cout, (int)H,
                                (int)W, (int)KH, (int)KW, (int)ph, (int)pw, (int)Cin,
                                Fo(mask, Nb * H * W * Cin, "mask"), P<float>(dx), cur_stream()),
         "f32_conv_dgrad");
}

void f32_conv_wgrad(Tensor x, Tensor dy, Tensor slab, int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t OH,
                    int64_t OW, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t Cout, int64_t splits) {
  check(x, at::kFloat, Nb * H * W * C, "x");
  check(dy, at::kFloat, Nb * OH * OW * Cout, "dy");
  TORCH_CHECK(splits >= 1 && splits <= 65535, "splits");
  check(slab, at::kFloat, splits * (KH * KW * C + 1) * Cout, "slab");
  hip_ok(mnistx::f32_conv_wgrad(P<const float>(x), P<const float>(dy), (int)Nb, (int)H, (int)W, (int)C, (int)OH,
                                (int)OW, (int)KH, (int)KW, (int)ph, (int)pw, (int)Cout, (int)splits, P<float>(slab),
                                cur_stream()),
         "f32_conv_wgrad");
}

// Split count the fp32 conv weight gradient prefers: the LDS-halo kernel's resident
// grid (one partial per workgroup) when it covers the geometry, else -1 (GEMM rule).
int64_t f32_conv_wgrad_pref_splits(int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW, int64_t KH, int64_t KW,
                                   int64_t ph, int64_t pw, int64_t Cout) {
  if (mnistx::f32_halo_wgrad_ok((int)H, (int)W, (int)C, (int)OH, (int)OW, (int)KH, (int)KW, (int)ph, (int)pw,
                                (int)Cout))
    return mnistx::f32_halo_wgrad_grid();
  if (mnistx::f32_conv1_ok((int)H, (int)W, (int)C, (int)OH, (int)OW, (int)KH, (int)KW, (int)ph, (int)pw, (int)Cout))
    return mnistx::f32_conv1_wgrad_grid();
  return -1;
}

void f32_maxpool_fwd(Tensor x, Tensor y, Tensor arg, int64_t Nb, int64_t H, int64_t W, int64_t C) {
  const int64_t OH = (H + 1) / 2, OW = (W + 1) / 2;
  check(x, at::kFloat, Nb * H * W * C, "x");
  check(y, at::kFloat, Nb * OH * OW * C, "y");
  check(arg, at::kByte, Nb * OH * OW * C, "arg");
  hip_ok(mnistx::f32_maxpool_fwd(P<const float>(x), (int)Nb, (int)H, (int)W, (int)C, (int)OH, (int)OW, P<float>(y),
                                 P<uint8_t>(arg), cur_stream()),
         "f32_maxpool_fwd");
}

void f32_maxpool_bwd(Tensor dy, Tensor arg, Tensor y, bool relu_mask, Tensor dx, int64_t Nb, int64_t H, int64_t W,
                     int64_t C) {
  const int64_t OH = (H + 1) / 2, OW = (W + 1) / 2;
  check(dy, at::kFloat, Nb * OH * OW * C, "dy");
  check(arg, at::kByte, Nb * OH * OW * C, "arg");
  check(y, at::kFloat, Nb * OH * OW * C, "y");
  check(dx, at::kFloat, Nb * H * W * C, "dx");
  hip_ok(mnistx::f32_maxpool_bwd(P<const float>(dy), P<const uint8_t>(arg), P<const float>(y), relu_mask ? 1 : 0,
                                 (int)Nb, (int)H, (int)W, (int)C, (int)OH, (int)OW, P<float>(dx), cur_stream()),
         "f32_maxpool_bwd");
}

void f32_lrn_fwd(Tensor x, Tensor y, int64_t P_, int64_t C, int64_t r, double bias, double alpha, double beta) {
  TORCH_CHECK(C <= 64, "f32 LRN: C <= 64");
  check(x, at::kFloat, P_ * C, "x");
  check(y, at::kFloat, P_ * C, "y");
  hip_ok(mnistx::f32_lrn_fwd(P<const float>(x), P_, (int)C, (int)r, (float)bias, (float)alpha, (float)beta,
                             P<float>(y), cur_stream()),
         "f32_lrn_fwd");
}

void f32_lrn_bwd(Tensor x, Tensor dy, Tensor dx, int64_t P_, int64_t C, int64_t r, double bias, double alpha,
                 double beta, bool relu_mask) {
  TORCH_CHECK(C <= 64, "f32 LRN: C <= 64");
  check(x, at::kFloat, P_ * C, "x");
  check(dy, at::kFloat, P_ * C, "dy");
  check(dx, at::kFloat, P_ * C, "dx");
  hip_ok(mnistx::f32_lrn_bwd(P<const float>(x), P<const float>(dy), P_, (int)C, (int)r, (float)bias, (float)alpha,
                             (float)beta, relu_mask ? 1 : 0, P<float>(dx), cur_stream()),
         "f32_lrn_bwd");
}

// fp32 conv1 (28x28x1 -> 32, 5x5 SAME) + bias + ReLU + 2x2 max-pool in one kernel, and its
// weight gradient from dL/d pool + the codes (tests/test_f32_gpu.py)
bool f32_conv1_pool_ok(int64_t H, int64_t W, int64_t C, int64_t OH, int64_t OW, int64_t KH, int64_t KW, int64_t ph,
                       int64_t pw, int64_t Cout) {
  return mnistx::f32_conv1_ok((int)H, (int)W, (int)C, (int)OH, (int)OW, (int)KH, (int)KW, (int)ph, (int)pw, (int)Cout);
}
void f32_conv1_fwd_pool(Tensor x, Tensor w, optional<Tensor> bias, Tensor y, Tensor arg, int64_t Nb) {
  check(x, at::kFloat, Nb * 784, "x");
  check(w, at::kFloat, 25 * 32, "w");
  check(y, at::kFloat, Nb * 196 * 32, "y");
  check(arg, at::kByte, Nb * 196 * 32, "arg");
  TORCH_CHECK(((uintptr_t)y.data_ptr() % 16) == 0 && ((uintptr_t)arg.data_ptr() % 4) == 0, "y / arg alignment");
  hip_ok(mnistx::f32_conv1_fwd_pool(P<const float>(x), P<const float>(w), (int)Nb, Fo(bias, 32, "bias"), P<float>(y),
                                    P<uint8_t>(arg), cur_stream()),
         "f32_conv1_fwd_pool");
}
int64_t f32_conv1_wgrad_unpool_grid() { return mnistx::f32_conv1_wgrad_unpool_grid(); }
void f32_conv1_wgrad_unpool(Tensor x, Tensor dp, Tensor codes, Tensor slab, int64_t Nb, int64_t splits) {
  check(x, at::kFloat, Nb * 784, "x");
  check(dp, at::kFloat, Nb * 196 * 32, "dp");
  check(codes, at::kByte, Nb * 196 * 32, "codes");
  TORCH_CHECK(splits >= 1 && splits <= 65535, "splits");
  check(slab, at::kFloat, splits * 26 * 32, "slab");
  hip_ok(mnistx::f32_conv1_wgrad_unpool(P<const float>(x), P<const float>(dp), P<const uint8_t>(codes), (int)Nb,
                                        (int)splits, P<float>(slab), cur_stream()),
         "f32_conv1_wgrad_unpool");
}
// with norm1's backward folded in: dn = dL/d norm1, p1 = pool1 (the LRN input), radius 4
void f32_conv1_wgrad_lrn(Tensor x, Tensor dn, Tensor p1, Tensor codes, Tensor slab, int64_t Nb, int64_t splits,
                         double bias, double alpha, double beta) {
  check(x, at::kFloat, Nb * 784, "x");
  check(dn, at::kFloat, Nb * 196 * 32, "dn");
  check(p1, at::kFloat, Nb * 196 * 32, "p1");
  check(codes, at::kByte, Nb * 196 * 32, "codes");
  for (const Tensor* t : {&x, &dn, &p1, &codes})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "x / dn / p1 / codes must be 16-byte aligned");
  TORCH_CHECK(Nb >= 1 && Nb * 196 * 32 * 4 < (int64_t)INT32_MAX * 2, "Nb");
  TORCH_CHECK(splits >= 1 && splits <= 65535, "splits");
  check(slab, at::kFloat, splits * 26 * 32, "slab");
  hip_ok(mnistx::f32_conv1_wgrad_lrn(P<const float>(x), P<const float>(dn), P<const float>(p1), P<const uint8_t>(codes),
                                     (int)Nb, (int)splits, (float)bias, (float)alpha, (float)beta, P<float>(slab),
                                     cur_stream()),
         "f32_conv1_wgrad_lrn");
}

// fp32 LRN + 2x2 max-pool fused (the reference's norm2 -> pool2) and its backward
bool f32_lrn_pool_ok(int64_t H, int64_t W, int64_t C, int64_t r) {
  return mnistx::f32_lrn_pool_ok((int)H, (int)W, (int)C, (int)r);
}
void f32_lrn_pool_fwd(Tensor x, Tensor y, Tensor arg, int64_t Nb, int64_t H, int64_t W, int64_t C, int64_t r,
                      double bias, double alpha, double beta) {
  check(x, at::kFloat, Nb * H * W * C, "x");
  check(y, at::kFloat, Nb * (H / 2) * (W / 2) * C, "y");
  check(arg, at::kByte, Nb * (H / 2) * (W / 2) * C, "arg");
  hip_ok(mnistx::f32_lrn_pool_fwd(P<const float>(x), (int)Nb, (int)H, (int)W, (int)C, (int)r, (float)bias,
                                  (float)alpha, (float)beta, P<float>(y), P<uint8_t>(arg), cur_stream()),
         "f32_lrn_pool_fwd");
}
void f32_lrn_pool_bwd(Tensor x, Tensor dy, Tensor arg, Tensor dx, int64_t Nb, int64_t H, int64_t W, int64_t C,
                      int64_t r, double bias, double alpha, double beta, bool relu_mask) {
  check(x, at::kFloat, Nb * H * W * C, "x");
  check(dy, at::kFloat, Nb * (H / 2) * (W / 2) * C, "dy");
  check(arg, at::kByte, Nb * (H / 2) * (W / 2) * C, "arg");
  check(dx, at::kFloat, Nb * H * W * C, "dx");
  hip_ok(mnistx::f32_lrn_pool_bwd(P<const float>(x), P<const float>(dy), P<const uint8_t>(arg), (int)Nb, (int)H,
                                  (int)W, (int)C, (int)r, (float)bias, (float)alpha, (float)beta, relu_mask ? 1 : 0,
                                  P<float>(dx), cur_stream()),
         "f32_lrn_pool_bwd");
}

void f32_softmax_ce(Tensor logits, int64_t ldl, optional<Tensor> labels, int64_t B, int64_t NC, double scale,
                    optional<Tensor> dlogits, int64_t ldd, optional<Tensor> stats, optional<Tensor> probs,
                    optional<Tensor> work) {
  TORCH_CHECK(ldl >= NC, "ldl < NC");
  check(logits, at::kFloat, span(B, ldl, NC), "logits");
  const int32_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    check(*labels, at::kInt, B, "labels");
    lab = P<const int32_t>(*labels);
  }
  float* dl = nullptr;
  if (dlogits.has_value() && dlogits->defined()) {
    TORCH_CHECK(lab != nullptr && ldd >= NC, "dlogits needs labels and ldd >= NC");
    check(*dlogits, at::kFloat, B * ldd, "dlogits");
    dl = P<float>(*dlogits);
  }
  float* st = nullptr;
  if (stats.has_value() && stats->defined()) {
    check(*stats, at::kFloat, 8, "stats");
    st = P<float>(*stats);
  }
  float* pr = nullptr;
  if (probs.has_value() && probs->defined()) {
    check(*probs, at::kFloat, B * NC, "probs");
    pr = P<float>(*probs);
  }
  float* wk = nullptr;
  if (work.has_value() && work->defined()) {
    check(*work, at::kFloat, 4 * 1024 + 1, "work");
    wk = P<float>(*work);
  }
  hip_ok(mnistx::f32_softmax_ce(P<const float>(logits), (int)ldl, lab, (int)B, (int)NC, (float)scale, dl, (int)ldd,
                                st, pr, wk, cur_stream()),
         "f32_softmax_ce");
}

void f32_prep_images(Tensor src, Tensor idx, Tensor lab_src, Tensor out, Tensor lab_out, int64_t HW, int64_t Csrc,
                     int64_t Cdst) {
  const int64_t B = idx.numel();
  check(idx, at::kLong, B, "idx");
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.is_contiguous(), "src: uint8 GPU tensor");
  TORCH_CHECK(src.numel() % (HW * Csrc) == 0, "src size");
  TORCH_CHECK(Csrc == Cdst || Csrc == 1, "channels: equal or 1 -> C replication");
  check(lab_src, at::kInt, src.numel() / (HW * Csrc), "lab_src");
  check(out, at::kFloat, B * HW * Cdst, "out");
  check(lab_out, at::kInt, B, "lab_out");
  hip_ok(mnistx::f32_prep_images(P<const uint8_t>(src), P<const int64_t>(idx), P<const int32_t>(lab_src), (int)B,
                                 (int)HW, (int)Csrc, (int)Cdst, P<float>(out), P<int32_t>(lab_out), cur_stream()),
         "f32_prep_images");
}

}  // namespace

PYBIND11_MODULE(_kernels, m) {
  m.def("f32_dense_fwd", &f32_dense_fwd);
  m.def("f32_dense_dgrad", &f32_dense_dgrad);
  m.def("f32_dense_wgrad", &f32_dense_wgrad);
  m.def("f32_wgrad_splits_cap", [](int64_t din, int64_t dout, int64_t b) {
    return (int64_t)mnistx::f32_wgrad_splits_cap((int)din, (int)dout, (int)b);
  }, "slab partials the fp32 256 x 256 weight-gradient path writes for this shape (0: not that path)");
  m.def("f32_conv_fwd", &f32_conv_fwd);
  m.def("f32_conv_dgrad", &f32_conv_dgrad);
  m.def("f32_conv_wgrad", &f32_conv_wgrad);
  m.def("f32_conv_wgrad_pref_splits", &f32_conv_wgrad_pref_splits);
  m.def("f32_maxpool_fwd", &f32_maxpool_fwd);
  m.def("f32_maxpool_bwd", &f32_maxpool_bwd);
  m.def("f32_lrn_fwd", &f32_lrn_fwd);
  m.def("f32_lrn_bwd", &f32_lrn_bwd);
  m.def("f32_conv1_pool_ok", &f32_conv1_pool_ok);
  m.def("f32_conv1_fwd_pool", &f32_conv1_fwd_pool);
  m.def("f32_conv1_wgrad_unpool_grid", &f32_conv1_wgrad_unpool_grid);
  m.def("f32_conv1_wgrad_unpool", &f32_conv1_wgrad_unpool);
  m.def("f32_conv1_wgrad_lrn", &f32_conv1_wgrad_lrn);
  m.def("f32_lrn_pool_ok", &f32_lrn_pool_ok);
  m.def("f32_lrn_pool_fwd", &f32_lrn_pool_fwd);
  m.def("f32_lrn_pool_bwd", &f32_lrn_pool_bwd);
  m.def("f32_softmax_ce", &f32_softmax_ce, py::arg("logits"), py::arg("ldl"), py::arg("labels"), py::arg("B"),
        py::arg("NC"), py::arg("scale"), py::arg("dlogits"), py::arg("ldd"), py::arg("stats"), py::arg("probs"),
        py::arg("work") = py::none());
  m.def("f32_prep_images", &f32_prep_images);
  // test hook: cap every persistent kernel's grid (0 = off) so small-batch oracle tests run
  // the multi-iteration (several tiles per block) paths the benchmark batches run
  m.def("set_grid_cap", [](int64_t n) { mnistx::set_grid_cap((int)n); });
  // pin / unpin host memory the caller mapped itself (the PS shm data plane's slots, so the
  // worker's gradient / parameter copies are DMA, not staged through a bounce buffer)
  m.def("host_register", [](uintptr_t addr, int64_t nbytes) {
    return hipHostRegister((void*)addr, (size_t)nbytes, hipHostRegisterDefault) == hipSuccess;
  });
  m.def("host_unregister", [](uintptr_t addr) { return hipHostUnregister((void*)addr) == hipSuccess; });
  m.def("set_gemm256", &mnistx::set_gemm256, "route the GEMMs that fill the GPU to gemm256.hip (A/B switch)");
  m.def("gemm256_enabled", &mnistx::gemm256_enabled);
  m.def("set_gemm256_debug", [](int64_t b) { mnistx::set_gemm256_debug((int)b); });
  m.def("set_reserve_cus", [](int64_t n) { mnistx::set_reserve_cus((int)n); });
  m.def("reserve_cus", []() { return (int64_t)mnistx::reserve_cus(); });
  m.def("clock_mark", [](Tensor out, int64_t slot) {
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous() && slot >= 0 &&
                    slot < out.numel(), "clock_mark: int64 GPU buffer with the slot in range");
    hip_ok(mnistx::clock_mark((uint64_t*)out.data_ptr<int64_t>(), (int)slot, cur_stream()), "clock_mark");
  });
  m.def("coresidency_probe", [](Tensor out, int64_t blocks, int64_t threads, int64_t lds_bytes, int64_t spin_ticks) {
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kLong && out.is_contiguous() && out.numel() >= 2 * blocks,
                "coresidency_probe: int64 GPU buffer of 2 * blocks stamps");
    hip_ok(mnistx::coresidency_probe((uint64_t*)out.data_ptr<int64_t>(), (int)blocks, (int)threads, (int)lds_bytes,
                                     (int)spin_ticks, cur_stream()), "coresidency_probe");
  });
  m.def("grid_cap", []() { return (int64_t)mnistx::grid_cap(); });
  m.doc() = "MI355X (gfx950) HIP kernels for the MNIST trainer";
  m.def("dense_fwd", &dense_fwd, py::arg("x"), py::arg("w"), py::arg("out"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("ldx"), py::arg("ldw"), py::arg("ldc"), py::arg("bias"), py::arg("bias_n"), py::arg("relu"),
        py::arg("mask"), py::arg("ldm"), py::arg("tile") = -1);
  m.def("dense_dgrad", &dense_dgrad, py::arg("dy"), py::arg("w"), py::arg("out"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("lddy"), py::arg("ldw"), py::arg("ldc"), py::arg("mask"), py::arg("ldm"),
        py::arg("tile") = -1);
  m.def("set_tile192", [](int64_t on) { mnistx::set_tile192((int)on); },
        "A/B switch of gemm.hip's 192-column tiles (MNISTX_TILE192)");
  m.def("set_reduce_fused", [](int64_t on) { mnistx::set_reduce_fused((int)on); },
        "A/B switch of the one-launch split-K reduce (MNISTX_REDUCE_FUSED)");
  m.def("reduce_fused_enabled", []() { return mnistx::reduce_fused_enabled() != 0; });
  m.def("dense_wgrad", &dense_wgrad, py::arg("x"), py::arg("dy"), py::arg("slab"), py::arg("Din"), py::arg("Dout"),
        py::arg("B"), py::arg("ldx"), py::arg("lddy"), py::arg("with_bias"), py::arg("splits"), py::arg("tile") = -1);
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("out"), py::arg("Nb"), py::arg("H"), py::arg("W"),
        py::arg("C"), py::arg("OH"), py::arg("OW"), py::arg("KH"), py::arg("KW"), py::arg("ph"), py::arg("pw"),
        py::arg("Cout"), py::arg("bias"), py::arg("bias_n"), py::arg("relu"), py::arg("lrn_r") = 0,
        py::arg("lrn_bias") = 0.0, py::arg("lrn_alpha") = 0.0, py::arg("lrn_beta") = 0.0);
  m.def("set_f32_halo_fwd_variant", [](int64_t v) { mnistx::set_f32_halo_fwd_variant((int)v); });
  m.def("set_halo_variants", [](int64_t f, int64_t d) { mnistx::set_halo_variants((int)f, (int)d); });
  m.def("conv_dgrad", &conv_dgrad);
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("slab"), py::arg("Nb"), py::arg("H"),
        py::arg("W"), py::arg("C"), py::arg("OH"), py::arg("OW"), py::arg("KH"), py::arg("KW"), py::arg("ph"),
        py::arg("pw"), py::arg("Cout"), py::arg("with_bias"), py::arg("splits"), py::arg("lrn_r") = 0,
        py::arg("lrn_bias") = 0.0, py::arg("lrn_alpha") = 0.0, py::arg("lrn_beta") = 0.0);
  m.def("prep_images", &prep_images);
  m.def("dense_wgrad_group", &dense_wgrad_group);
  m.def("conv_wgrad_pref_splits", &conv_wgrad_pref_splits);
  m.def("perm_positions", &perm_positions, py::arg("out"), py::arg("start"), py::arg("N"), py::arg("seed"), py::arg("h"),
        py::arg("lab_src") = py::none(), py::arg("lab_out") = py::none());
  m.def("prep_images_perm", &prep_images_perm);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("lrn_fwd", &lrn_fwd);
  m.def("lrn_bwd", &lrn_bwd);
  m.def("lrn_pool_supported", &lrn_pool_supported);
  m.def("lrn_pool_fwd", &lrn_pool_fwd, py::arg("x"), py::arg("y"), py::arg("arg"), py::arg("Nb"), py::arg("H"),
        py::arg("W"), py::arg("C"), py::arg("r"), py::arg("bias"), py::arg("alpha"), py::arg("beta"),
        py::arg("nonneg") = false);
  m.def("lrn_set_packed", [](bool on) { mnistx::lrn_set_packed(on ? 1 : 0); });
  m.def("lrn_pool_bwd", &lrn_pool_bwd);
  m.def("softmax_ce", &softmax_ce, py::arg("logits"), py::arg("ldl"), py::arg("labels"), py::arg("B"), py::arg("NC"),
        py::arg("scale"), py::arg("dlogits"), py::arg("ldd"), py::arg("stats"), py::arg("probs"),
        py::arg("work") = py::none(), py::arg("defer_stats") = false, py::arg("dbias") = py::none());
  m.def("softmax_ce_dbias_blocks",
        [](int64_t B, int64_t ldl) { return (int64_t)mnistx::softmax_ce_dbias_blocks((int)B, (int)ldl); });
  m.def("splitk_reduce", &splitk_reduce);
  m.def("splitk_reduce_multi", &splitk_reduce_multi);
  m.def("mlp_head_supported", &mlp_head_supported);
  m.def("ce_tail_supported", &ce_tail_supported);
  m.def("ce_tail_blocks", [](int64_t nb) { return (int64_t)mnistx::ce_tail_blocks((int)nb); });
  m.def("ce_tail", &ce_tail, py::arg("x"), py::arg("w5t"), py::arg("b5"), py::arg("nc"), py::arg("labels"),
        py::arg("nb"), py::arg("scale"), py::arg("logits"), py::arg("dl") = py::none(), py::arg("dx") = py::none(),
        py::arg("stats"), py::arg("work") = py::none(), py::arg("defer_stats") = false, py::arg("dbias") = py::none());
  m.def("mlp_head", &mlp_head, py::arg("x"), py::arg("w3t"), py::arg("b3"), py::arg("n1"), py::arg("w4t"),
        py::arg("b4"), py::arg("n2"), py::arg("w5t"), py::arg("b5"), py::arg("nc"), py::arg("labels"), py::arg("nb"),
        py::arg("scale"), py::arg("h3"), py::arg("h4"), py::arg("logits"), py::arg("dl") = py::none(),
        py::arg("dh4") = py::none(), py::arg("dh3") = py::none(), py::arg("dx") = py::none(), py::arg("stats"),
        py::arg("work"), py::arg("defer_stats") = false, py::arg("dbias") = py::none());
  m.def("fused_optimizer", &fused_optimizer, py::arg("params"), py::arg("grads"), py::arg("mom"), py::arg("ema"),
        py::arg("bf"), py::arg("segs"), py::arg("step"), py::arg("lr0"), py::arg("decay_rate"),
        py::arg("decay_steps"), py::arg("momentum"), py::arg("nesterov"), py::arg("use_momentum"),
        py::arg("grad_scale"), py::arg("ema_max"), py::arg("l2") = py::none(), py::arg("guard") = py::none(),
        py::arg("guard_want") = 0, py::arg("guard_err") = py::none(), py::arg("guard_id") = 0,
        py::arg("fin") = py::none(), py::arg("perm") = py::none());
  m.def("set_opt_fin_fused", [](int64_t on) { mnistx::set_opt_fin_fused((int)on); },
        "A/B switch of the optimizer launch running the step's finalize (MNISTX_OPT_FIN_FUSED)");
  m.def("opt_fin_fused_enabled", []() { return mnistx::opt_fin_fused_enabled() != 0; });
  m.def("fused_optimizer_blocks", [](Tensor segs) {
    TORCH_CHECK(!segs.is_cuda() && segs.scalar_type() == at::kLong && segs.dim() == 2, "segs: CPU int64 [n,14]");
    auto a = segs.accessor<int64_t, 2>();
    std::vector<mnistx::OptSeg> sv(segs.size(0));
    for (int64_t i = 0; i < segs.size(0); ++i) sv[i].n = a[i][1];
    return (int64_t)mnistx::fused_optimizer_blocks(sv.data(), (int)sv.size());
  });
  m.def("finalize_step", &finalize_step, py::arg("step"), py::arg("stats"), py::arg("l2"), py::arg("wds"),
        py::arg("nw"), py::arg("loss_ema"), py::arg("n_ema"), py::arg("batch"), py::arg("increment"),
        py::arg("l2_ranges") = py::none(), py::arg("ce_work") = py::none(), py::arg("ce_nblk") = 0);
  m.def("mlp_head_blocks", [](int64_t nb) { return (int64_t)mnistx::mlp_head_blocks((int)nb); });
  m.def("cast_f32_bf16_padded", &cast_f32_bf16_padded);
  m.def("convpool_supported", &convpool_supported);
  m.def("convpool_rows", &convpool_rows);
  m.def("gemm_tile", &gemm_tile);
  m.def("convpool_reduce_args", &convpool_reduce_args);
  m.def("convpool_fwd", &convpool_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("bias_n"),
        py::arg("pooled"), py::arg("arg"), py::arg("B"), py::arg("cin"), py::arg("cout"), py::arg("ks"),
        py::arg("pad"), py::arg("h"), py::arg("w_"), py::arg("u8") = py::none(), py::arg("idx") = py::none(),
        py::arg("lrn_out") = py::none(), py::arg("lrn_bias") = 0.0, py::arg("lrn_alpha") = 0.0,
        py::arg("lrn_beta") = 0.0, py::arg("lrn_r") = 0);
  // u8: the forward reads a uint8 dataset (3 channels: the fold needs bf16 input)
  m.def("convpool_fwd_lrn_ok", [](int64_t cin, int64_t cout, int64_t ks, int64_t pad, int64_t h, int64_t w, bool u8) {
    const int cfg = cp_geo(cin, cout, ks, pad, h, w).cfg;
    return (cfg == 2 && mnistx::refc1_fwd_lrn_ok()) || (cfg == 3 && !u8 && mnistx::refc1_fwd3_ok());
  }, py::arg("cin"), py::arg("cout"), py::arg("ks"), py::arg("pad"), py::arg("h"), py::arg("w"), py::arg("u8") = false);
  m.def("convpool_wgrad", &convpool_wgrad, py::arg("x"), py::arg("dP"), py::arg("arg"), py::arg("slab"),
        py::arg("grid"), py::arg("B"), py::arg("cin"), py::arg("cout"), py::arg("ks"), py::arg("pad"), py::arg("h"),
        py::arg("w_"), py::arg("u8") = py::none(), py::arg("idx") = py::none(), py::arg("lrn_p") = py::none(),
        py::arg("lrn_bias") = 0.0, py::arg("lrn_alpha") = 0.0, py::arg("lrn_beta") = 0.0, py::arg("lrn_r") = 0);
  m.def("convpool_u8_input", &convpool_u8_input);
  m.def("convpool_dgrad", &convpool_dgrad, py::arg("dP"), py::arg("arg"), py::arg("w"), py::arg("dx"), py::arg("B"),
        py::arg("cin"), py::arg("cout"), py::arg("ks"), py::arg("pad"), py::arg("h"), py::arg("w_"),
        py::arg("grid_cap") = 0);
  m.def("convpool_arg_bytes", &convpool_arg_bytes);
  m.def("convpool_has_dgrad", &convpool_has_dgrad);
  m.def("convpool_wgrad_grid", &convpool_wgrad_grid);
  m.def("lenet_band_fwd", &lenet_band_fwd, py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("b1n"),
        py::arg("w2"), py::arg("b2"), py::arg("B"), py::arg("p2"), py::arg("arg2"), py::arg("p1") = py::none(),
        py::arg("arg1") = py::none(), py::arg("idx") = py::none(), py::arg("prof") = py::none());
  m.def("lenet_bwd", &lenet_bwd, py::arg("x"), py::arg("p1"), py::arg("dp2"), py::arg("arg2"),
        py::arg("w2"), py::arg("B"), py::arg("slab1"), py::arg("slab2"), py::arg("grid"), py::arg("idx") = py::none(),
        py::arg("prof") = py::none());
  m.def("lenet_bwd_blocks", [](int64_t B) {
    const int n = mnistx::lenet_bwd_blocks((int)B);
    TORCH_CHECK(n > 0, "lenet_bwd_blocks: occupancy query failed");
    return (int64_t)n;
  });
  m.def("refc1_wgrad", &refc1_wgrad, py::arg("x"), py::arg("dn"), py::arg("p1"), py::arg("arg"), py::arg("slab"),
        py::arg("grid"), py::arg("B"), py::arg("lrn_bias"), py::arg("lrn_alpha"), py::arg("lrn_beta"),
        py::arg("u8") = py::none(), py::arg("idx") = py::none(), py::arg("cin") = 1);
  m.def("refc1_set_skip", [](int64_t s) { mnistx::refc1_set_skip((int)s); });
  m.def("refc1_set_fwd_variant", [](int64_t v) { mnistx::refc1_set_fwd_variant((int)v); });
  m.def("refc1_wgrad_blocks", [](int64_t B) {
    const int n = mnistx::refc1_wgrad_blocks((int)B);
    TORCH_CHECK(n > 0, "refc1_wgrad_blocks: occupancy query failed");
    return (int64_t)n;
  });
  m.attr("ARCH") = "gfx950";
}
