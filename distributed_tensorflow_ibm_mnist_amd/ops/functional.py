"""Shape-aware wrappers around the HIP kernels (``csrc/kernels``).

Conventions (see ``csrc/kernels/gemm.hip``):
* activations: bf16, NHWC, channel count padded to a multiple of 8 (pad lanes 0);
* dense activations: bf16 ``[B, D_pad]``;
* weights: a bf16 copy in the reference layout (``[KH, KW, Cin, Cout]`` /
  ``[Din, Dout]``) zero-padded to the activation padding; fp32 masters live in
  the optimizer's flat buffer;
* weight gradients: fp32 in the *unpadded* reference layout, produced by
  split-K slabs + ``splitk_reduce`` (deterministic).

Every function takes optional ``out=`` buffers so the executor can run with a
static arena (and under hipGraph capture); tests call them allocation-style.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import torch

from ._ext import kernels

BK = 32
BK_WG = 32           # K rows per step of the split-K weight-gradient GEMMs (gemm.hip BK_WG)
# Split-K target for weight-gradient GEMMs (workgroups per launch): ~8 per CU.
TARGET_BLOCKS = 2048
# Dense weight gradients with only a few output tiles (LeNet fc3/fc4/fc5) aim for
# ~2 per CU instead: with the counted-vmcnt 4-deep prefetch (gemm.hip) a block
# keeps its own loads in flight, and fewer splits mean a smaller fp32 slab to
# reduce (fc3 at B=65536: S=64 24.9 us vs S=147 ~34 us; LeNet-5 step 0.761 ->
# 0.744 ms).  Gather-bound im2col weight gradients and many-tile dense ones
# (reference CNN conv2 / local3) measured faster at 2048 (4.16 vs 4.78 ms/step).
# Round 3, with the head weight gradients grouped on 64x128 tiles: 256 (~1 per CU)
# beat 512 in 5 of 5 same-box pairs, LeNet-5 0.5255 vs 0.5291 ms/step on average
# (128: 0.5293, 384: 0.5260, 768: 0.5342, 1024: 0.5402; profiles/r3/lenet/wgrad_blocks/).
TARGET_BLOCKS_FEW_TILES = int(os.environ.get("MNISTX_WGRAD_BLOCKS", "256"))
# Round 6, the grouped head weight gradients (LeNet fc3 / fc4 / fc5 in one launch): 192 --
# kernel tables on one box: gemm_wg_group 34.2 -> 31.8 us, split-K reduce 8.4 -> 7.8 us; step
# pairs on very noisy boxes 7 of 11 for 192.  The standalone few-tile ones (reference local4)
# stay at 256: 1.8388 vs 1.8406 ms at 192, 3 pairs (profiles/r6/lenet_wgb/)
TARGET_BLOCKS_GROUPED = int(os.environ.get("MNISTX_WGRAD_BLOCKS_GROUPED", "192"))
# 128x128-tile dense weight gradients (reference local3): ~2 splits (bench/micro_wgrad.py
# ref: S=2 155.9 us, S=3 165.0, S=8 154.4, S=16 197.1 -- the fewest splits that fill
# the GPU keep the slab smallest; round 3, whole reference-CNN step: 256 / 400 / 600 / 800
# within noise, 2.19-2.22 ms, profiles/r3/refcnn/wgrad_blocks_big/)
# Round 4 (dense-GEMM epilogue and ROWS conv in): 1000 (local3 S = 5, the SLAB_CAP limit)
# beat 400 (S = 2) in 3 of 3 same-box pairs, 2.114-2.121 vs 2.135-2.144 ms/step
# (profiles/r4/gemm_epi/ab_wgrad_blocks_big.txt; standalone sweep micro_wgrad_local3_tiles.txt)
TARGET_BLOCKS_BIG_TILES = int(os.environ.get("MNISTX_WGRAD_BLOCKS_BIG", "1000"))

def pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def gemm_tile(M: int, N: int) -> Tuple[int, int]:
    """Tile of a weight-gradient GEMM: mirror of ``tile_code(M, N, wgrad=true)``
    in gemm.hip (checked against ``kernels().gemm_tile`` by the GPU tests).
    Small tiles give every K-split many workgroups, which keeps the
    deterministic split-K slab (splits x M x N fp32) small."""
    if N <= 16:
        return 64, 16
    if N <= 32:
        return 64, 32
    if N <= 64:
        return 64, 64
    if N <= 128:        # the whole N in one tile: the M operand is read once
        return (64, 128) if M >= 256 else (64, 64)
    if math.ceil(M / 128) * math.ceil(N / 128) < 128:
        return 64, 64
    return 128, 128


# column tile of the grouped head weight gradients (gemm.hip wg_group_bn, same variable)
GROUP_BN = 128   # gemm.hip wg_group_bn(): fc3 / fc4 outputs in ONE column tile
# (64-row tiles: 128-row ones measured equal, 0.4576-0.4599 vs 0.4557-0.4598 ms/step on one
# box, profiles/r4/lenet_head/group_bm_ab.txt)
GROUP_BM = 64
SLAB_CAP = 16 << 20   # fp32 elements of split-K partials (64 MB)


def pick_splits(M: int, N: int, K: int, target: Optional[int] = None, min_k: int = 256,
                dense: bool = False, grouped: bool = False) -> int:
    """Split-K factor for a weight-gradient GEMM: fill the CUs (``target``
    workgroups), but keep every split >= min_k reduction elements and the fp32
    slab under SLAB_CAP.  ``grouped``: one problem of a dense_wgrad_group launch
    (64x64 tiles)."""
    bm, bn = (GROUP_BM, GROUP_BN) if grouped else gemm_tile(M, N)
    tiles = math.ceil(M / bm) * math.ceil(N / bn)
    if target is None:
        if dense and (bm, bn) == (128, 128):
            target = TARGET_BLOCKS_BIG_TILES
        else:
            target = (TARGET_BLOCKS_GROUPED if grouped else TARGET_BLOCKS_FEW_TILES) if (dense and tiles < 64) \
                else TARGET_BLOCKS
    s = max(1, math.ceil(target / tiles))
    s = min(s, max(1, K // min_k), max(1, SLAB_CAP // max(1, M * N)))
    return eff_splits(K, s)


def eff_splits(K: int, s: int) -> int:
    s = max(1, s)
    kchunk = max(BK_WG, (math.ceil(K / s) + BK_WG - 1) // BK_WG * BK_WG)
    return math.ceil(K / kchunk)


def same_pad(k: int) -> int:
    return (k - 1) // 2


def conv_out_hw(h: int, w: int, kh: int, kw: int, padding: str) -> Tuple[int, int]:
    if padding == "SAME":
        return h, w
    return h - kh + 1, w - kw + 1


def conv_pads(kh: int, kw: int, padding: str) -> Tuple[int, int]:
    return (same_pad(kh), same_pad(kw)) if padding == "SAME" else (0, 0)


def weight_to_bf16(w: torch.Tensor, pad_in: int, pad_out: int) -> torch.Tensor:
    """fp32 reference-layout weight -> zero-padded bf16 copy (GPU kernel)."""
    K = kernels()
    if w.dim() == 4:
        kh, kw, ci, co = w.shape
        G, I, J = kh * kw, ci, co
        out = torch.empty(kh, kw, pad_in, pad_out, dtype=torch.bfloat16, device=w.device)
    else:
        I, J = w.shape
        G = 1
        out = torch.empty(pad_in, pad_out, dtype=torch.bfloat16, device=w.device)
    K.cast_f32_bf16_padded(w.contiguous(), out, G, I, J, pad_in, pad_out)
    return out


# ------------------------------------------------------------------ convolution
def conv2d(x: torch.Tensor, w_bf: torch.Tensor, bias: Optional[torch.Tensor], padding: str = "SAME",
           relu: bool = True, bias_n: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    N, H, W, C = x.shape
    kh, kw, ci, co = w_bf.shape
    assert ci == C, (ci, C)
    OH, OW = conv_out_hw(H, W, kh, kw, padding)
    ph, pw = conv_pads(kh, kw, padding)
    if out is None:
        out = torch.empty(N, OH, OW, co, dtype=torch.bfloat16, device=x.device)
    kernels().conv_fwd(x, w_bf, out, N, H, W, C, OH, OW, kh, kw, ph, pw, co, bias,
                       bias.numel() if (bias is not None and bias_n is None) else (bias_n or 0), relu)
    return out


def conv2d_dgrad(dy: torch.Tensor, w_bf: torch.Tensor, in_hw: Tuple[int, int], padding: str = "SAME",
                 mask: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    N, OH, OW, co = dy.shape
    kh, kw, ci, co2 = w_bf.shape
    assert co == co2
    H, W = in_hw
    ph, pw = conv_pads(kh, kw, padding)
    if out is None:
        out = torch.empty(N, H, W, ci, dtype=torch.bfloat16, device=dy.device)
    kernels().conv_dgrad(dy, w_bf, out, N, OH, OW, co, H, W, kh, kw, ph, pw, ci, mask)
    return out


def conv2d_wgrad(x: torch.Tensor, dy: torch.Tensor, kh: int, kw: int, padding: str, cin: int, cout: int,
                 with_bias: bool = True, splits: Optional[int] = None, slab: Optional[torch.Tensor] = None,
                 dw: Optional[torch.Tensor] = None, db: Optional[torch.Tensor] = None):
    """Returns (dW fp32 [kh,kw,cin,cout], db fp32 [cout] or None)."""
    N, H, W, C = x.shape
    _, OH, OW, CO = dy.shape
    ph, pw = conv_pads(kh, kw, padding)
    M = kh * kw * C + (1 if with_bias else 0)
    P = N * OH * OW
    S = pick_splits(M, CO, P) if splits is None else eff_splits(P, splits)
    if slab is None:
        slab = torch.empty(S * M * CO, dtype=torch.float32, device=x.device)
    K = kernels()
    S = K.conv_wgrad(x, dy, slab, N, H, W, C, OH, OW, kh, kw, ph, pw, CO, with_bias, S)
    if dw is None:
        dw = torch.empty(kh, kw, cin, cout, dtype=torch.float32, device=x.device)
    if with_bias and db is None:
        db = torch.empty(cout, dtype=torch.float32, device=x.device)
    K.splitk_reduce(slab, S, M, CO, kh * kw, C, cin, cout, kh * kw * C, dw, db if with_bias else None, 1.0)
    return dw, (db if with_bias else None)


# ------------------------------------------------------------------ dense
def dense(x: torch.Tensor, w_bf: torch.Tensor, bias: Optional[torch.Tensor], relu: bool,
          out_dtype: torch.dtype = torch.bfloat16, bias_n: Optional[int] = None,
          out: Optional[torch.Tensor] = None) -> torch.Tensor:
    B, Kd = x.shape
    K2, N = w_bf.shape
    assert Kd == K2, (Kd, K2)
    if out is None:
        out = torch.empty(B, N, dtype=out_dtype, device=x.device)
    bn = (bias.numel() if bias is not None else 0) if bias_n is None else bias_n
    kernels().dense_fwd(x, w_bf, out, B, N, Kd, Kd, N, out.shape[1], bias, bn, relu, None, 0)
    return out


def dense_dgrad(dy: torch.Tensor, w_bf: torch.Tensor, mask: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    B, N = dy.shape
    Din, N2 = w_bf.shape
    assert N == N2
    if out is None:
        out = torch.empty(B, Din, dtype=torch.bfloat16, device=dy.device)
    kernels().dense_dgrad(dy, w_bf, out, B, Din, N, N, N, Din, mask, Din)
    return out


def dense_wgrad(x: torch.Tensor, dy: torch.Tensor, din: int, dout: int, with_bias: bool = True,
                splits: Optional[int] = None, slab: Optional[torch.Tensor] = None,
                dw: Optional[torch.Tensor] = None, db: Optional[torch.Tensor] = None):
    B, Dp = x.shape
    _, Np = dy.shape
    M = Dp + (1 if with_bias else 0)
    S = pick_splits(M, Np, B, dense=True) if splits is None else eff_splits(B, splits)
    if slab is None:
        slab = torch.empty(S * M * Np, dtype=torch.float32, device=x.device)
    K = kernels()
    S = K.dense_wgrad(x, dy, slab, Dp, Np, B, Dp, Np, with_bias, S)
    if dw is None:
        dw = torch.empty(din, dout, dtype=torch.float32, device=x.device)
    if with_bias and db is None:
        db = torch.empty(dout, dtype=torch.float32, device=x.device)
    K.splitk_reduce(slab, S, M, Np, 1, Dp, din, dout, Dp, dw, db if with_bias else None, 1.0)
    return dw, (db if with_bias else None)


# ------------------------------------------------------------------ pooling / LRN / loss
def maxpool2x2(x: torch.Tensor, out: Optional[torch.Tensor] = None, arg: Optional[torch.Tensor] = None):
    N, H, W, C = x.shape
    OH, OW = (H + 1) // 2, (W + 1) // 2
    if out is None:
        out = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device=x.device)
    if arg is None:
        arg = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=x.device)
    kernels().maxpool_fwd(x, out, arg, N, H, W, C, OH, OW)
    return out, arg


def maxpool2x2_bwd(dy: torch.Tensor, arg: torch.Tensor, y: torch.Tensor, in_hw: Tuple[int, int],
                   relu_mask: bool = True, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    N, OH, OW, C = dy.shape
    H, W = in_hw
    if out is None:
        out = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dy.device)
    kernels().maxpool_bwd(dy, arg, y, relu_mask, out, N, H, W, C, OH, OW)
    return out


def lrn(x: torch.Tensor, r: int, bias: float, alpha: float, beta: float,
        out: Optional[torch.Tensor] = None) -> torch.Tensor:
    C = x.shape[-1]
    P = x.numel() // C
    if out is None:
        out = torch.empty_like(x)
    kernels().lrn_fwd(x, out, P, C, r, bias, alpha, beta)
    return out


def lrn_bwd(x: torch.Tensor, dy: torch.Tensor, r: int, bias: float, alpha: float, beta: float,
            relu_mask: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    C = x.shape[-1]
    P = x.numel() // C
    if out is None:
        out = torch.empty_like(x)
    kernels().lrn_bwd(x, dy, out, P, C, r, bias, alpha, beta, relu_mask)
    return out


def softmax_ce(logits: torch.Tensor, labels: torch.Tensor, n_classes: int, scale: Optional[float] = None,
               dlogits: Optional[torch.Tensor] = None, stats: Optional[torch.Tensor] = None,
               want_grad: bool = True):
    """Fused softmax-CE fwd+bwd.  Returns (dlogits bf16 [B, ld] or None, stats f32[8])."""
    B, ld = logits.shape
    if scale is None:
        scale = 1.0 / B
    if stats is None:
        stats = torch.zeros(8, dtype=torch.float32, device=logits.device)
    if want_grad and dlogits is None:
        dlogits = torch.empty(B, ld, dtype=torch.bfloat16, device=logits.device)
    kernels().softmax_ce(logits, ld, labels, B, n_classes, scale, dlogits if want_grad else None, ld, stats, None)
    return dlogits, stats


def softmax_probs(logits: torch.Tensor, n_classes: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    B, ld = logits.shape
    if out is None:
        out = torch.empty(B, n_classes, dtype=torch.float32, device=logits.device)
    kernels().softmax_ce(logits, ld, None, B, n_classes, 1.0, None, ld, None, out)
    return out
