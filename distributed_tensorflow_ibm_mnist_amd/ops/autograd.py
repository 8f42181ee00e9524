"""``torch.autograd.Function`` wrappers over the CDNA4 HIP kernels.

These make the kernels composable from ordinary PyTorch code (any model, any
optimizer); the fused training executor (``runtime/executor.py``) calls the
same kernels without autograd for the static-plan fast path.  Conventions
(``ops/functional.py``): activations are bf16 NHWC with channel counts padded
to a multiple of 8 (the padding lanes stay exactly 0); weights are fp32
``nn.Parameter`` masters in the reference layout (``[KH, KW, Cin, Cout]``,
``[Din, Dout]``) cast to a padded bf16 copy per call; weight gradients come
back fp32 from the deterministic split-K reduce.

Replaces the TF graph ops of SURVEY.md §2.3 N1-N9 (Conv2D, Conv2DBackprop*,
BiasAdd/Relu, MatMul, MaxPool, LRN, SparseSoftmaxCrossEntropyWithLogits) at
mnist_input.py:142-226 for user-defined models.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import functional as Fk
from ._ext import kernels


def _bf16c(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).contiguous()


def _relu_mask(dy: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    return (dy * (y > 0)).to(torch.bfloat16).contiguous()


class Conv2dFn(torch.autograd.Function):
    """y = [relu](conv2d(x, W) + b), stride 1, SAME/VALID (implicit-GEMM MFMA kernels)."""

    @staticmethod
    def forward(ctx, x, w, b, padding: str, relu: bool, cout_pad: int):
        kh, kw, cin, cout = w.shape
        x = _bf16c(x)
        w_bf = Fk.weight_to_bf16(w.detach(), x.shape[-1], cout_pad)
        y = Fk.conv2d(x, w_bf, b.detach().contiguous() if b is not None else None, padding, relu,
                      bias_n=cout if b is not None else 0)
        ctx.save_for_backward(x, w_bf, y)
        ctx.meta = (kh, kw, cin, cout, padding, relu, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_bf, y = ctx.saved_tensors
        kh, kw, cin, cout, padding, relu, has_b = ctx.meta
        g = _relu_mask(dy, y) if relu else _bf16c(dy)
        dw, db = Fk.conv2d_wgrad(x, g, kh, kw, padding, cin, cout, with_bias=has_b)
        dx = None
        if ctx.needs_input_grad[0]:
            if x.shape[-1] % 8 or w_bf.shape[-1] % 8:
                raise NotImplementedError("conv dgrad needs channel counts padded to multiples of 8")
            dx = Fk.conv2d_dgrad(g, w_bf, (x.shape[1], x.shape[2]), padding)
        return dx, dw, db, None, None, None


class ConvReluPoolFn(torch.autograd.Function):
    """Fused conv5x5 + bias + ReLU + 2x2/2 max-pool (csrc/kernels/convpool.hip);
    the full-resolution conv output never exists.  Geometries: see
    ``kernels().convpool_supported``."""

    @staticmethod
    def forward(ctx, x, w, b, pad: int, cout_pad: int):
        K = kernels()
        x = _bf16c(x)
        N, H, W, C = x.shape
        kh, kw, cin, cout = w.shape
        geo = (C, cout_pad, kh, pad, H, W)
        if K.convpool_supported(*geo) < 0:
            raise ValueError(f"no fused conv+pool kernel for geometry {geo}")
        w_bf = Fk.weight_to_bf16(w.detach(), C, cout_pad)
        OH, OW = H + 2 * pad - kh + 1, W + 2 * pad - kw + 1
        pooled = torch.empty(N, OH // 2, OW // 2, cout_pad, dtype=torch.bfloat16, device=x.device)
        arg = torch.empty(N, OH // 2, OW // 2, cout_pad, dtype=torch.uint8, device=x.device)
        K.convpool_fwd(x, w_bf, b.detach().contiguous(), cout, pooled, arg, N, *geo)
        ctx.save_for_backward(x, w_bf, arg)
        ctx.meta = (geo, cin, cout)
        ctx.mark_non_differentiable(arg)
        return pooled, arg

    @staticmethod
    def backward(ctx, dP, _darg):
        K = kernels()
        x, w_bf, arg = ctx.saved_tensors
        geo, cin, cout = ctx.meta
        N = x.shape[0]
        dP = _bf16c(dP)
        KM = K.convpool_rows(*geo)
        grid = max(1, min(1024, (N + 3) // 4))
        slab = torch.empty(grid * KM * geo[1], dtype=torch.float32, device=x.device)
        K.convpool_wgrad(x, dP, arg, slab, grid, N, *geo)
        G, Ip, I, brow = K.convpool_reduce_args(*geo, cin)
        kh = geo[2]
        dw = torch.empty(kh, kh, cin, cout, dtype=torch.float32, device=x.device)
        db = torch.empty(cout, dtype=torch.float32, device=x.device)
        K.splitk_reduce(slab, grid, KM, geo[1], G, Ip, I, cout, brow, dw, db, 1.0)
        dx = None
        if ctx.needs_input_grad[0]:
            if not K.convpool_has_dgrad(*geo):
                raise NotImplementedError(f"no fused dgrad for geometry {geo} (use Conv2d + MaxPool2x2)")
            dx = torch.empty_like(x)
            K.convpool_dgrad(dP, arg, w_bf, dx, N, *geo)
        return dx, dw, db, None, None


class DenseFn(torch.autograd.Function):
    """y = [relu](x @ W + b) on MFMA (bias/ReLU fused in the epilogue)."""

    @staticmethod
    def forward(ctx, x, w, b, relu: bool, out_pad: int, out_fp32: bool):
        din, dout = w.shape
        ctx.in_shape = x.shape
        x = _bf16c(x.reshape(x.shape[0], -1))
        w_bf = Fk.weight_to_bf16(w.detach(), x.shape[1], out_pad)
        y = Fk.dense(x, w_bf, b.detach().contiguous() if b is not None else None, relu,
                     out_dtype=torch.float32 if out_fp32 else torch.bfloat16, bias_n=dout if b is not None else 0)
        ctx.save_for_backward(x, w_bf, y)
        ctx.meta = (din, dout, relu, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_bf, y = ctx.saved_tensors
        din, dout, relu, has_b = ctx.meta
        g = _relu_mask(dy, y) if relu else _bf16c(dy)
        dw, db = Fk.dense_wgrad(x, g, din, dout, with_bias=has_b)
        dx = Fk.dense_dgrad(g, w_bf).view(ctx.in_shape) if ctx.needs_input_grad[0] else None
        return dx, dw, db, None, None, None


class MaxPool2x2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _bf16c(x)
        y, arg = Fk.maxpool2x2(x)
        ctx.save_for_backward(arg, y)
        ctx.hw = (x.shape[1], x.shape[2])
        return y

    @staticmethod
    def backward(ctx, dy):
        arg, y = ctx.saved_tensors
        return Fk.maxpool2x2_bwd(_bf16c(dy), arg, y, ctx.hw, relu_mask=False)


class LRNFn(torch.autograd.Function):
    """TF local response normalization across channels (alpha not divided by the window)."""

    @staticmethod
    def forward(ctx, x, r: int, bias: float, alpha: float, beta: float):
        x = _bf16c(x)
        ctx.save_for_backward(x)
        ctx.p = (r, bias, alpha, beta)
        return Fk.lrn(x, r, bias, alpha, beta)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return Fk.lrn_bwd(x, _bf16c(dy), *ctx.p), None, None, None, None


class SoftmaxCrossEntropyFn(torch.autograd.Function):
    """Mean sparse softmax cross-entropy; the same kernel pass produces dlogits,
    the top-1 correct count and a non-finite flag (returned as ``stats``)."""

    @staticmethod
    def forward(ctx, logits, labels, n_classes: int):
        logits = logits.float().contiguous()
        B = logits.shape[0]
        dl, stats = Fk.softmax_ce(logits, labels.to(torch.int32).contiguous(), n_classes, scale=1.0 / B)
        ctx.save_for_backward(dl)
        ctx.mark_non_differentiable(stats)
        return stats[0] / B, stats

    @staticmethod
    def backward(ctx, dloss, _dstats):
        (dl,) = ctx.saved_tensors
        return dl.float() * dloss, None, None


def conv2d(x, w, b=None, padding: str = "SAME", relu: bool = True, cout_pad: Optional[int] = None):
    return Conv2dFn.apply(x, w, b, padding, relu, cout_pad or Fk.pad8(w.shape[-1]))


def conv_relu_pool(x, w, b, padding: str = "SAME", cout_pad: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    pad = (w.shape[0] - 1) // 2 if padding == "SAME" else 0
    return ConvReluPoolFn.apply(x, w, b, pad, cout_pad or Fk.pad8(w.shape[-1]))


def dense(x, w, b=None, relu: bool = True, out_pad: Optional[int] = None, out_fp32: bool = False):
    return DenseFn.apply(x, w, b, relu, out_pad or Fk.pad8(w.shape[1]), out_fp32)


def maxpool2x2(x):
    return MaxPool2x2Fn.apply(x)


def lrn(x, r: int = 4, bias: float = 1.0, alpha: float = 0.001 / 9.0, beta: float = 0.75):
    return LRNFn.apply(x, r, bias, alpha, beta)


def softmax_cross_entropy(logits, labels, n_classes: int):
    """Returns (mean loss, stats f32[8]: [sum CE, #correct, nonfinite flag, ...])."""
    return SoftmaxCrossEntropyFn.apply(logits, labels, n_classes)
