"""``nn.Module`` layers over the HIP kernels (``ops/autograd.py``) and a builder
that turns a registry ``ModelSpec`` (``models/registry.py``) into an ordinary
trainable ``nn.Sequential`` -- the library face of the framework: any PyTorch
optimizer / training loop can drive the CDNA4 kernels.

Parameters keep the TF names of the reference (``conv1/weights`` ...,
mnist_input.py:136-205) in :meth:`HipModel.named_tf_parameters`, so checkpoints
(``ckpt/saver.py``) and the oracle (``models/torch_ref.py``) line up.
"""
from __future__ import annotations

from typing import Dict, Iterator, Optional, Tuple

import torch
from torch import nn

from ..models.spec import LRN, Conv, Dense, MaxPool, ModelSpec
from . import autograd as A
from . import functional as Fk
from ._ext import kernels


class Conv2d(nn.Module):
    def __init__(self, cin: int, cout: int, k: int = 5, padding: str = "SAME", relu: bool = True, name: str = "conv"):
        super().__init__()
        self.name, self.padding, self.relu = name, padding, relu
        self.weight = nn.Parameter(torch.zeros(k, k, cin, cout))
        self.bias = nn.Parameter(torch.zeros(cout))

    def forward(self, x):
        return A.conv2d(x, self.weight, self.bias, self.padding, self.relu)


class ConvReluPool(nn.Module):
    """conv + bias + ReLU + 2x2/2 max-pool as one fused kernel (returns the pooled map)."""

    def __init__(self, cin: int, cout: int, k: int = 5, padding: str = "SAME", name: str = "conv"):
        super().__init__()
        self.name, self.padding = name, padding
        self.weight = nn.Parameter(torch.zeros(k, k, cin, cout))
        self.bias = nn.Parameter(torch.zeros(cout))

    def forward(self, x):
        return A.conv_relu_pool(x, self.weight, self.bias, self.padding)[0]


class MaxPool2x2(nn.Module):
    def forward(self, x):
        return A.maxpool2x2(x)


class LocalResponseNorm(nn.Module):
    def __init__(self, r: int = 4, bias: float = 1.0, alpha: float = 0.001 / 9.0, beta: float = 0.75):
        super().__init__()
        self.p = (r, bias, alpha, beta)

    def forward(self, x):
        return A.lrn(x, *self.p)


class Linear(nn.Module):
    def __init__(self, din: int, dout: int, relu: bool = True, out_pad: Optional[int] = None, out_fp32: bool = False,
                 name: str = "dense"):
        super().__init__()
        self.name, self.relu, self.out_pad, self.out_fp32 = name, relu, out_pad, out_fp32
        self.weight = nn.Parameter(torch.zeros(din, dout))
        self.bias = nn.Parameter(torch.zeros(dout))

    def forward(self, x):
        return A.dense(x, self.weight, self.bias, self.relu, self.out_pad, self.out_fp32)


class SoftmaxCrossEntropy(nn.Module):
    def __init__(self, n_classes: int):
        super().__init__()
        self.n_classes = n_classes
        self.last_stats: Optional[torch.Tensor] = None

    def forward(self, logits, labels):
        loss, stats = A.softmax_cross_entropy(logits, labels, self.n_classes)
        self.last_stats = stats
        return loss


class HipModel(nn.Sequential):
    """A ModelSpec as modules; input [B, H, W, C] (any float dtype), output fp32
    logits [B, max(16, pad8(classes))] (columns >= num_classes are 0)."""

    def __init__(self, spec: ModelSpec, fuse_convpool: bool = True):
        mods = []
        h, w = spec.input_hw
        c = spec.in_channels
        layers = spec.layers
        i = 0
        first = True
        while i < len(layers):
            L = layers[i]
            nxt = layers[i + 1] if i + 1 < len(layers) else None
            if isinstance(L, Conv):
                pad = (L.kh - 1) // 2 if L.padding == "SAME" else 0
                geo = (c, Fk.pad8(L.cout), L.kh, pad, h, w)
                fuse = (fuse_convpool and L.relu and isinstance(nxt, MaxPool) and L.kh == L.kw
                        and kernels().convpool_supported(*geo) >= 0
                        and (first or kernels().convpool_has_dgrad(*geo)))
                m = (ConvReluPool if fuse else Conv2d)(L.cin, L.cout, L.kh, L.padding,
                                                      **({} if fuse else {"relu": L.relu}), name=L.name)
                m.tf_names = (f"{L.name}/weights", f"{L.name}/biases")
                mods.append(m)
                if L.padding == "VALID":
                    h, w = h - L.kh + 1, w - L.kw + 1
                c = Fk.pad8(L.cout)
                if fuse:
                    h, w = h // 2, w // 2
                    i += 2
                    first = False
                    continue
            elif isinstance(L, MaxPool):
                mods.append(MaxPool2x2())
                h, w = (h + 1) // 2, (w + 1) // 2
            elif isinstance(L, LRN):
                mods.append(LocalResponseNorm(L.depth_radius, L.bias, L.alpha, L.beta))
            elif isinstance(L, Dense):
                last = i == len(layers) - 1
                if not isinstance(layers[i - 1], Dense) and i > 0:
                    assert c == (L.din // (h * w)), "flatten needs an unpadded channel count"
                m = Linear(L.din, L.dout, L.relu, out_pad=max(16, Fk.pad8(L.dout)) if last else None,
                           out_fp32=last, name=L.name)
                m.tf_names = (f"{L.name}/weights", f"{L.name}/biases")
                mods.append(m)
                c = Fk.pad8(L.dout)
            first = False
            i += 1
        super().__init__(*mods)
        self.spec = spec

    def named_tf_parameters(self) -> Iterator[Tuple[str, nn.Parameter]]:
        for m in self:
            if hasattr(m, "tf_names"):
                yield m.tf_names[0], m.weight
                yield m.tf_names[1], m.bias

    @torch.no_grad()
    def load_tf_params(self, params: Dict[str, torch.Tensor]) -> None:
        for n, p in self.named_tf_parameters():
            p.copy_(params[n])

    def forward(self, x):
        h, w = self.spec.input_hw
        x = x.reshape(-1, h, w, self.spec.in_channels)
        return super().forward(x)
