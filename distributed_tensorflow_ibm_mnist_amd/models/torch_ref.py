"""Pure-PyTorch fp32 implementation of a ``ModelSpec`` — the numerical oracle.

This is *not* the compute path on MI355X (that is ``runtime.executor`` on the
HIP kernels); it is what every HIP kernel is tested against
and what ``--impl torch`` runs as the plain-PyTorch baseline.

TF semantics reproduced exactly:
* SAME padding for stride-1 convs and 2x2/2 pools (pad after, like TF).
* ``tf.nn.lrn``: ``sqr_sum = Σ_{|c'-c|<=r} x²``, ``y = x (bias + α·sqr_sum)^-β``
  — α is NOT divided by the window size (unlike ``nn.LocalResponseNorm``).
* Flatten in NHWC order (``mnist_input.py:177-180``).
* ``l2_loss(w) = Σw²/2``; total loss = CE mean + Σ wd·l2_loss (``mnist_input.py:
  113,224-231``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from .spec import Conv, Dense, LRN, MaxPool, ModelSpec


def truncated_normal_(t: torch.Tensor, std: float, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """``tf.truncated_normal_initializer``: N(0, std) re-drawn outside ±2 std."""
    with torch.no_grad():
        flat = t.view(-1)
        n = flat.numel()
        out = torch.empty(0, dtype=t.dtype, device=t.device)
        while out.numel() < n:
            s = torch.randn(max(2 * (n - out.numel()), 64), generator=generator, dtype=torch.float64)
            s = s[s.abs() <= 2.0]
            out = torch.cat([out, s[: n - out.numel()].to(t.dtype).to(t.device)])
        flat.copy_(out * std)
    return t


def init_params(spec: ModelSpec, seed: int = 0, device: str | torch.device = "cpu") -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    params: Dict[str, torch.Tensor] = {}
    for L in spec.weights():
        if isinstance(L, Conv):
            w = torch.empty(L.kh, L.kw, L.cin, L.cout)
            b = torch.full((L.cout,), float(L.b_init))
        else:
            w = torch.empty(L.din, L.dout)
            b = torch.full((L.dout,), float(L.b_init))
        truncated_normal_(w, L.w_std, g)
        params[f"{L.name}/weights"] = w.to(device)
        params[f"{L.name}/biases"] = b.to(device)
    return params


def lrn_tf(x_nchw: torch.Tensor, r: int, bias: float, alpha: float, beta: float) -> torch.Tensor:
    sq = x_nchw * x_nchw
    c = x_nchw.shape[1]
    padded = F.pad(sq, (0, 0, 0, 0, r, r))
    s = sum(padded[:, i:i + c] for i in range(2 * r + 1))
    return x_nchw * torch.pow(bias + alpha * s, -beta)


def _pool_same(x: torch.Tensor, k: int, s: int, padding: str) -> torch.Tensor:
    if padding == "SAME":
        h, w = x.shape[-2:]
        oh, ow = math.ceil(h / s), math.ceil(w / s)
        ph = max((oh - 1) * s + k - h, 0)
        pw = max((ow - 1) * s + k - w, 0)
        if ph or pw:
            x = F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=float("-inf"))
    return F.max_pool2d(x, k, s)


def forward(spec: ModelSpec, params: Dict[str, torch.Tensor], x: torch.Tensor,
            keep_activations: bool = False) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """x: [B, H*W*C] or [B, H, W, C] (NHWC).  Returns (logits [B, classes], acts)."""
    h, w = spec.input_hw
    x = x.reshape(-1, h, w, spec.in_channels).permute(0, 3, 1, 2)  # NCHW for torch ops
    acts: Dict[str, torch.Tensor] = {}
    flat = False
    for L in spec.layers:
        if isinstance(L, Conv):
            wt = params[f"{L.name}/weights"].permute(3, 2, 0, 1)  # [Cout,Cin,KH,KW]
            if L.padding == "SAME":
                ph, pw = L.kh - 1, L.kw - 1
                x = F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
            x = F.conv2d(x, wt) + params[f"{L.name}/biases"].view(1, -1, 1, 1)
            if L.relu:
                x = F.relu(x)
        elif isinstance(L, MaxPool):
            x = _pool_same(x, L.k, L.s, L.padding)
        elif isinstance(L, LRN):
            x = lrn_tf(x, L.depth_radius, L.bias, L.alpha, L.beta)
        elif isinstance(L, Dense):
            if not flat:
                x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # NHWC flatten
                flat = True
            x = x @ params[f"{L.name}/weights"] + params[f"{L.name}/biases"]
            if L.relu:
                x = F.relu(x)
        if keep_activations:
            acts[L.name] = x.permute(0, 2, 3, 1) if x.dim() == 4 else x
    return x, acts


def losses(spec: ModelSpec, params: Dict[str, torch.Tensor], logits: torch.Tensor,
           labels: torch.Tensor) -> Dict[str, torch.Tensor]:
    """All entries of the reference 'losses' collection plus total_loss."""
    out: Dict[str, torch.Tensor] = {}
    for L in spec.weights():
        if L.wd is not None:
            wgt = params[f"{L.name}/weights"]
            out[f"{L.name}/weight_loss"] = float(L.wd) * 0.5 * (wgt * wgt).sum()
    out["cross_entropy"] = F.cross_entropy(logits, labels.long())
    out["total_loss"] = sum(out.values())
    return out


def accuracy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """top-1 batch accuracy (the intent of mnist_input.py:237-243, fixed per Q4)."""
    return (logits.argmax(dim=1) == labels.long()).float().mean()


class TorchModel(torch.nn.Module):
    """nn.Module wrapper (params as nn.Parameters under their TF names)."""

    def __init__(self, spec: ModelSpec, params: Dict[str, torch.Tensor]):
        super().__init__()
        self.spec = spec
        self.names: List[str] = list(params)
        self.plist = torch.nn.ParameterList([torch.nn.Parameter(params[n].clone()) for n in self.names])

    def params(self) -> Dict[str, torch.Tensor]:
        return {n: p for n, p in zip(self.names, self.plist)}

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return forward(self.spec, self.params(), x)[0]
