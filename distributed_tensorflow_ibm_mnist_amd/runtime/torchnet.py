"""Plain-PyTorch replica with the same interface as ``HipNet``.

Used for (a) the CPU test path (multi-process gloo tests of data-parallel and
parameter-server logic, the BASELINE "MLP single-process CPU" config), and
(b) ``--impl torch``: the PyTorch-ROCm baseline (MIOpen convolutions,
hipBLASLt GEMMs, bf16 autocast) that the HIP kernels are measured against.
It shares ``FlatParams`` (flat fp32 params/grads/slots) so checkpoints, DP
buckets and PS transfers are identical between the two implementations.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch
import torch.nn.functional as F

from ..models import torch_ref
from ..models.spec import Conv, Dense, ModelSpec
from .params import FlatParams, OptConfig


def torch_update(fp: FlatParams, cfg: OptConfig, grad_scale: float = 1.0) -> None:
    """Reference-semantics update (same math as the fused K9 kernel)."""
    with torch.no_grad():
        step = int(fp.step.item())
        lr = cfg.lr_at(step)
        wd = torch.zeros_like(fp.params)
        for i, e in enumerate(fp.entries):
            if e.wd:
                wd[e.off:e.off + e.n] = e.wd
            if e.l2_index >= 0:
                v = fp.params[e.off:e.off + e.n]
                fp.l2[e.l2_index] += (v * v).sum()
        g = fp.grads * grad_scale + wd * fp.params
        if cfg.use_momentum:
            fp.mom.mul_(cfg.momentum).add_(g)
            upd = g + cfg.momentum * fp.mom if cfg.nesterov else fp.mom
        else:
            upd = g
        fp.params.sub_(lr * upd)
        if cfg.ema_max >= 0:
            d = min(cfg.ema_max, (1.0 + step) / (10.0 + step))
            fp.ema.sub_((1.0 - d) * (fp.ema - fp.params))


class TorchNet:
    def __init__(self, spec: ModelSpec, batch: int, device, init: Dict[str, torch.Tensor],
                 opt: Optional[OptConfig] = None, autocast: Optional[bool] = None):
        dev = torch.device(device)
        self.spec, self.B, self.device = spec, batch, dev
        self.opt = opt or OptConfig()
        specs = []
        for L in spec.weights():
            shp = (L.kh, L.kw, L.cin, L.cout) if isinstance(L, Conv) else (L.din, L.dout)
            specs.append((f"{L.name}/weights", shp, L.wd))
            specs.append((f"{L.name}/biases", (L.cout if isinstance(L, Conv) else L.dout,), None))
        self.fp = FlatParams.build(specs, init, dev)
        H, W = spec.input_hw
        self.autocast = (dev.type == "cuda") if autocast is None else autocast
        xdt = torch.bfloat16 if dev.type == "cuda" else torch.float32
        self.x0 = torch.zeros(batch, H, W, spec.in_channels, dtype=xdt, device=dev)
        self.labels = torch.zeros(batch, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(8, dtype=torch.float32, device=dev)
        self.eval_stats = torch.zeros(8, dtype=torch.float32, device=dev)
        names = [e.name for e in self.fp.wd_entries]
        self.loss_names = [n.replace("/weights", "/weight_loss") for n in names] + ["cross_entropy", "total_loss"]
        self.loss_ema = torch.zeros(3 * len(self.loss_names), dtype=torch.float32, device=dev)
        self.grad_ready_hooks: List[Callable[[int], None]] = []
        self.n_classes = spec.num_classes
        self._logits: Optional[torch.Tensor] = None
        self._loss: Optional[torch.Tensor] = None
        self._leaf: Optional[torch.Tensor] = None
        self._acts: Dict[str, torch.Tensor] = {}
        self.keep_activations = False

    def _params(self, leaf: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {e.name: leaf[e.off:e.off + e.n].view(e.shape) for e in self.fp.entries}

    def forward(self, nb: Optional[int] = None, grad: bool = True, defer_head: bool = False) -> torch.Tensor:
        nb = self.B if nb is None else nb
        leaf = self.fp.params.detach().requires_grad_(grad)
        self._leaf = leaf
        x = self.x0[:nb].float() if not self.autocast else self.x0[:nb]
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.autocast):
            logits, acts = torch_ref.forward(self.spec, self._params(leaf), x, keep_activations=self.keep_activations)
        self._acts = acts
        self._logits = logits.float()
        return self._logits

    def loss_and_grad(self, nb: Optional[int] = None, scale: Optional[float] = None) -> None:
        nb = self.B if nb is None else nb
        if self._leaf is None or not self._leaf.requires_grad:
            self.forward(nb, grad=True)
        lab = self.labels[:nb].long()
        loss = F.cross_entropy(self._logits, lab, reduction="sum")
        with torch.no_grad():
            self.stats[0] += loss.detach()
            self.stats[1] += (self._logits.argmax(1) == lab).sum().float()
            if not torch.isfinite(loss.detach()):
                self.stats[2] = 1.0
        self._loss = loss * ((1.0 / nb) if scale is None else scale)

    def backward(self, nb: Optional[int] = None) -> None:
        (g,) = torch.autograd.grad(self._loss, self._leaf)
        self.fp.grads.copy_(g)
        self._leaf = None
        for i in range(len(self.spec.layers) - 1, -1, -1):
            if isinstance(self.spec.layers[i], (Conv, Dense)):
                for h in self.grad_ready_hooks:
                    h(i)

    def update(self, grad_scale: float = 1.0, increment: bool = True, batch_for_stats: Optional[int] = None) -> None:
        torch_update(self.fp, self.opt, grad_scale)
        self.finalize(batch_for_stats or self.B, increment)

    def finalize(self, batch: int, increment: bool = True) -> None:
        fp = self.fp
        with torch.no_grad():
            ce = self.stats[0] / batch
            acc = self.stats[1] / batch
            wl = [float(e.wd) * 0.5 * fp.l2[e.l2_index] for e in fp.wd_entries]
            total = ce + (sum(wl) if wl else 0.0)
            vals = wl + [ce, total]
            for i, v in enumerate(vals):
                e = self.loss_ema[3 * i:3 * i + 3]
                e[0] = 0.9 * e[0] + 0.1 * v
                e[1] += 1
                e[2] = e[0] / (1 - 0.9 ** e[1])
            self.stats[4] = ce
            self.stats[5] = acc
            self.stats[6] = total
            self.stats[7] += 1
            self.stats[0] = 0
            self.stats[1] = 0
            fp.l2.zero_()
            if increment:
                fp.step += 1

    def train_step(self, grad_scale: float = 1.0) -> None:
        self.forward()
        self.loss_and_grad()
        self.backward()
        self.update(grad_scale)

    def eval_batch(self, nb: int, stats: Optional[torch.Tensor] = None) -> torch.Tensor:
        st = self.eval_stats if stats is None else stats
        with torch.no_grad():
            logits = self.forward(nb, grad=False)
            lab = self.labels[:nb].long()
            st[0] += F.cross_entropy(logits, lab, reduction="sum")
            st[1] += (logits.argmax(1) == lab).sum().float()
        return st

    def probs(self, nb: int) -> torch.Tensor:
        with torch.no_grad():
            return torch.softmax(self.forward(nb, grad=False)[:, : self.n_classes], 1)

    def activation(self, layer_name: str) -> torch.Tensor:
        return self._acts[layer_name]

    def layer_activation(self, layer_name: str, n: int) -> torch.Tensor:
        """``<layer>/<layer>:0`` (main.py:97-100) for the first n images of the
        current batch, recomputed without autograd (monitoring only)."""
        n = max(1, min(n, self.B))
        with torch.no_grad():
            x = self.x0[:n].float() if not self.autocast else self.x0[:n]
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.autocast):
                _, acts = torch_ref.forward(self.spec, self._params(self.fp.params), x, keep_activations=True)
        return acts[layer_name]

    def read_stats(self) -> Dict[str, float]:
        s = self.stats.detach().cpu().tolist()
        return {"cross_entropy": s[4], "accuracy": s[5], "total_loss": s[6], "nan": s[2]}
