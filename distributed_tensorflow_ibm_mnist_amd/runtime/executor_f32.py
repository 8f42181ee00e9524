"""Reference-precision execution plan: fp32 activations, fp32 MFMA (``--precision fp32``).

The reference trains in fp32 (``mnist_input.py:86,107``: ``dtype = tf.float32``).
``HipNet`` (the default) runs bf16 activations / bf16 MFMA operands with fp32
accumulation; ``HipNetF32`` runs the same model specs with every activation,
weight operand and gradient in fp32 on the ``csrc/kernels/f32.hip`` kernels
(``v_mfma_f32_16x16x4_f32`` GEMM engine with implicit-GEMM conv loaders, fp32
max-pool / LRN / softmax-CE).  The f32 launchers route the reference CNN's convs
to dedicated kernels: conv2 (14x14, 32 -> 64) fwd / dgrad / wgrad on LDS-halo
tiles (``conv_halo_f32.hip``, the bf16 halo design in fp32), conv1 (28x28x1 ->
32) fwd / wgrad on shifted-copy image tiles (``conv1_f32.hip``); pool and LRN run
as 16-byte-vector kernels.  At B=16384 that took the fp32 step from 26.0 to
~19 ms (``profiles/r3/fp32/``).  Optimizer, EMA, LR schedule, loss EMA and the
deterministic split-K reduce are the shared K9 / misc.hip kernels, so the
checkpoint layout, hooks and data-parallel buckets are identical.

Layer semantics follow the reference graph exactly: conv + bias + ReLU
(``mnist_input.py:142-145``), 2x2/2 SAME max-pool (first maximum wins), LRN across
channels, dense + bias (+ ReLU).  ReLU backward masks are folded into the producer of
each gradient, as in the bf16 plan.  Two pairs run fused (``fuse=True``, default):
conv1 + pool1 (ConvPoolF: the 1.64 GB conv1 output and its gradient never reach HBM at
B = 16384) and norm2 + pool2 (LRNPoolF: the 822 MB LRN output and its gradient); both
keep the unfused pair's arithmetic (tests/test_f32_gpu.py compares them).
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional

import torch

from ..models.spec import Conv, Dense, LRN, MaxPool, ModelSpec
from ..ops import functional as Fk
from ..ops._ext import kernels
from .executor import HipNet
from .params import FlatParams, OptConfig


def _f32(*shape, device) -> torch.Tensor:
    return torch.zeros(*shape, dtype=torch.float32, device=device)


def wgrad_splits(M: int, N: int, K: int, target: int = 2048, min_k: int = 256, cap: int = 1024) -> int:
    """Split-K factor of an fp32 weight-gradient GEMM (64x64 tiles): fill the CUs
    while keeping every split >= min_k reduction elements."""
    tiles = math.ceil(M / 64) * math.ceil(N / 64)
    return int(max(1, min(math.ceil(target / tiles), max(1, K // min_k), cap)))


class _L:
    has_params = False
    idx = -1

    def fwd(self, nb: int) -> None: ...

    def bwd_weight(self, nb: int, dy: torch.Tensor) -> None: ...

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None: ...


class ConvF(_L):
    has_params = True

    def __init__(self, spec: Conv, x: torch.Tensor, in_relu: bool, fp: FlatParams, B: int, dev):
        self.spec, self.name, self.x, self.in_relu, self.fp = spec, spec.name, x, in_relu, fp
        _, self.H, self.W, self.C = x.shape
        self.OH, self.OW = Fk.conv_out_hw(self.H, self.W, spec.kh, spec.kw, spec.padding)
        self.ph, self.pw = Fk.conv_pads(spec.kh, spec.kw, spec.padding)
        self.out = _f32(B, self.OH, self.OW, spec.cout, device=dev)
        self.wname, self.bname = f"{spec.name}/weights", f"{spec.name}/biases"
        self.M = spec.kh * spec.kw * self.C + 1
        # the LDS-halo weight gradient (conv_halo_f32.hip) writes one partial per resident
        # workgroup; other geometries use the split-K GEMM rule
        pref = kernels().f32_conv_wgrad_pref_splits(self.H, self.W, self.C, self.OH, self.OW, spec.kh, spec.kw,
                                                    self.ph, self.pw, spec.cout) if dev.type == "cuda" else -1
        self.halo_wg = pref > 0
        self.splits = pref if self.halo_wg else wgrad_splits(self.M, spec.cout, B * self.OH * self.OW)
        self.slab = _f32(self.splits * self.M * spec.cout, device=dev)

    def fwd(self, nb: int) -> None:
        s = self.spec
        kernels().f32_conv_fwd(self.x, self.fp.param_view(self.wname), self.out, nb, self.H, self.W, self.C, self.OH,
                               self.OW, s.kh, s.kw, self.ph, self.pw, s.cout, self.fp.param_view(self.bname), s.relu)

    def bwd_weight(self, nb: int, dy: torch.Tensor) -> None:
        s, K = self.spec, kernels()
        S = min(self.splits, max(1, nb)) if self.halo_wg else \
            min(self.splits, wgrad_splits(self.M, s.cout, nb * self.OH * self.OW))
        K.f32_conv_wgrad(self.x, dy, self.slab, nb, self.H, self.W, self.C, self.OH, self.OW, s.kh, s.kw, self.ph,
                         self.pw, s.cout, S)
        K.splitk_reduce(self.slab, S, self.M, s.cout, s.kh * s.kw, self.C, self.C, s.cout, s.kh * s.kw * self.C,
                        self.fp.grad_view(self.wname), self.fp.grad_view(self.bname), 1.0)

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None:
        if dx is None:
            return
        s = self.spec
        kernels().f32_conv_dgrad(dy, self.fp.param_view(self.wname), dx, nb, self.OH, self.OW, s.cout, self.H, self.W,
                                 s.kh, s.kw, self.ph, self.pw, self.C, self.x if self.in_relu else None)


class PoolF(_L):
    def __init__(self, spec: MaxPool, x: torch.Tensor, in_relu: bool, B: int, dev):
        assert spec.k == 2 and spec.s == 2 and spec.padding == "SAME", "2x2/2 SAME pooling only"
        self.spec, self.name, self.x, self.in_relu = spec, spec.name, x, in_relu
        _, self.H, self.W, self.C = x.shape
        self.out = _f32(B, (self.H + 1) // 2, (self.W + 1) // 2, self.C, device=dev)
        self.arg = torch.zeros(self.out.shape, dtype=torch.uint8, device=dev)

    def fwd(self, nb: int) -> None:
        kernels().f32_maxpool_fwd(self.x, self.out, self.arg, nb, self.H, self.W, self.C)

    def bwd_data(self, nb: int, dy, dx) -> None:
        if dx is not None:
            kernels().f32_maxpool_bwd(dy, self.arg, self.out, self.in_relu, dx, nb, self.H, self.W, self.C)


class LRNF(_L):
    def __init__(self, spec: LRN, x: torch.Tensor, in_relu: bool, B: int, dev):
        self.spec, self.name, self.x, self.in_relu = spec, spec.name, x, in_relu
        self.C = x.shape[-1]
        self.out = torch.zeros_like(x)

    def _p(self, nb: int) -> int:
        return nb * (self.x[0].numel() // self.C)

    def fwd(self, nb: int) -> None:
        s = self.spec
        kernels().f32_lrn_fwd(self.x, self.out, self._p(nb), self.C, s.depth_radius, s.bias, s.alpha, s.beta)

    folded = False   # the backward runs inside the preceding ConvPoolF's weight gradient

    def bwd_data(self, nb: int, dy, dx) -> None:
        if dx is not None and not self.folded:
            s = self.spec
            kernels().f32_lrn_bwd(self.x, dy, dx, self._p(nb), self.C, s.depth_radius, s.bias, s.alpha, s.beta,
                                  self.in_relu)


class ConvPoolF(_L):
    """conv1 (28x28x1 -> 32, 5x5 SAME) + bias + ReLU + 2x2/2 max-pool as one kernel
    (conv1_f32.hip): the conv output is never materialised; the weight gradient un-pools
    dL/d pool through the codes inside its staging.  First layer only (no data gradient)."""
    has_params = True

    def __init__(self, conv: Conv, pool: MaxPool, x: torch.Tensor, fp: FlatParams, B: int, dev):
        self.spec, self.pool_spec, self.name, self.x, self.fp = conv, pool, conv.name, x, fp
        self.in_relu = False
        _, self.H, self.W, self.C = x.shape
        self.out = _f32(B, self.H // 2, self.W // 2, conv.cout, device=dev)
        self.arg = torch.zeros(self.out.shape, dtype=torch.uint8, device=dev)
        self.wname, self.bname = f"{conv.name}/weights", f"{conv.name}/biases"
        self.M = conv.kh * conv.kw * self.C + 1
        # the unfused conv1 weight gradient's split count: same image -> block assignment and
        # summation order, so the two graphs' gradients are bitwise equal
        ph, pw = Fk.conv_pads(conv.kh, conv.kw, conv.padding)
        self.splits = kernels().f32_conv_wgrad_pref_splits(self.H, self.W, self.C, self.H, self.W, conv.kh, conv.kw,
                                                           ph, pw, conv.cout)
        self.slab = _f32(self.splits * self.M * conv.cout, device=dev)

    @staticmethod
    def fits(conv, pool, x: torch.Tensor) -> bool:
        if not (isinstance(conv, Conv) and isinstance(pool, MaxPool) and conv.relu and pool.k == 2 and pool.s == 2
                and pool.padding == "SAME"):
            return False
        _, H, W, C = x.shape
        OH, OW = Fk.conv_out_hw(H, W, conv.kh, conv.kw, conv.padding)
        ph, pw = Fk.conv_pads(conv.kh, conv.kw, conv.padding)
        return bool(kernels().f32_conv1_pool_ok(H, W, C, OH, OW, conv.kh, conv.kw, ph, pw, conv.cout))

    def fwd(self, nb: int) -> None:
        kernels().f32_conv1_fwd_pool(self.x, self.fp.param_view(self.wname), self.fp.param_view(self.bname),
                                     self.out, self.arg, nb)

    # (LRN spec, dL/d LRN output): the following norm1's backward runs inside this weight
    # gradient (conv1_f32_wgrad_lrn_k), dL/d pool1 is never written
    lrn_fold: Optional[tuple] = None

    def bwd_weight(self, nb: int, dy: torch.Tensor) -> None:
        s, K = self.spec, kernels()
        S = min(self.splits, max(1, nb))
        if self.lrn_fold is not None:
            ls, dn = self.lrn_fold
            K.f32_conv1_wgrad_lrn(self.x, dn, self.out, self.arg, self.slab, nb, S, ls.bias, ls.alpha, ls.beta)
        else:
            K.f32_conv1_wgrad_unpool(self.x, dy, self.arg, self.slab, nb, S)
        K.splitk_reduce(self.slab, S, self.M, s.cout, s.kh * s.kw, self.C, self.C, s.cout, s.kh * s.kw * self.C,
                        self.fp.grad_view(self.wname), self.fp.grad_view(self.bname), 1.0)

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None:
        assert dx is None, "ConvPoolF is a first layer"

    def conv_output(self, n: int) -> torch.Tensor:
        """The unpooled bias+ReLU conv output of the first n images (monitoring only)."""
        s = self.spec
        ph, pw = Fk.conv_pads(s.kh, s.kw, s.padding)
        out = torch.empty(n, self.H, self.W, s.cout, dtype=torch.float32, device=self.x.device)
        kernels().f32_conv_fwd(self.x, self.fp.param_view(self.wname), out, n, self.H, self.W, self.C, self.H,
                               self.W, s.kh, s.kw, ph, pw, s.cout, self.fp.param_view(self.bname), s.relu)
        return out


class LRNPoolF(_L):
    """LRN then 2x2/2 max-pool in one pass (the reference's norm2 -> pool2): the LRN output
    is never materialised; the backward un-pools and runs the LRN backward in one kernel.
    Outputs, codes and gradients are bitwise the unfused LRNF + PoolF pair's."""

    def __init__(self, lrn: LRN, pool: MaxPool, x: torch.Tensor, in_relu: bool, B: int, dev):
        self.spec, self.pool_spec, self.name, self.x, self.in_relu = lrn, pool, lrn.name, x, in_relu
        _, self.H, self.W, self.C = x.shape
        self.out = _f32(B, self.H // 2, self.W // 2, self.C, device=dev)
        self.arg = torch.zeros(self.out.shape, dtype=torch.uint8, device=dev)

    @staticmethod
    def fits(lrn, pool, x: torch.Tensor) -> bool:
        if not (isinstance(lrn, LRN) and isinstance(pool, MaxPool) and pool.k == 2 and pool.s == 2
                and pool.padding == "SAME"):
            return False
        _, H, W, C = x.shape
        return bool(kernels().f32_lrn_pool_ok(H, W, C, lrn.depth_radius))

    def fwd(self, nb: int) -> None:
        s = self.spec
        kernels().f32_lrn_pool_fwd(self.x, self.out, self.arg, nb, self.H, self.W, self.C, s.depth_radius, s.bias,
                                   s.alpha, s.beta)

    def bwd_data(self, nb: int, dy, dx) -> None:
        if dx is not None:
            s = self.spec
            kernels().f32_lrn_pool_bwd(self.x, dy, self.arg, dx, nb, self.H, self.W, self.C, s.depth_radius,
                                       s.bias, s.alpha, s.beta, self.in_relu)

    def lrn_output(self, n: int) -> torch.Tensor:
        s = self.spec
        out = torch.empty(n, self.H, self.W, self.C, dtype=torch.float32, device=self.x.device)
        kernels().f32_lrn_fwd(self.x, out, n * self.H * self.W, self.C, s.depth_radius, s.bias, s.alpha, s.beta)
        return out


class DenseF(_L):
    has_params = True

    def __init__(self, spec: Dense, x: torch.Tensor, in_relu: bool, fp: FlatParams, B: int, dev):
        self.spec, self.name, self.in_relu, self.fp = spec, spec.name, in_relu, fp
        self.x = x.view(B, -1)
        assert self.x.shape[1] == spec.din, f"{spec.name}: flatten {self.x.shape[1]} != din {spec.din}"
        self.out = _f32(B, spec.dout, device=dev)
        self.wname, self.bname = f"{spec.name}/weights", f"{spec.name}/biases"
        # slab capacity: the 64x64-tile split, or the 256x256 path's own (one round of blocks)
        self.splits = max(wgrad_splits(spec.din + 1, spec.dout, B), kernels().f32_wgrad_splits_cap(spec.din, spec.dout, B))
        self.slab = _f32(self.splits * (spec.din + 1) * spec.dout, device=dev)

    def fwd(self, nb: int) -> None:
        s = self.spec
        kernels().f32_dense_fwd(self.x, self.fp.param_view(self.wname), self.out, nb, s.dout, s.din, s.dout,
                                self.fp.param_view(self.bname), s.relu)

    def bwd_weight(self, nb: int, dy: torch.Tensor) -> None:
        s, K = self.spec, kernels()
        S = min(self.splits, max(wgrad_splits(s.din + 1, s.dout, nb), K.f32_wgrad_splits_cap(s.din, s.dout, nb)))
        S = K.f32_dense_wgrad(self.x, dy.view(-1, s.dout), self.slab, nb, s.din, s.dout, S)   # partials written
        K.splitk_reduce(self.slab, S, s.din + 1, s.dout, 1, s.din, s.din, s.dout, s.din,
                        self.fp.grad_view(self.wname), self.fp.grad_view(self.bname), 1.0)

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None:
        if dx is not None:
            s = self.spec
            kernels().f32_dense_dgrad(dy.view(-1, s.dout), self.fp.param_view(self.wname), dx.view(-1, s.din), nb,
                                      s.din, s.dout, self.x if self.in_relu else None)


class HipNetF32:
    """One fp32 model replica on one GPU: the HipNet interface (forward /
    loss_and_grad / backward / update, eval, probs, stats) on fp32 kernels."""

    precision = "fp32"

    def __init__(self, spec: ModelSpec, batch: int, device, init: Dict[str, torch.Tensor],
                 opt: Optional[OptConfig] = None, fuse: bool = True):
        """``fuse``: conv1 + pool1 and LRN + pool runs as one kernel each where the kernels
        cover the geometry (ConvPoolF, LRNPoolF); False keeps the reference's layer-by-layer
        graph (tests compare the two)."""
        dev = torch.device(device)
        assert dev.type == "cuda", "HipNetF32 runs the HIP kernels (use --impl=torch on CPU)"
        self.spec, self.B, self.device = spec, batch, dev
        self.opt = opt or OptConfig()
        specs = []
        for L in spec.weights():
            shp = (L.kh, L.kw, L.cin, L.cout) if isinstance(L, Conv) else (L.din, L.dout)
            specs.append((f"{L.name}/weights", shp, L.wd))
            specs.append((f"{L.name}/biases", (L.cout if isinstance(L, Conv) else L.dout,), None))
        self.fp = FlatParams.build(specs, init, dev, bf16_copies=False)   # kernels read the fp32 masters
        H, W = spec.input_hw
        self.x0 = _f32(batch, H, W, spec.in_channels, device=dev)
        self.labels = torch.zeros(batch, dtype=torch.int32, device=dev)
        self.layers: List[_L] = []
        x, in_relu = self.x0, False
        skip = -1
        for i, L in enumerate(spec.layers):
            if i == skip:
                continue
            nxt = spec.layers[i + 1] if i + 1 < len(spec.layers) else None
            if fuse and i == 0 and ConvPoolF.fits(L, nxt, x):
                lay = ConvPoolF(L, nxt, x, self.fp, batch, dev)
                skip, in_relu = i + 1, False
            elif fuse and LRNPoolF.fits(L, nxt, x):
                lay = LRNPoolF(L, nxt, x, in_relu, batch, dev)
                skip, in_relu = i + 1, False
            elif isinstance(L, Conv):
                lay = ConvF(L, x, in_relu, self.fp, batch, dev)
                in_relu = L.relu
            elif isinstance(L, MaxPool):
                lay = PoolF(L, x, in_relu, batch, dev)
                in_relu = False
            elif isinstance(L, LRN):
                lay = LRNF(L, x, in_relu, batch, dev)
                in_relu = False
            elif isinstance(L, Dense):
                lay = DenseF(L, x, in_relu, self.fp, batch, dev)
                in_relu = L.relu
            else:
                raise TypeError(L)
            lay.idx = i
            self.layers.append(lay)
            x = lay.out
        assert isinstance(self.layers[-1], DenseF), "model must end in a Dense"
        self.logits = self.layers[-1].out
        self.n_classes = spec.num_classes
        self.dlogits = torch.zeros_like(self.logits)
        self.dbuf: List[Optional[torch.Tensor]] = [None] + [torch.zeros_like(l.out) for l in self.layers[:-1]]
        # norm1's backward folded into conv1's weight gradient (reference CNN: conv1 + pool1 ->
        # norm1, radius 4 over 32 channels); MNISTX_F32_FOLD_LRN=0 keeps the separate LRN backward
        self.fold_lrn = False
        L0, L1 = self.layers[0], self.layers[1] if len(self.layers) > 1 else None
        if (fuse and isinstance(L0, ConvPoolF) and isinstance(L1, LRNF) and L1.x is L0.out and L1.C == 32
                and L1.spec.depth_radius == 4 and not L1.in_relu and os.environ.get("MNISTX_F32_FOLD_LRN", "1") != "0"):
            L0.lrn_fold = (L1.spec, self.dbuf[2])
            L1.folded = True
            self.fold_lrn = True
        self.stats = _f32(8, device=dev)
        self.eval_stats = _f32(8, device=dev)
        self.ce_work = _f32(4 * 1024 + 1, device=dev)
        names = [e.name for e in self.fp.wd_entries]
        self.loss_names = [n.replace("/weights", "/weight_loss") for n in names] + ["cross_entropy", "total_loss"]
        self.loss_ema = _f32(3 * len(self.loss_names), device=dev)
        self.grad_ready_hooks: List[Callable[[int], None]] = []
        self.hook_layers: Optional[set] = None
        self.idx_buf: Optional[torch.Tensor] = None
        self.head = None

    # shared with the bf16 plan: K9 update + finalisation, stats readback
    update = HipNet.update
    finalize = HipNet.finalize
    _fin_args = HipNet._fin_args
    read_stats = HipNet.read_stats

    def can_gather_input(self) -> bool:
        return False

    def bind_u8_input(self, images_u8: torch.Tensor) -> bool:
        return False

    def forward(self, nb: Optional[int] = None, from_x0: bool = False, defer_head: bool = False) -> torch.Tensor:
        nb = self.B if nb is None else nb
        for lay in self.layers:
            lay.fwd(nb)
        return self.logits

    def loss_and_grad(self, nb: Optional[int] = None, scale: Optional[float] = None) -> None:
        nb = self.B if nb is None else nb
        kernels().f32_softmax_ce(self.logits, self.logits.shape[1], self.labels, nb, self.n_classes,
                                 (1.0 / nb) if scale is None else scale, self.dlogits, self.logits.shape[1],
                                 self.stats, None, self.ce_work)

    def backward(self, nb: Optional[int] = None) -> None:
        nb = self.B if nb is None else nb
        dy = self.dlogits
        for i in range(len(self.layers) - 1, -1, -1):
            lay = self.layers[i]
            if lay.has_params:
                lay.bwd_weight(nb, dy)
                if self.hook_layers is None or lay.idx in self.hook_layers:
                    for h in self.grad_ready_hooks:
                        h(lay.idx)
            dx = self.dbuf[i]
            lay.bwd_data(nb, dy, dx)
            dy = dx

    def train_step(self, grad_scale: float = 1.0) -> None:
        self.forward()
        self.loss_and_grad()
        self.backward()
        self.update(grad_scale)

    def eval_batch(self, nb: int, stats: Optional[torch.Tensor] = None) -> torch.Tensor:
        st = self.eval_stats if stats is None else stats
        self.forward(nb)
        kernels().f32_softmax_ce(self.logits, self.logits.shape[1], self.labels, nb, self.n_classes, 1.0, None,
                                 self.logits.shape[1], st, None, self.ce_work)
        return st

    def probs(self, nb: int) -> torch.Tensor:
        self.forward(nb)
        out = torch.empty(nb, self.n_classes, dtype=torch.float32, device=self.device)
        kernels().f32_softmax_ce(self.logits, self.logits.shape[1], None, nb, self.n_classes, 1.0, None,
                                 self.logits.shape[1], None, out, None)
        return out

    def activation(self, layer_name: str) -> torch.Tensor:
        """A layer's output tensor (a fused pair's pool output under either name's pool)."""
        for lay in self.layers:
            if lay.name == layer_name and not isinstance(lay, (ConvPoolF, LRNPoolF)):
                return lay.out
            if getattr(lay, "pool_spec", None) is not None and lay.pool_spec.name == layer_name:
                return lay.out
        raise KeyError(layer_name)

    def layer_activation(self, layer_name: str, n: int) -> torch.Tensor:
        """``<layer>/<layer>:0`` (main.py:97-100) for the first n images: the conv ReLU output
        itself (recomputed for a fused conv + pool, monitoring only)."""
        n = max(1, min(n, self.B))
        for lay in self.layers:
            if lay.name == layer_name and isinstance(lay, ConvPoolF):
                return lay.conv_output(n)
            if lay.name == layer_name and isinstance(lay, LRNPoolF):
                return lay.lrn_output(n)
        return self.activation(layer_name)[:n]
