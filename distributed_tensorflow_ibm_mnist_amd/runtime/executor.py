"""Static execution plan for a ``ModelSpec`` on the HIP kernels.

This replaces TF's graph executor for the reference model: the
forward, the *explicit* backward and the fused update of one training step are
a fixed sequence of kernel launches over buffers allocated once for a given
batch size (an arena), so the whole step can be captured into a hipGraph
(``runtime/graph.py``) and replayed with no host work.

Design points (MI355X-first, not a port of the TF graph):
* activations bf16 NHWC, channels padded to 8 → every operand load is 16 B;
* ReLU backward is fused into whichever kernel produces the gradient
  (dgrad epilogue, pool-backward, LRN-backward), never a separate pass;
* bias gradients ride in the weight-gradient GEMM as a virtual ones column;
* weight gradients are written straight into the flat gradient buffer, and a
  per-layer "grads ready" hook lets the data-parallel layer launch RCCL
  all-reduce of finished buckets while earlier layers are still in backward;
* loss / accuracy / NaN flag stay on device (``stats``); the host reads them
  only when it logs (no per-step sync).
"""
from __future__ import annotations

import os

import dataclasses
from typing import Callable, Dict, List, Optional, Tuple

import torch

from ..models.spec import Conv, Dense, LRN, MaxPool, ModelSpec
from ..ops import functional as Fk
from ..ops._ext import kernels
from .params import FlatParams, OptConfig


def _bf16(*shape, device) -> torch.Tensor:
    return torch.zeros(*shape, dtype=torch.bfloat16, device=device)


def _reduce(red: Optional[list], slab: torch.Tensor, geo: Tuple[int, ...], wdst: torch.Tensor,
            bdst: torch.Tensor) -> None:
    """Split-K reduce of one weight gradient: now, or queued on ``red``.
    geo = (splits, M, N, G, Ipad, I, J, bias_row) of splitk_reduce."""
    if red is None:
        kernels().splitk_reduce(slab, *geo, wdst, bdst, 1.0)
    else:
        red.append((slab, geo, wdst, bdst))


class _Layer:
    name: str
    has_params = False
    out: torch.Tensor          # output activation buffer [B, ...]

    def fwd(self, nb: int) -> None: ...

    # backward = weight gradient (off the critical path: side stream) + data gradient.
    # ``red``: a list collecting this layer's split-K reduce (see HipNet._flush_reduce)
    # instead of launching it right away.
    def bwd_weight(self, nb: int, dy: torch.Tensor, slab: torch.Tensor, red: Optional[list] = None) -> None:
        pass

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None:
        pass

    def bwd(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor], slab=None) -> None:
        if self.has_params:
            self.bwd_weight(nb, dy, slab)
        self.bwd_data(nb, dy, dx)


class ConvLayer(_Layer):
    has_params = True

    def __init__(self, spec: Conv, x: torch.Tensor, in_relu: bool, first: bool, fp: FlatParams, B: int, dev):
        self.spec, self.name, self.x, self.in_relu, self.first, self.fp = spec, spec.name, x, in_relu, first, fp
        _, self.H, self.W, self.C = x.shape
        self.OH, self.OW = Fk.conv_out_hw(self.H, self.W, spec.kh, spec.kw, spec.padding)
        self.Cp = Fk.pad8(spec.cout)
        self.ph, self.pw = Fk.conv_pads(spec.kh, spec.kw, spec.padding)
        self.out = _bf16(B, self.OH, self.OW, self.Cp, device=dev)
        self.wname, self.bname = f"{spec.name}/weights", f"{spec.name}/biases"
        self.M_wg = spec.kh * spec.kw * self.C + 1
        # the LDS-halo weight gradient (conv_halo.hip) wants one partial per resident block
        self.pref = (kernels().conv_wgrad_pref_splits(B, self.H, self.W, self.C, self.OH, self.OW, spec.kh, spec.kw,
                                                      self.ph, self.pw, self.Cp, True) if dev.type == "cuda" else -1)
        self.splits = max(Fk.pick_splits(self.M_wg, self.Cp, B * self.OH * self.OW), self.pref)
        self.slab_elems = self.splits * self.M_wg * self.Cp

    # (LRN spec, LRN input): the preceding LRN is applied while this conv stages its
    # input (forward and weight gradient), so the LRN output is never written
    # (HipNet.fold_lrn_fwd; reference CNN norm1 -> conv2 on the LDS-halo kernels)
    lrn_pre: Optional[tuple] = None

    def _xin(self):
        if self.lrn_pre is None:
            return self.x, {}
        ls, xp = self.lrn_pre
        return xp, {"lrn_r": ls.depth_radius, "lrn_bias": ls.bias, "lrn_alpha": ls.alpha, "lrn_beta": ls.beta}

    def fwd(self, nb: int) -> None:
        s = self.spec
        x, lrn = self._xin()
        kernels().conv_fwd(x, self.fp.bf16_view(self.wname), self.out, nb, self.H, self.W, self.C, self.OH,
                           self.OW, s.kh, s.kw, self.ph, self.pw, self.Cp, self.fp.param_view(self.bname), s.cout,
                           s.relu, **lrn)

    def bwd_weight(self, nb: int, dy: torch.Tensor, slab: torch.Tensor, red: Optional[list] = None) -> None:
        s = self.spec
        K = kernels()
        req = self.pref if self.pref > 0 else Fk.pick_splits(self.M_wg, self.Cp, nb * self.OH * self.OW)
        x, lrn = self._xin()
        S = K.conv_wgrad(x, dy, slab, nb, self.H, self.W, self.C, self.OH, self.OW, s.kh, s.kw, self.ph, self.pw,
                         self.Cp, True, req, **lrn)
        _reduce(red, slab, (S, self.M_wg, self.Cp, s.kh * s.kw, self.C, s.cin, s.cout, s.kh * s.kw * self.C),
                self.fp.grad_view(self.wname), self.fp.grad_view(self.bname))

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None:
        if dx is not None:
            s = self.spec
            kernels().conv_dgrad(dy, self.fp.bf16_view(self.wname), dx, nb, self.OH, self.OW, self.Cp, self.H, self.W,
                                 s.kh, s.kw, self.ph, self.pw, self.C, self.x if self.in_relu else None)


class ConvPoolLayer(_Layer):
    """conv + bias + ReLU + 2x2 max-pool as ONE fused kernel (csrc/kernels/convpool.hip).

    Used when a ReLU conv is directly followed by a 2x2/2 pool and the geometry
    has a compile-time specialisation (LeNet-5 conv1/conv2, reference conv1).
    The full-resolution conv output is never materialised; backward rebuilds
    dY from the pooled gradient, argmax byte and ReLU mask inside the wgrad
    (and, when needed, dgrad) kernels.
    """
    has_params = True

    @staticmethod
    def supported(spec: Conv, pool: MaxPool, x_shape) -> bool:
        _, H, W, C = x_shape
        if not (spec.relu and spec.kh == spec.kw == 5 and pool.k == 2 and pool.s == 2 and pool.padding == "SAME"):
            return False
        pad = 2 if spec.padding == "SAME" else 0
        return kernels().convpool_supported(C, Fk.pad8(spec.cout), 5, pad, H, W) >= 0

    def __init__(self, spec: Conv, pool: MaxPool, x: torch.Tensor, first: bool, fp: FlatParams, B: int, dev,
                 need_dx: bool):
        self.spec, self.pool, self.name, self.x, self.first, self.fp = spec, pool, spec.name, x, first, fp
        _, self.H, self.W, self.C = x.shape
        self.pad = 2 if spec.padding == "SAME" else 0
        self.Cp = Fk.pad8(spec.cout)
        self.cfg = kernels().convpool_supported(self.C, self.Cp, 5, self.pad, self.H, self.W)
        OH, OW = Fk.conv_out_hw(self.H, self.W, 5, 5, spec.padding)
        self.PH, self.PW = OH // 2, OW // 2
        self.out = _bf16(B, self.PH, self.PW, self.Cp, device=dev)
        # argmax codes: one byte per channel, or (LeNet conv1) 4 bits each
        ab = kernels().convpool_arg_bytes(self.C, self.Cp, 5, self.pad, self.H, self.W)
        self.arg = torch.zeros(B, self.PH, self.PW, ab, dtype=torch.uint8, device=dev)
        self.wname, self.bname = f"{spec.name}/weights", f"{spec.name}/biases"
        self.KM = kernels().convpool_rows(self.C, self.Cp, 5, self.pad, self.H, self.W)
        self.red = kernels().convpool_reduce_args(*self._geo(), spec.cin)   # (G, Ipad, I, bias_row)
        # one resident wave of wgrad workgroups (occupancy query; 1024 without a GPU)
        self.grid = kernels().convpool_wgrad_grid(*self._geo()) if dev.type == "cuda" else 1024
        self.slab_elems = self.grid * self.KM * self.Cp
        self.can_dgrad = kernels().convpool_has_dgrad(*self._geo())
        if need_dx and not self.can_dgrad:
            raise ValueError(f"{spec.name}: fused dgrad not available for this geometry")

    def _geo(self):
        return (self.C, self.Cp, 5, self.pad, self.H, self.W)

    # first layer only: read a resident dataset (uint8, or bf16 normalised once)
    # through the batch index (fused K10): (images [n, H*W], idx [B])
    u8: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
    use_u8 = False

    def _src(self) -> dict:
        if self.u8 is None or not self.use_u8:
            return {}
        if self.u8[0].dtype == torch.uint8:
            return {"u8": self.u8[0], "idx": self.u8[1]}
        return {"idx": self.u8[1]}          # x is the bf16 dataset (_xin)

    def _xin(self) -> torch.Tensor:
        """The kernels' x argument: the input buffer, or the bf16 dataset it gathers from."""
        if self.u8 is not None and self.use_u8 and self.u8[0].dtype == torch.bfloat16:
            return self.u8[0]
        return self.x

    # (LRN spec, LRN output): the following LRN is written by this layer's forward launch
    # (reference CNN conv1 -> norm1, lenet_band.hip refc1n_fwd_k; HipNet.fold_lrn_fwd1)
    lrn_out: Optional[tuple] = None

    def fwd(self, nb: int) -> None:
        lrn = {}
        if self.lrn_out is not None:
            ls, out = self.lrn_out
            lrn = dict(lrn_out=out, lrn_bias=ls.bias, lrn_alpha=ls.alpha, lrn_beta=ls.beta, lrn_r=ls.depth_radius)
        kernels().convpool_fwd(self._xin(), self.fp.bf16_view(self.wname), self.fp.param_view(self.bname),
                               self.spec.cout, self.out, self.arg, nb, *self._geo(), **self._src(), **lrn)

    skip_dgrad = False

    # (LRN spec, dL/d(LRN output)): the following LRN's backward is applied inside this
    # layer's weight-gradient staging (reference CNN norm1, HipNet.fold_lrn)
    lrn_fold: Optional[tuple] = None

    def _refc1(self, ls) -> bool:
        """The reference CNN's conv1 (28x28x1 or x3 -> 32, SAME) under norm1 (radius 4, beta
        0.75): refc1_wgrad replaces the folded convpool_wgrad (MNISTX_REFC1_WGRAD=0 keeps the
        latter).  3 channels (the reference's DLI records): bf16 input only (the batch, or the
        resident dataset through the batch index)."""
        if self.C == 3 and "u8" in self._src():
            return False
        return (self.C in (1, 3) and self.Cp == 32 and self.spec.cout == 32 and self.pad == 2
                and self.H == self.W == 28 and ls.depth_radius == 4 and float(ls.beta) == 0.75
                and os.environ.get("MNISTX_REFC1_WGRAD", "1") != "0")

    def bwd_weight(self, nb: int, dy: torch.Tensor, slab: torch.Tensor, red: Optional[list] = None) -> None:
        K = kernels()
        if self.lrn_fold is not None and self._refc1(self.lrn_fold[0]):
            # reference conv1 + norm1: the MFMA pool-phase kernel (refc1_wgrad.hip), same slab layout
            ls, dn = self.lrn_fold
            grid = min(self.grid, K.refc1_wgrad_blocks(nb))
            K.refc1_wgrad(self._xin(), dn, self.out, self.arg, slab, grid, nb, ls.bias, ls.alpha, ls.beta,
                          **self._src(), cin=self.C)
        elif self.lrn_fold is not None:
            ls, dn = self.lrn_fold
            grid = min(self.grid, max(1, (nb + 3) // 4))
            K.convpool_wgrad(self._xin(), dn, self.arg, slab, grid, nb, *self._geo(), **self._src(), lrn_p=self.out,
                             lrn_bias=ls.bias, lrn_alpha=ls.alpha, lrn_beta=ls.beta, lrn_r=ls.depth_radius)
        else:
            grid = min(self.grid, max(1, (nb + 3) // 4))
            K.convpool_wgrad(self._xin(), dy, self.arg, slab, grid, nb, *self._geo(), **self._src())
        G, Ip, I, brow = self.red
        _reduce(red, slab, (grid, self.KM, self.Cp, G, Ip, I, self.spec.cout, brow),
                self.fp.grad_view(self.wname), self.fp.grad_view(self.bname))

    dgrad_cap = 0   # persistent dgrad blocks (0: one resident wave); set when backward overlaps

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None:
        if dx is not None and not self.skip_dgrad:
            kernels().convpool_dgrad(dy, self.arg, self.fp.bf16_view(self.wname), dx, nb, *self._geo(),
                                     grid_cap=self.dgrad_cap)


class PoolLayer(_Layer):
    def __init__(self, spec: MaxPool, x: torch.Tensor, in_relu: bool, B: int, dev):
        assert spec.k == 2 and spec.s == 2 and spec.padding == "SAME", "2x2/2 SAME pooling only"
        self.spec, self.name, self.x, self.in_relu = spec, spec.name, x, in_relu
        _, self.H, self.W, self.C = x.shape
        self.OH, self.OW = (self.H + 1) // 2, (self.W + 1) // 2
        self.out = _bf16(B, self.OH, self.OW, self.C, device=dev)
        self.arg = torch.zeros(B, self.OH, self.OW, self.C, dtype=torch.uint8, device=dev)

    def fwd(self, nb: int) -> None:
        kernels().maxpool_fwd(self.x, self.out, self.arg, nb, self.H, self.W, self.C, self.OH, self.OW)

    def bwd_data(self, nb: int, dy, dx) -> None:
        if dx is not None:
            kernels().maxpool_bwd(dy, self.arg, self.out, self.in_relu, dx, nb, self.H, self.W, self.C, self.OH,
                                  self.OW)


class LRNLayer(_Layer):
    def __init__(self, spec: LRN, x: torch.Tensor, in_relu: bool, B: int, dev):
        self.spec, self.name, self.x, self.in_relu = spec, spec.name, x, in_relu
        self.C = x.shape[-1]
        self.out = torch.zeros_like(x)

    def _p(self, nb):
        return nb * (self.x[0].numel() // self.C)

    skip_fwd = False   # the following conv applies this LRN while staging (HipNet.fold_lrn_fwd)

    def fwd(self, nb: int) -> None:
        if self.skip_fwd:
            return
        s = self.spec
        kernels().lrn_fwd(self.x, self.out, self._p(nb), self.C, s.depth_radius, s.bias, s.alpha, s.beta)

    def bwd_data(self, nb: int, dy, dx) -> None:
        if dx is not None and not self.skip_bwd:
            s = self.spec
            kernels().lrn_bwd(self.x, dy, dx, self._p(nb), self.C, s.depth_radius, s.bias, s.alpha, s.beta,
                              self.in_relu)

    skip_bwd = False   # the preceding conv+pool layer applies this LRN's backward (HipNet.fold_lrn)


class LRNPoolLayer(_Layer):
    """LRN followed by a 2x2/2 SAME max-pool as ONE kernel each way (misc.hip
    lrn_pool_fwd_k / lrn_pool_bwd_k): the reference CNN's norm2 -> pool2
    (mnist_input.py:168-172).  The full-resolution LRN output and its gradient are
    never materialised; results are bitwise those of LRNLayer + PoolLayer."""

    @staticmethod
    def supported(lrn: LRN, pool: MaxPool, x_shape) -> bool:
        _, H, W, C = x_shape
        return (pool.k == 2 and pool.s == 2 and pool.padding == "SAME"
                and kernels().lrn_pool_supported(H, W, C, lrn.depth_radius))

    def __init__(self, lrn: LRN, pool: MaxPool, x: torch.Tensor, in_relu: bool, B: int, dev):
        self.spec, self.pool, self.name, self.x, self.in_relu = lrn, pool, pool.name, x, in_relu
        _, self.H, self.W, self.C = x.shape
        self.out = _bf16(B, self.H // 2, self.W // 2, self.C, device=dev)
        self.arg = torch.zeros(B, self.H // 2, self.W // 2, self.C, dtype=torch.uint8, device=dev)

    def fwd(self, nb: int) -> None:
        s = self.spec
        kernels().lrn_pool_fwd(self.x, self.out, self.arg, nb, self.H, self.W, self.C, s.depth_radius, s.bias,
                               s.alpha, s.beta, nonneg=self.in_relu)   # post-ReLU input: the packed kernel

    def bwd_data(self, nb: int, dy, dx) -> None:
        if dx is not None:
            s = self.spec
            kernels().lrn_pool_bwd(self.x, dy, self.arg, dx, nb, self.H, self.W, self.C, s.depth_radius, s.bias,
                                   s.alpha, s.beta, self.in_relu)


class DenseLayer(_Layer):
    has_params = True

    def __init__(self, spec: Dense, x: torch.Tensor, in_relu: bool, first: bool, last: bool, fp: FlatParams, B: int,
                 dev):
        self.spec, self.name, self.in_relu, self.first, self.last, self.fp = spec, spec.name, in_relu, first, last, fp
        self.x = x.view(B, -1)
        self.Dp = self.x.shape[1]
        self.Np = Fk.pad8(spec.dout) if not last else max(16, Fk.pad8(spec.dout))
        self.out = torch.zeros(B, self.Np, dtype=torch.float32 if last else torch.bfloat16, device=dev)
        self.wname, self.bname = f"{spec.name}/weights", f"{spec.name}/biases"
        self.M_wg = self.Dp + 1
        # slab sized for the larger of the standalone and the grouped (64x64-tile) split
        self.splits = max(Fk.pick_splits(self.M_wg, self.Np, B, dense=True),
                          Fk.pick_splits(self.M_wg, self.Np, B, dense=True, grouped=True))
        self.slab_elems = self.splits * self.M_wg * self.Np

    def fwd(self, nb: int) -> None:
        s = self.spec
        kernels().dense_fwd(self.x, self.fp.bf16_view(self.wname), self.out, nb, self.Np, self.Dp, self.Dp, self.Np,
                            self.Np, self.fp.param_view(self.bname), s.dout, s.relu, None, 0)

    def bwd_weight(self, nb: int, dy: torch.Tensor, slab: torch.Tensor, red: Optional[list] = None) -> None:
        K = kernels()
        dy2 = dy.view(-1, self.Np)
        S = K.dense_wgrad(self.x, dy2, slab, self.Dp, self.Np, nb, self.Dp, self.Np, True,
                          Fk.pick_splits(self.M_wg, self.Np, nb, dense=True))
        self.reduce_wgrad(S, slab, red)

    # (per-block fp32 dlogits column sums [blocks, Np], blocks): set by the softmax-CE /
    # fused-head launch of the step; the last layer's bias gradient is their sum instead of
    # the bias row of the bf16-dlogits GEMM (the reference computes it in tf.float32,
    # mnist_input.py:203-205,224-226)
    ce_bias: Optional[Tuple[torch.Tensor, int]] = None

    def reduce_wgrad(self, S: int, slab: torch.Tensor, red: Optional[list] = None) -> None:
        """Queue (or run) the split-K reduce of an S-split weight-gradient slab."""
        s = self.spec
        bgrad = self.fp.grad_view(self.bname)
        cb = self.ce_bias
        _reduce(red, slab, (S, self.M_wg, self.Np, 1, self.Dp, s.din, s.dout, self.Dp),
                self.fp.grad_view(self.wname), bgrad if cb is None else bgrad[:0])
        if cb is not None:
            # bias only (G = 0): sum of the CE kernel's block partials, rows = blocks
            _reduce(red, cb[0], (cb[1], 1, self.Np, 0, 1, 0, s.dout, 0), bgrad[:0], bgrad)
            self.ce_bias = None

    def bwd_data(self, nb: int, dy: torch.Tensor, dx: Optional[torch.Tensor]) -> None:
        if dx is not None:
            dy2 = dy.view(-1, self.Np)
            kernels().dense_dgrad(dy2, self.fp.bf16_view(self.wname), dx.view(-1, self.Dp), nb, self.Dp, self.Np,
                                  self.Np, self.Np, self.Dp, self.x if self.in_relu else None, self.Dp)


def _weight_pads(spec: ModelSpec) -> Dict[str, Tuple[int, int]]:
    """(I_pad, J_pad) of every weight's bf16 copy, following activation padding."""
    pads: Dict[str, Tuple[int, int]] = {}
    c = spec.in_channels
    flat: Optional[int] = None
    layers = spec.layers
    for i, L in enumerate(layers):
        if isinstance(L, Conv):
            cout_p = Fk.pad8(L.cout)
            pads[f"{L.name}/weights"] = (c, cout_p)
            c = cout_p
        elif isinstance(L, Dense):
            din_p = flat if flat is not None else None
            if din_p is None:
                din_p = L.din  # flatten of a spatial map (channels must be unpadded)
            last = i == len(layers) - 1
            dout_p = max(16, Fk.pad8(L.dout)) if last else Fk.pad8(L.dout)
            pads[f"{L.name}/weights"] = (din_p, dout_p)
            flat = dout_p
    return pads


class HipNet:
    """One model replica on one GPU: buffers + kernels for fwd / bwd / update."""

    # head blocks whose CE partials the next finalize combines (deferred statistics;
    # class default so subclasses with their own heads, e.g. HipNetF32, never defer)
    _ce_defer_blocks = 0

    def __init__(self, spec: ModelSpec, batch: int, device, init: Dict[str, torch.Tensor],
                 opt: Optional[OptConfig] = None, fuse_convpool: bool = True, overlap_backward: bool = False,
                 fuse_head: bool = True, fuse_lrnpool: Optional[bool] = None, fused_lenet_bwd: bool = True,
                 fold_lrn_fwd: bool = False):
        dev = torch.device(device)
        if fuse_lrnpool is None:
            fuse_lrnpool = os.environ.get("MNISTX_FUSE_LRNPOOL", "1") != "0"
        self.spec, self.B, self.device = spec, batch, dev
        self.opt = opt or OptConfig()
        pads = _weight_pads(spec)
        specs = []
        for L in spec.weights():
            shp = (L.kh, L.kw, L.cin, L.cout) if isinstance(L, Conv) else (L.din, L.dout)
            specs.append((f"{L.name}/weights", shp, L.wd))
            specs.append((f"{L.name}/biases", (L.cout if isinstance(L, Conv) else L.dout,), None))
        self.fp = FlatParams.build(specs, init, dev, pads)
        H, W = spec.input_hw
        self.x0 = _bf16(batch, H, W, spec.in_channels, device=dev)
        self.labels = torch.zeros(batch, dtype=torch.int32, device=dev)
        self.layers: List[_Layer] = []
        x, in_relu = self.x0, False
        n = len(spec.layers)
        i = 0
        while i < n:
            L = spec.layers[i]
            nxt = spec.layers[i + 1] if i + 1 < n else None
            if (fuse_convpool and isinstance(L, Conv) and isinstance(nxt, MaxPool) and not in_relu
                    and ConvPoolLayer.supported(L, nxt, x.shape)):
                # the fused dgrad exists only for interior layers whose geometry has it
                lay = ConvPoolLayer(L, nxt, x, i == 0, self.fp, batch, dev, need_dx=False)
                if i > 0 and not lay.can_dgrad:
                    lay = None
                if lay is not None:
                    lay.idx = i
                    self.layers.append(lay)
                    x, in_relu = lay.out, False
                    i += 2
                    continue
            if (fuse_lrnpool and dev.type == "cuda" and isinstance(L, LRN) and isinstance(nxt, MaxPool)
                    and LRNPoolLayer.supported(L, nxt, x.shape)):
                lay = LRNPoolLayer(L, nxt, x, in_relu, batch, dev)
                lay.idx = i
                self.layers.append(lay)
                x, in_relu = lay.out, False
                i += 2
                continue
            if isinstance(L, Conv):
                lay = ConvLayer(L, x, in_relu, i == 0, self.fp, batch, dev)
                in_relu = L.relu
            elif isinstance(L, MaxPool):
                lay = PoolLayer(L, x, in_relu, batch, dev)
                in_relu = False
            elif isinstance(L, LRN):
                lay = LRNLayer(L, x, in_relu, batch, dev)
                in_relu = False
            elif isinstance(L, Dense):
                if x.dim() == 4:  # NHWC flatten (mnist_input.py:177-180); padded channels would break it
                    assert x[0].numel() == L.din, f"{L.name}: flatten {x[0].numel()} != din {L.din}"
                lay = DenseLayer(L, x, in_relu, i == 0, i == n - 1, self.fp, batch, dev)
                in_relu = L.relu
            else:
                raise TypeError(L)
            lay.idx = i
            self.layers.append(lay)
            x = lay.out
            i += 1
        assert isinstance(self.layers[-1], DenseLayer) and self.layers[-1].last, "model must end in a Dense"
        self.logits = self.layers[-1].out
        self.n_classes = spec.num_classes
        self.dlogits = _bf16(batch, self.logits.shape[1], device=dev)
        # per-block fp32 column sums of dlogits (the last layer's bias gradient, DenseLayer.ce_bias)
        self.ce_dbias = torch.zeros(1024 * 32, dtype=torch.float32, device=dev)
        # overlap_backward: every weight gradient (+ its split-K reduce) runs on a side
        # stream, concurrently with the data-gradient chain on the main stream (one
        # input-gradient buffer and one slab region per layer, so the streams never share
        # scratch).  Off by default: at B=65536 every kernel already fills the 256 CUs and
        # concurrent kernels only time-slice (profiles/r1_overlap/); the serial plan is the
        # same code with one slab.
        # overlap_backward="dense": only the dense weight gradients (latency-bound split-K
        # GEMMs with little work per CU) fork to the side stream, beside the conv backward
        # (measured 4 % SLOWER at B=65536 too: profiles/r1s2/ab_overlap_dense.txt).
        self.overlap_dense_only = overlap_backward == "dense"
        self.overlap = bool(overlap_backward) and dev.type == "cuda"
        # serial plan: every layer's split-K reduce is queued and flushed as ONE
        # multi-tensor launch per gradient bucket (``hook_layers``), so the layers
        # need disjoint slab regions, as with overlap
        self.defer_reduce = not self.overlap or self.overlap_dense_only
        self.dbuf: List[Optional[torch.Tensor]] = [None] + [torch.zeros_like(l.out, dtype=torch.bfloat16)
                                                           for l in self.layers[:-1]]
        sizes = [(getattr(l, "slab_elems", 0) + 3) // 4 * 4 for l in self.layers]
        disjoint = self.overlap or self.defer_reduce
        self.slab = torch.zeros(max(1, sum(sizes) if disjoint else max(sizes)), dtype=torch.float32, device=dev)
        self.slabs, off = [], 0
        for n in sizes:
            self.slabs.append(self.slab[off:off + n] if n else self.slab[:1])
            off += n if disjoint else 0
        if self.overlap:
            self.side = torch.cuda.Stream(device=dev)
            self.ev_dy = [torch.cuda.Event() for _ in self.layers]
            # (Co-residency budgets for the concurrent persistent conv kernels were all SLOWER
            # than the serial plan: profiles/r1s3/overlap_budget.txt -- the conv kernels are
            # LDS/issue-bound on the same units, so sharing a CU adds no throughput.)
        self.stats = torch.zeros(8, dtype=torch.float32, device=dev)
        self.eval_stats = torch.zeros(8, dtype=torch.float32, device=dev)
        # softmax-CE per-block partials + ticket: deterministic loss / accuracy sums
        self.ce_work = torch.zeros(4 * 1024 + 1, dtype=torch.float32, device=dev)
        names = [e.name for e in self.fp.wd_entries]
        self.loss_names = [n.replace("/weights", "/weight_loss") for n in names] + ["cross_entropy", "total_loss"]
        self.loss_ema = torch.zeros(3 * len(self.loss_names), dtype=torch.float32, device=dev)
        self.grad_ready_hooks: List[Callable[[int], None]] = []
        # layers after whose weight gradient the hooks need reduced gradients (e.g. the
        # DP bucket triggers); None = every layer
        self.hook_layers: Optional[set] = None
        self.idx_buf: Optional[torch.Tensor] = None
        # fused dense head (mlp_head.hip): index of its first layer, or None
        self.head: Optional[int] = self._find_head() if (fuse_head and dev.type == "cuda") else None
        # "mlp" (LeNet-5's three-layer head) or "tail" (the reference CNN's softmax_linear +
        # softmax-CE + its masked data gradient as one launch, mlp_head.hip ce_tail_k;
        # MNISTX_CE_TAIL=0 keeps the GEMM + softmax_ce + dgrad launches)
        self.head_kind = "mlp" if self.head is not None else None
        if self.head is None and fuse_head and dev.type == "cuda" and os.environ.get("MNISTX_CE_TAIL", "1") != "0":
            self.head = self._find_tail()
            self.head_kind = "tail" if self.head is not None else None
        self._head_pending: Optional[int] = None   # nb of a deferred head (forward(defer_head=True))
        # the head's fc3/fc4/fc5 weight gradients as one grouped launch (gemm.hip
        # dense_wgrad_group)
        self.group_head_wgrad = (self.head_kind == "mlp"
                                 and all(l.Dp % 8 == 0 and l.Np % 8 == 0 for l in self.layers[self.head:]))
        self._group_S: Optional[list] = None
        self._head_grads = False                   # loss_and_grad already produced the head's dgrads
        # reference CNN: norm1's backward runs in conv1's weight-gradient staging (reads
        # dL/d norm1 + pool1, no pool-level gradient in HBM, no lrn_bwd launch)
        self.fold_lrn = False
        if dev.type == "cuda" and not self.overlap and os.environ.get("MNISTX_FOLD_LRN", "1") != "0":
            for k in range(len(self.layers) - 1):
                a, b = self.layers[k], self.layers[k + 1]
                if (isinstance(a, ConvPoolLayer) and a.cfg in (2, 3) and isinstance(b, LRNLayer) and b.x is a.out
                        and b.spec.depth_radius == 4 and b.C == 32 and k == 0):
                    a.lrn_fold = (b.spec, self.dbuf[k + 2])   # dL/d(LRN output) = the LRN's incoming gradient
                    b.skip_bwd = True
                    self.fold_lrn = True
        # reference CNN: norm1's forward written by conv1's forward launch from its pooled
        # registers (refc1n_fwd_k: no lrn_fwd_k pass over pool1); MNISTX_FOLD_LRN_FWD1=0 keeps
        # the separate LRN launch
        self.fold_lrn_fwd1 = False
        if dev.type == "cuda" and not fold_lrn_fwd and os.environ.get("MNISTX_FOLD_LRN_FWD1", "1") != "0":
            for k in range(len(self.layers) - 1):
                a, b = self.layers[k], self.layers[k + 1]
                if (k == 0 and isinstance(a, ConvPoolLayer) and isinstance(b, LRNLayer) and b.x is a.out
                        and b.spec.depth_radius == 4 and b.C == 32
                        and kernels().convpool_fwd_lrn_ok(*a._geo())):
                    a.lrn_out = (b.spec, b.out)
                    b.skip_fwd = True
                    self.fold_lrn_fwd1 = True
        # reference CNN: norm1's forward in conv2's input staging (LDS-halo fwd and weight-
        # gradient kernels read pool1 and normalise it; norm1 never written).  Opt-in
        # (fold_lrn_fwd=True): the LRN math in both staging loops costs more than the 67 us
        # lrn_fwd launch it removes (2.25-2.28 vs 2.22-2.24 ms/step, profiles/r2/README.md)
        self.fold_lrn_fwd = False
        if dev.type == "cuda" and fold_lrn_fwd and os.environ.get("MNISTX_CONV_HALO", "1") != "0":
            for k in range(len(self.layers) - 1):
                a, b = self.layers[k], self.layers[k + 1]
                if (isinstance(a, LRNLayer) and isinstance(b, ConvLayer) and b.x is a.out and a.C == 32
                        and a.spec.depth_radius == 4 and not a.in_relu and (b.H, b.W, b.C) == (14, 14, 32)
                        and (b.spec.kh, b.spec.kw, b.spec.padding) == (5, 5, "SAME") and b.Cp % 32 == 0):
                    b.lrn_pre = (a.spec, a.x)
                    a.skip_fwd = True
                    self.fold_lrn_fwd = True
        # LeNet-5: conv1+pool1+conv2+pool2 forward as ONE banded-MFMA kernel (lenet_band.hip)
        # on x0 or the resident dataset (bf16, or uint8 normalised while staging);
        # MNISTX_BAND_FWD=0 runs the two convpool kernels instead
        self.band_fwd = self._find_c2d_c1w() and os.environ.get("MNISTX_BAND_FWD", "1") != "0"
        # LeNet-5: the conv stack's whole backward (conv2 dgrad + both weight gradients) as ONE
        # kernel (lenet_bwd.hip): dP1 stays in LDS, the weight gradients accumulate in
        # registers per block; fused_lenet_bwd=False runs the three convpool kernels
        self.fused_bwd = self.band_fwd and fused_lenet_bwd and not self.overlap
        self.bwd_u8: Optional[torch.Tensor] = None    # uint8 twin of a bound bf16 dataset (bind_u8_input)
        if self.fused_bwd:
            res = kernels().lenet_bwd_blocks(batch)
            self.lb_grid = res          # the slabs' partial count: per-step grids never exceed it
            self.lb_slab1 = torch.zeros(res * 32 * 8, dtype=torch.float32, device=dev)
            self.lb_slab2 = torch.zeros(res * 208 * 16, dtype=torch.float32, device=dev)

    @property
    def bucket_lockout(self) -> set:
        """Spec indices of the layers after whose grad-ready hook the next backward kernel is a
        persistent one-resident-wave kernel that takes every CU (measured: a collective-sized
        probe on another stream does not start until it retires, bench/dp_coresidency.py,
        profiles/r5/dp_coresidency/).  parallel/dp.plan_buckets never closes a bucket there.
          * fused head + fused LeNet conv backward: the head already produced every data
            gradient, so fc3's hook is followed directly by lenet_bwd_k;
          * an interior conv layer: its data gradient (conv5_halo dgrad / convpool_dgrad)."""
        out = set()
        if self.head is not None and self.fused_bwd:
            out.add(self.layers[self.head].idx)
        for lay in self.layers[1:]:
            if isinstance(lay, (ConvLayer, ConvPoolLayer)):
                out.add(lay.idx)
        return out

    def _find_c2d_c1w(self) -> bool:
        if self.device.type != "cuda" or len(self.layers) < 2:
            return False
        l0, l1 = self.layers[0], self.layers[1]
        return (isinstance(l0, ConvPoolLayer) and isinstance(l1, ConvPoolLayer) and l0.cfg == 0 and l1.cfg == 1
                and l1.x is l0.out)

    def _find_head(self) -> Optional[int]:
        """LeNet-5's fc3 -> fc4 -> fc5 tail (400 -> 120 -> 84 -> 10 with ReLUs on the
        hidden layers) runs as ONE kernel with softmax-CE and its data gradients."""
        if len(self.layers) < 4:
            return None
        i = len(self.layers) - 3
        l3, l4, l5 = self.layers[i:]
        if not all(isinstance(l, DenseLayer) for l in (l3, l4, l5)):
            return None
        dims = (l3.Dp, l3.Np, l4.Dp, l4.Np, l5.Dp, l5.Np)
        if dims != (400, 120, 120, 88, 88, 16) or l3.in_relu or not (l3.spec.relu and l4.spec.relu) or l5.spec.relu:
            return None
        if not kernels().mlp_head_supported(400, 120, 88, 16, l3.spec.dout, l4.spec.dout, l5.spec.dout, self.B):
            return None
        # the kernel stages transposed, tile-padded weight copies (W^T rows = output units)
        self.fp.enable_transposed({l3.wname: (128, 416), l4.wname: (96, 128), l5.wname: (16, 96)})
        return i

    def _find_tail(self) -> Optional[int]:
        """The reference CNN's softmax_linear (192 -> 10, no ReLU, on local4's ReLU output,
        mnist_input.py:195-203) + softmax-CE (+ dL/d local4, masked by local4 > 0) as ONE
        kernel (mlp_head.hip ce_tail_k)."""
        if len(self.layers) < 2:
            return None
        i = len(self.layers) - 1
        l5 = self.layers[i]
        if not (isinstance(l5, DenseLayer) and (l5.Dp, l5.Np) == (192, 16) and l5.in_relu and not l5.spec.relu
                and l5.spec.din == 192):
            return None
        if not kernels().ce_tail_supported(192, l5.spec.dout, self.B):
            return None
        self.fp.enable_transposed({l5.wname: (16, 192)})
        return i

    def _run_head(self, nb: int, scale: float, grads: bool, stats: torch.Tensor) -> None:
        i = self.head
        # training statistics: the per-block CE partials are combined by this step's
        # finalize_k (no agent-scope fence / ticket inside the head; ce_stats.h)
        defer = grads and stats is self.stats and self.ce_work is not None
        if self.head_kind == "tail":
            l5 = self.layers[i]
            K = kernels()
            K.ce_tail(l5.x, self.fp.bf16t_view(l5.wname), self.fp.param_view(l5.bname), l5.spec.dout, self.labels,
                      nb, scale, l5.out, dl=self.dlogits if grads else None, dx=self.dbuf[i] if grads else None,
                      stats=stats, work=self.ce_work, defer_stats=defer, dbias=self.ce_dbias if grads else None)
            if grads:
                l5.ce_bias = (self.ce_dbias, K.ce_tail_blocks(nb))
            if defer:
                self._ce_defer_blocks = K.ce_tail_blocks(nb)
            return
        l3, l4, l5 = self.layers[i:]
        fp = self.fp
        kernels().mlp_head(l3.x, fp.bf16t_view(l3.wname), fp.param_view(l3.bname), l3.spec.dout,
                           fp.bf16t_view(l4.wname), fp.param_view(l4.bname), l4.spec.dout,
                           fp.bf16t_view(l5.wname), fp.param_view(l5.bname), l5.spec.dout,
                           self.labels, nb, scale, l3.out, l4.out, l5.out,
                           dl=self.dlogits if grads else None, dh4=self.dbuf[i + 2] if grads else None,
                           dh3=self.dbuf[i + 1] if grads else None, dx=self.dbuf[i] if grads else None,
                           stats=stats, work=self.ce_work, defer_stats=defer,
                           dbias=self.ce_dbias if grads else None)
        if grads:
            l5.ce_bias = (self.ce_dbias, kernels().mlp_head_blocks(nb))
        if defer:
            self._ce_defer_blocks = kernels().mlp_head_blocks(nb)

    def can_gather_input(self) -> bool:
        """Whether ``bind_u8_input`` would accept a resident dataset (checked BEFORE the
        caller builds a normalised bf16 copy of it)."""
        first = self.layers[0]
        return (isinstance(first, ConvPoolLayer) and self.spec.in_channels in (1, 3)
                and bool(kernels().convpool_u8_input(*first._geo())))

    def bind_u8_input(self, images: torch.Tensor, bwd_images: Optional[torch.Tensor] = None) -> bool:
        """Training steps read a resident dataset [n, H*W] directly through ``idx_buf``
        (filled by DeviceLoader(idx_out=...)), fusing the gather (K10,
        mnist_input.py:37-39) into the first fused conv's staging -- its forward and
        its weight gradient -- so no normalised batch is written and re-read:
          * uint8: normalised x/255 - 0.5 inside the kernels;
          * bf16: the dataset normalised ONCE (DeviceDataset.bf16_images, bitwise the
            per-step prep) -- 2x the uint8 footprint (94 MB for MNIST, nothing next
            to 288 GB of HBM) for no per-step conversion work.
        Eval / inference keep using ``x0``.  Returns False when the first layer
        cannot (Cin != 1 etc.).  ``bwd_images``: the same rows as uint8, read by the fused
        LeNet-5 conv backward when ``images`` is the bf16 copy (half the input bytes; its
        in-kernel normalisation is bitwise the bf16 copy's, tests/test_lenet_bwd_gpu.py)."""
        first = self.layers[0]
        H, W = self.spec.input_hw
        C = self.spec.in_channels
        # 3 channels (the reference CNN on its 3-channel records): the bf16 dataset only -- the
        # conv1 weight gradient (refc1_wgrad) gathers bf16 NHWC rows
        if not (isinstance(first, ConvPoolLayer) and C in (1, 3)
                and images.dtype in ((torch.uint8, torch.bfloat16) if C == 1 else (torch.bfloat16,))
                and images.dim() == 2 and images.shape[1] == H * W * C and images.device == self.device
                and kernels().convpool_u8_input(*first._geo())):
            return False
        self.idx_buf = torch.zeros(self.B, dtype=torch.int64, device=self.device)
        first.u8 = (images.contiguous(), self.idx_buf)
        ok_bwd = (self.fused_bwd and bwd_images is not None and images.dtype == torch.bfloat16
                  and bwd_images.dtype == torch.uint8
                  and tuple(bwd_images.shape) == tuple(images.shape) and bwd_images.device == self.device)
        self.bwd_u8 = bwd_images.contiguous() if ok_bwd else None
        return True

    # ------------------------------------------------------------------ step parts
    def forward(self, nb: Optional[int] = None, from_x0: bool = False, defer_head: bool = False) -> torch.Tensor:
        """Training forward reads the bound uint8 source when there is one;
        ``from_x0`` forces the bf16 ``x0`` buffer (eval / inference / tests).
        ``defer_head``: a fused dense head is left to ``loss_and_grad`` (which then
        runs head forward + softmax-CE + head data gradients as one kernel), so the
        logits are only valid after it."""
        nb = self.B if nb is None else nb
        first = self.layers[0]
        if isinstance(first, ConvPoolLayer):
            first.use_u8 = first.u8 is not None and not from_x0
        stop = self.head if (defer_head and self.head is not None) else len(self.layers)
        start = 0
        if self.band_fwd and stop >= 2:
            self._band_forward(nb)
            start = 2
        for lay in self.layers[start:stop]:
            lay.fwd(nb)
        self._head_pending = nb if stop < len(self.layers) else None
        return self.logits

    def _band_forward(self, nb: int) -> None:
        """conv1 -> pool1 -> conv2 -> pool2 in one launch; writes both layers' pooled
        outputs and argmax codes in the convpool layouts the backward kernels read."""
        l0, l1 = self.layers[0], self.layers[1]
        fp = self.fp
        src = l0._src()   # {} (x0) | {"idx"} (bf16 dataset = _xin()) | {"u8", "idx"} (uint8 dataset)
        # for the fused backward: ONE 16-byte record per pool1 window (channels 0-5 + the code
        # word, lenet_band.hip P1OUT 2) in l0.out; the unfused backward reads the convpool layouts
        kernels().lenet_band_fwd(src.get("u8", l0._xin()), fp.bf16_view(l0.wname), fp.param_view(l0.bname), l0.spec.cout,
                                 fp.bf16_view(l1.wname), fp.param_view(l1.bname), nb, l1.out, l1.arg,
                                 p1=l0.out, arg1=None if self.fused_bwd else l0.arg, idx=src.get("idx"))

    def _fused_conv_backward(self, nb: int, dp2: torch.Tensor, pending: list) -> None:
        """LeNet-5 conv1+conv2 backward in one launch (lenet_bwd.hip) reading the band
        forward's pool1 / argmax outputs and dL/d pool2; both layers' weight / bias gradients
        go to split-K slabs reduced with the other queued layers (``pending``)."""
        l0, l1 = self.layers[0], self.layers[1]
        fp = self.fp
        src = l0._src()
        K = kernels()
        grid = min(self.lb_grid, K.lenet_bwd_blocks(nb))   # less any CUs reserved for collectives
        x = src.get("u8", l0._xin())
        if self.bwd_u8 is not None and l0.use_u8 and "idx" in src:
            x = self.bwd_u8        # the uint8 copy of the bound bf16 dataset: half the bytes
        K.lenet_bwd(x, l0.out, dp2, l1.arg, fp.bf16_view(l1.wname), nb,
                    self.lb_slab1, self.lb_slab2, grid, idx=src.get("idx"))
        _reduce(pending, self.lb_slab2, (grid, 208, 16, 25, 8, l1.spec.cin, l1.spec.cout, 200),
                fp.grad_view(l1.wname), fp.grad_view(l1.bname))
        _reduce(pending, self.lb_slab1, (grid, 32, 8, 25, 1, 1, l0.spec.cout, 25),
                fp.grad_view(l0.wname), fp.grad_view(l0.bname))

    def loss_and_grad(self, nb: Optional[int] = None, scale: Optional[float] = None) -> None:
        nb = self.B if nb is None else nb
        if self._head_pending is not None:
            assert self._head_pending == nb, "loss_and_grad batch differs from the deferred forward"
            self._run_head(nb, (1.0 / nb) if scale is None else scale, True, self.stats)
            self._head_pending, self._head_grads = None, True
            return
        # training statistics deferred to this step's finalize_k, as for the fused head
        ld = self.logits.shape[1]
        nblk = kernels().softmax_ce_dbias_blocks(nb, ld)
        self._ce_defer_blocks = kernels().softmax_ce(
            self.logits, ld, self.labels, nb, self.n_classes,
            (1.0 / nb) if scale is None else scale, self.dlogits, ld, self.stats,
            None, self.ce_work, defer_stats=self.ce_work is not None,
            dbias=self.ce_dbias if nblk > 0 else None)
        self.layers[-1].ce_bias = (self.ce_dbias, nblk) if nblk > 0 else None

    def backward(self, nb: Optional[int] = None) -> None:
        """Data-gradient chain on the current stream; each layer's weight gradient
        forks to the side stream as soon as its dY exists (event), and grad-ready
        hooks (DP all-reduce launches) are issued from the side stream so RCCL
        waits on exactly that work.  Joins before returning."""
        nb = self.B if nb is None else nb
        dy = self.dlogits
        pending: list = []          # split-K reduces queued on the main stream
        side_pending: list = []     # ... and on the side stream
        main = torch.cuda.current_stream(self.device) if self.overlap else None
        if self.overlap:
            self.side.wait_stream(main)
        # fused head: its three weight gradients run as ONE grouped split-K launch
        self._group_S = None
        if self.group_head_wgrad and self._head_grads and self.defer_reduce and not self.overlap:
            # before the fused conv backward: launched after it instead (the conv backward then
            # reads the band forward's pool1 records with ~110 MB less traffic in between) the
            # step measured 11 us SLOWER same-box (profiles/r6/order/)
            hl = self.layers[self.head:]
            dys = [self.dbuf[self.head + 1], self.dbuf[self.head + 2], self.dlogits]
            self._group_S = kernels().dense_wgrad_group(
                [l.x for l in hl], [d.view(-1, l.Np) for d, l in zip(dys, hl)],
                [self.slabs[self.head + k] for k in range(3)], [l.Dp for l in hl], [l.Np for l in hl], nb,
                [Fk.pick_splits(l.M_wg, l.Np, nb, dense=True, grouped=True) for l in hl])
        for i in range(len(self.layers) - 1, -1, -1):
            lay = self.layers[i]
            dx = self.dbuf[i]
            if i == 1 and self.fused_bwd:
                self._fused_conv_backward(nb, dy, pending)
                for li in (self.layers[1].idx, self.layers[0].idx):
                    if self.grad_ready_hooks and (self.hook_layers is None or li in self.hook_layers):
                        self._flush_reduce(pending)
                        for h in self.grad_ready_hooks:
                            h(li)
                break
            if lay.has_params:
                # the first layer has no data gradient: its weight gradient IS the tail of
                # the critical path, so it runs on the main stream while the side drains
                if self.overlap and i > 0 and (not self.overlap_dense_only or isinstance(lay, DenseLayer)):
                    self.ev_dy[i].record(main)
                    self.side.wait_event(self.ev_dy[i])
                    with torch.cuda.stream(self.side):
                        lay.bwd_weight(nb, dy, self.slabs[i], side_pending)
                        if self.grad_ready_hooks and (self.hook_layers is None or lay.idx in self.hook_layers):
                            self._flush_reduce(side_pending)
                            for h in self.grad_ready_hooks:
                                h(lay.idx)
                elif self.defer_reduce and self._group_S is not None and i >= self.head:
                    lay.reduce_wgrad(self._group_S[i - self.head], self.slabs[i], pending)
                    if self.grad_ready_hooks and (self.hook_layers is None or lay.idx in self.hook_layers):
                        self._flush_reduce(pending)
                        for h in self.grad_ready_hooks:
                            h(lay.idx)
                elif self.defer_reduce:
                    lay.bwd_weight(nb, dy, self.slabs[i], pending)
                    if self.grad_ready_hooks and (self.hook_layers is None or lay.idx in self.hook_layers):
                        self._flush_reduce(pending)
                        for h in self.grad_ready_hooks:
                            h(lay.idx)
                else:
                    lay.bwd_weight(nb, dy, self.slabs[i])
                    for h in self.grad_ready_hooks:
                        h(lay.idx)
            if not (self._head_grads and i >= self.head):   # the fused head wrote these already
                lay.bwd_data(nb, dy, dx)
            dy = dx
        self._head_grads = False
        self._flush_reduce(pending)
        if self.overlap:
            with torch.cuda.stream(self.side):
                self._flush_reduce(side_pending)
            main.wait_stream(self.side)

    @staticmethod
    def _flush_reduce(pending: list) -> None:
        """One multi-tensor split-K reduce (one launch per pass) for the queued layers."""
        if not pending:
            return
        geo = torch.tensor([g for _, g, _, _ in pending], dtype=torch.int64)
        kernels().splitk_reduce_multi([p[0] for p in pending], [p[2] for p in pending],
                                      [p[3] for p in pending], geo, [1.0] * len(pending))
        pending.clear()

    def update(self, grad_scale: float = 1.0, increment: bool = True, batch_for_stats: Optional[int] = None) -> None:
        # the step's finalize rides on the optimizer launch (its last block runs it: one launch
        # fewer per step, misc.hip fused_opt_k; the launcher falls back to two launches)
        # and, when a loader offers it (next_input_job: DeviceLoader.lookahead_job), the next
        # batch's shuffle rows + labels run in extra blocks of the same launch
        job = self.next_input_job() if getattr(self, "next_input_job", None) is not None else None
        self.fp.apply(self.opt, grad_scale, fin=self._fin_args(batch_for_stats or self.B, increment), perm=job)

    def _fin_args(self, batch: int, increment: bool) -> tuple:
        """finalize_step's arguments after `step` (consumes the deferred CE block count)."""
        fp = self.fp
        nw = len(fp.wd_entries)
        nblk = getattr(self, "_ce_defer_blocks", 0)   # HipNetF32 borrows this method
        self._ce_defer_blocks = 0
        return (self.stats, fp.l2 if nw else None, fp.wds if nw else None, nw, self.loss_ema, len(self.loss_names),
                batch, increment, fp.l2_ranges if nw else None, self.ce_work if nblk else None, nblk)

    def finalize(self, batch: int, increment: bool = True) -> None:
        kernels().finalize_step(self.fp.step, *self._fin_args(batch, increment))

    def train_step(self, grad_scale: float = 1.0) -> None:
        self.forward(defer_head=True)
        self.loss_and_grad()
        self.backward()
        self.update(grad_scale)

    # ------------------------------------------------------------------ eval
    def eval_batch(self, nb: int, stats: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Forward only on x0[:nb] / labels[:nb]; accumulates loss/correct into stats."""
        st = self.eval_stats if stats is None else stats
        self.forward(nb, from_x0=True, defer_head=True)
        if self._head_pending is not None:
            self._run_head(nb, 1.0, False, st)
            self._head_pending = None
            return st
        kernels().softmax_ce(self.logits, self.logits.shape[1], self.labels, nb, self.n_classes, 1.0, None,
                             self.logits.shape[1], st, None, self.ce_work)
        return st

    def probs(self, nb: int) -> torch.Tensor:
        self.forward(nb, from_x0=True)
        return Fk.softmax_probs(self.logits[:nb], self.n_classes)

    # ------------------------------------------------------------------ introspection
    def activation(self, layer_name: str) -> torch.Tensor:
        for lay in self.layers:
            if lay.name == layer_name:
                return lay.out
        raise KeyError(layer_name)

    def layer_activation(self, layer_name: str, n: int) -> torch.Tensor:
        """The reference's ``<layer>/<layer>:0`` tensor (main.py:97-100) for the first
        ``n`` images of the current batch: a conv layer's bias+ReLU output BEFORE
        pooling.  A fused conv+pool layer never materialises it, so it is recomputed
        here with the unfused implicit-GEMM conv kernel (monitoring only, every
        ``test_interval`` steps).  Channel padding is kept; callers strip it."""
        for lay in self.layers:
            if lay.name != layer_name:
                continue
            n = max(1, min(n, self.B))
            if not isinstance(lay, ConvPoolLayer):
                return lay.out[:n]
            s = lay.spec
            OH, OW = Fk.conv_out_hw(lay.H, lay.W, s.kh, s.kw, s.padding)
            x = lay.x
            # decided by the binding, not by ``use_u8``: that flag belongs to the last EAGER
            # forward (an eval pass clears it) and hipGraph replays of the training step never
            # run the Python forward, so it can be stale while training still reads the dataset
            if lay.u8 is not None:
                # training reads a resident dataset through the batch index: those rows, normalised
                ds, idx = lay.u8
                rows = ds[idx[:n]]
                if rows.dtype == torch.uint8:
                    rows = (rows.float() / 255.0 - 0.5).to(torch.bfloat16)
                x = rows.view(n, lay.H, lay.W, lay.C)
            out = torch.empty(n, OH, OW, lay.Cp, dtype=torch.bfloat16, device=self.device)
            kernels().conv_fwd(x, self.fp.bf16_view(lay.wname), out, n, lay.H, lay.W, lay.C, OH, OW, s.kh, s.kw,
                               lay.pad, lay.pad, lay.Cp, self.fp.param_view(lay.bname), s.cout, True)
            return out
        raise KeyError(layer_name)

    def read_stats(self) -> Dict[str, float]:
        s = self.stats.detach().cpu().tolist()
        return {"cross_entropy": s[4], "accuracy": s[5], "total_loss": s[6], "nan": s[2]}
