"""Flat parameter / gradient / optimizer-slot buffers (device resident).

All trainable variables live in ONE contiguous fp32 buffer (and so do their
gradients, momentum slots and EMA shadows), laid out in the reference's
creation order (``mnist_input.py:137-205``).  This gives:

* one fused optimizer launch for every tensor (K9, ``csrc/kernels/misc.hip``):
  L2 weight decay, SGD / momentum / Nesterov, the staircase LR schedule
  (``mnist_input.py:252-256``, read from the device-side global step — no host
  sync, hipGraph capturable), the weight EMA with TF's
  ``min(decay, (1+t)/(10+t))`` (``mnist_input.py:265-267``), and the refresh of
  the zero-padded bf16 weight copies the GEMM kernels read;
* contiguous gradient buckets for RCCL all-reduce (``parallel/dp.py``);
* a single buffer to send/receive in parameter-server mode (``parallel/ps.py``).
"""
from __future__ import annotations

import dataclasses
import math
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import torch


@dataclasses.dataclass
class OptConfig:
    lr0: float = 0.1
    decay_rate: float = 0.1
    decay_steps: int = 0          # <= 0: constant learning rate
    momentum: float = 0.0
    nesterov: bool = False
    use_momentum: bool = False
    ema_max: float = 0.9999       # MOVING_AVERAGE_DECAY (mnist_input.py:20); < 0 disables

    @staticmethod
    def from_spec(spec, decay_steps: int, decay_rate: float, ema: float = 0.9999) -> "OptConfig":
        """From a parameter-manager ``OptimizerSpec``."""
        lr = spec.learning_rate
        return OptConfig(lr0=float(lr), decay_rate=float(decay_rate), decay_steps=int(decay_steps),
                         momentum=float(spec.momentum), nesterov=bool(spec.nesterov),
                         use_momentum=spec.name == "momentum", ema_max=ema)

    def lr_at(self, step: int) -> float:
        if self.decay_steps <= 0:
            return self.lr0
        return self.lr0 * self.decay_rate ** (step // self.decay_steps)


@dataclasses.dataclass
class Entry:
    name: str
    shape: Tuple[int, ...]
    wd: Optional[float]
    off: int
    n: int
    G: int
    I: int
    J: int
    Ip: int
    Jp: int
    bf_off: int
    l2_index: int   # -1: not tracked


def _f32_bits(x: float) -> int:
    return struct.unpack("<i", struct.pack("<f", float(x)))[0]


class FlatParams:
    def __init__(self, entries: List[Entry], total: int, bf_total: int, device: torch.device):
        self.entries = entries
        self.by_name = {e.name: e for e in entries}
        self.total = total
        self.device = device
        self.params = torch.zeros(total, dtype=torch.float32, device=device)
        self.grads = torch.zeros(total, dtype=torch.float32, device=device)
        self.mom = torch.zeros(total, dtype=torch.float32, device=device)
        self.ema = torch.zeros(total, dtype=torch.float32, device=device)
        self.bf16 = torch.zeros(max(bf_total, 1), dtype=torch.bfloat16, device=device)
        self.step = torch.zeros(1, dtype=torch.int64, device=device)
        self.wd_entries = [e for e in entries if e.l2_index >= 0]
        # [per-tensor sum(w^2) | one partial per fused-optimizer block (misc.hip OPT_CHUNK =
        # 512 elements)]: the partials are combined in block order (deterministic)
        n_opt_blocks = sum(-(-e.n // 512) for e in entries)
        self.l2 = torch.zeros(max(len(self.wd_entries), 1) + n_opt_blocks, dtype=torch.float32, device=device)
        self.wds = torch.tensor([float(e.wd) for e in self.wd_entries] or [0.0], dtype=torch.float32,
                                device=device)
        # name -> (offset in bf16, Jt, It): optional transposed bf16 copies W^T [Jt][It]
        self.bft: Dict[str, Tuple[int, int, int]] = {}
        self._build_segs()
        # finalize_step: {weight index, first, end fused-optimizer block} per tracked weight
        ranges, b = [], 0
        for e in entries:
            nb = -(-e.n // 512)
            if e.l2_index >= 0:
                ranges.append([e.l2_index, b, b + nb])
            b += nb
        self.l2_ranges = torch.tensor(ranges or [[0, 0, 0]], dtype=torch.int32, device=device)

    def _build_segs(self) -> None:
        rows = []
        for e in self.entries:
            t = self.bft.get(e.name)
            rows.append([e.off, e.n, e.G, e.I, e.J, e.Ip, e.Jp, e.bf_off, _f32_bits(e.wd or 0.0),
                         e.l2_index + 1, t[0] if t else -1, t[1] if t else 0, t[2] if t else 0, 0])
        self.segs = torch.tensor(rows, dtype=torch.int64)

    def enable_transposed(self, tdims: Dict[str, Tuple[int, int]]) -> None:
        """Also keep a transposed, zero-padded bf16 copy W^T [Jt][It] of these 2-D
        weights, rewritten by every optimizer step (the fused dense head stages
        them into LDS with straight 16-byte copies instead of transposing)."""
        off = (self.bf16.numel() + 7) // 8 * 8
        for name, (Jt, It) in tdims.items():
            e = self.by_name[name]
            assert e.G == 1 and Jt >= e.J and It >= e.I, name
            self.bft[name] = (off, int(Jt), int(It))
            off = (off + Jt * It + 7) // 8 * 8
        grown = torch.zeros(off, dtype=torch.bfloat16, device=self.device)
        grown[:self.bf16.numel()].copy_(self.bf16)
        self.bf16 = grown
        self._build_segs()
        self.refresh_bf16()

    def bf16t_view(self, name: str) -> torch.Tensor:
        off, Jt, It = self.bft[name]
        return self.bf16[off:off + Jt * It].view(Jt, It)

    # -- construction -----------------------------------------------------
    @classmethod
    def build(cls, specs: Sequence[Tuple[str, Tuple[int, ...], Optional[float]]],
              init: Dict[str, torch.Tensor], device, pads: Optional[Dict[str, Tuple[int, int]]] = None,
              bias_names_have_no_bf16: bool = True, bf16_copies: bool = True) -> "FlatParams":
        """specs: (name, shape, wd) in creation order.  pads: name -> (I_pad, J_pad)
        for tensors that get a bf16 copy (weights; 4-D = [KH,KW,I,J], 2-D = [I,J]).
        bf16_copies=False: no bf16 copies at all (the fp32 plan reads the masters)."""
        pads = pads or {}
        entries: List[Entry] = []
        off = 0
        bf_off = 0
        l2i = 0
        for name, shape, wd in specs:
            shape = tuple(int(s) for s in shape)
            n = math.prod(shape)
            if len(shape) == 4:
                G, I, J = shape[0] * shape[1], shape[2], shape[3]
            elif len(shape) == 2:
                G, I, J = 1, shape[0], shape[1]
            else:
                G, I, J = 1, 1, shape[0]
            has_bf = bf16_copies and (len(shape) >= 2 or not bias_names_have_no_bf16)
            Ip, Jp = pads.get(name, (I, J))
            e = Entry(name, shape, wd, off, n, G, I, J, Ip, Jp, bf_off if has_bf else -1,
                      l2i if (wd is not None and len(shape) >= 2) else -1)
            if e.l2_index >= 0:
                l2i += 1
            if has_bf:
                bf_off += G * Ip * Jp
                bf_off = (bf_off + 7) // 8 * 8   # keep every copy 16-byte aligned
            entries.append(e)
            off += n
        fp = cls(entries, off, bf_off, torch.device(device))
        fp.load_state({k: v for k, v in init.items() if k in fp.by_name}, ema_too=True)
        return fp

    # -- views ------------------------------------------------------------
    def _view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        e = self.by_name[name]
        return buf[e.off:e.off + e.n].view(e.shape)

    def param_view(self, name: str) -> torch.Tensor:
        return self._view(self.params, name)

    def grad_view(self, name: str) -> torch.Tensor:
        return self._view(self.grads, name)

    def mom_view(self, name: str) -> torch.Tensor:
        return self._view(self.mom, name)

    def ema_view(self, name: str) -> torch.Tensor:
        return self._view(self.ema, name)

    def bf16_view(self, name: str) -> torch.Tensor:
        e = self.by_name[name]
        assert e.bf_off >= 0, f"{name} has no bf16 copy"
        n = e.G * e.Ip * e.Jp
        v = self.bf16[e.bf_off:e.bf_off + n]
        if len(e.shape) == 4:
            return v.view(e.shape[0], e.shape[1], e.Ip, e.Jp)
        return v.view(e.Ip, e.Jp)

    def names(self) -> List[str]:
        return [e.name for e in self.entries]

    # -- state --------------------------------------------------------------
    def load_state(self, values: Dict[str, torch.Tensor], ema_too: bool = False,
                   ema_values: Optional[Dict[str, torch.Tensor]] = None,
                   mom_values: Optional[Dict[str, torch.Tensor]] = None) -> None:
        with torch.no_grad():
            for name, v in values.items():
                self.param_view(name).copy_(v.reshape(self.by_name[name].shape))
                if ema_too:
                    self.ema_view(name).copy_(v.reshape(self.by_name[name].shape))
            for name, v in (ema_values or {}).items():
                self.ema_view(name).copy_(v.reshape(self.by_name[name].shape))
            for name, v in (mom_values or {}).items():
                self.mom_view(name).copy_(v.reshape(self.by_name[name].shape))
        self.refresh_bf16()

    def refresh_bf16(self) -> None:
        """Rebuild the padded bf16 copies from the fp32 masters (GPU kernel)."""
        if self.device.type != "cuda":
            return
        from ..ops._ext import kernels
        K = kernels()
        for e in self.entries:
            if e.bf_off >= 0:
                K.cast_f32_bf16_padded(self.param_view(e.name).contiguous(), self.bf16[e.bf_off:], e.G, e.I, e.J,
                                       e.Ip, e.Jp)
        with torch.no_grad():
            for name in self.bft:
                e = self.by_name[name]
                self.bf16t_view(name)[:e.J, :e.I].copy_(self.param_view(name).reshape(e.I, e.J).t())

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {e.name: self.param_view(e.name).detach().cpu().clone() for e in self.entries}

    # -- K9 -------------------------------------------------------------------
    def apply(self, cfg: OptConfig, grad_scale: float = 1.0, track_l2: bool = True, fin: Optional[tuple] = None,
              perm: Optional[tuple] = None) -> None:
        """``fin``: finalize_step's arguments after ``step`` -- the step's finalize then runs
        in the same launch (HipNet.update); ``perm``: the next batch's perm_positions job
        (DeviceLoader.lookahead_job), run by extra blocks of the launch."""
        from ..ops._ext import kernels
        kernels().fused_optimizer(self.params, self.grads, self.mom, self.ema, self.bf16, self.segs, self.step,
                                  cfg.lr0, cfg.decay_rate, cfg.decay_steps, cfg.momentum, cfg.nesterov,
                                  cfg.use_momentum, grad_scale, cfg.ema_max,
                                  self.l2 if (track_l2 and self.wd_entries) else None, fin=fin, perm=perm)
