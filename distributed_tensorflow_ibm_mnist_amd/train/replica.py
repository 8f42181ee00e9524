"""One training replica: model executor + on-device input pipeline + DP wiring.

Bridges the session/hook layer (host-side, step-count driven) and the device
(`HipNet` on the HIP kernels, or `TorchNet` for CPU / the PyTorch baseline).
The host keeps a mirror of the global step so hooks never read device memory
on the hot path; device state (loss, accuracy, NaN flag) is read only when a
hook asks for it.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..data.device_loader import DeviceDataset, DeviceLoader, eval_batches
from ..models import torch_ref
from ..models.spec import ModelSpec
from ..parallel.dp import DataParallel
from ..runtime.params import FlatParams, OptConfig


def build_net(impl: str, spec: ModelSpec, batch: int, device, init, opt: OptConfig, precision: str = "bf16"):
    if impl == "hip" and precision == "fp32":
        from ..runtime.executor_f32 import HipNetF32
        return HipNetF32(spec, batch, device, init, opt)
    if impl == "hip":
        assert precision == "bf16", f"unknown precision {precision!r}"
        from ..runtime.executor import HipNet
        return HipNet(spec, batch, device, init, opt)
    from ..runtime.torchnet import TorchNet
    return TorchNet(spec, batch, device, init, opt)


def state_tensors(net, include_momentum: bool = True) -> Dict[str, np.ndarray]:
    """Device state -> checkpoint dict with the reference's variable names."""
    fp: FlatParams = net.fp
    out: Dict[str, np.ndarray] = {}
    params = fp.params.detach().cpu().numpy()
    ema = fp.ema.detach().cpu().numpy()
    mom = fp.mom.detach().cpu().numpy()
    for e in fp.entries:
        sl = slice(e.off, e.off + e.n)
        out[e.name] = params[sl].reshape(e.shape).copy()
        if net.opt.ema_max >= 0:
            out[f"{e.name}/ExponentialMovingAverage"] = ema[sl].reshape(e.shape).copy()
        if include_momentum and net.opt.use_momentum:
            out[f"{e.name}/Momentum"] = mom[sl].reshape(e.shape).copy()
    out["global_step"] = np.asarray(int(fp.step.item()), dtype=np.int64)
    le = net.loss_ema.detach().cpu().numpy().reshape(-1, 3)
    for i, name in enumerate(net.loss_names):
        out[f"{name}/avg"] = np.asarray(le[i, 2], dtype=np.float32)
        out[f"{name}/avg/biased"] = np.asarray(le[i, 0], dtype=np.float32)
        out[f"{name}/avg/local_step"] = np.asarray(le[i, 1], dtype=np.float32)
    return out


def load_state(net, tensors: Dict[str, np.ndarray], strict: bool = True) -> int:
    fp: FlatParams = net.fp
    missing = [e.name for e in fp.entries if e.name not in tensors]
    if missing and strict:
        raise KeyError(f"checkpoint lacks {missing}")
    vals = {n: torch.from_numpy(np.asarray(tensors[n])) for n in fp.names() if n in tensors}
    emas = {n: torch.from_numpy(np.asarray(tensors[f"{n}/ExponentialMovingAverage"])) for n in fp.names()
            if f"{n}/ExponentialMovingAverage" in tensors}
    moms = {n: torch.from_numpy(np.asarray(tensors[f"{n}/Momentum"])) for n in fp.names()
            if f"{n}/Momentum" in tensors}
    fp.load_state(vals, ema_too=not emas, ema_values=emas, mom_values=moms)
    step = int(np.asarray(tensors.get("global_step", 0)))
    fp.step.fill_(step)
    le = net.loss_ema.view(-1, 3)
    for i, name in enumerate(net.loss_names):
        if f"{name}/avg/biased" in tensors:
            le[i, 0] = float(tensors[f"{name}/avg/biased"])
            le[i, 1] = float(tensors[f"{name}/avg/local_step"])
            le[i, 2] = float(tensors[f"{name}/avg"])
    return step


class Replica:
    def __init__(self, spec: ModelSpec, impl: str, batch: int, device, init: Dict[str, torch.Tensor], opt: OptConfig,
                 train_images: torch.Tensor, train_labels: torch.Tensor, src_channels: int,
                 eval_images: Optional[torch.Tensor] = None, eval_labels: Optional[torch.Tensor] = None,
                 seed: int = 0, shard: bool = True, use_graph: bool = True, bucket_mb: float = 4.0,
                 group=None, standalone: bool = False, fused_input=False, precision: str = "bf16",
                 dp_graph: bool = False):
        self.spec, self.impl, self.B, self.device = spec, impl, batch, torch.device(device)
        self.net = build_net(impl, spec, batch, self.device, init, opt, precision)
        # standalone: a parameter-server worker (no data-parallel group of its own)
        dp_on = dist.is_initialized() and not standalone
        self.world = dist.get_world_size(group) if dp_on else 1
        self.rank = dist.get_rank(group) if dp_on else 0
        self.dp = DataParallel(self.net, group=group, bucket_cap_mb=bucket_mb, world=self.world)
        self.train_ds = DeviceDataset(train_images, train_labels, self.device, hw=784, channels=src_channels)
        self.eval_ds = (DeviceDataset(eval_images, eval_labels, self.device, hw=784, channels=src_channels)
                        if eval_images is not None else None)
        # --input_mode u8 / bf16 (HIP; --fused_input = u8): the first fused conv gathers the
        # resident training set (uint8, or normalised once to bf16) through the batch index
        mode = "u8" if fused_input is True else (fused_input or "prep")
        # eligibility first: a model that cannot gather (3-channel input, fp32 executor) never
        # gets a normalised bf16 copy of the whole split built for nothing
        fused_in = (impl == "hip" and mode != "prep" and getattr(self.net, "can_gather_input", lambda: True)()
                    and self.net.bind_u8_input(self.train_ds.images if mode == "u8" else self.train_ds.bf16_images(),
                                                bwd_images=None if mode == "u8" else self.train_ds.images))
        self.loader = DeviceLoader(self.train_ds, self.net.x0, self.net.labels, rank=self.rank, world=self.world,
                                   seed=seed, shard=shard, idx_out=self.net.idx_buf if fused_in else None)
        # hipGraph: single replica, or (dp_graph) the DP step with its RCCL all-reduces captured
        self.use_graph = (use_graph and impl == "hip" and self.device.type == "cuda"
                          and (self.world == 1 or (dp_graph and dist.get_backend(group) == "nccl")))
        self._graph = None
        self.global_step = 0
        self.examples_per_step = batch * self.world

    # ------------------------------------------------------------------ steps
    def _body(self) -> None:
        self.dp.train_step()

    def step(self) -> None:
        self.loader.next()
        if self.use_graph and self._graph is None:
            from ..runtime.graph import StepGraph
            # the warm-up inside StepGraph IS this step (on the batch just loaded);
            # capture itself executes nothing, so exactly one update happens here
            self._graph = StepGraph(self._body, warmup=1)
        elif self.use_graph:
            self._graph.replay()
        else:
            self._body()
        self.global_step += 1

    def sync_step_from_device(self) -> None:
        self.global_step = int(self.net.fp.step.item())

    def learning_rate(self) -> float:
        return self.net.opt.lr_at(self.global_step)

    def read_stats(self) -> Dict[str, float]:
        # local replica's last step (no collective: hooks run on the chief only)
        return self.net.read_stats()

    def evaluate(self, max_examples: Optional[int] = None) -> Dict[str, float]:
        """Full (or capped) pass over the eval split; returns loss / accuracy."""
        if self.eval_ds is None:
            return {"loss": float("nan"), "accuracy": float("nan")}
        st = self.net.eval_stats
        st.zero_()
        n = 0
        for nb in eval_batches(self.eval_ds, self.net.x0, self.net.labels):
            self.net.eval_batch(nb, st)
            n += nb
            if max_examples and n >= max_examples:
                break
        # local pass (no collective, so chief-only hooks can call it safely)
        v = (st[:2] / max(n, 1)).tolist()
        return {"loss": v[0], "accuracy": v[1]}

    def inject_nan(self) -> None:
        with torch.no_grad():
            self.net.fp.params[0] = float("nan")
        self.net.fp.refresh_bf16()

    def synchronize(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
