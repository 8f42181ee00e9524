"""Chief-only training monitor — the in-repo equivalent of DLI's ``monitor_cb.CMonitor``.

The reference registers, on the chief (``main.py:75-109``):
``SummaryHist`` (weights / biases / activations of conv1, conv2, local3, local4),
``SummaryNorm2`` (weight L2 norms), ``SummaryGradient`` (gradient histograms),
``SummaryGWRatio`` (gradient/weight ratio) and the scalars ``train loss``,
``train accuracy``, ``test loss``, ``test accuracy``, merged into a TRAIN and a
TEST collection written by ``_LoggerHook`` every ``test_interval`` steps to
``train_dir/log``.  ``monitor_cb`` itself is not in the repository [DLI]; this
class reproduces each summary type as TensorBoard event data under the same
names.  Unlike the reference (Q5), "test" scalars come from a real pass over
the held-out split, not from the next training batch.

Activations are the reference's ``<layer>/<layer>:0`` tensors (``main.py:97-100``):
a conv layer's bias+ReLU output BEFORE pooling (conv1: ``[n,28,28,32]``), for the
first ``sample`` images of the last batch.  Where conv and pool run as one fused
kernel that tensor never exists, so the executor recomputes it for the sample with
the unfused conv kernel (``HipNet.layer_activation``); dense layers expose their
live output buffers.  Channel padding is stripped.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from .events import EventFileWriter, histogram_value, scalar_value, summary

DLMAO_TRAIN_SUMMARIES = "DLMAO_TRAIN_SUMMARIES"
DLMAO_TEST_SUMMARIES = "DLMAO_TEST_SUMMARIES"


class Monitor:
    def __init__(self, log_dir: str, test_interval: int, max_steps: int, replica, sample: int = 64,
                 eval_examples: Optional[int] = 10000, log=print):
        self.log_dir = log_dir
        self.test_interval, self.max_steps = test_interval, max_steps
        self.replica = replica
        self.sample = sample
        self.eval_examples = eval_examples
        self.writer = EventFileWriter(log_dir)
        self.log = log
        self._train: List[Tuple[str, Callable[[], bytes]]] = []
        self._test: List[Tuple[str, Callable[[], bytes]]] = []
        self._test_cache: Dict[str, float] = {}

    # ---- registration API (names as in monitor_cb) ------------------------
    def _fp(self):
        return self.replica.net.fp

    def SummaryHist(self, kind: str, layer: str) -> None:
        """kind: 'weight' | 'bias' | 'activation'."""
        tag = f"{layer}/{kind}"
        if kind == "weight":
            fn = lambda: self._fp().param_view(f"{layer}/weights").detach().float().cpu().numpy()  # noqa: E731
        elif kind == "bias":
            fn = lambda: self._fp().param_view(f"{layer}/biases").detach().float().cpu().numpy()  # noqa: E731
        elif kind == "activation":
            fn = lambda: self._activation(layer)  # noqa: E731
        else:
            raise ValueError(kind)
        self._train.append((tag, lambda: histogram_value(tag, fn())))

    def SummaryNorm2(self, kind: str, layer: str) -> None:
        tag = f"{layer}/{kind}_norm2"
        name = f"{layer}/weights" if kind == "weight" else f"{layer}/biases"
        self._train.append((tag, lambda: scalar_value(tag, float(self._fp().param_view(name).norm().item()))))

    def SummaryGradient(self, kind: str = "weight", loss=None) -> None:
        fp = self._fp()
        for e in fp.entries:
            if kind == "weight" and not e.name.endswith("/weights"):
                continue
            tag = f"gradient/{e.name}"
            self._train.append((tag, (lambda n=e.name, t=tag: histogram_value(t, self._grad(n)))))

    def SummaryGWRatio(self) -> None:
        fp = self._fp()
        for e in fp.entries:
            if not e.name.endswith("/weights"):
                continue
            tag = f"gw_ratio/{e.name}"

            def fn(n=e.name, t=tag):
                w = float(self._fp().param_view(n).norm().item())
                g = float(np.linalg.norm(self._grad(n)))
                return scalar_value(t, g / w if w > 0 else 0.0)
            self._train.append((tag, fn))

    def SummaryScalar(self, name: str, source: Optional[str] = None) -> None:
        """'train loss' / 'train accuracy' / 'test loss' / 'test accuracy'."""
        if name.startswith("test"):
            key = "loss" if "loss" in name else "accuracy"
            self._test.append((name, lambda k=key, n=name: scalar_value(n, self._test_cache.get(k, float("nan")))))
        else:
            key = "total_loss" if "loss" in name else "accuracy"
            self._train.append((name, lambda k=key, n=name: scalar_value(n, self.replica.read_stats()[k])))

    def register_reference_summaries(self, layers=("conv1", "conv2", "local3", "local4")) -> None:
        """The exact registration block of main.py:95-107 (layers present in the model)."""
        names = {e.name.split("/")[0] for e in self._fp().entries}
        for layer in layers:
            if layer not in names:
                continue
            self.SummaryHist("weight", layer)
            self.SummaryHist("bias", layer)
            self.SummaryHist("activation", layer)
            self.SummaryNorm2("weight", layer)
        self.SummaryGradient("weight")
        self.SummaryGWRatio()
        for s in ("train loss", "train accuracy", "test loss", "test accuracy"):
            self.SummaryScalar(s)

    # ---- helpers --------------------------------------------------------------
    def _grad(self, name: str) -> np.ndarray:
        g = self._fp().grad_view(name).detach().float().cpu().numpy()
        w = max(1, self.replica.world)
        return g / w

    def _activation(self, layer: str) -> np.ndarray:
        net = self.replica.net
        try:
            a = net.layer_activation(layer, self.sample)
        except KeyError:
            return np.zeros(1)
        a = a[: self.sample].detach().float().cpu().numpy()
        spec = {L.name: L for L in self.replica.spec.layers}.get(layer)
        real = getattr(spec, "cout", None) or getattr(spec, "dout", None)
        if real is not None and a.shape[-1] > real:
            a = a[..., :real]
        return a

    # ---- writers ----------------------------------------------------------------
    def write_train(self, step: int) -> None:
        vals = [fn() for _, fn in self._train]
        if vals:
            self.writer.add_summary(summary(vals), step)

    def write_test(self, step: int) -> None:
        res = self.replica.evaluate(self.eval_examples)
        self._test_cache = res
        vals = [fn() for _, fn in self._test]
        if vals:
            self.writer.add_summary(summary(vals), step)
        self.log(f"step {step}: test loss {res['loss']:.4f}  test accuracy {res['accuracy']:.4f}")

    def flush(self) -> None:
        self.writer.flush()

    def close(self) -> None:
        self.writer.close()
