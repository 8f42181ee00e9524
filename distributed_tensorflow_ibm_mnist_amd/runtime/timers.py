"""Step-phase timing with HIP events.

``PhaseTimer.mark(name)`` records an event on the current stream; after a step
``close()`` synchronizes once and accumulates the time between consecutive
marks per phase.  The DP step marks: forward, loss (softmax-CE), backward
(which launches the bucketed all-reduces on RCCL's stream), allreduce_wait (the
part of the gradient exchange NOT hidden behind backward), update (fused
optimizer + finalize).  Eager only: a hipGraph replay has no phase boundaries.
Replaces the reference's implicit TF StepCounterHook timing (main.py:140-146).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Tuple

import torch


class PhaseTimer:
    def __init__(self, device):
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self._marks: List[Tuple[str, object]] = []
        self.total: "OrderedDict[str, float]" = OrderedDict()
        self.steps = 0

    def _event(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        import time
        return time.perf_counter()

    def mark(self, name: str) -> None:
        self._marks.append((name, self._event()))

    def close(self) -> None:
        if len(self._marks) < 2:
            self._marks.clear()
            return
        if self.gpu:
            self._marks[-1][1].synchronize()
        for (_, a), (name, b) in zip(self._marks[:-1], self._marks[1:]):
            ms = a.elapsed_time(b) if self.gpu else (b - a) * 1e3
            self.total[name] = self.total.get(name, 0.0) + ms
        self.steps += 1
        self._marks.clear()

    def summary(self) -> Dict[str, float]:
        n = max(self.steps, 1)
        return {k: round(v / n, 4) for k, v in self.total.items()}
