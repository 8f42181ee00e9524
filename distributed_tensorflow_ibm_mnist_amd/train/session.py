"""``MonitoredTrainingSession`` equivalent (``main.py:140-156`` [TF1-lib]).

* restores the latest checkpoint of ``checkpoint_dir`` on start (chief reads,
  then the state is broadcast to every data-parallel replica), so a restarted
  job resumes at its last global step;
* installs TF's default chief hooks: checkpoint saver (600 s + start + end),
  summary saver (every 100 steps), step counter (every 100 steps);
* drives ``before_run`` / step / ``after_run`` hooks; ``should_stop`` turns true
  when a hook requests it (``StopAtStepHook``);
* on exit runs ``end`` hooks — the final checkpoint — unless the session is
  leaving because of an error (a NaN loss must not overwrite a good checkpoint).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from ..ckpt.saver import Saver, latest_checkpoint, write_graph_pbtxt
from ..obs.events import EventFileWriter
from .hooks import (CheckpointSaverHook, RunContext, SessionRunHook, StepCounterHook, SummarySaverHook)
from .replica import load_state, state_tensors


class MonitoredTrainingSession:
    def __init__(self, replica, is_chief: bool, checkpoint_dir: Optional[str], hooks: List[SessionRunHook],
                 save_checkpoint_secs: Optional[float] = 600, save_checkpoint_steps: Optional[int] = None,
                 save_summaries_steps: int = 100, log_step_count_steps: int = 100, max_to_keep: int = 5,
                 meta: Optional[dict] = None, log=print, restore: bool = True):
        self.replica = replica
        self.is_chief = is_chief
        self.checkpoint_dir = checkpoint_dir
        self.hooks = list(hooks)
        self.saver = Saver(max_to_keep=max_to_keep)
        self.meta = meta or {}
        self.log = log
        self._ctx = RunContext(self)
        self._writer: Optional[EventFileWriter] = None
        self.stats_event = None
        self.restored_from: Optional[str] = None
        if restore:
            self._restore()
        if is_chief and checkpoint_dir:
            self._writer = EventFileWriter(checkpoint_dir)
            if save_checkpoint_secs or save_checkpoint_steps:
                self.hooks.append(CheckpointSaverHook(save_checkpoint_secs, save_checkpoint_steps))
            if save_summaries_steps:
                self.hooks.append(SummarySaverHook(self._writer, save_summaries_steps))
            write_graph_pbtxt(checkpoint_dir, state_tensors(replica.net))
        if is_chief and log_step_count_steps:
            self.hooks.append(StepCounterHook(log_step_count_steps, self._writer, replica.examples_per_step, log))

    # ------------------------------------------------------------------ session surface used by hooks
    @property
    def global_step(self) -> int:
        return self.replica.global_step

    @property
    def stats(self) -> torch.Tensor:
        return self.replica.net.stats

    def record_stats_event(self) -> None:
        if self.stats.is_cuda:
            if self.stats_event is None:
                self.stats_event = torch.cuda.Event()
            self.stats_event.record()

    def read_stats(self):
        return self.replica.read_stats()

    def learning_rate(self) -> float:
        return self.replica.learning_rate()

    def synchronize(self) -> None:
        self.replica.synchronize()

    def inject_nan(self) -> None:
        self.replica.inject_nan()

    def save_checkpoint(self) -> Optional[str]:
        if not (self.is_chief and self.checkpoint_dir):
            return None
        kw = {}
        if hasattr(self.replica, "fetch_state"):
            # PS mode: the PS tasks own masters/slots/EMA; pull them, write one data shard per PS
            self.replica.fetch_state()
            kw = {"num_shards": self.replica.client.k, "shard_of": self.replica.client.shard_of()}
        tensors = state_tensors(self.replica.net)
        return self.saver.save(self.checkpoint_dir, self.global_step, tensors, meta=self.meta, **kw)

    def _restore(self) -> None:
        r = self.replica
        prefix = latest_checkpoint(self.checkpoint_dir) if self.checkpoint_dir else None
        if prefix is not None and (self.is_chief or r.world > 1):
            # every DP rank sees the same shared train_dir on one node; the chief's copy wins
            if self.is_chief:
                load_state(r.net, Saver.restore(prefix))
                self.restored_from = prefix
                self.log(f"Restored from {prefix}")
        r.dp.broadcast_state(0)
        r.sync_step_from_device()
        loader = getattr(r, "loader", None)
        if loader is not None and hasattr(loader, "seek"):
            loader.seek(r.global_step)     # the data order resumes where the checkpoint left it

    # ------------------------------------------------------------------ loop
    def __enter__(self):
        for h in self.hooks:
            h.begin(self)
        for h in self.hooks:
            h.after_create_session(self)
        return self

    def should_stop(self) -> bool:
        return self._ctx.stop_requested

    def run(self) -> None:
        for h in self.hooks:
            h.before_run(self._ctx)
        if self._ctx.stop_requested:
            return
        self.replica.step()
        for h in self.hooks:
            h.after_run(self._ctx)

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None:
            for h in self.hooks:
                h.end(self)
        if self._writer is not None:
            self._writer.close()
        return False
