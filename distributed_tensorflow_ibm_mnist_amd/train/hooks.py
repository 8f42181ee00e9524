"""Session hooks (TF ``SessionRunHook`` semantics, host-side, no per-step sync).

Reference hook set (``main.py:111-139``) plus the defaults TF's
``MonitoredTrainingSession`` adds on the chief [TF1-lib]:

* ``StopAtStepHook(last_step)``      — stop once the (shared) global step reaches it
* ``NanTensorHook``                  — NaN/Inf loss raises ``NanLossDuringTrainingError``;
                                       the flag is set on device by the softmax-CE
                                       kernel and read one step late (pinned async copy)
* ``LoggerHook(test_interval)``      — the reference ``_LoggerHook``: every
                                       ``test_interval`` global steps write train
                                       summaries, then run a real eval and write test
                                       summaries (fixes Q5)
* ``CheckpointSaverHook``            — every ``save_secs`` (600) / ``save_steps``, at
                                       session start and at the end
* ``SummarySaverHook``               — loss/accuracy scalars every N steps
* ``StepCounterHook``                — ``global_step/sec`` and images/sec every N steps
* ``FaultInjectionHook``             — env-driven NaN / kill / exit injection (T6)
"""
from __future__ import annotations

import os
import signal
import sys
import time
from typing import Optional

import torch


class NanLossDuringTrainingError(RuntimeError):
    def __str__(self):
        return "NaN loss during training."


class RunContext:
    def __init__(self, session):
        self.session = session
        self.stop_requested = False

    def request_stop(self) -> None:
        self.stop_requested = True


class SessionRunHook:
    def begin(self, session) -> None: ...
    def after_create_session(self, session) -> None: ...
    def before_run(self, ctx: RunContext) -> None: ...
    def after_run(self, ctx: RunContext) -> None: ...
    def end(self, session) -> None: ...


class StopAtStepHook(SessionRunHook):
    def __init__(self, last_step: Optional[int] = None, num_steps: Optional[int] = None):
        if (last_step is None) == (num_steps is None):
            raise ValueError("exactly one of last_step / num_steps")
        self.last_step, self.num_steps = last_step, num_steps

    def after_create_session(self, session) -> None:
        if self.num_steps is not None:
            self.last_step = session.global_step + self.num_steps

    def begin(self, session) -> None:
        self.after_create_session(session)

    def before_run(self, ctx: RunContext) -> None:
        if ctx.session.global_step >= self.last_step:
            ctx.request_stop()

    def after_run(self, ctx: RunContext) -> None:
        if ctx.session.global_step >= self.last_step:
            ctx.request_stop()


class NanTensorHook(SessionRunHook):
    """Asynchronous NaN guard: the device flag (``stats[2]``, set by the
    softmax-CE / finalize kernels and never cleared, so no step is missed) is copied to
    a pinned host mirror with a non-blocking copy every ``every_n_steps`` steps and
    checked one step later -- a NaN at step k is raised by step k + N, with one host
    sync per N steps instead of per step.  ``end`` does a final synchronous check."""

    def __init__(self, fail_on_nan_loss: bool = True, every_n_steps: int = 1, log=print):
        self.fail, self.every = fail_on_nan_loss, max(1, every_n_steps)
        self.log = log
        self._host: Optional[torch.Tensor] = None
        self._n = 0
        self._pending = False
        self.checks = 0                 # host syncs taken (tests: one per N steps)

    def _check(self, session) -> None:
        if self._pending:
            if session.stats_event is not None:
                session.stats_event.synchronize()
            self.checks += 1
            self._pending = False
            if float(self._host[0]) != 0.0:
                self.log(f"NaN loss detected at global step {session.global_step}")
                if self.fail:
                    raise NanLossDuringTrainingError()
                print("Model diverged with loss = NaN.", file=sys.stderr)

    def _record(self, s) -> None:
        if self._host is None:
            self._host = torch.zeros(1, dtype=torch.float32, pin_memory=s.stats.is_cuda)
        self._host.copy_(s.stats[2:3], non_blocking=True)
        s.record_stats_event()
        self._pending = True

    def after_run(self, ctx: RunContext) -> None:
        s = ctx.session
        self._check(s)
        self._n += 1
        if self._n % self.every == 0:
            self._record(s)

    def end(self, session) -> None:
        self._check(session)
        self._record(session)            # the steps since the last mirror copy
        self._check(session)


class LoggerHook(SessionRunHook):
    """The reference ``_LoggerHook`` (main.py:111-135), on the chief."""

    def __init__(self, test_interval: int, monitor):
        self.test_interval = max(1, int(test_interval))
        self.monitor = monitor

    def begin(self, session) -> None:
        self._next = (session.global_step // self.test_interval + 1) * self.test_interval

    def after_run(self, ctx: RunContext) -> None:
        s = ctx.session
        gs = s.global_step
        if gs >= self._next:
            self._next += self.test_interval
            self.monitor.write_train(gs)
            self.monitor.write_test(gs)


class CheckpointSaverHook(SessionRunHook):
    def __init__(self, save_secs: Optional[float] = 600, save_steps: Optional[int] = None):
        self.save_secs = save_secs if save_secs and save_secs > 0 else None
        self.save_steps = save_steps if save_steps and save_steps > 0 else None
        self._last_time = time.time()
        self._last_step = -1

    def after_create_session(self, session) -> None:
        # TF saves right after the session is created (step of restore / 0)
        self._save(session)

    def after_run(self, ctx: RunContext) -> None:
        s = ctx.session
        due = False
        if self.save_steps and s.global_step - max(self._last_step, 0) >= self.save_steps:
            due = True
        if self.save_secs and time.time() - self._last_time >= self.save_secs:
            due = True
        if due:
            self._save(s)

    def end(self, session) -> None:
        if session.global_step != self._last_step:
            self._save(session)

    def _save(self, session) -> None:
        # The NaN guard reads the device flag only every N steps (NanTensorHook), so a save
        # can fall between a NaN step and its detection: read the flag synchronously here
        # (one sync per checkpoint) and never write poisoned parameters -- a restart would
        # restore them and fail again.
        st = getattr(session, "stats", None)
        if st is not None and float(st[2]) != 0.0:
            raise NanLossDuringTrainingError()
        session.save_checkpoint()
        self._last_step = session.global_step
        self._last_time = time.time()


class SummarySaverHook(SessionRunHook):
    def __init__(self, writer, save_steps: int = 100):
        self.writer, self.every = writer, max(1, save_steps)

    def after_run(self, ctx: RunContext) -> None:
        s = ctx.session
        if s.global_step % self.every == 0:
            st = s.read_stats()
            self.writer.add_scalars({"loss": st["total_loss"], "cross_entropy": st["cross_entropy"],
                                     "accuracy": st["accuracy"], "learning_rate": s.learning_rate()},
                                    s.global_step)


class StepCounterHook(SessionRunHook):
    def __init__(self, every_n_steps: int = 100, writer=None, images_per_step: int = 0, log=print):
        self.every, self.writer, self.ips, self.log = max(1, every_n_steps), writer, images_per_step, log
        self._t = None
        self._s = None

    def after_create_session(self, session) -> None:
        self._t, self._s = time.time(), session.global_step

    def after_run(self, ctx: RunContext) -> None:
        s = ctx.session
        if s.global_step - self._s >= self.every:
            s.synchronize()
            now = time.time()
            rate = (s.global_step - self._s) / max(now - self._t, 1e-9)
            msg = f"global_step/sec: {rate:.4g}"
            if self.ips:
                msg += f"  images/sec: {rate * self.ips:.4g}"
            self.log(msg)
            if self.writer is not None:
                self.writer.add_scalars({"global_step/sec": rate}, s.global_step)
            self._t, self._s = now, s.global_step


class FaultInjectionHook(SessionRunHook):
    """T6 fault injection, driven by environment variables:

    MNIST_FI_NAN_AT_STEP=k          poison the loss at global step k (NaN hook must fire)
    MNIST_FI_KILL_RANK_AT_STEP=r:k  SIGKILL rank r at global step k (restart/resume tests)
    MNIST_FI_EXIT_AT_STEP=k         clean sys.exit(17) at global step k
    MNIST_FI_EVERY_ATTEMPT=1        also inject after a torchrun elastic restart
                                    (default: only on attempt 0, so --max-restarts
                                    recovers instead of re-failing at the same step)
    """

    def __init__(self, rank: int = 0):
        self.rank = rank
        attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if attempt > 0 and os.environ.get("MNIST_FI_EVERY_ATTEMPT", "0") != "1":
            for k in ("MNIST_FI_NAN_AT_STEP", "MNIST_FI_KILL_RANK_AT_STEP", "MNIST_FI_EXIT_AT_STEP"):
                os.environ.pop(k, None)
        self.nan_at = int(os.environ.get("MNIST_FI_NAN_AT_STEP", "-1"))
        kr = os.environ.get("MNIST_FI_KILL_RANK_AT_STEP", "")
        self.kill_rank, self.kill_at = (int(kr.split(":")[0]), int(kr.split(":")[1])) if ":" in kr else (-1, -1)
        self.exit_at = int(os.environ.get("MNIST_FI_EXIT_AT_STEP", "-1"))

    def active(self) -> bool:
        return self.nan_at >= 0 or self.kill_at >= 0 or self.exit_at >= 0

    def before_run(self, ctx: RunContext) -> None:
        s = ctx.session
        if self.nan_at >= 0 and s.global_step == self.nan_at:
            s.inject_nan()

    def after_run(self, ctx: RunContext) -> None:
        gs = ctx.session.global_step
        if self.kill_at >= 0 and gs >= self.kill_at and self.rank == self.kill_rank:
            sys.stdout.flush()
            os.kill(os.getpid(), signal.SIGKILL)
        if self.exit_at >= 0 and gs >= self.exit_at:
            sys.stdout.flush()
            os._exit(17)
