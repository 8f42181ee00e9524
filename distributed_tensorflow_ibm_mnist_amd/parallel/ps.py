"""Asynchronous parameter-server mode (``main.py:56-62,80-82``).

Reference semantics (between-graph replication, TF1 ``replica_device_setter``):
variables live on the PS tasks; every worker pulls them, computes gradients on
its own batch and pushes them; the PS applies each push as it arrives (no
aggregation, no staleness bound, Hogwild-style); every push increments the
shared ``global_step`` and ``StopAtStepHook`` compares that shared step.

MI355X realisation:
* one process per GPU; PS and workers talk with point-to-point send/recv over
  RCCL (``nccl`` backend: every (PS, worker) pair gets its own communicator and
  stream, so pushes from different workers progress independently over their
  direct xGMI links) or gloo on CPU;
* the PS keeps the fp32 masters, momentum slots and EMA shadows of ITS shard
  and applies each push with the fused K9 kernel on its GPU;
* k > 1 PS tasks own contiguous, byte-balanced ranges of the flat parameter
  buffer at tensor granularity (TF placed variables round-robin; here the
  12.85 MB ``local3/weights`` simply gets a PS of its own when k >= 2);
* the PS polls posted receives (``Work.is_completed``) and serves whichever
  worker is ready first — true asynchronous apply in arrival order;
* shutdown (Q9): when the global step reaches ``max_steps`` PS 0 answers with a
  stop flag; workers send DONE to every PS; a PS exits once all workers are done.

Wire protocol per exchange, worker -> PS j: ctrl f64[8] = (kind, want_state,
worker_step, global_step_seen, ...) then (GRAD) the fp32 gradient slice;
PS j -> worker: ctrl f64[8] = (global_step, stop, ...) then the fp32 parameter
slice, then (STATE) EMA and momentum slices.
"""
from __future__ import annotations

import os
import signal
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..runtime.params import FlatParams, OptConfig

HELLO, GRAD, STATE, DONE = 0.0, 1.0, 2.0, 3.0
CTRL = 8


def _staged() -> bool:
    return dist.get_backend() == "gloo"


def send(t: torch.Tensor, dst: int) -> None:
    """p2p send; gloo moves GPU tensors through host memory."""
    if t.is_cuda and _staged():
        t = t.cpu()
    dist.send(t.contiguous(), dst)


def recv(t: torch.Tensor, src: Optional[int] = None) -> int:
    if t.is_cuda and _staged():
        h = torch.empty(t.shape, dtype=t.dtype)
        r = dist.recv(h, src)
        t.copy_(h)
        return r
    return dist.recv(t, src)


def shard_ranges(fp: FlatParams, num_ps: int) -> List[Tuple[int, int, List[str]]]:
    """Contiguous byte-balanced ranges of whole tensors: [(start, end, names)]."""
    ents = fp.entries
    if num_ps > len(ents):
        raise ValueError(f"{num_ps} parameter servers for {len(ents)} tensors")
    cum = np.cumsum([e.n for e in ents])
    bounds = [0]
    for j in range(1, num_ps):
        i = int(np.searchsorted(cum, fp.total * j / num_ps)) + 1
        i = max(i, bounds[-1] + 1)
        i = min(i, len(ents) - (num_ps - j))
        bounds.append(i)
    bounds.append(len(ents))
    out = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        out.append((ents[a].off, ents[b - 1].off + ents[b - 1].n, [e.name for e in ents[a:b]]))
    return out


class ParameterServer:
    def __init__(self, ps_index: int, num_ps: int, num_workers: int, specs, init: Dict[str, torch.Tensor],
                 opt: OptConfig, device, max_steps: int, restore: Optional[Dict[str, np.ndarray]] = None,
                 log=print):
        self.j, self.k, self.W = ps_index, num_ps, num_workers
        self.device = torch.device(device)
        full = FlatParams.build(specs, {}, "cpu")
        self.start, self.end, self.names = shard_ranges(full, num_ps)[ps_index]
        mine = [s for s in specs if s[0] in self.names]
        self.fp = FlatParams.build(mine, {n: init[n] for n in self.names}, self.device,
                                   pads={})  # bf16 copy unused by the PS; kernel refreshes it harmlessly
        self.opt = opt
        self.max_steps = max_steps
        self.log = log
        # T6 fault injection: MNIST_FI_KILL_RANK_AT_STEP=r:k SIGKILLs this PS (rank r) at global step k
        kr = os.environ.get("MNIST_FI_KILL_RANK_AT_STEP", "")
        self._kill = tuple(int(v) for v in kr.split(":")) if ":" in kr else (-1, -1)
        self.global_step = 0
        if restore is not None:
            from ..train.replica import load_state  # noqa: F401  (names match)
            vals = {n: torch.from_numpy(np.asarray(restore[n])) for n in self.names if n in restore}
            emas = {n: torch.from_numpy(np.asarray(restore[f"{n}/ExponentialMovingAverage"])) for n in self.names
                    if f"{n}/ExponentialMovingAverage" in restore}
            moms = {n: torch.from_numpy(np.asarray(restore[f"{n}/Momentum"])) for n in self.names
                    if f"{n}/Momentum" in restore}
            self.fp.load_state(vals, ema_too=not emas, ema_values=emas, mom_values=moms)
            self.global_step = int(np.asarray(restore.get("global_step", 0)))
            self.fp.step.fill_(self.global_step)
        self.applied = 0
        self.per_worker = [0] * num_workers

    def _ctrl(self) -> torch.Tensor:
        return torch.zeros(CTRL, dtype=torch.float64, device=self.device)

    def _apply(self) -> None:
        if self.device.type == "cuda":
            self.fp.apply(self.opt, 1.0, track_l2=False)
        else:
            from ..runtime.torchnet import torch_update
            torch_update(self.fp, self.opt, 1.0)
            self.fp.l2.zero_()

    def _reply(self, w_rank: int, want_state: bool) -> None:
        c = self._ctrl()
        c[0] = float(self.global_step)
        c[1] = 1.0 if (self.j == 0 and self.global_step >= self.max_steps) else 0.0
        c[2] = float(self.applied)
        send(c, w_rank)
        send(self.fp.params, w_rank)
        if want_state:
            send(self.fp.ema, w_rank)
            send(self.fp.mom, w_rank)

    def _handle(self, r: int, ctrl: List[float], done: set) -> bool:
        """Process one message from worker rank r; returns False for DONE."""
        kind = ctrl[0]
        if kind == DONE:
            done.add(r)
            return False
        if kind == GRAD:
            recv(self.fp.grads, r)
            if self.j == 0 and self.global_step >= self.max_steps:
                # in-flight push after the stop point: answer with the stop flag, do not apply
                self._reply(r, want_state=ctrl[1] > 0)
                return True
            if self.j != 0:
                # LR / EMA schedule follows the global step owned by PS 0
                self.global_step = int(ctrl[3])
                self.fp.step.fill_(self.global_step)
            self._apply()
            self.applied += 1
            self.per_worker[r - self.k] += 1
            if self.j == 0:
                self.global_step += 1
                self.fp.step.fill_(self.global_step)
            if self._kill[0] == dist.get_rank() and self.global_step >= self._kill[1]:
                self.log(f"[ps {self.j}] fault injection: SIGKILL at global step {self.global_step}")
                sys.stdout.flush()
                os.kill(os.getpid(), signal.SIGKILL)
        self._reply(r, want_state=ctrl[1] > 0)
        return True

    def serve(self) -> Dict[str, int]:
        """Run until every worker has sent DONE, serving workers in arrival order."""
        ranks = [self.k + i for i in range(self.W)]
        done: set = set()
        self.log(f"[ps {self.j}] serving {len(self.names)} tensor(s), {self.end - self.start} params, "
                 f"{self.W} worker(s)")
        if dist.get_backend() == "gloo":
            # gloo: blocking receive from ANY source = the next worker to push
            while len(done) < self.W:
                c = torch.zeros(CTRL, dtype=torch.float64)
                r = dist.recv(c)
                self._handle(r, c.tolist(), done)
        else:
            # RCCL: one posted receive per (PS, worker) communicator, polled for completion
            bufs = {r: self._ctrl() for r in ranks}
            works = {r: dist.irecv(bufs[r], r) for r in ranks}
            idle = 0
            while len(done) < self.W:
                progressed = False
                for r in ranks:
                    if r in done or not works[r].is_completed():
                        continue
                    works[r].wait()
                    if self._handle(r, bufs[r].tolist(), done):
                        bufs[r] = self._ctrl()
                        works[r] = dist.irecv(bufs[r], r)
                    progressed = True
                if not progressed:
                    idle += 1
                    time.sleep(0.00005 if idle < 1000 else 0.0005)
                else:
                    idle = 0
        self.log(f"[ps {self.j}] done: applied {self.applied} update(s), per worker {self.per_worker}, "
                 f"global_step {self.global_step}")
        return {"applied": self.applied, "global_step": self.global_step}


class PSClient:
    """Worker side: push gradients / pull parameters of every PS shard."""

    def __init__(self, net, num_ps: int):
        self.net = net
        self.k = num_ps
        self.ranges = shard_ranges(net.fp, num_ps)
        self.global_step = 0
        self.stop = False
        dev = net.fp.params.device
        self._c = torch.zeros(CTRL, dtype=torch.float64, device=dev)

    def _exchange(self, kind: float, want_state: bool = False) -> Optional[Dict[str, np.ndarray]]:
        fp = self.net.fp
        state: Dict[str, np.ndarray] = {}
        # push to every PS first (they work in parallel), then collect replies
        for j, (a, b, _) in enumerate(self.ranges):
            c = self._c.clone()
            c[0] = kind
            c[1] = 1.0 if want_state else 0.0
            c[3] = float(self.global_step)
            send(c, j)
            if kind == GRAD:
                send(fp.grads[a:b], j)
        for j, (a, b, names) in enumerate(self.ranges):
            r = torch.empty_like(self._c)
            recv(r, j)
            recv(fp.params[a:b], j)
            if want_state:
                recv(fp.ema[a:b], j)
                recv(fp.mom[a:b], j)
            if j == 0:
                vals = r.tolist()
                self.global_step = int(vals[0])
                self.stop = vals[1] > 0
        fp.step.fill_(self.global_step)
        fp.refresh_bf16()
        return state if want_state else None

    def hello(self) -> None:
        self._exchange(HELLO)

    def push_pull(self) -> None:
        self._exchange(GRAD)

    def fetch_state(self) -> None:
        self._exchange(STATE, want_state=True)

    def done(self) -> None:
        for j in range(self.k):
            c = self._c.clone()
            c[0] = DONE
            send(c, j)

    def shard_of(self) -> Dict[str, int]:
        out = {}
        for j, (_, _, names) in enumerate(self.ranges):
            for n in names:
                out[n] = j
                out[f"{n}/ExponentialMovingAverage"] = j
                out[f"{n}/Momentum"] = j
        return out


class PSWorkerReplica:
    """A worker replica in PS mode: same executor/input pipeline as ``Replica``
    but no local optimizer — gradients go to the PS tasks, fresh parameters
    and the shared global step come back."""

    def __init__(self, base, num_ps: int):
        self.base = base                  # a train.replica.Replica (built with world=1 semantics)
        self.net = base.net
        self.spec = base.spec
        self.client = PSClient(base.net, num_ps)
        self.world = 1
        self.examples_per_step = base.B
        self.device = base.device
        self.loader = base.loader
        self.eval_ds = base.eval_ds
        self.dp = base.dp
        self.client.hello()

    @property
    def global_step(self) -> int:
        return self.client.global_step

    def sync_step_from_device(self) -> None:
        pass

    def step(self) -> None:
        net = self.net
        self.loader.next()
        net.forward(defer_head=True)
        net.loss_and_grad()
        net.backward()
        net.finalize(net.B, increment=False)
        self.client.push_pull()

    @property
    def stop_requested(self) -> bool:
        return self.client.stop

    def learning_rate(self) -> float:
        return self.net.opt.lr_at(self.global_step)

    def read_stats(self):
        return self.net.read_stats()

    def evaluate(self, max_examples=None):
        return self.base.evaluate(max_examples)

    def inject_nan(self) -> None:
        self.base.inject_nan()

    def synchronize(self) -> None:
        self.base.synchronize()

    def fetch_state(self) -> None:
        self.client.fetch_state()

    def finish(self) -> None:
        self.client.done()
