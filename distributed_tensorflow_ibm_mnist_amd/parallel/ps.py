"""Asynchronous parameter-server mode (``main.py:56-62,80-82``).

Reference semantics (between-graph replication, TF1 ``replica_device_setter``):
variables live on the PS tasks; every worker pulls them, computes gradients on
its own batch and pushes them; the PS applies each push as it arrives (no
aggregation, no staleness bound, Hogwild-style; ``mnist_input.py:261-264``);
every push increments the shared ``global_step`` and ``StopAtStepHook``
compares that shared step.

MI355X realisation -- ONE serve loop, two planes:

* **control plane** (SURVEY C3): tiny int64 messages on a gloo group over the
  rendezvous TCPStore.  The PS blocks in a host ``recv`` from ANY worker and so
  serves workers strictly in arrival order.  Nothing on any GPU waits for an
  idle worker: no posted-but-unmatched receive kernels, no polling of device
  work, no host sync on a device ctrl tensor.
* **data plane** (``Transport``), chosen per run:
  - ``shm`` (default with GPU workers on one host): the PS is a CPU task, as the
    reference's are (``replica_device_setter`` puts the variables on /job:ps).  Its shard's
    fp32 master / momentum / EMA live in host memory and a native loop
    (``csrc/host/ps_shm.h``, GIL released) serves every gradient push straight from a
    shared-memory segment: the worker DMAs its slice into its pinned push slot and
    publishes a sequence word, the PS checks the stamp, applies the update (bitwise
    ``torch_update``), copies the parameters into the worker's reply slot and publishes
    the reply word the worker spins on.  No GPU work on the PS (a GPU PS time-slices the
    workers' GPU) and no Python or control message per update: 23 us of PS time per
    update on an MI355X host against 61 us for ``ipc`` (``profiles/r5/ps/``).  Control
    words (HELLO / STATE / DONE / RESET) stay on gloo: a worker raises a pending flag
    first so the native loop hands over to Python.  A worker notices a dead PS by its pid.
  - ``ipc``: one-sided copies over xGMI peer memory into a GPU PS.  Each PS
    exports (hipIpc/dmabuf, via ``torch.multiprocessing.reductions``) a
    gradient mailbox and a parameter reply slot per worker plus a state slot.
    A worker copies its gradient slice straight into its mailbox on the PS GPU
    (a DMA over its direct xGMI link), synchronises its own stream and only
    THEN announces the push on the control plane; the PS applies the fused K9
    optimizer reading the mailbox in place, snapshots the parameters into the
    worker's reply slot, synchronises and answers; the worker pulls the
    snapshot with one peer copy.  Every copy is bounded DMA work, and several
    processes can share one GPU (the 1-GPU rehearsal runs the same code).
  - ``host``: gloo send/recv of the slices on the control group (tagged apart
    from control words), staged through host memory for GPU tensors.  The CPU
    test path, and a fallback.
  (RCCL point-to-point is deliberately not used: its matched send/recv pairs
  are GPU kernels that spin until the peer arrives, and RCCL refuses two
  ranks on one GPU, so it could never be exercised on a 1-GPU box.)
* the PS keeps the fp32 masters, momentum slots and EMA shadows of ITS shard;
  k > 1 PS tasks own contiguous, byte-balanced tensor ranges of the flat
  parameter buffer (TF placed variables round-robin; here the 12.85 MB
  ``local3/weights`` simply gets a PS of its own when k >= 2);
* every worker pushes to every PS, so each PS sees the same pushes (in its
  own arrival order); each PS applies the first ``max_steps - start`` it
  receives and counts its own global step, so in an uninterrupted run all
  shards end on the same update count (the reference's async PS made no
  stronger promise).  After a restart every shard resumes from the
  checkpoint's single ``global_step`` (PS 0's count when the chief fetched the
  state); shard j's tensors may have been fetched up to W-1 pushes away from
  that count, so restarted shards can end up to W-1 updates apart (the
  checkpoint keeps the reference's one global_step variable; no per-shard step);
* shutdown (Q9): once its global step reaches ``max_steps`` PS 0 answers with
  a stop flag; workers send DONE to every PS; a PS exits when all are done.
* the worker computes the weight-decay loss terms (``mnist_input.py:112-114``)
  from the parameters its forward used, so logged ``total_loss`` and the
  ``*/weight_loss/avg`` EMAs include them in PS mode too.

Push integrity (both transports): every gradient slice travels with an int64
sequence stamp in its last 8 bytes -- the worker's local step, also announced in
the control word.  The host transport checks it on arrival; the ``ipc`` PS hands
the mailbox's stamp and the expected value to the fused K9 kernel, which skips
the update on a mismatch and records the worker in an error word the PS reads
after its reply sync.  A stale, misdirected or torn push is never applied: the
PS raises ``PushIntegrityError`` naming the worker (fault injection:
``MNIST_FI_CORRUPT_PUSH=worker:local_step``).

``ipc`` needs peer access between every worker GPU and every PS GPU
(``torch.cuda.can_device_access_peer``); the transport is agreed collectively,
and a cluster where any pair lacks it falls back to ``host`` with the reason
logged (``MNISTX_PS_STRICT=1`` makes that an error).

Control words (int64[8]) worker -> PS: (kind, want_state, worker_local_step,
new generation for RESET); PS -> worker: (global_step, stop, applied).

Session recovery (``MonitoredTrainingSession`` recreates its session on
``AbortedError`` / ``UnavailableError``, and the workers outlive a PS restart:
``/root/reference/main.py:140-146`` [TF1-lib]).  The control store lives in the
chief (``cluster.py``), so it outlives any parameter server.  When a PS dies, the
workers keep their processes, their hipGraphs and their input position:

1. a worker's exchange fails on the dead peer (gloo connection error);
2. the PS is restarted (``parallel/supervisor.py`` relaunches just that process,
   or an operator does): it restores its shard from the latest checkpoint and
   opens session generation g+1 in the store;
3. the worker waits for g+1, sends RESET(g+1) to every PS on the old group (the
   surviving PS tasks are blocked in their any-source receive there; the dead one
   just errors), and every rank joins generation g+1 and sets the data plane up again;
4. the worker re-sends the interrupted exchange -- as a parameter pull only to the
   PS tasks that already took its gradient, so no push is applied twice.

Surviving PS tasks keep their parameters and step counts; the restarted one resumes
from the checkpoint (TF's PS recovery made the same promise).  Not covered: two PS
tasks restarting at once, or a worker dying (the supervisor restarts the whole job).
"""
from __future__ import annotations

import os
import re
import signal
import sys
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..runtime.params import FlatParams, OptConfig

HELLO, GRAD, STATE, DONE, RESET = 0, 1, 2, 3, 4
FATAL_KEY = "mnistx/fatal"      # set by a PS that stops on an error no restart would fix
EXIT_FATAL = 86                 # a PS's exit code for such an error: the supervisor never restarts it
CTRL = 8
TAG_CTRL, TAG_DATA = 1, 2


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


# The shm data plane's CPU parameter server streams every byte of its shard through host
# memory per update (params, grads, momentum, EMA, weight decay: 32 bytes per parameter):
# 23 us for LeNet-5's 61.7 K parameters, but 2.4 ms of apply + 2.2 ms of reply copy for the
# reference CNN's 3.46 M (bench/ps_capacity.py).  Above this many parameters per
# shard the GPU parameter server of ``ipc`` (HBM-speed apply, xGMI peer copies) serves instead.
SHM_MAX_SHARD_PARAMS = 1 << 20


def max_shard_params(specs_or_fp, num_ps: int) -> int:
    """Parameters of the largest PS shard (shard_ranges' split) -- the same number on every
    rank, computed from the model's parameter specs or a FlatParams."""
    fp = specs_or_fp if isinstance(specs_or_fp, FlatParams) else FlatParams.build(specs_or_fp, {}, "cpu")
    size = {e.name: e.n for e in fp.entries}
    return max(sum(size[n] for n in names) for _, _, names in shard_ranges(fp, num_ps))


def default_transport(device: torch.device, shard_params: int = 0) -> str:
    """The PS data plane when none is asked for; every rank resolves the same one.

    GPU ranks: ``shm`` -- a CPU parameter server serving pinned shared memory natively (23 us
    of PS time per update at LeNet-5 size vs 61 us for the GPU PS of ``ipc``, and the PS
    never time-slices a worker's GPU: profiles/r5/ps/) -- for shards up to
    SHM_MAX_SHARD_PARAMS (``MNISTX_PS_SHM_MAX_PARAMS``); larger shards (the reference CNN)
    ``ipc``, whose apply runs at HBM speed (profiles/r6/ps/).  setup_transport falls back to
    ``host`` when the ranks span hosts or a GPU lacks peer access.  CPU runs: ``host`` (gloo).
    ``shard_params`` 0 = unknown (treated as small)."""
    if torch.device(device).type != "cuda":
        return "host"
    limit = int(os.environ.get("MNISTX_PS_SHM_MAX_PARAMS", str(SHM_MAX_SHARD_PARAMS)))
    return "shm" if shard_params <= limit else "ipc"


def _sync(t: torch.Tensor) -> None:
    if t.is_cuda:
        torch.cuda.current_stream(t.device).synchronize()


def is_peer_loss(e: BaseException) -> bool:
    """A control-plane failure that a lost / restarted peer explains: torch's
    ``DistBackendError`` / ``DistNetworkError``, or gloo's connection-closed / reset /
    timeout errors (raised as plain RuntimeError by some builds).  Never a
    ``PushIntegrityError`` or a HIP / torch compute error."""
    if isinstance(e, PushIntegrityError):
        return False
    if isinstance(e, PeerLostError):
        return True
    for name in ("DistBackendError", "DistNetworkError", "DistStoreError"):
        t = getattr(dist, name, None)
        if t is not None and isinstance(e, t):
            return True
    msg = str(e).lower()
    # explicit HIP / CUDA error forms only (a device string such as "cuda:0" inside a gloo
    # transport error is not a compute error)
    if re.search(r"\bhip ?error|\bcuda ?error|\bhip runtime error|device-side assert|\bhipgraph\w*error", msg):
        return False             # e.g. hipErrorLaunchTimeOut: a compute failure, re-raised at once
    # only gloo's own transport errors (plain RuntimeError in some builds): the word gloo
    # together with a connection / timeout symptom
    return "gloo" in msg and any(k in msg for k in ("connection", "connect", "timed out", "timeout", "reset by peer",
                                                    "broken pipe", "socket", "closed", "eof"))


class PushIntegrityError(RuntimeError):
    """A gradient push whose sequence stamp does not match its control word."""


def slot_len(n: int) -> int:
    """Elements of one push slot: the slice padded to an even count + an int64 stamp."""
    return (n + 1) // 2 * 2 + 2


def stamp_view(slot: torch.Tensor) -> torch.Tensor:
    """The int64 stamp in the last 8 bytes of a push slot (1-D float32 view)."""
    return slot[-2:].view(torch.int64)


def corrupt_push_at() -> Tuple[int, int]:
    """MNIST_FI_CORRUPT_PUSH=worker:local_step -> that push carries a wrong stamp."""
    v = os.environ.get("MNIST_FI_CORRUPT_PUSH", "")
    return tuple(int(x) for x in v.split(":")) if ":" in v else (-1, -1)


# ---------------------------------------------------------------------------- transports
class HostTransport:
    """Slices travel as gloo messages on the control group (tag TAG_DATA)."""
    name = "host"

    def __init__(self, group, num_ps: int, num_workers: int):
        self.g, self.k, self.W = group, num_ps, num_workers

    def _send(self, t: torch.Tensor, dst: int) -> None:
        dist.send(t.detach().cpu().contiguous() if t.is_cuda else t.contiguous(), dst, group=self.g, tag=TAG_DATA)

    def _recv(self, t: torch.Tensor, src: int) -> None:
        if t.is_cuda:
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src, group=self.g, tag=TAG_DATA)
            t.copy_(h)
        else:
            dist.recv(t, src, group=self.g, tag=TAG_DATA)

    # -- PS side
    def ps_setup(self, ps, is_me: bool) -> None:
        if is_me:
            n = ps.fp.total
            self.n = n
            self.slot = torch.zeros(slot_len(n), dtype=torch.float32)     # host staging: checked on arrival
            self.grad_in = torch.zeros_like(ps.fp.grads)

    def ps_take_grads(self, ps, r: int, expect: int) -> torch.Tensor:
        dist.recv(self.slot, r, group=self.g, tag=TAG_DATA)
        got = int(stamp_view(self.slot))
        if got != expect:
            raise PushIntegrityError(f"PS {ps.j}: push from worker {r - self.k} carries stamp {got}, its control "
                                     f"word announced {expect}: gradient rejected")
        self.grad_in.copy_(self.slot[:self.n])
        return self.grad_in

    def ps_guard(self, r: int, expect: int):
        return None               # checked on the host in ps_take_grads

    def ps_check(self, ps, final: bool = False) -> None:
        pass

    def ps_stage_reply(self, ps, r: int, want_state: bool) -> None:
        pass

    def ps_after_ctrl(self, ps, r: int, want_state: bool) -> None:
        self._send(ps.fp.params, r)
        if want_state:
            self._send(ps.fp.ema, r)
            self._send(ps.fp.mom, r)

    # -- worker side
    def worker_open(self, w_index: int, ranges) -> None:
        self.wi = w_index

    def worker_before_ctrl(self, j: int, kind: int, grads: Optional[torch.Tensor]) -> None:
        pass

    def worker_after_ctrl(self, j: int, kind: int, grads: Optional[torch.Tensor]) -> None:
        if kind == GRAD:
            self._send(grads, j)          # the stamped slot (PSClient._stage)

    def worker_pull(self, j: int, params: torch.Tensor, ema: torch.Tensor, mom: torch.Tensor, state: bool) -> None:
        self._recv(params, j)
        if state:
            self._recv(ema, j)
            self._recv(mom, j)


class IpcTransport:
    """One-sided xGMI peer copies into / out of PS-owned device buffers.

    Per worker the PS exports a stamped gradient mailbox, a parameter reply slot and
    an optimizer-state slot.  The PS answers once an event recorded after the reply
    copy has completed (an event sync on that copy, not a stream-wide sync).  Inter-
    process events -- the worker's stream waiting on the PS's event instead -- were
    measured and rejected: on this runtime the waiting stream is released ~68 ms after
    the producer's work completes (``bench/ipc_event_probe.py``,
    ``profiles/r3/ps/ipc_event_probe.txt``)."""
    name = "ipc"

    def __init__(self, group, num_ps: int, num_workers: int):
        self.g, self.k, self.W = group, num_ps, num_workers
        self.peer: Dict[int, Dict[str, torch.Tensor]] = {}

    def ps_setup(self, ps, is_me: bool) -> None:
        """Collective over the control group: PS j exports, everyone else imports."""
        from torch.multiprocessing.reductions import reduce_tensor
        for j in range(self.k):
            obj = [None]
            if is_me and ps.j == j:
                n, dev = ps.fp.total, ps.fp.params.device
                self.n = n
                self.grad_in = torch.zeros(self.W, slot_len(n), dtype=torch.float32, device=dev)
                self.reply = torch.zeros(self.W, n, dtype=torch.float32, device=dev)
                self.state = torch.zeros(self.W, 2, n, dtype=torch.float32, device=dev)   # one slot per worker
                # K9 guard: error word (device) + its pinned host mirror, refreshed by an async copy
                self.err = torch.zeros(1, dtype=torch.int32, device=dev)
                self.err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
                self.err_ev = torch.cuda.Event()
                torch.cuda.synchronize(dev)
                obj = [{k: reduce_tensor(t) for k, t in
                        (("grad_in", self.grad_in), ("reply", self.reply), ("state", self.state))}]
            dist.broadcast_object_list(obj, src=j, group=self.g)
            if ps is None:                          # a worker maps every PS's buffers
                self.peer[j] = {k: fn(*args) for k, (fn, args) in obj[0].items()}

    def ps_take_grads(self, ps, r: int, expect: int) -> torch.Tensor:
        return self.grad_in[r - self.k, :self.n]   # the worker wrote it before announcing

    def ps_guard(self, r: int, expect: int):
        """(stamp pointer tensor, expected, error word, id) for the K9 kernel's check."""
        return stamp_view(self.grad_in[r - self.k]), expect, self.err, r - self.k + 1

    def ps_stage_reply(self, ps, r: int, want_state: bool) -> None:
        i = r - self.k
        self.reply[i].copy_(ps.fp.params)
        if want_state:
            self.state[i, 0].copy_(ps.fp.ema)
            self.state[i, 1].copy_(ps.fp.mom)
        self.err_host.copy_(self.err, non_blocking=True)
        self.err_ev.record()
        self.err_ev.synchronize()                 # reply + error word landed before the ctrl reply

    def ps_check(self, ps, final: bool = False) -> None:
        """A push the K9 guard rejected (never applied) is a hard error naming the worker,
        raised at the reply that follows it (the error word's host mirror is current)."""
        if final:
            self.err_ev.synchronize()
        bad = int(self.err_host[0])
        if bad:
            raise PushIntegrityError(f"PS {ps.j}: push from worker {bad - 1} failed its sequence-stamp check "
                                     f"(stale or torn mailbox): gradient not applied")

    def ps_after_ctrl(self, ps, r: int, want_state: bool) -> None:
        pass

    def worker_open(self, w_index: int, ranges) -> None:
        self.wi = w_index

    def worker_before_ctrl(self, j: int, kind: int, grads: Optional[torch.Tensor]) -> None:
        if kind == GRAD:
            self.peer[j]["grad_in"][self.wi].copy_(grads)   # the stamped slot (PSClient._stage)
            _sync(grads)                          # landed in the PS's HBM before we announce it

    def worker_after_ctrl(self, j: int, kind: int, grads: Optional[torch.Tensor]) -> None:
        pass

    def worker_pull(self, j: int, params: torch.Tensor, ema: torch.Tensor, mom: torch.Tensor, state: bool) -> None:
        params.copy_(self.peer[j]["reply"][self.wi])
        if state:
            ema.copy_(self.peer[j]["state"][self.wi, 0])
            mom.copy_(self.peer[j]["state"][self.wi, 1])


class PeerLostError(RuntimeError):
    """A parameter server process of the shm data plane is gone (the worker saw its pid die
    while it waited for a reply): recovered like a lost gloo peer."""


# per-worker control words of the shm segment (csrc/host/ps_shm.h PsCtrl)
C_PUSH_SEQ, C_PENDING, C_REPLY_SEQ, C_REPLY_GSTEP, C_REPLY_STOP, C_REPLY_APPLIED = range(6)
PS_CTRL, PS_BAD_STAMP, PS_KILL, PS_IDLE_TIMEOUT = range(4)


def _align(v: int, a: int) -> int:
    return (v + a - 1) // a * a


class ShmLayout:
    """Byte layout of one PS shard's segment (mirrored by csrc/host/ps_shm.h): a 4096-byte
    header page (int64: magic, n, W, PS pid, generation), then per worker (page-aligned blocks): control words
    int64[16], the stamped push slot, the reply parameters, the optimizer-state reply."""
    HDR, MAGIC = 4096, 0x6D6E69737870735F     # a header PAGE: every worker block is page-aligned

    def __init__(self, n: int, W: int):
        self.n, self.W = n, W
        self.slot_floats = slot_len(n)
        self.ctrl_off = 0
        self.push_off = 128
        self.reply_off = _align(self.push_off + 4 * self.slot_floats, 64)
        self.state_off = _align(self.reply_off + 4 * n, 64)
        self.wblock = _align(self.state_off + 8 * n, 4096)
        self.total = self.HDR + W * self.wblock

    def native(self) -> List[int]:
        return [self.n, self.W, self.slot_floats, self.wblock, self.ctrl_off, self.push_off, self.reply_off]


class ShmSegment:
    """A PS shard's shared-memory segment: a /dev/shm file mapped by the PS (creator) and
    every worker; the PS unlinks the name once everyone has mapped it, so nothing is left
    behind even when a process is SIGKILLed."""

    def __init__(self, path: str, lay: ShmLayout, create: bool, gen: int = 0):
        import mmap
        self.path, self.lay = path, lay
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                # reserve every page now: a /dev/shm smaller than the segment then
                # fails here with ENOSPC -- setup_transport falls back to the host transport --
                # instead of a SIGBUS when some process first touches a page past the limit
                try:
                    os.posix_fallocate(fd, 0, lay.total)
                except OSError:
                    os.close(fd)
                    fd = -1
                    os.unlink(path)
                    raise
            self.mm = mmap.mmap(fd, lay.total, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            if fd >= 0:
                os.close(fd)
        import ctypes
        self._cbuf = ctypes.c_char.from_buffer(self.mm)
        self.addr = ctypes.addressof(self._cbuf)
        self.hdr = np.frombuffer(self.mm, dtype=np.int64, count=32, offset=0)
        self.ctrl = [np.frombuffer(self.mm, dtype=np.int64, count=16, offset=lay.HDR + w * lay.wblock + lay.ctrl_off)
                     for w in range(lay.W)]
        self.push = [torch.frombuffer(self.mm, dtype=torch.float32, count=lay.slot_floats,
                                      offset=lay.HDR + w * lay.wblock + lay.push_off) for w in range(lay.W)]
        self.reply = [torch.frombuffer(self.mm, dtype=torch.float32, count=lay.n,
                                       offset=lay.HDR + w * lay.wblock + lay.reply_off) for w in range(lay.W)]
        self.state = [torch.frombuffer(self.mm, dtype=torch.float32, count=2 * lay.n,
                                       offset=lay.HDR + w * lay.wblock + lay.state_off).view(2, lay.n)
                      for w in range(lay.W)]
        self.pinned = False
        if create:
            self.hdr[:] = 0
            self.hdr[0], self.hdr[1], self.hdr[2], self.hdr[3], self.hdr[4] = lay.MAGIC, lay.n, lay.W, os.getpid(), gen

    @property
    def ps_pid(self) -> int:
        return int(self.hdr[3])

    def pin(self, worker: Optional[int] = None) -> bool:
        """hipHostRegister the mapping (a GPU worker's copies become DMA): only the
        worker's own block when ``worker`` is given (registering faults every page in, so
        pinning the whole segment from every worker would touch every other worker's
        block), else the whole segment."""
        from ..ops._ext import kernels
        if worker is None:
            self._pin_at, n = self.addr, self.lay.total
        else:
            self._pin_at, n = self.addr + self.lay.HDR + worker * self.lay.wblock, self.lay.wblock
        self.pinned = bool(kernels().host_register(self._pin_at, n))
        return self.pinned

    def close(self) -> None:
        if self.mm is None:
            return
        if self.pinned:
            from ..ops._ext import kernels
            kernels().host_unregister(self._pin_at)
            self.pinned = False
        self.hdr = self.ctrl = self.push = self.reply = self.state = None
        self._cbuf = None
        try:
            self.mm.close()
        except BufferError:       # a caller still holds a view; the mapping goes with the process
            pass
        self.mm = None


def _pid_alive(pid: int) -> bool:
    """True while ``pid`` runs (a zombie -- dead, not yet reaped -- counts as gone)."""
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except OSError:
        return True


class ShmTransport:
    """Same-host data plane with the parameter server on the CPU (csrc/host/ps_shm.h).

    The PS keeps its shard's fp32 master / momentum / EMA in host memory and a native
    loop (GIL released) serves the gradient pushes straight from a shared-memory segment:
    no GPU work on the PS -- which would time-slice the workers' GPU -- and no Python or
    control-plane message per update.  A worker DMAs its gradient slice into its pinned
    push slot, stamps it and publishes the sequence word; the PS applies it (bitwise
    runtime/torchnet.torch_update), copies the parameters into the worker's reply slot and
    publishes the reply word, on which the worker spins before DMAing them back.  HELLO /
    STATE / DONE / RESET keep the gloo control words; a worker raises its pending flag
    first so the native loop hands over to Python.  A worker notices a dead PS by its pid
    (same host) and recovers as from a lost gloo peer."""
    name = "shm"

    def __init__(self, group, num_ps: int, num_workers: int):
        self.g, self.k, self.W = group, num_ps, num_workers
        self.segs: Dict[int, ShmSegment] = {}
        self.seg: Optional[ShmSegment] = None

    # -- PS side
    def ps_setup(self, ps, is_me: bool) -> None:
        """Collective over the control group: PS j creates its segment, every worker maps
        it, then the names are unlinked."""
        import uuid
        self.fallback = ""
        for j in range(self.k):
            obj = [None]
            if is_me and ps.j == j:
                lay = ShmLayout(ps.fp.total, self.W)
                gen = ps.cluster.gen if ps.cluster is not None else 0
                path = f"/dev/shm/mnistx_ps{j}_{os.getpid()}_{gen}_{uuid.uuid4().hex[:8]}"
                try:
                    self.seg = ShmSegment(path, lay, create=True, gen=gen)
                except OSError as e:      # e.g. ENOSPC: /dev/shm smaller than the segment
                    obj = [{"fallback": f"PS {j}: {lay.total / 2**20:.0f} MiB segment: {e}"}]
                    dist.broadcast_object_list(obj, src=j, group=self.g)
                    self.fallback = obj[0]["fallback"]
                    continue
                self.wd = torch.zeros(ps.fp.total, dtype=torch.float32)
                for e in ps.fp.entries:
                    if e.wd:
                        self.wd[e.off:e.off + e.n] = e.wd
                self.last_seq = np.zeros(self.W, dtype=np.int64)
                self.per_worker = np.array(ps.per_worker, dtype=np.int64)   # survives a rejoin
                self.arrivals = np.zeros(ps.max_steps + 16, dtype=np.int32)
                self.narr = 0
                self.cursor = self.W - 1
                obj = [{"path": path, "n": ps.fp.total}]
            dist.broadcast_object_list(obj, src=j, group=self.g)
            if "fallback" in obj[0]:
                self.fallback = self.fallback or obj[0]["fallback"]
            elif ps is None:
                self.segs[j] = ShmSegment(obj[0]["path"], ShmLayout(obj[0]["n"], self.W), create=False)
        dist.barrier(group=self.g)
        if self.seg is not None:
            os.unlink(self.seg.path)
        if self.fallback:                 # every rank saw the same broadcasts: all fall back together
            self.close()

    def ps_take_grads(self, ps, r: int, expect: int) -> torch.Tensor:
        raise RuntimeError("shm transport: gradients never travel on the control plane")

    def ps_guard(self, r: int, expect: int):
        return None

    def ps_check(self, ps, final: bool = False) -> None:
        pass

    def ps_stage_reply(self, ps, r: int, want_state: bool) -> None:
        i = r - self.k
        self.seg.reply[i].copy_(ps.fp.params)
        if want_state:
            self.seg.state[i][0].copy_(ps.fp.ema)
            self.seg.state[i][1].copy_(ps.fp.mom)

    def ps_after_ctrl(self, ps, r: int, want_state: bool) -> None:
        pass

    def clear_pending(self, r: int) -> None:
        self.seg.ctrl[r - self.k][C_PENDING] = 0

    def native_serve(self, ps, kill_step: int, idle_timeout: float) -> Tuple[int, int]:
        """Run the native loop until a control message is pending (or an error / the kill
        step); the PS's counters follow it."""
        from .. import _host
        o = ps.opt
        fp = ps.fp
        marks = sorted(k for k, v in ps.marks.items() if not v)
        ms = np.array(marks or [-1], dtype=np.int64)
        mt = np.zeros(len(ms), dtype=np.float64)
        ph = np.array([ps.phase_s["idle"], ps.phase_s["apply"], ps.phase_s["reply"]], dtype=np.float64)
        rc, who, gstep, applied, rejected, narr, cursor = _host.ps_shm_serve(
            self.seg.addr, self.seg.lay.native(), fp.params.data_ptr(), fp.mom.data_ptr(), fp.ema.data_ptr(),
            self.wd.data_ptr(),
            [o.lr0, o.decay_rate, float(o.decay_steps), o.momentum, float(o.nesterov), float(o.use_momentum),
             o.ema_max],
            [ps.global_step, ps.max_steps, ps.applied, ps.rejected, kill_step, self.narr, self.cursor],
            self.per_worker.ctypes.data, self.last_seq.ctypes.data, self.arrivals.ctypes.data, len(self.arrivals),
            ms.ctypes.data, mt.ctypes.data, len(marks), ph.ctypes.data, idle_timeout)
        ps.arrivals.extend(int(w) for w in self.arrivals[self.narr:narr])
        self.narr, self.cursor = narr, cursor
        ps.global_step, ps.applied, ps.rejected = gstep, applied, rejected
        ps.per_worker[:] = [int(v) for v in self.per_worker]
        fp.step.fill_(gstep)
        ps.phase_s.update(idle=float(ph[0]), apply=float(ph[1]), reply=float(ph[2]))
        for k, t in zip(marks, mt):
            if t:
                ps.marks[k] = float(t)
        return rc, who

    def close(self) -> None:
        for s in list(self.segs.values()) + ([self.seg] if self.seg is not None else []):
            s.close()
        self.segs.clear()
        self.seg = None

    # -- worker side
    def worker_open(self, w_index: int, ranges) -> None:
        self.wi = w_index
        if getattr(self, "want_pin", False):
            self.pin()

    def pin(self) -> None:
        for s in self.segs.values():
            s.pin(self.wi)

    def worker_before_ctrl(self, j: int, kind: int, grads: Optional[torch.Tensor]) -> None:
        # a control word follows on gloo: the PS's native loop must hand over to Python
        self.segs[j].ctrl[self.wi][C_PENDING] = 1

    def worker_after_ctrl(self, j: int, kind: int, grads: Optional[torch.Tensor]) -> None:
        pass

    def worker_pull(self, j: int, params: torch.Tensor, ema: torch.Tensor, mom: torch.Tensor, state: bool) -> None:
        s = self.segs[j]
        params.copy_(s.reply[self.wi], non_blocking=True)
        if state:
            ema.copy_(s.state[self.wi][0], non_blocking=True)
            mom.copy_(s.state[self.wi][1], non_blocking=True)


def make_transport(name: str, group, num_ps: int, num_workers: int):
    if name == "shm":
        return ShmTransport(group, num_ps, num_workers)
    if name == "ipc":
        return IpcTransport(group, num_ps, num_workers)
    if name in ("host", "gloo"):
        return HostTransport(group, num_ps, num_workers)
    raise ValueError(f"unknown PS transport {name!r} (shm | ipc | host)")


def ipc_reachable(group, num_ps: int, device) -> Tuple[bool, str]:
    """Collective: can every worker GPU map and copy every PS GPU's memory?
    Ranks 0..k-1 are the PS tasks; each rank reports its device, each worker checks
    ``can_device_access_peer`` towards every PS device, and the verdict is agreed."""
    dev = torch.device(device)
    mine = dev.index if dev.type == "cuda" else -1
    devs = [None] * dist.get_world_size(group)
    dist.all_gather_object(devs, mine, group=group)
    me = dist.get_rank(group)
    reason = ""
    if mine < 0 or any(d is None or d < 0 for d in devs):
        reason = "a rank is not on a GPU"
    elif me >= num_ps:
        for j in range(num_ps):
            if devs[j] != mine and not torch.cuda.can_device_access_peer(mine, devs[j]):
                reason = f"worker GPU {mine} has no peer access to PS {j}'s GPU {devs[j]}"
                break
    flag = torch.tensor([0 if reason else 1], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if int(flag) == 0 and not reason:
        reason = "another rank lacks peer access to a PS GPU"
    return bool(int(flag)), reason


def setup_transport(name: str, group, num_ps: int, num_workers: int, ps=None, device=None, log=print):
    """Collective: every PS and worker rank calls this once, in the same order.
    ``ipc`` is downgraded to ``host`` (reason logged) unless every worker can reach
    every PS GPU; ``MNISTX_PS_STRICT=1`` raises instead."""
    if name == "shm":
        import socket
        hosts = [None] * dist.get_world_size(group)
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) > 1:
            if os.environ.get("MNISTX_PS_STRICT", "0") == "1":
                raise RuntimeError("PS shm transport needs every rank on one host")
            log(f"[ps] shm data plane needs one host (ranks on {sorted(set(hosts))}): using the host transport")
            name = "host"
    if name == "ipc":
        ok, why = ipc_reachable(group, num_ps, device if device is not None else torch.device("cpu"))
        if not ok:
            if os.environ.get("MNISTX_PS_STRICT", "0") == "1":
                raise RuntimeError(f"PS ipc transport unavailable: {why}")
            log(f"[ps] ipc data plane unavailable ({why}): using the host transport")
            name = "host"
    tx = make_transport(name, group, num_ps, num_workers)
    tx.ps_setup(ps, ps is not None)
    if getattr(tx, "fallback", ""):
        if os.environ.get("MNISTX_PS_STRICT", "0") == "1":
            raise RuntimeError(f"PS shm transport unavailable: {tx.fallback}")
        log(f"[ps] shm data plane unavailable ({tx.fallback}): using the host transport")
        name = "host"
        tx = make_transport(name, group, num_ps, num_workers)
        tx.ps_setup(ps, ps is not None)
    if name == "shm" and ps is None and device is not None and torch.device(device).type == "cuda":
        tx.want_pin = True        # pinned at worker_open, once the worker's block is known
    return tx


# ---------------------------------------------------------------------------- PS
class ParameterServer:
    def __init__(self, ps_index: int, num_ps: int, num_workers: int, specs, init: Dict[str, torch.Tensor],
                 opt: OptConfig, device, max_steps: int, restore: Optional[Dict[str, np.ndarray]] = None,
                 log=print, transport: str = "", group=None, cluster=None):
        self.j, self.k, self.W = ps_index, num_ps, num_workers
        self.device = torch.device(device)
        transport = transport or default_transport(self.device, max_shard_params(specs, num_ps))
        if transport == "shm":
            self.device = torch.device("cpu")      # the shm PS is a CPU task: the GPUs are the workers'
        self.max_steps = max_steps
        self.group = group
        self.cluster = cluster
        self.transport_name = transport
        full = FlatParams.build(specs, {}, "cpu")
        self.start, self.end, self.names = shard_ranges(full, num_ps)[ps_index]
        mine = [s for s in specs if s[0] in self.names]
        self.fp = FlatParams.build(mine, {n: init[n] for n in self.names}, self.device, pads={})
        self.opt = opt
        self.max_steps = max_steps
        self.log = log
        # T6 fault injection: MNIST_FI_KILL_RANK_AT_STEP=r:k SIGKILLs this PS (rank r) at global step k
        # (attempt 0 only, like train/hooks.FaultInjectionHook, unless MNIST_FI_EVERY_ATTEMPT=1)
        kr = os.environ.get("MNIST_FI_KILL_RANK_AT_STEP", "")
        restarted = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0 or \
            os.environ.get("MNISTX_PS_RESTART", "0") == "1"
        if restarted and os.environ.get("MNIST_FI_EVERY_ATTEMPT", "0") != "1":
            kr = ""
        self._kill = tuple(int(v) for v in kr.split(":")) if ":" in kr else (-1, -1)
        self.global_step = 0
        if restore is not None:
            vals = {n: torch.from_numpy(np.asarray(restore[n])) for n in self.names if n in restore}
            emas = {n: torch.from_numpy(np.asarray(restore[f"{n}/ExponentialMovingAverage"])) for n in self.names
                    if f"{n}/ExponentialMovingAverage" in restore}
            moms = {n: torch.from_numpy(np.asarray(restore[f"{n}/Momentum"])) for n in self.names
                    if f"{n}/Momentum" in restore}
            self.fp.load_state(vals, ema_too=not emas, ema_values=emas, mom_values=moms)
            self.global_step = int(np.asarray(restore.get("global_step", 0)))
        self.fp.step.fill_(self.global_step)
        self.applied = 0
        self.rejected = 0
        self.per_worker = [0] * num_workers
        self.arrivals: List[int] = []            # worker index of every applied push, in order
        self.tx = setup_transport(transport, group, num_ps, num_workers, ps=self,
                                  device=self.device, log=log)
        # global-step values at which serve() records a wall-clock mark (bench.py --mode ps)
        self.marks: Dict[int, float] = {}

    def _apply(self, grads: torch.Tensor, guard=None) -> None:
        fp = self.fp
        if self.device.type == "cuda":
            from ..ops._ext import kernels
            o = self.opt
            gk = {}
            if guard is not None:    # the kernel skips the update if the mailbox stamp != expected
                gk = dict(guard=guard[0], guard_want=guard[1], guard_err=guard[2], guard_id=guard[3])
            kernels().fused_optimizer(fp.params, grads, fp.mom, fp.ema, fp.bf16, fp.segs, fp.step, o.lr0,
                                      o.decay_rate, o.decay_steps, o.momentum, o.nesterov, o.use_momentum, 1.0,
                                      o.ema_max, None, **gk)
        else:
            from ..runtime.torchnet import torch_update
            if grads is not fp.grads:
                fp.grads.copy_(grads)
            torch_update(fp, self.opt, 1.0)
            fp.l2.zero_()

    def _reply(self, r: int, want_state: bool) -> None:
        self.tx.ps_stage_reply(self, r, want_state)
        self.tx.ps_check(self)
        c = torch.zeros(CTRL, dtype=torch.int64)
        c[0] = self.global_step
        c[1] = int(self.global_step >= self.max_steps)
        c[2] = self.applied
        dist.send(c, r, group=self.group, tag=TAG_CTRL)
        self.tx.ps_after_ctrl(self, r, want_state)

    def _rejoin(self, gen: int, r: int) -> None:
        from .cluster import rejoin
        if self.cluster is None or gen <= self.cluster.gen:
            return                        # a stale RESET (this generation is already joined)
        self.log(f"[ps {self.j}] worker {r - self.k} reports a restarted parameter server: "
                 f"rejoining session generation {gen} at global step {self.global_step}")
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        rejoin(self.cluster, gen)
        old_tx = self.tx
        self.tx = setup_transport(self.transport_name, self.group, self.k,
                                  self.W, ps=self, device=self.device, log=self.log)
        if hasattr(old_tx, "close"):
            old_tx.close()
        self.rejoins = getattr(self, "rejoins", 0) + 1

    def serve(self) -> Dict[str, int]:
        """``_serve`` on the PS stream; a ``PushIntegrityError`` is published to the
        store first, so the workers stop instead of waiting for a recovery."""
        try:
            return self._serve_stream()
        except PushIntegrityError as e:
            if self.cluster is not None and self.cluster.store is not None:
                self.cluster.store.set(FATAL_KEY, f"PS {self.j}: {e}")
            raise

    def _serve_stream(self) -> Dict[str, int]:
        """Run until every worker has sent DONE, serving workers in arrival order.

        On a GPU the PS works on a high-priority stream (``MNISTX_PS_PRIORITY=0`` turns
        it off): its apply + reply are a few small kernels and copies that every worker
        is blocked on, while the workers' step graphs are long and can wait -- with
        workers sharing the PS's GPU, a default-priority PS queue waits behind them."""
        if self.device.type != "cuda" or os.environ.get("MNISTX_PS_PRIORITY", "1") == "0":
            return self._serve()
        lo, hi = torch.cuda.Stream.priority_range()
        s = torch.cuda.Stream(device=self.device, priority=hi)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            res = self._serve()
        torch.cuda.current_stream(self.device).wait_stream(s)
        return res

    def _serve(self) -> Dict[str, int]:
        done: set = set()
        self.phase_s = {"idle": 0.0, "apply": 0.0, "reply": 0.0}
        self.log(f"[ps {self.j}] serving {len(self.names)} tensor(s), {self.end - self.start} params, "
                 f"{self.W} worker(s), transport {self.tx.name}")
        t0 = time.perf_counter()
        # host seconds per phase of the serve loop (bench.py --mode ps reports them):
        # idle = blocked waiting for the next worker's control word
        ph = self.phase_s
        clk = time.perf_counter
        c = torch.zeros(CTRL, dtype=torch.int64)
        while len(done) < self.W:
            if self.tx.name == "shm":
                # gradient pushes are served natively until a worker announces a control word
                kill = self._kill[1] if self._kill[0] == dist.get_rank() else -1
                rc, who = self.tx.native_serve(self, kill, float(os.environ.get("MNISTX_PS_IDLE_TIMEOUT", "1800")))
                if rc == PS_BAD_STAMP:
                    raise PushIntegrityError(f"PS {self.j}: push from worker {who} failed its sequence-stamp check "
                                             f"(stale or torn push slot): gradient not applied")
                if rc == PS_KILL:
                    self.log(f"[ps {self.j}] fault injection: SIGKILL at global step {self.global_step}")
                    sys.stdout.flush()
                    os.kill(os.getpid(), signal.SIGKILL)
                if rc == PS_IDLE_TIMEOUT:
                    raise RuntimeError(f"PS {self.j}: no push or control word for MNISTX_PS_IDLE_TIMEOUT s")
            ta = clk()
            r = dist.recv(c, group=self.group, tag=TAG_CTRL)     # any source: the next worker to arrive
            tb = clk()
            ph["idle"] += tb - ta
            if self.tx.name == "shm":
                self.tx.clear_pending(r)
            kind, want_state, wstep = int(c[0]), bool(c[1]), int(c[2])
            if kind == DONE:
                done.add(r)
                continue
            if kind == RESET:             # another PS restarted: rejoin at the announced generation
                self._rejoin(int(c[3]), r)
                continue
            if kind == GRAD:
                g = self.tx.ps_take_grads(self, r, wstep)
                if self.global_step < self.max_steps:
                    self._apply(g, self.tx.ps_guard(r, wstep))
                    self.global_step += 1
                    self.fp.step.fill_(self.global_step)
                    self.applied += 1
                    self.per_worker[r - self.k] += 1
                    self.arrivals.append(r - self.k)
                else:
                    self.rejected += 1            # in flight past the stop point: answered, not applied
                if self._kill[0] == dist.get_rank() and self.global_step >= self._kill[1]:
                    self.log(f"[ps {self.j}] fault injection: SIGKILL at global step {self.global_step}")
                    sys.stdout.flush()
                    os.kill(os.getpid(), signal.SIGKILL)
            tc = clk()
            ph["apply"] += tc - tb
            self._reply(r, want_state)
            ph["reply"] += clk() - tc
            if self.global_step in self.marks and not self.marks[self.global_step]:
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                self.marks[self.global_step] = time.perf_counter()
        self.tx.ps_check(self, final=True)
        if hasattr(self.tx, "close"):
            self.tx.close()
        dt = time.perf_counter() - t0
        self.log(f"[ps {self.j}] done: applied {self.applied} update(s), per worker {self.per_worker}, "
                 f"rejected {self.rejected}, global_step {self.global_step}, {self.applied / max(dt, 1e-9):.1f} "
                 f"updates/s")
        return {"applied": self.applied, "global_step": self.global_step, "per_worker": list(self.per_worker),
                "seconds": dt, "phase_s": dict(ph)}


# ---------------------------------------------------------------------------- worker
class PSClient:
    """Worker side: push gradients / pull parameters of every PS shard."""

    def __init__(self, net, num_ps: int, num_workers: int, worker_index: int, group=None, transport: str = "",
                 cluster=None, log=print):
        self.net = net
        self.k, self.W, self.wi = num_ps, num_workers, worker_index
        self.group = group
        self.cluster = cluster            # PS-mode Cluster (store + generation): enables session recovery
        self.log = log
        self.transport_name = transport
        self.recoveries = 0
        # shm data plane: longest wait for a reply word before the PS counts as lost
        # (MNISTX_PS_REPLY_TIMEOUT; default the cluster's collective timeout, else 600 s)
        to = getattr(cluster, "timeout", None) if cluster is not None else None
        self.reply_timeout_s = float(os.environ.get(
            "MNISTX_PS_REPLY_TIMEOUT", to.total_seconds() if hasattr(to, "total_seconds") else 600.0))
        self.ranges = shard_ranges(net.fp, num_ps)
        self.global_step = 0
        self.stop = False
        self._open_transport()
        self.local_step = 0
        self._pending: set = set()         # PS tasks holding this exchange's control word, reply not taken
        self._pending_state = False
        self._corrupt = corrupt_push_at()
        # data-plane accounting (bench.py --mode ps): host seconds and bytes of the GRAD
        # exchanges; push = stage + copy/send + announce to every PS, pull = wait for the
        # replies + copy the parameters back (so it includes the PS's service time)
        self.comm = {"push_s": 0.0, "reply_wait_s": 0.0, "push_bytes": 0, "pull_bytes": 0, "msgs": 0}
        self._pull_ev: List[Tuple] = []      # (start, end) CUDA events around the pull copies

    def _open_transport(self) -> None:
        """Collective with every PS (setup_transport) -- at start and after a rejoin."""
        dev = self.net.fp.params.device
        old = getattr(self, "tx", None)
        if old is not None and hasattr(old, "close"):
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)     # no copy of ours still reads the old mapping
            old.close()
        self.tx = setup_transport(self.transport_name or default_transport(dev, max_shard_params(self.net.fp, self.k)),
                                  self.group, self.k, self.W,
                                  device=dev)
        self.tx.worker_open(self.wi, self.ranges)
        # one stamped push slot per PS shard: the slice + its int64 sequence stamp, sent as ONE message
        # (host) / ONE peer copy (ipc)
        stage_dev = dev if self.tx.name == "ipc" else torch.device("cpu")
        self.slots = [torch.zeros(slot_len(b - a), dtype=torch.float32, device=stage_dev) for a, b, _ in self.ranges]

    def recover(self, err: BaseException, timeout_s: Optional[float] = None) -> None:
        """Session recreation after a parameter server failed (module docstring): wait
        for the restarted PS's generation, RESET the survivors, rejoin, re-open the data
        plane.  Re-raises ``err`` when there is no store or no PS comes back in time."""
        from .cluster import current_gen, rejoin
        cl = self.cluster
        if cl is None or cl.store is None:
            raise err
        self.log(f"[worker {self.wi}] An error was raised ({type(err).__name__}: {str(err).splitlines()[0][:160]}). "
                 f"This may be due to a preemption in a connected parameter server. The current session "
                 f"will be recreated.")
        if timeout_s is None:
            timeout_s = float(os.environ.get("MNISTX_PS_RECOVERY_TIMEOUT", "300"))
        t_end = time.time() + timeout_s

        def fatal() -> bool:               # the PS failed on purpose (e.g. a rejected push): no recovery
            if cl.store.check([FATAL_KEY]):
                self.log(f"[worker {self.wi}] parameter server reported a fatal error: "
                         f"{cl.store.get(FATAL_KEY).decode()[:300]}")
                return True
            return False

        # checked before AND after the generation compare: a restarted PS that opened the next
        # generation must not pull the survivors past a rejected push
        if fatal():
            raise err
        gen = current_gen(cl)
        while gen <= cl.gen:
            if fatal():
                raise err
            if time.time() > t_end:
                self.log(f"[worker {self.wi}] no parameter server came back within {timeout_s:.0f} s")
                raise err
            time.sleep(0.05)
            gen = current_gen(cl)
        if fatal():
            raise err
        # a surviving PS that took this exchange's control word is blocked sending its reply
        # (gloo sends complete only when matched): take those replies on the old group first
        fp = self.net.fp
        for j in sorted(self._pending):
            a, b, _ = self.ranges[j]
            try:
                dist.recv(torch.zeros(CTRL, dtype=torch.int64), j, group=self.group, tag=TAG_CTRL)
                self.tx.worker_pull(j, fp.params[a:b], fp.ema[a:b], fp.mom[a:b], self._pending_state)
            except Exception:
                pass
        self._pending.clear()
        for j in range(self.k):            # best effort: the dead PS is not there to hear it
            c = torch.zeros(CTRL, dtype=torch.int64)
            c[0], c[3] = RESET, gen
            try:
                self.tx.worker_before_ctrl(j, RESET, None)
                dist.send(c, j, group=self.group, tag=TAG_CTRL)
            except Exception:
                pass
        if self.net.fp.params.is_cuda:
            torch.cuda.synchronize(self.net.fp.params.device)
        rejoin(cl, gen)
        self._open_transport()
        self.recoveries += 1
        self.log(f"[worker {self.wi}] session recreated: joined generation {gen}")

    def _stage(self, j: int, a: int, b: int) -> torch.Tensor:
        slot = self.slots[j]
        slot[:b - a].copy_(self.net.fp.grads[a:b])
        stamp = self.local_step
        if self._corrupt == (self.wi, self.local_step):
            stamp += 1000                                   # fault injection: a stale-looking push
        stamp_view(slot).fill_(stamp)
        return slot

    def _exchange(self, kind: int, want_state: bool = False) -> None:
        """One exchange with every PS; on a control-plane failure (a PS died) the session
        is recreated and the exchange re-sent -- as a pull only to the PS tasks that
        already took this push.  Any other error (HIP, torch, a rejected push) is re-raised
        at once instead of waiting for a recovery that cannot come."""
        took: set = set()
        while True:
            try:
                return self._exchange_once(kind, want_state, took)
            except RuntimeError as e:
                if not is_peer_loss(e):
                    raise
                self.recover(e)

    def _exchange_once(self, kind: int, want_state: bool, took: set) -> None:
        if kind == GRAD and self.tx.name == "shm" and not took:
            return self._exchange_shm(took)
        fp = self.net.fp
        t0 = time.perf_counter()
        # announce to every PS first (they work in parallel), then collect the replies
        for j, (a, b, _) in enumerate(self.ranges):
            kj = HELLO if (kind == GRAD and j in took) else kind
            g = self._stage(j, a, b) if kj == GRAD else None
            self.tx.worker_before_ctrl(j, kj, g)
            c = torch.zeros(CTRL, dtype=torch.int64)
            c[0], c[1], c[2] = kj, int(want_state), self.local_step
            dist.send(c, j, group=self.group, tag=TAG_CTRL)
            self._pending.add(j)
            self._pending_state = want_state
            self.tx.worker_after_ctrl(j, kj, g)
            if kj == GRAD:
                took.add(j)
        t1 = time.perf_counter()
        wait = 0.0
        evs = None
        if kind == GRAD and fp.params.is_cuda and len(self._pull_ev) < 4096:
            evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for j, (a, b, _) in enumerate(self.ranges):
            r = torch.zeros(CTRL, dtype=torch.int64)
            tw = time.perf_counter()
            dist.recv(r, j, group=self.group, tag=TAG_CTRL)
            wait += time.perf_counter() - tw
            if evs is not None and j == 0:
                evs[0].record()
            self.tx.worker_pull(j, fp.params[a:b], fp.ema[a:b], fp.mom[a:b], want_state)
            self._pending.discard(j)
            if j == 0:
                self.global_step = int(r[0])
                self.stop = bool(r[1])
        if kind == GRAD:
            if evs is not None:
                evs[1].record()
                self._pull_ev.append(evs)
            c = self.comm
            c["push_s"] += t1 - t0
            c["reply_wait_s"] += wait
            c["push_bytes"] += sum(sl.numel() * 4 for sl in self.slots)
            c["pull_bytes"] += fp.total * 4
            c["msgs"] += 1
        fp.step.fill_(self.global_step)
        fp.refresh_bf16()

    def _exchange_shm(self, took: set) -> None:
        """GRAD on the shm data plane: DMA the gradient slices into the push slots, stamp and
        publish them, spin on the reply words, DMA the parameters back.  No control message:
        the PS's native loop (csrc/host/ps_shm.h) serves the push."""
        fp = self.net.fp
        tx = self.tx
        wi = tx.wi
        t0 = time.perf_counter()
        for j, (a, b, _) in enumerate(self.ranges):
            tx.segs[j].push[wi][:b - a].copy_(fp.grads[a:b], non_blocking=True)
        if fp.grads.is_cuda:
            torch.cuda.current_stream(fp.grads.device).synchronize()    # the slices are in the slots
        stamp = self.local_step
        if self._corrupt == (self.wi, self.local_step):
            stamp += 1000                                   # fault injection: a stale-looking push
        for j in range(self.k):
            seg = tx.segs[j]
            stamp_view(seg.push[wi]).fill_(stamp)
            seg.ctrl[wi][C_PUSH_SEQ] = self.local_step      # publish (x86 stores stay in order)
            took.add(j)
        t1 = time.perf_counter()
        wait = 0.0
        evs = None
        if fp.params.is_cuda and len(self._pull_ev) < 4096:
            evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for j, (a, b, _) in enumerate(self.ranges):
            seg = tx.segs[j]
            ctrl = seg.ctrl[wi]
            tw = time.perf_counter()
            spins = 0
            while int(ctrl[C_REPLY_SEQ]) != self.local_step:
                spins += 1
                if spins & 0x3ff == 0:
                    if not _pid_alive(seg.ps_pid):
                        raise PeerLostError(f"parameter server {j} (pid {seg.ps_pid}) is gone")
                    # a PS that is alive but stuck (e.g. blocked in a control recv from a
                    # worker that died between its pending flag and its message): bounded by
                    # the reply deadline, then recovered like a lost peer
                    if time.perf_counter() - tw > self.reply_timeout_s:
                        raise PeerLostError(f"parameter server {j} (pid {seg.ps_pid}) sent no reply within "
                                            f"{self.reply_timeout_s:.0f} s")
                    # back off once the reply is clearly not imminent (a PS apply is < 10 ms)
                    time.sleep(0 if spins < (1 << 16) else 50e-6)
            wait += time.perf_counter() - tw
            if evs is not None and j == 0:
                evs[0].record()
            fp.params[a:b].copy_(seg.reply[wi][:b - a], non_blocking=True)
            if j == 0:
                self.global_step = int(ctrl[C_REPLY_GSTEP])
                self.stop = bool(ctrl[C_REPLY_STOP])
        if evs is not None:
            evs[1].record()
            self._pull_ev.append(evs)
        c = self.comm
        c["push_s"] += t1 - t0
        c["reply_wait_s"] += wait
        c["push_bytes"] += fp.total * 4 + 8 * self.k      # slices + their stamps
        c["pull_bytes"] += fp.total * 4
        c["msgs"] += 1
        fp.step.fill_(self.global_step)
        fp.refresh_bf16()

    def comm_summary(self) -> Dict[str, float]:
        """Per GRAD message: push host us (stage + copy + announce) and its GB/s, the wait
        for the PS reply, the pull copy's device us (events) and its GB/s."""
        c = self.comm
        n = max(1, c["msgs"])
        if self._pull_ev:
            torch.cuda.synchronize()
            pull_ms = sum(a.elapsed_time(b) for a, b in self._pull_ev) / len(self._pull_ev)
        else:
            pull_ms = float("nan")
        push_us = c["push_s"] / n * 1e6
        pull_us = pull_ms * 1e3
        return {"msgs": c["msgs"], "push_us": round(push_us, 1),
                "push_GBps": round(c["push_bytes"] / n / max(push_us, 1e-9) / 1e3, 3),
                "reply_wait_us": round(c["reply_wait_s"] / n * 1e6, 1),
                "pull_us": round(pull_us, 1),
                "pull_GBps": round(c["pull_bytes"] / n / max(pull_us, 1e-9) / 1e3, 3) if pull_us == pull_us else None,
                "bytes_per_push": c["push_bytes"] // n, "bytes_per_pull": c["pull_bytes"] // n}

    def hello(self) -> None:
        self._exchange(HELLO)

    def push_pull(self) -> None:
        self.local_step += 1
        self._exchange(GRAD)

    def fetch_state(self) -> None:
        self._exchange(STATE, want_state=True)

    def done(self) -> None:
        """DONE to every PS, through the same recovery as an exchange: a PS that dies
        while the workers shut down is relaunched and still hears every DONE.  The
        store's done key (which makes a relaunched PS give up in-place recovery) is set
        only once every PS has been told: until then this worker can still rejoin."""
        told: set = set()
        while True:
            try:
                for j in range(self.k):
                    if j in told:
                        continue
                    c = torch.zeros(CTRL, dtype=torch.int64)
                    c[0] = DONE
                    self.tx.worker_before_ctrl(j, DONE, None)
                    dist.send(c, j, group=self.group, tag=TAG_CTRL)
                    told.add(j)
                if self.cluster is not None and self.cluster.store is not None:
                    from .cluster import DONE_KEY
                    self.cluster.store.set(f"{DONE_KEY}/rank{dist.get_rank()}", "1")
                return
            except RuntimeError as e:
                if not is_peer_loss(e):
                    raise
                self.recover(e)
                told.clear()              # a new generation: every PS (re)counts DONE from scratch

    def shard_of(self) -> Dict[str, int]:
        out = {}
        for j, (_, _, names) in enumerate(self.ranges):
            for n in names:
                out[n] = j
                out[f"{n}/ExponentialMovingAverage"] = j
                out[f"{n}/Momentum"] = j
        return out


def weight_l2_into(fp: FlatParams) -> None:
    """sum(w^2) of every weight-decayed tensor into the per-tensor L2 slots that
    ``finalize`` turns into the ``*/weight_loss`` terms (``mnist_input.py:112-114``);
    PS workers run no local optimizer, which is what fills them otherwise."""
    if not fp.wd_entries:
        return
    with torch.no_grad():
        sq = torch.stack([fp.param_view(e.name).float().square().sum() for e in fp.wd_entries])
        fp.l2[:len(fp.wd_entries)].copy_(sq)


class PSWorkerReplica:
    """A worker replica in PS mode: same executor/input pipeline as ``Replica``
    but no local optimizer — gradients go to the PS tasks, fresh parameters
    and the shared global step come back."""

    def __init__(self, base, num_ps: int, num_workers: int, worker_index: int, group=None, transport: str = "",
                 cluster=None, log=print):
        self.base = base                  # a train.replica.Replica (built with world=1 semantics)
        self.net = base.net
        self.spec = base.spec
        self.client = PSClient(base.net, num_ps, num_workers, worker_index, group=group, transport=transport,
                               cluster=cluster, log=log)
        self.world = 1
        self.examples_per_step = base.B
        self.device = base.device
        self.loader = base.loader
        self.eval_ds = base.eval_ds
        self.dp = base.dp
        # T6-style slow worker (async test): MNIST_FI_SLOW_WORKER=task:seconds sleeps every step
        sw = os.environ.get("MNIST_FI_SLOW_WORKER", "")
        self._sleep = float(sw.split(":")[1]) if ":" in sw and int(sw.split(":")[0]) == worker_index else 0.0
        self.client.hello()
        self._cluster, self._nw = cluster, num_workers
        self._started = False

    def _start_barrier(self) -> None:
        """MNISTX_PS_START_BARRIER=1: before its FIRST push (its first step computed, graphs
        captured) every worker waits on the cluster store until all have got there -- for runs
        that must see every worker contribute (tests); async PS semantics are unchanged after
        the start.  Without it a worker whose start-up is slower (the chief's graph capture and
        initial checkpoint) can find a short job already finished, as TF's workers can."""
        self._started = True
        cl = self._cluster
        if os.environ.get("MNISTX_PS_START_BARRIER", "0") != "1" or cl is None or cl.store is None:
            return
        key = f"mnistx/started/gen{cl.gen}"
        cl.store.add(key, 1)
        t_end = time.time() + 300
        while int(cl.store.add(key, 0)) < self._nw and time.time() < t_end:
            time.sleep(0.005)

    @property
    def global_step(self) -> int:
        return self.client.global_step

    def sync_step_from_device(self) -> None:
        pass

    def _compute(self) -> None:
        """forward + CE + backward + L2 terms + stats: no communication, so one hipGraph."""
        net = self.net
        net.forward(defer_head=True)
        net.loss_and_grad()
        net.backward()
        weight_l2_into(net.fp)
        net.finalize(net.B, increment=False)

    _graph = None

    def step(self) -> None:
        self.loader.next()
        if getattr(self.base, "use_graph", False):
            if self._graph is None:
                from ..runtime.graph import StepGraph
                self._graph = StepGraph(self._compute, warmup=1)   # the warm-up computes this step
            else:
                self._graph.replay()
        else:
            self._compute()
        if self._sleep:
            time.sleep(self._sleep)
        if not self._started:
            self._start_barrier()
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
