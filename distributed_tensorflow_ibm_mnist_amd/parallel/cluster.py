"""Cluster setup — the equivalent of ``setup_distribute()`` (``main.py:42-68``).

Modes:

* **local** — no ``--worker_hosts`` and no torchrun environment: one process,
  the reference's ``create_local_server`` path (``main.py:63-66``; task_id forced 0);
* **dp** — torchrun env (``WORLD_SIZE`` > 1), or ``--worker_hosts`` without
  ``--ps_hosts`` (the reference would silently train unshared per-worker copies,
  Q10; we treat it as synchronous data parallel);
* **ps** — ``--ps_hosts`` + ``--worker_hosts`` + ``--job_name`` + ``--task_id``:
  1..k parameter-server ranks followed by the workers
  (rank(ps k) = k, rank(worker i) = num_ps + i), a gloo control group over a
  TCPStore hosted by the CHIEF (worker 0's ``host:port``), so the store outlives a
  parameter server: a restarted PS opens the next *session generation* (a fresh
  ``PrefixStore`` namespace) and the surviving processes rejoin it in place
  (``rejoin`` below; ``MonitoredTrainingSession``'s session recreation,
  ``/root/reference/main.py:140-146`` [TF1-lib]).

Device: one process per GPU; ``LOCAL_RANK`` if set, else rank modulo the
visible device count.
"""
from __future__ import annotations

import dataclasses
import datetime
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


@dataclasses.dataclass
class Cluster:
    mode: str                       # local | dp | ps
    job_name: str
    task_id: int
    ps_hosts: List[str]
    worker_hosts: List[str]
    rank: int = 0
    world: int = 1
    num_ps: int = 0
    num_workers: int = 1
    master: str = ""
    device: Optional[torch.device] = None
    backend: str = ""
    transport: str = ""             # PS-mode data plane (shm | ipc | host)
    store: Optional[object] = None  # PS mode: the chief-hosted TCPStore (survives PS restarts)
    gen: int = 0                    # PS mode: session generation of the current control group
    timeout: Optional[datetime.timedelta] = None

    @property
    def is_chief(self) -> bool:
        """main.py:73: the chief is worker task 0."""
        return self.job_name != "ps" and self.task_id == 0

    @property
    def spec(self) -> Dict[str, List[str]]:
        d: Dict[str, List[str]] = {}
        if self.worker_hosts:
            d["worker"] = self.worker_hosts
        if self.ps_hosts:
            d["ps"] = self.ps_hosts
        return d


def _split(s: Optional[str]) -> List[str]:
    return [h.strip() for h in (s or "").split(",") if h.strip()]


def _norm_host(hp: str) -> str:
    host, _, port = hp.rpartition(":")
    if host in ("localhost", "", "0.0.0.0"):
        host = "127.0.0.1"
    return f"{host}:{port}"


def pick_device(rank: int, want_gpu: bool) -> torch.device:
    if not want_gpu or not torch.cuda.is_available():
        return torch.device("cpu")
    lr = os.environ.get("LOCAL_RANK")
    n = torch.cuda.device_count()
    idx = int(lr) if lr is not None else rank
    return torch.device("cuda", idx % max(n, 1))   # several ranks may share a GPU (gloo rehearsal)


def _attempt_store(rank: int, world: int, timeout: datetime.timedelta):
    """The env:// (torchrun) store, namespaced by the elastic restart attempt.

    torchrun keeps ONE store across ``--max-restarts`` attempts, and a fresh
    process numbers its process groups from 0 again, so without a namespace the
    restarted ranks can read the previous attempt's keys -- gloo pair addresses
    of dead processes ("Connection refused"), or a stale RCCL unique id (a hang)."""
    store, _, _ = next(dist.rendezvous("env://", rank, world, timeout=timeout))
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    return dist.PrefixStore(f"mnistx/attempt{attempt}", store)


GEN_KEY = "mnistx/gen"
DONE_KEY = "mnistx/done"        # + /rank<r>: a PS-mode worker that has started its shutdown
EXIT_NO_INPLACE = 87            # a restarted PS that cannot rejoin in place (supervisor.py: whole-job restart)


def _gen_prefix(gen: int) -> str:
    return f"mnistx/gen{gen}"


def _ps_store(cl: "Cluster", to: datetime.timedelta):
    """PS mode: the TCPStore lives in the chief (worker 0), which every recovery needs
    alive anyway; parameter servers and the other workers are clients."""
    host, _, port = cl.master.rpartition(":")
    is_master = cl.job_name == "worker" and cl.task_id == 0
    return dist.TCPStore(host, int(port), is_master=is_master, timeout=to, wait_for_workers=False)


def rejoin(cl: "Cluster", gen: int) -> None:
    """Leave the current control group and join session generation ``gen`` (every
    rank of the job does, the restarted PS included); blocks until all have."""
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:                       # a dead peer's pairs may not close cleanly
            pass
    dist.init_process_group("gloo", store=dist.PrefixStore(_gen_prefix(gen), cl.store), rank=cl.rank,
                            world_size=cl.world, timeout=cl.timeout)
    cl.gen = gen


def current_gen(cl: "Cluster") -> int:
    return int(cl.store.add(GEN_KEY, 0))


def setup_distribute(job_name: str = "", ps_hosts: str = "", worker_hosts: str = "", task_id: int = 0,
                     want_gpu: bool = True, timeout_s: float = 600.0, log=print,
                     ps_backend: str = "", dp_backend: str = "", ps_shard_params: int = 0) -> Cluster:
    ps, workers = _split(ps_hosts), _split(worker_hosts)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    to = datetime.timedelta(seconds=timeout_s)
    if workers:
        cl = Cluster("ps" if ps else "dp", job_name or "worker", int(task_id), ps, workers)
        log("Cluster spec: ", cl.spec)                               # main.py:57
        if cl.mode == "ps":
            if cl.job_name not in ("ps", "worker"):
                raise ValueError('job_name must be "ps" or "worker"')
            cl.num_ps, cl.num_workers = len(ps), len(workers)
            n = len(ps) if cl.job_name == "ps" else len(workers)
            if not 0 <= cl.task_id < n:
                raise ValueError(f"task_id {cl.task_id} out of range for job {cl.job_name} ({n} tasks)")
            cl.rank = cl.task_id if cl.job_name == "ps" else len(ps) + cl.task_id
            cl.world = len(ps) + len(workers)
            cl.master = _norm_host(workers[0])
        else:
            if cl.job_name == "ps":
                raise ValueError("job_name=ps without --ps_hosts")
            cl.num_workers = len(workers)
            cl.rank, cl.world = cl.task_id, len(workers)
            cl.master = _norm_host(workers[0])
        cl.device = pick_device(cl.rank, want_gpu)
        cl.backend = "nccl" if cl.device.type == "cuda" else "gloo"
        if cl.mode == "dp" and dp_backend:
            cl.backend = dp_backend
        if cl.mode == "ps":
            # PS mode: the process group is the gloo control plane; gradients and
            # parameters move on the PS data plane (parallel/ps.py): a CPU PS serving a
            # shared-memory segment natively ("shm", one host; default on GPU for shards up
            # to 1 M parameters), xGMI peer copies into a GPU PS ("ipc", default on GPU for
            # larger shards: ps.default_transport) or gloo messages staged through host ("host").
            cl.backend = "gloo"
            t = {"": "", "gloo": "host", "host": "host", "ipc": "ipc", "shm": "shm"}.get(ps_backend)
            if t is None:
                raise ValueError(f"--ps_backend={ps_backend!r}: expected shm | ipc | host (gloo)")
            from .ps import default_transport
            cl.transport = t or default_transport(cl.device, ps_shard_params)
            if cl.transport == "shm" and cl.job_name == "ps":
                cl.device = torch.device("cpu")    # the shm PS is a CPU task: it never opens a GPU
        if cl.device.type == "cuda":
            torch.cuda.set_device(cl.device)
        cl.timeout = to
        if cl.mode == "ps":
            cl.store = _ps_store(cl, to)
            gen = 0
            if cl.job_name == "ps" and cl.store.add(f"mnistx/ps{cl.task_id}/starts", 1) > 1:
                # a restarted parameter server: open the next session generation; the
                # surviving workers / PS tasks notice the failure and rejoin it -- unless a
                # worker has already finished (it can never rejoin, so the new generation
                # would wait for it until the collective timeout): exit with EXIT_NO_INPLACE
                # and let the supervisor restart the whole job from the checkpoint instead
                gone = [r for r in range(cl.num_ps, cl.world) if cl.store.check([f"{DONE_KEY}/rank{r}"])]
                if gone:
                    log(f"[ps {cl.task_id}] restarted after rank(s) {gone} finished: no in-place recovery")
                    raise SystemExit(EXIT_NO_INPLACE)
                gen = int(cl.store.add(GEN_KEY, 1))
                log(f"[ps {cl.task_id}] restarted: opening session generation {gen}")
            rejoin(cl, gen)
            return cl
        kw = {"device_id": cl.device} if cl.backend == "nccl" else {}
        dist.init_process_group(cl.backend, init_method=f"tcp://{cl.master}", rank=cl.rank, world_size=cl.world,
                                timeout=to, **kw)
        return cl
    if env_world > 1:
        rank = int(os.environ.get("RANK", "0"))
        cl = Cluster("dp", "worker", rank, [], [], rank=rank, world=env_world, num_workers=env_world)
        cl.device = pick_device(rank, want_gpu)
        cl.backend = dp_backend or ("nccl" if cl.device.type == "cuda" else "gloo")
        if cl.device.type == "cuda":
            torch.cuda.set_device(cl.device)
        kw = {"device_id": cl.device} if cl.backend == "nccl" else {}
        dist.init_process_group(cl.backend, timeout=to, store=_attempt_store(rank, env_world, to),
                                rank=rank, world_size=env_world, **kw)
        return cl
    # local server (main.py:63-66): single process, task 0
    cl = Cluster("local", job_name or "worker", 0, [], [])
    cl.device = pick_device(0, want_gpu)
    if cl.device.type == "cuda":
        torch.cuda.set_device(cl.device)
    return cl


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
