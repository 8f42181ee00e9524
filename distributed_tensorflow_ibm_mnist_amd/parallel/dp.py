"""Synchronous data parallelism: RCCL all-reduce of gradient buckets over xGMI.

The reference has no synchronous DP (no ``SyncReplicasOptimizer``,
``mnist_input.py:261-264``); BASELINE's north star adds it.

Design for MI355X:
* one process per GPU, ``torch.distributed`` with the ``nccl`` backend (= RCCL);
* gradients live in ONE flat fp32 buffer (``runtime/params.py``) so buckets are
  plain contiguous slices — no packing copies;
* buckets are cut at layer boundaries in *backward* order and launched from the
  executor's grads-ready hook with ``async_op=True``: RCCL runs on its own HIP
  stream after an event wait on the compute stream, so the all-reduce of a
  finished bucket overlaps the backward of the layers below it.  For the
  reference CNN the 12.85 MB ``local3/weights`` gradient (92.7 % of the bytes)
  is ready after local3's wgrad and overlaps the whole conv backward;
* every bucket except the last overlaps the backward still to run, so the cap is
  small (bench/main default 0.125 MB): LeNet-5's 236 KB fc bucket is reduced
  while conv2/conv1 backward (~80 % of backward time) runs, leaving a 10 KB
  latency-bound conv bucket at the end; the reference CNN gets [softmax+local4]
  0.8 MB, [local3] 12.85 MB (ring per-link bound on xGMI: ~2·7/8·S / 153 GB/s
  ≈ 150 µs), [conv2], [conv1];
* where the local3 all-reduce runs, reference CNN at the BASELINE batch
  (B=16384/GPU, ``profiles/r3/dp_overlap/refcnn_b16384_step_timeline.txt``,
  rocprofv3 kernel trace of a 2.47 ms step): the bucket is ready at 1.16 ms
  (after the local3 wgrad GEMM + split-K reduce); 1.2 ms of backward follows.
  The first 650 µs of it leave room for the RCCL kernel on every CU -- local3
  dgrad is a 1600-workgroup GEMM (2 per CU, retiring in waves), lrn_pool_bwd
  uses no LDS, conv2 wgrad is one 69 KB-LDS workgroup per CU -- and only then
  does the conv2 dgrad halo kernel take 148 KB of each CU's 160 KB LDS for
  315 µs.  A ~150 µs ring all-reduce therefore fits before the one kernel that
  could lock it out, so no compute grid is capped.  Not yet measured: the ring
  kernel's actual CU share on a multi-GPU node (a one-rank RCCL group issues no
  kernel, so the one-GPU trace pins when the bucket is ready, not the contention);
* split-K weight-gradient reduces of a bucket's layers are flushed as ONE
  multi-tensor launch just before its all-reduce (``HipNet.hook_layers``);
* ``work.wait()`` only makes the compute stream wait (no host block); the
  gradient average is folded into the fused optimizer (grad_scale = 1/world).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..models.spec import Conv, Dense


@dataclasses.dataclass
class Bucket:
    start: int
    end: int
    layers: List[int]

    @property
    def nbytes(self) -> int:
        return (self.end - self.start) * 4


def plan_buckets(net, cap_bytes: int) -> List[Bucket]:
    fp = net.fp
    spec = net.spec
    order = [i for i, L in enumerate(spec.layers) if isinstance(L, (Conv, Dense))]
    rng: Dict[int, tuple] = {}
    for i in order:
        name = spec.layers[i].name
        w, b = fp.by_name[f"{name}/weights"], fp.by_name[f"{name}/biases"]
        rng[i] = (min(w.off, b.off), max(w.off + w.n, b.off + b.n))
    buckets: List[Bucket] = []
    cur: Optional[Bucket] = None
    for k, i in enumerate(reversed(order)):
        s, e = rng[i]
        if cur is None:
            cur = Bucket(s, e, [i])
        else:
            assert e == cur.start, "parameter layout must be contiguous in layer order"
            cur.start = s
            cur.layers.append(i)
        if cur.nbytes >= cap_bytes or k == len(order) - 1:
            buckets.append(cur)
            cur = None
    return buckets


class DataParallel:
    def __init__(self, net, group=None, bucket_cap_mb: float = 1.0, overlap: bool = True,
                 world: Optional[int] = None, force_collectives: bool = False):
        """``force_collectives``: issue the bucket all-reduces even with one rank (a
        one-GPU rehearsal of the RCCL path, e.g. hipGraph capture of the DP step)."""
        self.net = net
        self.group = group
        if world is None:
            world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.world = world
        self.active = world > 1 or force_collectives
        self.buckets = plan_buckets(net, int(bucket_cap_mb * (1 << 20)))
        self.trigger = {b.layers[-1]: b for b in self.buckets}
        self.pending: list = []
        self.overlap = overlap
        # comm_enabled = False skips the all-reduces (replicas drift apart): only for
        # measuring how much of a step the collectives leave exposed (bench.py)
        self.comm_enabled = True
        if self.active:
            net.grad_ready_hooks.append(self._hook)
            if hasattr(net, "hook_layers"):       # reduced gradients are needed only at bucket triggers
                net.hook_layers = set(self.trigger)

    def _hook(self, layer_index: int) -> None:
        if not self.overlap or not self.comm_enabled:
            return
        b = self.trigger.get(layer_index)
        if b is not None:
            self.pending.append(dist.all_reduce(self.net.fp.grads[b.start:b.end], group=self.group, async_op=True))

    def sync_grads(self) -> None:
        if not self.active or not self.comm_enabled:
            return
        if not self.overlap:
            for b in self.buckets:
                self.pending.append(dist.all_reduce(self.net.fp.grads[b.start:b.end], group=self.group,
                                                    async_op=True))
        for w in self.pending:
            w.wait()
        self.pending.clear()

    def train_step(self, timer=None) -> None:
        """One DP step; ``timer`` (runtime/timers.PhaseTimer) records phase boundaries."""
        net = self.net
        if timer is None:
            net.forward(defer_head=True)
            net.loss_and_grad()
            net.backward()
            self.sync_grads()
            net.update(grad_scale=1.0 / self.world)
            return
        timer.mark("start")
        net.forward(defer_head=True)
        timer.mark("forward")
        net.loss_and_grad()
        timer.mark("loss")
        net.backward()
        timer.mark("backward")
        self.sync_grads()
        timer.mark("allreduce_wait")
        net.update(grad_scale=1.0 / self.world)
        timer.mark("update")
        timer.close()

    def measure_buckets(self, reps: int = 20, warmup: int = 3) -> List[Dict[str, float]]:
        """Each gradient bucket's all-reduce ALONE (outside any step): mean time of
        ``reps`` back-to-back all-reduces of a scratch copy of the bucket, host-timed
        between device synchronisations and a barrier; ring bus bandwidth
        busbw = 2(N-1)/N * bytes / t (the per-link figure to compare with xGMI's
        ~153 GB/s), algbw = bytes / t.  Collective: every rank calls it."""
        import time
        out = []
        if not self.active:
            return out
        dev = self.net.fp.grads.device
        n = self.world
        for b in self.buckets:
            buf = self.net.fp.grads[b.start:b.end].clone()
            for _ in range(warmup):
                dist.all_reduce(buf, group=self.group)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            dist.barrier(group=self.group)
            t0 = time.perf_counter()
            for _ in range(reps):
                dist.all_reduce(buf, group=self.group)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t = (time.perf_counter() - t0) / reps
            tt = torch.tensor([t], dtype=torch.float64, device=dev if dist.get_backend(self.group) == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=self.group)     # the slowest rank's view
            t = float(tt.item())
            out.append({"mb": round(b.nbytes / 2 ** 20, 4),
                        "layers": [self.net.spec.layers[i].name for i in b.layers],
                        "allreduce_us": round(t * 1e6, 2),
                        "busbw_GBps": round(2 * (n - 1) / n * b.nbytes / t / 1e9, 3),
                        "algbw_GBps": round(b.nbytes / t / 1e9, 3)})
        return out

    def broadcast_state(self, src: int = 0) -> None:
        """Make every replica start from the chief's parameters / slots / step."""
        if self.world == 1:
            return
        fp = self.net.fp
        for t in (fp.params, fp.ema, fp.mom, fp.step):
            dist.broadcast(t, src, group=self.group)
        fp.refresh_bf16()

    def global_stats(self) -> Dict[str, float]:
        """Average the last-step loss / accuracy over replicas (logging only)."""
        s = self.net.stats[4:7].clone()
        if self.world > 1:
            dist.all_reduce(s, group=self.group)
            s /= self.world
        v = s.tolist()
        return {"cross_entropy": v[0], "accuracy": v[1], "total_loss": v[2]}

    def describe(self) -> str:
        lines = [f"data parallel: world={self.world}, {len(self.buckets)} gradient bucket(s)"]
        for k, b in enumerate(self.buckets):
            names = [self.net.spec.layers[i].name for i in b.layers]
            lines.append(f"  bucket {k}: {b.nbytes / 1e6:.3f} MB [{', '.join(names)}] -> RCCL all-reduce "
                         f"(async, launched after {names[-1]} wgrad)")
        return "\n".join(lines)
