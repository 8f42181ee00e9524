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
* whether an all-reduce issued mid-backward actually overlaps is a question of CU
  residency, measured on one MI355X with an RCCL-footprint probe kernel launched on a
  second stream while each persistent compute kernel runs (``bench/dp_coresidency.py``,
  ``profiles/r5/dp_coresidency/``; first-block start as a fraction of the kernel):

  ====================================  ===========  ===========  ==============
  kernel (one resident wave)            probe 0 KB   16-32 KB     16-32 KB, R=8
  ====================================  ===========  ===========  ==============
  ``lenet_bwd_k`` (LeNet, 157 KB LDS)   0.14         0.94 (waits) 0.12
  ``lenet_band_fwd_k``                  0.76 (waits) 0.81 (waits) 0.18
  ``conv5_halo_k`` dgrad (ref conv2)    0.07         0.94 (waits) 0.06
  ``conv5_halo_wgrad_k`` (ref conv2)    0.07         0.08         0.08
  ``refc1_wgrad_k`` (ref conv1+norm1)   0.14         0.14         0.13
  ====================================  ===========  ===========  ==============

  so a collective that needs LDS cannot start beside the LeNet fused backward or the
  reference CNN's conv2 dgrad, and starts at once when the persistent grids leave
  ``R`` CUs free (``kernels.set_reserve_cus``: one per XCD);
* bucket plan (``plan_buckets``): buckets close once they reach the cap (bench / CLI
  default 0.125 MB) but never right before a CU-locking kernel (``HipNet.bucket_lockout``):
  there the all-reduce could only start after it, so it would just add one more
  latency-bound collective.  LeNet-5 (fused head + fused conv backward) therefore has ONE
  246 KB bucket at the end of backward -- its gradient is latency-bound on xGMI either
  way, and one collective is one latency -- and needs no reserve.  The reference CNN gets
  [softmax+local4] 0.8 MB, [local3] 12.85 MB (ring per-link bound: ~2·7/8·S / 153 GB/s
  ≈ 150 µs, issued after the local3 weight gradient with 1.2 ms of backward still to run)
  and [conv2+conv1] at the end;
* with world > 1 and more than one bucket, ``DataParallel`` reserves ``RESERVE_CUS`` = 8
  CUs from the persistent kernels for the whole step so the early buckets' all-reduce
  kernels are never locked out (cost per kernel: interleaved A/B in
  ``profiles/r5/dp_coresidency/``); one GPU and one-bucket plans reserve nothing.  The
  one-block-per-tile GEMMs size themselves for the CUs left too (``gemm256.hip``
  ``num_cus``): local3's forward (256 tiles = one round of 256 CUs, two of 248) goes back
  to gemm.hip's finer tiles, and the split-K weight gradient recounts its splits;
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


def plan_buckets(net, cap_bytes: int, lockout: Optional[set] = None) -> List[Bucket]:
    """Contiguous buckets in backward order, closed once they reach ``cap_bytes`` --
    except at a layer in ``lockout`` (default ``net.bucket_lockout``): the backward
    kernel right after that layer's grad-ready hook occupies every CU (a persistent,
    LDS-filling kernel), so an all-reduce issued there could not start before it ends
    and would only add one more latency-bound collective; the bucket grows on instead."""
    fp = net.fp
    spec = net.spec
    if lockout is None:
        lockout = set(getattr(net, "bucket_lockout", ()) or ())
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
        if (cur.nbytes >= cap_bytes and i not in lockout) or k == len(order) - 1:
            buckets.append(cur)
            cur = None
    return buckets


class DataParallel:
    # CUs the persistent compute kernels leave free while an early bucket's all-reduce may
    # be in flight (one per XCD; kernels.set_reserve_cus)
    RESERVE_CUS = 8

    def __init__(self, net, group=None, bucket_cap_mb: float = 1.0, overlap: bool = True,
                 world: Optional[int] = None, force_collectives: bool = False,
                 reserve_cus: Optional[int] = None):
        """``force_collectives``: issue the bucket all-reduces even with one rank (a
        one-GPU rehearsal of the RCCL path, e.g. hipGraph capture of the DP step).
        ``reserve_cus``: CUs kept free of the persistent kernels (None = auto:
        RESERVE_CUS when world > 1 and some bucket is all-reduced before the backward
        ends, else 0)."""
        self.net = net
        self.group = group
        if world is None:
            world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.world = world
        self.active = world > 1 or force_collectives
        self.buckets = plan_buckets(net, int(bucket_cap_mb * (1 << 20)))
        self.trigger = {b.layers[-1]: b for b in self.buckets}
        if reserve_cus is None:
            reserve_cus = self.RESERVE_CUS if (world > 1 and overlap and len(self.buckets) > 1) else 0
        self.reserve_cus = int(reserve_cus)
        dev = getattr(getattr(net, "fp", None), "params", None)
        if dev is not None and dev.device.type == "cuda":
            from ..ops._ext import kernels
            kernels().set_reserve_cus(self.reserve_cus)
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
        lines = [f"data parallel: world={self.world}, {len(self.buckets)} gradient bucket(s), "
                 f"{self.reserve_cus} CU(s) reserved for collectives"]
        for k, b in enumerate(self.buckets):
            names = [self.net.spec.layers[i].name for i in b.layers]
            lines.append(f"  bucket {k}: {b.nbytes / 1e6:.3f} MB [{', '.join(names)}] -> RCCL all-reduce "
                         f"(async, launched after {names[-1]} wgrad)")
        return "\n".join(lines)
