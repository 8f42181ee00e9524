"""hipGraph capture of a whole training step.

At small batches the MNIST step is a few µs of MFMA work spread over ~30
kernels, so host launch cost (~3-5 µs per launch) would dominate.  The
executor allocates every buffer up front and its kernels never allocate or
synchronise, so forward + backward + fused update + finalisation capture into
one hipGraph and replay with a single launch.  (The batch gather runs just
before replay, outside the graph, because its source slice moves every step.)

Data parallel (N > 1): the step's RCCL bucket all-reduces (issued from the
grads-ready hooks, ``async_op=True``, joined by stream waits) are captured with
it when asked (``--hip_graph_dp`` / ``bench.py --graph 1``): RCCL kernels become
graph nodes on the communicator's stream, so a small-batch DP step replays with
one launch.  Off by default: at the BASELINE batch (65536 / GPU) eager launches
already keep the GPU busy (profiles/r2/graph_vs_eager.md) and the 1..8-GPU curve
then runs one execution mode throughout.  Rehearsed on one GPU with a one-rank
RCCL group (tests/test_dp_graph_gpu.py).

With a process group up, capture runs in thread-local error mode: the RCCL
process group's watchdog thread keeps polling the events of earlier
collectives, and under the default global mode such a query during capture
fails the watchdog ("operation not permitted when stream is capturing").
"""
from __future__ import annotations

from typing import Callable

import torch


class StepGraph:
    def __init__(self, fn: Callable[[], None], warmup: int = 2):
        self.fn = fn
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        import torch.distributed as dist
        mode = "thread_local" if dist.is_available() and dist.is_initialized() else "global"
        with torch.cuda.graph(self.graph, capture_error_mode=mode):
            fn()
        torch.cuda.synchronize()

    def replay(self) -> None:
        self.graph.replay()
